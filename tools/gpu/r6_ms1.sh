#!/bin/bash
# one-plane-per-wave multi-scale sums (ms_rows1_kernel): tests, enhance-leg A/B against ms_rows_kernel, kernel stats
set -o pipefail
mkdir -p gpurun_out/r6
R=$GRAFT_REPO_ROOT
for bh in 16 20 24 32; do
  UPR_MSR1_BH=$bh timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "multiscale or multi_scale" > gpurun_out/r6/ms1_tests.log 2>&1 || { tail -30 gpurun_out/r6/ms1_tests.log; exit 1; }
  echo "BH $bh: $(tail -1 gpurun_out/r6/ms1_tests.log)"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_enhancers.py > gpurun_out/r6/ms1_tests2.log 2>&1 || { tail -30 gpurun_out/r6/ms1_tests2.log; exit 1; }
tail -1 gpurun_out/r6/ms1_tests2.log
: > gpurun_out/r6/ms1_ab.txt
for m in "1 16" "2 16" "2 20" "2 24" "2 32" "1 16" "2 16" "2 20"; do
  set -- $m; r=$(UPR_MS_ROWS=$1 UPR_MSR1_BH=$2 timeout -k 10 200 python bench.py --enhance --steps 50 --warmup 5 --no-traffic --cpu-seconds 0 --detail "" 2>/dev/null | grep '^{"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['multiscale']['avg_call_ms'], d['roofline']['avg_call_ms'])") || exit 1
  echo "UPR_MS_ROWS=$1 BH=$2 img/s, ms_call_ms, clahe_ms: $r" | tee -a gpurun_out/r6/ms1_ab.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/ms1_prof -o k --output-format csv -- python3 $R/bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $R/gpurun_out/r6/ms1_prof.log 2>&1 || exit 1
cut -c1-140 $R/gpurun_out/r6/ms1_prof/k_kernel_stats.csv
