#!/bin/bash
# multi-scale sums after the fma / branch-free accumulate change: tests + kernel stats + enhance leg
set -o pipefail
mkdir -p gpurun_out/r6
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "multiscale or multi_scale" > gpurun_out/r6/ms2_tests.log 2>&1 || { tail -30 gpurun_out/r6/ms2_tests.log; exit 1; }
tail -1 gpurun_out/r6/ms2_tests.log
for i in 1 2; do
timeout -k 10 200 python bench.py --enhance --steps 50 --warmup 5 --no-traffic --cpu-seconds 0 --detail "" 2>/dev/null | grep '^{"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('img/s', d['value'], 'ms_call', d['roofline']['multiscale']['avg_call_ms'], 'clahe', d['roofline']['avg_call_ms'])" || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/ms2_prof -o k --output-format csv -- python3 $R/bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $R/gpurun_out/r6/ms2_prof.log 2>&1 || exit 1
cut -c1-120 $R/gpurun_out/r6/ms2_prof/k_kernel_stats.csv | grep -v at::native
