#!/bin/bash
# ms_rows band height / prefetch A/B (fp32): per-scale sums test per variant, then the enhance leg's multiscale call time
set -o pipefail
mkdir -p gpurun_out/r6
: > gpurun_out/r6/msr_ab.txt
for v in "16 2" "8 2" "8 3" "16 1" "16 3" "32 2" "16 2" "8 2"; do
  set -- $v
  UPR_MSR_BH=$1 UPR_MSR_PF=$2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "multiscale" > gpurun_out/r6/msr_t.log 2>&1 || { tail -20 gpurun_out/r6/msr_t.log; exit 1; }
  r=$(UPR_MSR_BH=$1 UPR_MSR_PF=$2 timeout -k 10 200 python bench.py --enhance --steps 50 --warmup 5 --no-traffic --cpu-seconds 0 --detail "" 2>/dev/null | grep '^{"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['multiscale']['avg_call_ms'], d['roofline']['avg_call_ms'])") || exit 1
  echo "BH $1 PF $2 tests $(tail -1 gpurun_out/r6/msr_t.log | cut -c1-40) | img/s, ms_call_ms, clahe_ms: $r" | tee -a gpurun_out/r6/msr_ab.txt
done
