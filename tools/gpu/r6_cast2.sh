#!/bin/bash
# residual-head masked gradient with its fp16 copy: training tests, cast trace, train leg
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_bn_parity.py > gpurun_out/r6/cast2_tests.log 2>&1 || { tail -40 gpurun_out/r6/cast2_tests.log; exit 1; }
tail -1 gpurun_out/r6/cast2_tests.log
UPR_TRACE_CAST=1 timeout -k 10 300 python bench.py --train --amp --steps 1 --warmup 1 --cpu-seconds 0 --detail "" > gpurun_out/r6/cast2.json 2> gpurun_out/r6/cast2.err || { tail -20 gpurun_out/r6/cast2.err; exit 1; }
grep upr_cast gpurun_out/r6/cast2.err | sort | uniq -c || true
for i in 1 2; do
timeout -k 10 300 python bench.py --train --amp --steps 10 --warmup 2 --cpu-seconds 0 --detail "" 2>/dev/null | grep '^{"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('img/s', d['value'], 'step', r['step_ms'], 'conv', r['conv_ms'], 'nonconv', r['non_conv_ms'], 'parity', d['parity']['pass'])" || exit 1
done
