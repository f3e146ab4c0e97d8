#!/bin/bash
# the fp16-only stores regression test (bitwise on / off), the training tests, the preact+ASPP train leg
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_train.py -k "fp16_only_stores" > gpurun_out/r6/fp16only_test.log 2>&1 || { tail -40 gpurun_out/r6/fp16only_test.log; exit 1; }
grep -h "PASSED\|FAILED\|passed\|failed" gpurun_out/r6/fp16only_test.log | tail -2
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_bn_parity.py tests/test_gpu_modules.py > gpurun_out/r6/fp16only_tests.log 2>&1 || { tail -40 gpurun_out/r6/fp16only_tests.log; exit 1; }
tail -1 gpurun_out/r6/fp16only_tests.log
timeout -k 10 300 python bench.py --train --amp --variant preact_aspp --steps 10 --warmup 2 --cpu-seconds 0 --detail "" 2>/dev/null | grep '^{"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('preact_aspp img/s', d['value'], 'step', r['step_ms'], 'conv', r['conv_ms'], 'nonconv', r['non_conv_ms'])" || exit 1
