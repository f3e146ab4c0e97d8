#!/bin/bash
# FAM fp16-only branch outputs in the AMP training step: training tests, then the train leg
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_bn_parity.py > gpurun_out/r6/fam16_tests.log 2>&1 || { tail -40 gpurun_out/r6/fam16_tests.log; exit 1; }
tail -1 gpurun_out/r6/fam16_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --train --amp --steps 10 --warmup 2 --cpu-seconds 0 --detail "" 2>/dev/null | grep '^{"metric"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('img/s', d['value'], 'step', r['step_ms'], 'conv', r['conv_ms'], 'nonconv', r['non_conv_ms'], 'parity', json.dumps(d.get('parity'))[:300])" || exit 1
done
