# training GPU tests (train + modules) and the AMP train bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sh16
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_modules.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sh16/tests.log 2>&1
rc=$?; tail -3 gpurun_out/sh16/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/sh16/train.json 2> gpurun_out/sh16/train.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/sh16/train.json').read().strip().splitlines()[-1]); print('train amp', round(d['value'],1), 'img/s', round(d['ms_per_step'],2), 'ms')"
