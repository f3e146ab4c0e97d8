# training GPU tests + train bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tr2
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tr2/tests.log 2>&1 || { tail -40 gpurun_out/tr2/tests.log; exit 1; }
tail -2 gpurun_out/tr2/tests.log
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/tr2/train.json 2> gpurun_out/tr2/train.err || { tail -5 gpurun_out/tr2/train.err; exit 1; }
cat gpurun_out/tr2/train.json
