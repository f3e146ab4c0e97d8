# training-path GPU tests (run on the GPU box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tr
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 200 --timeout-method thread > gpurun_out/tr/train_tests.log 2>&1
