# loss modules + training tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/loss
timeout -k 10 500 python -u -m pytest tests/test_gpu_losses.py tests/test_gpu_train.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/loss/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|grad\[" gpurun_out/loss/tests.log | tail -60
exit $rc
