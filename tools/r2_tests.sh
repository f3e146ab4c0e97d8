# full -m gpu suite (no -x: report every failure), log under gpurun_out/r2t
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2t
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r2t/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/r2t/gpu_tests.log
exit $rc
