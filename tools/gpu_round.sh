# train tests, then inference GPU tests, then fp16 breakdown (run on the GPU box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tr
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -v --timeout 200 --timeout-method thread > gpurun_out/tr/train_tests.log 2>&1
rc=$?
echo "train tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_train.py > gpurun_out/tr/gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 3 > gpurun_out/tr/fp16pa.json 2> gpurun_out/tr/fp16pa.err
