# 64-pixel ring strips for the plain 64 -> 64 conv: conv parity + A/B (UPR_RING_WIDE64)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w64
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv2d or fp16 or full_size" > gpurun_out/w64/tests.log 2>&1
rc=$?; tail -2 gpurun_out/w64/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for w in 0 1; do
echo "w64=$w $(UPR_RING_WIDE64=$w timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes dec2p --iters 30 2>/dev/null)" >> gpurun_out/w64/cb.log || exit 1
done; done
cat gpurun_out/w64/cb.log
