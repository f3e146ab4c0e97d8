# halo-tiled wide kernel: conv op parity, A/B convbench (UPR_WIDE_HALO=0/1), fp16 preact+ASPP breakdown
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/halo
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv2d or full_size or fp16" > gpurun_out/halo/tests.log 2>&1
rc=$?; tail -3 gpurun_out/halo/tests.log; [ $rc -eq 0 ] || exit $rc
for h in 0 1 0 1; do
UPR_WIDE_HALO=$h timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,dec3,enc2c2 --iters 30 >> gpurun_out/halo/cb_$h.log 2>&1 || exit 1
done
cat gpurun_out/halo/cb_0.log gpurun_out/halo/cb_1.log
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 10 > gpurun_out/halo/fp16.json 2> gpurun_out/halo/fp16.err || exit $?
cat gpurun_out/halo/fp16.json
