# fp32 wide kernel: parity (conv ops + model), A/B per shape, bench breakdown
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w32
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py -x -q --timeout 200 --timeout-method thread -k "conv2d or fp32 or forward or configs or predict or rect or crop or full_size" > gpurun_out/w32/tests.log 2>&1 || { tail -30 gpurun_out/w32/tests.log; exit 1; }
tail -3 gpurun_out/w32/tests.log
S=bneck,enc1s2,enc2s2,enc3s2,fam_h,dec2,dec3,aspp18,fuse
UPR_WIDE32=0 timeout -k 10 120 python tools/convbench.py --dtype fp32 --shapes $S --iters 10 > gpurun_out/w32/cb_off.txt 2>&1 || exit 1
timeout -k 10 120 python tools/convbench.py --dtype fp32 --shapes $S --iters 10 > gpurun_out/w32/cb_on.txt 2>&1 || exit 1
paste gpurun_out/w32/cb_off.txt gpurun_out/w32/cb_on.txt
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --breakdown --steps 5 > gpurun_out/w32/bd.json 2> gpurun_out/w32/bd.err || exit 1
cat gpurun_out/w32/bd.json
