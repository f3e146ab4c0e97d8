# wide32 32-wide tiles: parity + A/B vs the halo kernel
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/n32
UPR_WIDE32_N32=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "conv2d or fp32 or rect or crop" > gpurun_out/n32/tests.log 2>&1 || { tail -30 gpurun_out/n32/tests.log; exit 1; }
tail -2 gpurun_out/n32/tests.log
for c in 0 1 2 3; do
  UPR_WIDE32_N32=$c timeout -k 10 120 python tools/convbench.py --dtype fp32 --shapes dec1,d2 --iters 10 > gpurun_out/n32/c$c.txt 2>&1 || exit 1
  echo "n32=$c"; grep fp32 gpurun_out/n32/c$c.txt
done
