# hwide4 direct-store (bottleneck + dec3 W 128) parity and timing; A/B vs the LDS epilogue / hwide3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-hw4ab2}
mkdir -p $out
UPR_HW4_128=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  echo "base (LDS epilogue, dec3 on hwide3)" >> $out/bench.txt
  UPR_HW4_DS=0 timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,bneckr,dec3,dec3p --iters 30 >> $out/bench.txt 2>&1 || exit $?
  echo "direct store (dec3 on hwide4)" >> $out/bench.txt
  UPR_HW4_128=1 timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,bneckr,dec3,dec3p --iters 30 >> $out/bench.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $out/bench.txt
