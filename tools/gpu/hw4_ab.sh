# hwide4 vs hwide3 on the bottleneck conv (same-box A/B) + parity tests of the conv families
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-hw4}
mkdir -p $out
UPR_HW4=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "conv2d_nhwc or fp16" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  UPR_HW4=0 timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck --iters 30 >> $out/bench.txt 2>&1 || exit $?
  UPR_HW4=1 timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck --iters 30 >> $out/bench.txt 2>&1 || exit $?
done
cat $out/bench.txt
