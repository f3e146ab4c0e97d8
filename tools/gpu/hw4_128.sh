# hwide4 (direct-store) for the dec3 W 128 convs (UPR_HW4_128=1) vs hwide3: conv parity + same-box A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-hw4128}
mkdir -p $out
UPR_HW4_128=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "conv2d_nhwc or fp16" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    echo "UPR_HW4_128=$v" >> $out/bench.txt
    UPR_HW4_128=$v timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes dec3,dec3p --iters 30 >> $out/bench.txt 2>&1 || exit $?
  done
done
cat $out/bench.txt
