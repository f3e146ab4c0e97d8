# hwide4 direct-store epilogue (UPR_HW4_DS=1, default) vs the LDS epilogue: conv parity + same-box A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-hw4ds}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for ds in 0 1; do
    echo "UPR_HW4_DS=$ds" >> $out/bench.txt
    UPR_HW4_DS=$ds timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,bneckr --iters 30 >> $out/bench.txt 2>&1 || exit $?
  done
done
cat $out/bench.txt
