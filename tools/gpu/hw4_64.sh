# hwide4 2-row tiles for the 64 -> 64 W 256 convs (dec2) vs the row ring: parity + same-box A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-hw464}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k conv2d_nhwc --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    echo "UPR_HW4_64=$v" >> $out/bench.txt
    UPR_HW4_64=$v timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes dec2p,dec2 --iters 30 >> $out/bench.txt 2>&1 || exit $?
  done
done
grep -v amdgpu $out/bench.txt
