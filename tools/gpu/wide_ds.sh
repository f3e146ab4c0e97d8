# gathered wide kernel direct-store epilogue (UPR_WIDE_DS=1, default) vs LDS epilogue: parity + same-box A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-wideds}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    echo "UPR_WIDE_DS=$v" >> $out/bench.txt
    UPR_WIDE_DS=$v timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes enc2s2,enc2c2,enc3s2,fuse,aspp6 --iters 30 >> $out/bench.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $out/bench.txt
