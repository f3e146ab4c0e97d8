# dilated hwide4 (ASPP branches) parity + same-box A/B vs the gathered wide kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-hw4dl}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "conv2d_nhwc" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    echo "UPR_HW4_DIL=$v" >> $out/bench.txt
    UPR_HW4_DIL=$v timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes aspp6,aspp12,aspp18 --iters 30 >> $out/bench.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $out/bench.txt
