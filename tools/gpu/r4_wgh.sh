# training-kernel checks: the wgrad / conv-layer / stride-2 dgrad / AMP oracle tests, then the
# AMP weight-gradient A/B (lib/libupr_prev.so vs lib/libupr.so) on the training shapes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-wgh}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -q -k "${TK:-wgrad or conv_layer or stride2 or amp_autocast}" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -15 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for L in prev new; do
  if [ $L = prev ]; then export UPR_LIB=$GRAFT_REPO_ROOT/retinex-image-enhancement_amd/lib/libupr_prev.so; else unset UPR_LIB; fi
  echo $L >> $out/bench.txt
  timeout -k 10 120 python tools/wgrad_bench.py >> $out/bench.txt 2>&1 || exit $?
  timeout -k 10 120 python tools/wgrad_bench.py --dy16 --shapes w32,p128 >> $out/bench.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $out/bench.txt
