# Same-box A/B of conv kernels: conv parity (the -m gpu conv cases, under the B env), then
# tools/convbench.py on $SHAPES alternating env A ($AENV) and env B ($BENV) $ROUNDS times.
#   AENV="UPR_HW4_DS=0" BENV="UPR_HW4_DS=1" SHAPES=bneck,bneckr bash tools/gpu/conv_ab.sh
# (the round-3 direct-store / dilated / 2-row-tile A/Bs in profiles/r3_*_ab.txt ran this way)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-convab}
mkdir -p $out
env ${BENV:-UPR_X=1} timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k conv2d_nhwc --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq ${ROUNDS:-2}); do
  for side in A B; do
    if [ $side = A ]; then e="${AENV:-UPR_X=0}"; else e="${BENV:-UPR_X=1}"; fi
    echo "$side: $e" >> $out/bench.txt
    env $e timeout -k 10 120 python tools/convbench.py --dtype ${DTYPE:-fp16} --shapes ${SHAPES:-bneck} --iters 30 >> $out/bench.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $out/bench.txt
