# dilated-hwide4 bank fix check + ring kernel timing and PMC
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-dlring}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k conv2d_nhwc --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes aspp6,aspp12,aspp18,bneck,dec1p,dec1,fam_h,dec2p,dec2 --iters 20 > $out/time.txt 2>&1 || exit $?
grep -v amdgpu $out/time.txt
PMC_SHAPES=aspp6,dec1p,dec1,fam_h,dec2p bash tools/gpu/pmc_conv.sh > /dev/null || exit $?
cp gpurun_out/pmcr_summary.txt $out/pmc_summary.txt
