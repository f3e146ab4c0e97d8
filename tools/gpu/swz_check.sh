# halo swizzle table change: conv parity on every halo-kernel route + timing + bank-conflict PMC
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-swz}
mkdir -p $out
for e in "UPR_X=1" "UPR_HW4=0" "UPR_WIDE_HALO=1"; do
  env $e timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k conv2d_nhwc --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
  rc=$?; echo "$e: $(tail -1 $out/tests.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes aspp6,aspp12,aspp18,bneck,bneckr,dec3,dec3p --iters 30 > $out/time.txt 2>&1 || exit $?
grep -v amdgpu $out/time.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA --kernel-trace -d gpurun_out/swz_pmc -o p --output-format csv -- python3 tools/convbench.py --dtype fp16 --shapes aspp6,bneck,dec3 --iters 3 > $out/pmc.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/swz_pmc --match hwide > $out/pmc_summary.txt
grep -E "==|BANK" $out/pmc_summary.txt
