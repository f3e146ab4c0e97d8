# multi-scale single pass re-check (tests + enhance leg + kernel stats), then PMC passes over the
# narrow-N fp16 ring convs (dec1p 32->32 @512^2, fam_h 32->64 @512^2, dec2p 64->64 @256^2)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5m}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "multiscale" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/profE -o p --output-format csv -- python3 bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $out/enh_prof.json 2>&1 || exit $?
SH=${PMC_SHAPES:-dec1p,fam_h,dec2p}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $out/pmc_a -o p --output-format csv -- python3 tools/convbench.py --dtype fp16 --shapes $SH --iters 3 > $out/pmc_a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace -d $out/pmc_b -o p --output-format csv -- python3 tools/convbench.py --dtype fp16 --shapes $SH --iters 3 > $out/pmc_b.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY --kernel-trace -d $out/pmc_c -o p --output-format csv -- python3 tools/convbench.py --dtype fp16 --shapes $SH --iters 3 > $out/pmc_c.log 2>&1 || exit 1
python3 tools/pmc_summary.py $out/pmc_a $out/pmc_b $out/pmc_c > $out/pmc_summary.txt
timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes $SH,dec1 --iters 30 > $out/convbench.txt 2>&1 || exit 1
cat $out/convbench.txt
