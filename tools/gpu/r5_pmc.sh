# PMC passes over the conv kernels on convbench shapes (4 HBM-resident input copies): issue / wait / MFMA
# busy, instruction mix + LDS, HBM bytes (FETCH_SIZE, WRITE_SIZE) -- one counter group per pass
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5pmc}
mkdir -p $out
SH=${PMC_SHAPES:-bneck,aspp6,aspp18,fuse1k,enc3s2,enc2s2,dec2p,dec1p,fam_h}
CB="tools/convbench.py --dtype fp16 --shapes $SH --iters 2 --bufs 4"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $out/pmc_a -o p --output-format csv -- python3 $CB > $out/pmc_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace -d $out/pmc_b -o p --output-format csv -- python3 $CB > $out/pmc_b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/pmc_c -o p --output-format csv -- python3 $CB > $out/pmc_c.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/pmc_d -o p --output-format csv -- python3 $CB > $out/pmc_d.log 2>&1 || exit 1
python3 tools/pmc_summary.py $out/pmc_a $out/pmc_b $out/pmc_c $out/pmc_d > $out/pmc_summary.txt
timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes $SH --iters 20 --bufs 4 > $out/convbench_bufs4.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/convbench_bufs4.txt
grep -E "^==|wait_any|MFMA_BUSY|FETCH|WRITE_SIZE" $out/pmc_summary.txt | head -80
