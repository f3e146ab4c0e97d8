# PMC passes over the fp16 ring kernels (dec1, fam_h, dec2) and the halo wide kernel (bneck)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SH=${PMC_SHAPES:-dec1,fam_h,dec2,bneck}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmcr_a -o p --output-format csv -- python3 tools/convbench.py --dtype ${PMC_DTYPE:-fp16} --shapes $SH --iters 3 > gpurun_out/pmcr_a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/pmcr_b -o p --output-format csv -- python3 tools/convbench.py --dtype ${PMC_DTYPE:-fp16} --shapes $SH --iters 3 > gpurun_out/pmcr_b.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/pmcr_c -o p --output-format csv -- python3 tools/convbench.py --dtype ${PMC_DTYPE:-fp16} --shapes $SH --iters 3 > gpurun_out/pmcr_c.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmcr_a gpurun_out/pmcr_b gpurun_out/pmcr_c > gpurun_out/pmcr_summary.txt
cat gpurun_out/pmcr_summary.txt
