#!/bin/bash
# PMC passes: hwide4 (UPR_HW2=0) vs conv_hw2 (UPR_HW2=${V:-3}) on bneck / aspp6
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r6pmc}
mkdir -p $out
SH=${PMC_SHAPES:-bneck,aspp6}
CB="tools/convbench.py --dtype fp16 --shapes $SH --iters 2 --bufs 4"
for v in 0 ${V:-3}; do
  export UPR_HW2=$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $out/v$v/pmc_a -o p --output-format csv -- python3 $CB > $out/v$v.pmc_a.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace -d $out/v$v/pmc_b -o p --output-format csv -- python3 $CB > $out/v$v.pmc_b.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY --kernel-trace -d $out/v$v/pmc_c -o p --output-format csv -- python3 $CB > $out/v$v.pmc_c.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $out/v$v/pmc_a $out/v$v/pmc_b $out/v$v/pmc_c > $out/v$v.summary.txt
  echo "=== UPR_HW2=$v"; cat $out/v$v.summary.txt
done
