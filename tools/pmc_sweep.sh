# rocprofv3 counter passes over one conv shape: PMC_CFGS="4,1 4,2" PMC_DT=fp32 PMC_SHAPE=dec1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { # name cfg dtype shape counters...
  local name=$1 cfg=$2 dt=$3 shape=$4; shift 4
  UPR_HALO=$cfg timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace -T -d gpurun_out/pmc_$name -o p --output-format csv -- python3 tools/convbench.py --dtype $dt --shapes $shape --iters 3 > gpurun_out/pmc_$name.log 2>&1 || exit 1
}
DT=${PMC_DT:-fp32}; SH=${PMC_SHAPE:-dec1}
DEF="4,1 4,2"
for cfg in ${PMC_CFGS:-$DEF}; do
  c=${DT}_${SH}_${cfg/,/_}
  run a_$c $cfg $DT $SH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  run b_$c $cfg $DT $SH SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
done
