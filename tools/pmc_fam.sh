# PMC counters of the fp16 preact+ASPP forward (1 timed step), per kernel. OUT=<dir>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-pmc}; mkdir -p $O
run() { local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $O/$n -o p --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --steps 1 --warmup 1 --cpu-seconds 0 --no-traffic --no-profile > $O/$n.log 2>&1 || exit 1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
run c FETCH_SIZE
run d WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
