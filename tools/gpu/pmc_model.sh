# rocprofv3 counter passes over one bench.py forward (all kernels); PMC_PREC=fp32|fp16
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PREC=${PMC_PREC:-fp32}
run() { # name counters...
  local name=$1; shift
  timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmcm_${PREC}_$name -o p --output-format csv -- python3 bench.py --precision $PREC --variant ${PMC_VARIANT:-plain} --steps 1 --warmup 1 --no-traffic --no-profile --cpu-seconds 0 > gpurun_out/pmcm_${PREC}_$name.log 2>&1 || exit 1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
