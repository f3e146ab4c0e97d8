# A/B of the wide-conv main loops + counter passes on the bottleneck shape
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ring2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "conv2d or fp16 or full_size" > $O/tests.log 2>&1 || exit 1
for k in 0 1 2; do
UPR_WIDE_KIND=$k timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,aspp6,aspp18,fuse,enc3s2,enc2s2,dec3 --iters 20 > $O/cb_$k.log 2>&1 || exit 1
done
for k in 0 1; do
UPR_WIDE_KIND=$k timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pa_$k -o p --output-format csv -- python3 tools/convbench.py --dtype fp16 --shapes bneck --iters 3 > $O/pa_$k.log 2>&1 || exit 1
UPR_WIDE_KIND=$k timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -d $O/pb_$k -o p --output-format csv -- python3 tools/convbench.py --dtype fp16 --shapes bneck --iters 3 > $O/pb_$k.log 2>&1 || exit 1
done
