#!/bin/bash
# round 6: conv_hw2 schedule variants (burst vs spread DMA issue) -- parity + A/B vs hwide4, then PMC
set -o pipefail
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
for v in 4 6; do
  UPR_HW2=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "conv2d_nhwc" > gpurun_out/r6/hw2b_tests_$v.log 2>&1 || { tail -30 gpurun_out/r6/hw2b_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r6/hw2b_tests_$v.log
done
: > gpurun_out/r6/hw2b_ab.txt
for v in 0 1 3 4 5 6 0 4 5 6; do
  echo "UPR_HW2=$v" >> gpurun_out/r6/hw2b_ab.txt
  UPR_HW2=$v timeout -k 10 120 python -u tools/convbench.py --shapes bneck,bneckr,aspp6,aspp18 --iters 40 --bufs 4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r6/hw2b_ab.txt || exit 1
done
cat gpurun_out/r6/hw2b_ab.txt
V=${PV:-6} bash tools/gpu/r6_pmc_hw2.sh 2>&1 | grep -E "^==|wait_any|per MFMA|MFMA_BUSY|BANK|LDS_IDX|SQ_WAVES|BUSY_CYCLES|WAVE_CYCLES|INSTS_LDS|INSTS_MFMA"
