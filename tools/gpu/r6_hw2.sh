#!/bin/bash
# round 6: two-blocks-per-CU 3x3 conv (conv_hw2.hip) -- parity of the conv cases, then A/B vs hwide4
set -o pipefail
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "conv2d_nhwc" > gpurun_out/r6/hw2_tests.log 2>&1 || { tail -30 gpurun_out/r6/hw2_tests.log; exit 1; }
tail -3 gpurun_out/r6/hw2_tests.log
for v in 0 1 2 3 0 1; do
  echo "UPR_HW2=$v" >> gpurun_out/r6/hw2_ab.txt
  UPR_HW2=$v timeout -k 10 120 python -u tools/convbench.py --shapes bneck,bneckr,aspp6,aspp12,aspp18 --iters 40 --bufs 4 >> gpurun_out/r6/hw2_ab.txt 2>&1 || exit 1
done
cat gpurun_out/r6/hw2_ab.txt
