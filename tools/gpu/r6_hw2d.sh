#!/bin/bash
# conv_hw2 fragment-read schedules (SCH 0/1/2) -- parity, then A/B vs hwide4
set -o pipefail
mkdir -p gpurun_out/r6
for v in 2 5; do
  UPR_HW2=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "conv2d_nhwc" > gpurun_out/r6/hw2d_tests_$v.log 2>&1 || { tail -30 gpurun_out/r6/hw2d_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r6/hw2d_tests_$v.log
done
: > gpurun_out/r6/hw2d_ab.txt
for v in 0 2 4 5 6 1 0 2 4 5; do
  echo "UPR_HW2=$v" >> gpurun_out/r6/hw2d_ab.txt
  UPR_HW2=$v timeout -k 10 120 python -u tools/convbench.py --shapes bneck,bneckr,aspp6,aspp18 --iters 40 --bufs 4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r6/hw2d_ab.txt || exit 1
done
cat gpurun_out/r6/hw2d_ab.txt
