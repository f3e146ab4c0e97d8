#!/bin/bash
# conv_hw2 operand-contiguity ablations (modes 7-9: garbage results, timing only)
set -o pipefail
mkdir -p gpurun_out/r6
: > gpurun_out/r6/hw2c_ab.txt
for v in 0 3 7 8 9 0 3 7 8 9; do
  echo "UPR_HW2=$v" >> gpurun_out/r6/hw2c_ab.txt
  UPR_HW2=$v timeout -k 10 120 python -u tools/convbench.py --shapes bneck,aspp6,aspp18 --iters 40 --bufs 4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r6/hw2c_ab.txt || exit 1
done
cat gpurun_out/r6/hw2c_ab.txt
