#!/bin/bash
# hwide4 bottleneck-form timing ablations (UPR_HW4_ABL: 1 no main-loop DMA, 4 no epilogue, 5 both, 7 + no LDS reads)
set -o pipefail
mkdir -p gpurun_out/r6
: > gpurun_out/r6/hw4_abl.txt
for a in 0 1 4 5 7 0 1 4 5 7; do
  echo "UPR_HW4_ABL=$a" >> gpurun_out/r6/hw4_abl.txt
  UPR_HW2=0 UPR_HW4_ABL=$a timeout -k 10 120 python -u tools/convbench.py --shapes bneck --iters 40 --bufs 4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r6/hw4_abl.txt || exit 1
done
cat gpurun_out/r6/hw4_abl.txt
