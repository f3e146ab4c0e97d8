#!/bin/bash
# (1) conv_hw2 schedules A/B (parity first); (2) hwide4 with pinned fragment reads vs the previous build
set -o pipefail
bash tools/gpu/r6_hw2d.sh || exit 1
: > gpurun_out/r6/hw4_sgb_ab.txt
for i in 1 2; do
  echo "A prev hwide4" >> gpurun_out/r6/hw4_sgb_ab.txt
  UPR_HW2=0 UPR_LIB=$GRAFT_REPO_ROOT/retinex-image-enhancement_amd/lib/libupr_prev.so timeout -k 10 120 python tools/convbench.py --shapes bneck,bneckr,aspp6,aspp18,dec3,dec3p,enc3s2,fuse1k,a1x1 --iters 30 --bufs 4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r6/hw4_sgb_ab.txt || exit 1
  echo "B pinned hwide4" >> gpurun_out/r6/hw4_sgb_ab.txt
  UPR_HW2=0 timeout -k 10 120 python tools/convbench.py --shapes bneck,bneckr,aspp6,aspp18,dec3,dec3p,enc3s2,fuse1k,a1x1 --iters 30 --bufs 4 2>&1 | grep -v amdgpu.ids >> gpurun_out/r6/hw4_sgb_ab.txt || exit 1
done
cat gpurun_out/r6/hw4_sgb_ab.txt
