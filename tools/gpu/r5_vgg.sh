#!/bin/bash
# VGG-shape convs: halo-tiled forms vs the gathered kernel (UPR_HALO=0)
set -e
mkdir -p gpurun_out
S=vgg1,vgg21,vgg2,vgg31,vgg3,dec3p,enc2c2,bneck
timeout -k 10 240 python -u tools/convbench.py --shapes $S --bufs 4 --iters 30 > gpurun_out/r5_vgg_halo.txt 2>&1
UPR_HALO=0 timeout -k 10 240 python -u tools/convbench.py --shapes $S --bufs 4 --iters 30 > gpurun_out/r5_vgg_gath.txt 2>&1
timeout -k 10 240 python -u tools/convbench.py --shapes $S --bufs 4 --iters 30 >> gpurun_out/r5_vgg_halo.txt 2>&1
UPR_HALO=0 timeout -k 10 240 python -u tools/convbench.py --shapes $S --bufs 4 --iters 30 >> gpurun_out/r5_vgg_gath.txt 2>&1
