#!/bin/bash
# preact+ASPP AMP train leg (stderr kept)
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python bench.py --train --amp --variant preact_aspp --steps 10 --warmup 2 --cpu-seconds 0 --detail "" > gpurun_out/r6/aspp_train.json 2> gpurun_out/r6/aspp_train.err
rc=$?; tail -30 gpurun_out/r6/aspp_train.err | grep -v amdgpu.ids; grep -h '^{"metric"' gpurun_out/r6/aspp_train.json | cut -c1-300; exit $rc
