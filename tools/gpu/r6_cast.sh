#!/bin/bash
# which autocast convs cast their fp16 operand (UPR_TRACE_CAST) in one plain AMP train step
set -o pipefail
mkdir -p gpurun_out/r6
UPR_TRACE_CAST=1 timeout -k 10 300 python bench.py --train --amp --steps 1 --warmup 1 --cpu-seconds 0 --detail "" > gpurun_out/r6/cast.json 2> gpurun_out/r6/cast.err || { tail -20 gpurun_out/r6/cast.err; exit 1; }
grep upr_cast gpurun_out/r6/cast.err | sort | uniq -c
