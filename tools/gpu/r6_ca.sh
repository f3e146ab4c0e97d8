#!/bin/bash
# content-aware fused saliency pass + cached letterbox taps: tests, then bench (fused vs three-kernel form)
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_gpu_enhancers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/ca_tests.log 2>&1 || { tail -40 gpurun_out/r6/ca_tests.log; exit 1; }
tail -2 gpurun_out/r6/ca_tests.log
UPR_CA_FUSED=0 timeout -k 10 200 python -u tools/enh_extra_bench.py > gpurun_out/r6/ca_bench_old.json 2>&1 || { cat gpurun_out/r6/ca_bench_old.json; exit 1; }
timeout -k 10 200 python -u tools/enh_extra_bench.py > gpurun_out/r6/ca_bench_new.json 2>&1 || { cat gpurun_out/r6/ca_bench_new.json; exit 1; }
grep -v amdgpu gpurun_out/r6/ca_bench_old.json gpurun_out/r6/ca_bench_new.json
