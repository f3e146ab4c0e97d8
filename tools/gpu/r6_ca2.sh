#!/bin/bash
# content-aware v2 (fp32 Laplacian in LDS, consumer-side min/max): tests, bench, kernel stats
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_gpu_enhancers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/ca2_tests.log 2>&1 || { tail -40 gpurun_out/r6/ca2_tests.log; exit 1; }
tail -2 gpurun_out/r6/ca2_tests.log
timeout -k 10 200 python -u tools/enh_extra_bench.py > gpurun_out/r6/ca2_bench.json 2>&1 || { cat gpurun_out/r6/ca2_bench.json; exit 1; }
grep -v amdgpu gpurun_out/r6/ca2_bench.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6/ca2_prof -o ca2 -- python3 $GRAFT_REPO_ROOT/tools/enh_extra_bench.py > $GRAFT_REPO_ROOT/gpurun_out/r6/ca2_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r6/ca2_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/r6/ca2_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -c1-160 {}
