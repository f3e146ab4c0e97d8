#!/bin/bash
# content-aware kernel stats + one SQ counter pass over the same bench
set -o pipefail
mkdir -p gpurun_out/r6
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_enhancers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/ca3_tests.log 2>&1 || { tail -40 gpurun_out/r6/ca3_tests.log; exit 1; }
tail -2 gpurun_out/r6/ca3_tests.log
timeout -k 10 200 python -u tools/enh_extra_bench.py 2>&1 | grep -v amdgpu | head -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/ca3_prof -o k --output-format csv -- python3 $R/tools/enh_extra_bench.py > $R/gpurun_out/r6/ca3_prof.log 2>&1 || { tail -20 $R/gpurun_out/r6/ca3_prof.log; exit 1; }
find $R/gpurun_out/r6/ca3_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -c1-150 {}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $R/gpurun_out/r6/ca3_pmc -o p --output-format csv -- python3 $R/tools/enh_extra_bench.py > $R/gpurun_out/r6/ca3_pmc.log 2>&1 || { tail -20 $R/gpurun_out/r6/ca3_pmc.log; exit 1; }
f=$(find $R/gpurun_out/r6/ca3_pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVE_CYCLES": n[k] += 1
for k, d in acc.items():
    if "ca_" in k:
        print(k, n[k], {c: round(v / max(n[k], 1)) for c, v in sorted(d.items())})
PY
