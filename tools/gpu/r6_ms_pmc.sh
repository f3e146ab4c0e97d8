#!/bin/bash
# ms_rows_kernel SQ counters (one pass) over the enhance leg + the new content-aware shape test
set -o pipefail
mkdir -p gpurun_out/r6
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_enhancers.py -k content_aware > gpurun_out/r6/ms_pmc_tests.log 2>&1 || { tail -30 gpurun_out/r6/ms_pmc_tests.log; exit 1; }
tail -1 gpurun_out/r6/ms_pmc_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d $R/gpurun_out/r6/ms_pmc -o p --output-format csv -- python3 $R/bench.py --enhance --steps 10 --warmup 2 --no-traffic --cpu-seconds 0 --detail "" > $R/gpurun_out/r6/ms_pmc.log 2>&1 || { tail -20 $R/gpurun_out/r6/ms_pmc.log; exit 1; }
f=$(find $R/gpurun_out/r6/ms_pmc -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:50]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVE_CYCLES": n[k] += 1
for k, d in acc.items():
    if "upr::" in k:
        print(k, n[k], {c: round(v / max(n[k], 1)) for c, v in sorted(d.items())})
PY
