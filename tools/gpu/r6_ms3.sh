#!/bin/bash
# ms_rows1 fma / branch-free accumulate A/B on one box (UPR_MS1_FMA=0 the previous form), kernel time from rocprofv3
set -o pipefail
mkdir -p gpurun_out/r6
R=$GRAFT_REPO_ROOT
for f in; do
UPR_MS1_FMA=$f timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "multiscale or multi_scale" > gpurun_out/r6/ms3_tests.log 2>&1 || { tail -30 gpurun_out/r6/ms3_tests.log; exit 1; }
echo "FMA=$f $(tail -1 gpurun_out/r6/ms3_tests.log)"
done
cd /tmp && export TMPDIR=/tmp
: > $R/gpurun_out/r6/ms3_ab.txt
for f in 0 1 0 1 0 1; do
  rm -rf $R/gpurun_out/r6/ms3_prof
  UPR_MS1_FMA=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/ms3_prof -o k --output-format csv -- python3 $R/bench.py --enhance --steps 30 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $R/gpurun_out/r6/ms3_prof.log 2>&1 || exit 1
  echo "FMA=$f $(python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/r6/ms3_prof/k_kernel_stats.csv')):
    if 'ms_rows1' in r['Name'] or 'ms_fin1' in r['Name']: print(r['Name'][:40], r['Calls'], r['AverageNs'], end=' | ')
")" | tee -a $R/gpurun_out/r6/ms3_ab.txt
done
