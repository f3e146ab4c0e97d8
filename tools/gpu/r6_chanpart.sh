#!/bin/bash
# channel-statistics loads in flight: training tests, then the train leg's kernel stats (chan_part rows)
set -o pipefail
mkdir -p gpurun_out/r6
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_bn_parity.py > gpurun_out/r6/chanpart_tests.log 2>&1 || { tail -40 gpurun_out/r6/chanpart_tests.log; exit 1; }
tail -1 gpurun_out/r6/chanpart_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/chanpart_prof -o k --output-format csv -- python3 $R/bench.py --train --amp --steps 8 --warmup 2 --cpu-seconds 0 --detail "" > $R/gpurun_out/r6/chanpart_prof.log 2>&1 || { tail -20 $R/gpurun_out/r6/chanpart_prof.log; exit 1; }
grep -h '^{"metric"' $R/gpurun_out/r6/chanpart_prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('img/s (profiled)', d['value'])"
python3 - $R/gpurun_out/r6/chanpart_prof/k_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'chan_part' in r['Name'] or 'bn_bwd_apply4' in r['Name']:
        print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
