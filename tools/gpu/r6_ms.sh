#!/bin/bash
# multi-scale register-streaming pass: parity, then the enhance leg A/B (UPR_MS_ROWS=0: tiled ms_sums3) with kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -o pipefail
out=gpurun_out/${CK:-r6ms}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "multiscale" tests/test_gpu_enhancers.py > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || { tail -40 $out/tests.log; exit $rc; }
for m in 0 1; do
  UPR_MS_ROWS=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/pe$m -o p --output-format csv -- python3 bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $out/enh$m.json 2>&1 || exit $?
  find $out/pe$m -name "*kernel_stats.csv" -exec cp {} $out/enhance_kernel_stats_rows$m.csv \; ; rm -rf $out/pe$m
  echo "UPR_MS_ROWS=$m"
  python3 -c "
import csv
for r in csv.DictReader(open('$out/enhance_kernel_stats_rows$m.csv')):
    print('  ', r['Name'][:60], r['Calls'], r['AverageNs'])
"
  grep -o '"value": [0-9.]*' $out/enh$m.json | head -1
done
# content-aware / letterbox kernel stats
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/pc -o p --output-format csv -- python3 tools/enh_extra_bench.py > $out/ca_bench.json 2>&1 || exit $?
find $out/pc -name "*kernel_stats.csv" -exec cp {} $out/ca_kernel_stats.csv \; ; rm -rf $out/pc
python3 -c "
import csv
for r in csv.DictReader(open('$out/ca_kernel_stats.csv')):
    print('  ', r['Name'][:60], r['Calls'], r['AverageNs'])
"
