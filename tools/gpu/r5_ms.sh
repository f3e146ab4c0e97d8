# enhancers: parity tests, the enhance leg, its rocprofv3 kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5ms}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "multiscale or clahe or lab or gray or quant" tests/test_gpu_enhancers.py > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/pe -o p --output-format csv -- python3 bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $out/enh.json 2>&1 || exit $?
find $out/pe -name "*kernel_stats.csv" -exec cp {} $out/enhance_kernel_stats.csv \; ; rm -rf $out/pe
python3 -c "
import csv
for r in csv.DictReader(open('$out/enhance_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], r['AverageNs'])
"
grep -o '"multiscale": {[^}]*}' $out/enh.json
