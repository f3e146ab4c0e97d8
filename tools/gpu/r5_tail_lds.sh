# retinex tail with LDS-staged bilinear windows: forward parity tests, then kernel stats (serialised fp16 / fp32)
# (the LDS-window tail kernel was removed after this run: profiles/r5_retinex_tail_ab.txt)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5taillds}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_api_surface.py > $out/tests.log 2>&1
rc=$?; tail -1 $out/tests.log; [ $rc -eq 0 ] || exit $rc
UPR_MS_STREAMS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/p16 -o k --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --no-nested --detail "" --steps 10 > $out/fp16.json 2>&1 || exit $?
UPR_MS_STREAMS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/p32 -o k --output-format csv -- python3 bench.py --cpu-seconds 0 --no-traffic --no-nested --detail "" --steps 5 > $out/fp32.json 2>&1 || exit $?
for f in p16 p32; do
  echo "== $f"; python3 -c "
import csv,glob
for p in glob.glob('$out/$f/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        if 'tail' in r['Name'] or 'fam_sa' in r['Name']: print('  %-50s %5s %8.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))
"
done
rm -rf $out/p16 $out/p32
