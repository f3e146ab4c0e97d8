# retinex tail A/B on one box: kernel stats of the fp16 preact+ASPP and fp32 forwards, 4-pixel form vs UPR_TAIL4=0
# (the UPR_TAIL4 switch and the 4-pixel kernel were removed after this A/B: profiles/r5_retinex_tail_ab.txt)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5tailab}
mkdir -p $out
for v in 1 0; do
  UPR_TAIL4=$v UPR_MS_STREAMS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/p16_$v -o k --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --no-nested --detail "" --steps 10 > $out/fp16_$v.json 2>&1 || exit $?
  UPR_TAIL4=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/p32_$v -o k --output-format csv -- python3 bench.py --cpu-seconds 0 --no-traffic --no-nested --detail "" --steps 5 > $out/fp32_$v.json 2>&1 || exit $?
done
for f in $out/p16_1 $out/p16_0 $out/p32_1 $out/p32_0; do
  echo "== $f"; python3 -c "
import csv,glob
for p in glob.glob('$f/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        if 'tail' in r['Name']: print('  %-50s %5s %8.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))
"
done
rm -rf $out/p16_* $out/p32_*
