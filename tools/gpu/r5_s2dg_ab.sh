# enc1.conv1 input gradient: LDS-filter phase kernel (default) vs the register-filter one (UPR_S2DG_REG=1)
# (the UPR_S2DG_REG switch was removed after this A/B: profiles/r5_s2dgrad_lds_ab.txt)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5s2ab}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "stride2 or full_step or g7" > $out/tests.log 2>&1
rc=$?; tail -1 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  UPR_S2DG_REG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p_$v -o k --output-format csv -- python3 bench.py --train --amp --steps 4 --warmup 1 --cpu-seconds 0 --detail "" > $out/train_$v.json 2>&1 || exit $?
  echo "== UPR_S2DG_REG=$v"; python3 -c "
import csv,glob
for p in glob.glob('$out/p_$v/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        if 's2dg' in r['Name']: print('  %-50s %5s %8.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))
"
done
rm -rf $out/p_*
