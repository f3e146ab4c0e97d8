# enhancers: parity tests, the enhance leg + kernel stats, then PMC passes over the enhance leg
# (issue / wait / LDS mix and HBM bytes per kernel: ms_sums3, clahe_hist, clahe_apply, scale_clamp)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5ep}
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
grep -o '"value": [0-9.]*' $out/enh.json | head -1; grep -o '"frac": [0-9.]*' $out/enh.json | head -2
E="python3 bench.py --enhance --steps 2 --warmup 1 --no-traffic --cpu-seconds 0 --detail \"\""
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $out/pmc_a -o p --output-format csv -- python3 bench.py --enhance --steps 2 --warmup 1 --no-traffic --cpu-seconds 0 --detail "" > $out/pmc_a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-trace -d $out/pmc_b -o p --output-format csv -- python3 bench.py --enhance --steps 2 --warmup 1 --no-traffic --cpu-seconds 0 --detail "" > $out/pmc_b.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/pmc_c -o p --output-format csv -- python3 bench.py --enhance --steps 2 --warmup 1 --no-traffic --cpu-seconds 0 --detail "" > $out/pmc_c.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/pmc_d -o p --output-format csv -- python3 bench.py --enhance --steps 2 --warmup 1 --no-traffic --cpu-seconds 0 --detail "" > $out/pmc_d.log 2>&1 || exit 1
python3 tools/pmc_summary.py $out/pmc_a $out/pmc_b $out/pmc_c $out/pmc_d > $out/pmc_summary.txt
grep -A40 "ms_sums3\|clahe_apply\|clahe_hist" $out/pmc_summary.txt | head -120
