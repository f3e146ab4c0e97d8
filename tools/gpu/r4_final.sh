# end-of-round evidence on the committed tree: the full -m gpu suite + smoke, the default bench line
# (configs[1]) and the fp16 configs[2] line, rocprofv3 kernel stats of both (serialised fp16), all under profiles-ready names
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r4final}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -2 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $out/bench_default.json 2> $out/bench_default.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/rp32 -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic --no-nested > $out/rp32.log 2>&1 || exit $?
UPR_MS_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/rp16 -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic --no-nested --precision fp16 --variant preact_aspp > $out/rp16.log 2>&1 || exit $?
find $out/rp32 -name "*kernel_stats.csv" -exec cp {} $out/fp32_plain_kernel_stats.csv \; ; find $out/rp16 -name "*kernel_stats.csv" -exec cp {} $out/fp16_pa_kernel_stats_serial.csv \; ; rm -rf $out/rp32 $out/rp16
grep -h '^{"metric"' $out/bench_default.json | cut -c1-400
