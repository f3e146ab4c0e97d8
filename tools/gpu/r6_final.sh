# round-6 evidence on the committed tree: the full -m gpu suite + smoke, the default bench line (configs[1]
# + nested fp16 / enhance / train_amp summaries, detail file), rocprofv3 kernel stats of fp32, fp16 (serialised),
# the enhance leg, the training step (+ its trace), content-aware / letterbox, the directory harness at 256^2 / 512^2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r6final}
mkdir -p $out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
  rc=$?; tail -2 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
fi
timeout -k 10 600 python bench.py --detail $out/bench_detail.json > $out/bench_default.json 2> $out/bench_default.err || exit $?
grep -h '^{"metric"' $out/bench_default.json | cut -c1-400
UPR_MS_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/rp32 -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic --no-nested --detail "" > $out/rp32.log 2>&1 || exit $?
UPR_MS_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/rp16 -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic --no-nested --precision fp16 --variant preact_aspp --detail "" > $out/rp16.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/rpe -o k --output-format csv -- python3 bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $out/rpe.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/rpt -o k --output-format csv -- python3 bench.py --train --amp --steps 4 --warmup 1 --cpu-seconds 0 --detail "" > $out/rpt.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/rpc -o k --output-format csv -- python3 tools/enh_extra_bench.py > $out/ca_bench.json 2>&1 || exit $?
find $out/rp32 -name "*kernel_stats.csv" -exec cp {} $out/fp32_plain_kernel_stats_serial.csv \; ; find $out/rp16 -name "*kernel_stats.csv" -exec cp {} $out/fp16_pa_kernel_stats_serial.csv \;
find $out/rpe -name "*kernel_stats.csv" -exec cp {} $out/enhance_kernel_stats.csv \; ; find $out/rpt -name "*kernel_stats.csv" -exec cp {} $out/train_kernel_stats.csv \; ; find $out/rpt -name "*kernel_trace.csv" -exec cp {} $out/train_kernel_trace.csv \;
find $out/rpc -name "*kernel_stats.csv" -exec cp {} $out/ca_kernel_stats.csv \;
rm -rf $out/rp32 $out/rp16 $out/rpe $out/rpt $out/rpc
timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --no-nested --breakdown --cpu-seconds 0 --no-traffic --detail "" > $out/fp16_layers.json 2> $out/fp16_layers.txt || exit $?
for s in 256 512; do
  timeout -k 10 300 python tools/harness_bench.py --n 32 --size $s > $out/harness_$s.json 2> $out/harness_$s.err || exit $?
  echo "harness $s $(cat $out/harness_$s.json)"
done
