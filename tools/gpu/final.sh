# end-of-session check on the committed tree: full -m gpu suite, smoke, configs[3] 1024^2 per-GPU shard and
# fp16 plain bench lines (two-stream executor)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-final}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -2 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --size 1024 --steps 5 --warmup 2 --cpu-seconds 0 --no-traffic --no-nested > $out/bench_fp16_1024.json 2> $out/bench_fp16_1024.err || exit $?
timeout -k 10 200 python bench.py --precision fp16 --steps 20 --cpu-seconds 0 --no-traffic --no-nested > $out/bench_fp16_plain.json 2> $out/bench_fp16_plain.err || exit $?
grep -h '^{"metric"' $out/bench_fp16_1024.json $out/bench_fp16_plain.json | cut -c1-300
