# rocprofv3 evidence for the bench's per-launch roofline numbers: the default (fp32, single-stream) bench,
# the fp16 preact+ASPP bench serialised (UPR_MS_STREAMS=0, every kernel's duration separable) and as it
# runs by default (two streams: overlapped kernels' trace durations stretch), plus the default bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-pe}
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-traffic --cpu-seconds 0 --no-nested > $out/bench_prof.json 2>&1 || exit $?
UPR_MS_STREAMS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof16s -o p --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --no-nested > $out/bench_prof16s.json 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof16 -o p --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --no-nested > $out/bench_prof16.json 2>&1 || exit $?
timeout -k 10 400 python bench.py > $out/bench_default.json 2> $out/bench_default.err || exit $?
cat $out/bench_default.json
