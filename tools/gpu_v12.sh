# Round validation of HEAD on the GPU box: all GPU tests, smoke, benches, rocprofv3 kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/v12
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-seconds 12 > $O/bench_fp32.json 2> $O/bench_fp32.err && \
timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 3 --breakdown > $O/bench_fp16pa.json 2> $O/bench_fp16pa.err && \
timeout -k 10 300 python bench.py --precision fp16 --cpu-seconds 3 > $O/bench_fp16.json 2> $O/bench_fp16.err && \
timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --size 1024 --cpu-seconds 0 --no-traffic --steps 5 > $O/bench_fp16pa_1024.json 2> $O/bench_fp16pa_1024.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp32 -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic > $O/rp32.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp16pa -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic --precision fp16 --variant preact_aspp > $O/rp16pa.log 2>&1
echo "rc=$?"
