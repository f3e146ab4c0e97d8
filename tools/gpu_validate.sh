cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1b
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1b/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1b/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/r1b/bench_fp32.json 2> gpurun_out/r1b/bench_fp32.err && \
timeout -k 10 300 python bench.py --precision fp16 --cpu-seconds 0 > gpurun_out/r1b/bench_fp16.json 2> gpurun_out/r1b/bench_fp16.err && \
timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 > gpurun_out/r1b/bench_fp16pa.json 2> gpurun_out/r1b/bench_fp16pa.err
