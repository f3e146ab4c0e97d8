# Full bench lines + rocprofv3 kernel stats for profiles/ (run on the GPU box)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
set -e
mkdir -p gpurun_out/prof
timeout -k 10 600 python bench.py > gpurun_out/prof/bench_fp32_plain.json 2> gpurun_out/prof/bench_fp32_plain.err
timeout -k 10 300 python bench.py --precision fp16 --cpu-seconds 0 > gpurun_out/prof/bench_fp16_plain.json 2> gpurun_out/prof/bench_fp16_plain.err
timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 > gpurun_out/prof/bench_fp16_pa.json 2> gpurun_out/prof/bench_fp16_pa.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/rp32 -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic > gpurun_out/prof/rp32.log 2>&1
