# rocprofv3 kernel stats of the default bench (fp32 plain) and fp16 preact+ASPP for profiles/ (run on the GPU box)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/rp32 -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic > gpurun_out/prof/rp32.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/rp16pa -o k --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-traffic --precision fp16 --variant preact_aspp > gpurun_out/prof/rp16pa.log 2>&1
