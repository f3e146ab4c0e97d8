cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bd
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 3 > gpurun_out/bd/fp16pa.json 2> gpurun_out/bd/fp16pa.err && \
timeout -k 10 200 python bench.py --precision fp16 --cpu-seconds 0 --no-traffic --breakdown --steps 3 > gpurun_out/bd/fp16.json 2> gpurun_out/bd/fp16.err && \
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --breakdown --steps 3 > gpurun_out/bd/fp32.json 2> gpurun_out/bd/fp32.err
