# fp32 + fp16 breakdown benches (no traffic passes, no cpu baseline)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bd2
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --breakdown --steps 5 > gpurun_out/bd2/fp32.json 2> gpurun_out/bd2/fp32.err || exit 1
cat gpurun_out/bd2/fp32.json
grep conv_igemm gpurun_out/bd2/fp32.err
