# state snapshot: train step bench (AMP, bs8 512^2), fp16 preact+aspp breakdown
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/st
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/st/train.json 2> gpurun_out/st/train.err || { tail -5 gpurun_out/st/train.err; exit 1; }
cat gpurun_out/st/train.json
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 5 > gpurun_out/st/fp16pa.json 2> gpurun_out/st/fp16pa.err || exit 1
cat gpurun_out/st/fp16pa.json
