# rocprofv3 kernel stats of the training bench (bs8 512^2 AMP)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp/rp -o k --output-format csv -- python3 bench.py --train --amp --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/tp/train.log 2>&1 || { tail -5 gpurun_out/tp/train.log; exit 1; }
find gpurun_out/tp -name "*kernel_stats.csv" | head -1
