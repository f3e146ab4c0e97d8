cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-tprof}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python3 bench.py --train --amp --steps 4 --warmup 1 --cpu-seconds 0 > $out/train_prof.json 2>&1 || exit $?
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/train_kernel_stats.csv \; ; find $out/prof -name "*kernel_trace.csv" -exec cp {} $out/train_kernel_trace.csv \; ; rm -rf $out/prof
