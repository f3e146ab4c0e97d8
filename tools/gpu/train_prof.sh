# configs[4] AMP training step: bench line (per-pass conv breakdown) + rocprofv3 kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-tp}
mkdir -p $out
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 0 > $out/train.json 2> $out/train.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python3 bench.py --train --amp --steps 4 --warmup 1 --cpu-seconds 0 > $out/train_prof.json 2>&1 || exit $?
