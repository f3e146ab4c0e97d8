# kernel traces: the fp16 preact+ASPP forward serialised (UPR_MS_STREAMS=0: every kernel's duration
# separable) and the configs[4] AMP training step; stats + traces copied out, raw dirs removed
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5p}
mkdir -p $out
UPR_MS_STREAMS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/p16 -o p --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --steps 10 --warmup 3 --no-traffic --cpu-seconds 0 --no-nested --detail "" > $out/fp16_prof.json 2>&1 || exit $?
find $out/p16 -name "*kernel_stats.csv" -exec cp {} $out/fp16_kernel_stats.csv \; ; find $out/p16 -name "*kernel_trace.csv" -exec cp {} $out/fp16_kernel_trace.csv \; ; rm -rf $out/p16
timeout -k 10 300 python bench.py --train --amp --steps 10 --warmup 3 --cpu-seconds 0 --detail $out/train_detail.json > $out/train.json 2> $out/train.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pt -o p --output-format csv -- python3 bench.py --train --amp --steps 4 --warmup 1 --cpu-seconds 0 --detail "" > $out/train_prof.json 2>&1 || exit $?
find $out/pt -name "*kernel_stats.csv" -exec cp {} $out/train_kernel_stats.csv \; ; find $out/pt -name "*kernel_trace.csv" -exec cp {} $out/train_kernel_trace.csv \; ; rm -rf $out/pt
python3 -c "import json;d=json.load(open('$out/train.json'));print('train', d['value'], d['ms_per_step'])"
