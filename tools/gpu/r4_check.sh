# round-4 check of a build: conv / full-size parity (incl. the shortcut program on hwide4),
# the training tests, the fp16 preact+ASPP layer breakdown, and the training bench + kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r4check}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "${TK:-conv2d or full_size or wgrad or conv_layer or stride2 or amp_autocast or full_size_bs8}" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 5 > $out/fp16pa.json 2> $out/fp16pa.err || exit $?
timeout -k 10 300 python bench.py --train --amp --steps 10 --warmup 3 --cpu-seconds 0 > $out/train.json 2> $out/train.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python3 bench.py --train --amp --steps 4 --warmup 1 --cpu-seconds 0 > $out/train_prof.json 2>&1 || exit $?
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/train_kernel_stats.csv \; ; rm -rf $out/prof
python3 -c "import json;d=json.loads(open('$out/train.json').read().strip().splitlines()[-1]);print('train',d['value'],d['ms_per_step'])"
