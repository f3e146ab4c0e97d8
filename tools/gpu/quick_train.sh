# quick check of a training-path change: selected GPU tests, the AMP training
# bench, and a kernel trace of the same run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-qt}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_modules.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "${TK:-bn or batchnorm or maxpool or amp_autocast or wgrad or determin}" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --train --amp --steps 10 --warmup 3 --cpu-seconds 0 > $out/train.json 2> $out/train.err || exit $?
python3 -c "import json;d=json.loads(open('$out/train.json').read().strip().splitlines()[-1]);print('train',d['value'],d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python3 bench.py --train --amp --steps 4 --warmup 1 --cpu-seconds 0 > $out/train_prof.json 2>&1 || exit $?
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/train_kernel_stats.csv \; ; find $out/prof -name "*kernel_trace.csv" -exec cp {} $out/train_kernel_trace.csv \; ; rm -rf $out/prof
