# training-path checks: the training GPU tests, the conv parity cases, then the configs[4] bench + kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r4train}
mkdir -p $out
timeout -k 10 800 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py tests/test_gpu_modules.py tests/test_gpu_api_surface.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --train --amp --steps 10 --warmup 3 --cpu-seconds 0 > $out/train.json 2> $out/train.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python3 bench.py --train --amp --steps 4 --warmup 1 --cpu-seconds 0 > $out/train_prof.json 2>&1 || exit $?
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/train_kernel_stats.csv \; ; rm -rf $out/prof
