# round-4 enhancer / loss checks: targeted -m gpu tests, the enhance bench leg, its rocprofv3 kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r4enh}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_api_surface.py tests/test_gpu_enhancers.py -m gpu -x -q -k "clahe or lab or quantize or gray or multiscale or three_channel or scratch or multi_scale_enhance or loss_terms or enhance" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --enhance --steps 20 --warmup 3 > $out/bench_enh.json 2> $out/bench_enh.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o enh -- python bench.py --enhance --steps 20 --warmup 3 --cpu-seconds 0 --no-traffic > $out/prof.log 2>&1 || exit $?
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/enh_kernel_stats.csv \;
cat $out/bench_enh.json
