# round-5 quick check: the tests touched this round, the enhancer bench + its rocprofv3 kernel
# summary, and the default bench line (compact stdout, full record in gpurun_out/$CK/detail.json)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5c}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py::test_multiscale_single_pass tests/test_gpu_parity.py::test_multiscale_kernel \
  tests/test_gpu_parity.py::test_multiscale_side_stream_matches_serial tests/test_gpu_enhancers.py \
  tests/test_gpu_train.py::test_scratch_more_streams_than_table tests/test_gpu_train.py::test_loss_without_reflectance \
  tests/test_gpu_train.py::test_dgrad_1x1_stride2_scatter tests/test_gpu_train.py::test_dgrad_3x3_stride2_phases \
  ${EXTRA_TESTS} > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --enhance --steps 20 --warmup 3 --detail $out/enh_detail.json > $out/enh.json 2> $out/enh.err || exit $?
cat $out/enh.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/profE -o p --output-format csv -- python3 bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $out/enh_prof.json 2>&1 || exit $?
[ -n "$NO_DEFAULT" ] && exit 0
timeout -k 10 500 python bench.py --detail $out/detail.json > $out/bench_default.json 2> $out/bench_default.err || exit $?
cat $out/bench_default.json | wc -c
