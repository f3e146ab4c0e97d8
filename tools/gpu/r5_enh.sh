# round-5 enhancer evidence: parity of the enhancer kernels, the enhance bench leg + its rocprofv3
# summary, content-aware / letterbox timings + rocprofv3 summary, the end-to-end harness at 256^2 / 512^2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5e}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "multiscale or clahe or lab or gray or quant" tests/test_gpu_enhancers.py > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --enhance --steps 20 --warmup 3 --detail $out/enh_detail.json > $out/enh.json 2> $out/enh.err || exit $?
cat $out/enh.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/profE -o p --output-format csv -- python3 bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $out/enh_prof.json 2>&1 || exit $?
timeout -k 10 200 python tools/enh_extra_bench.py > $out/extra.json 2> $out/extra.err || exit $?
cat $out/extra.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/profX -o p --output-format csv -- python3 tools/enh_extra_bench.py > $out/extra_prof.json 2>&1 || exit $?
timeout -k 10 300 python tools/harness_bench.py --n 32 --size 256 > $out/harness256.json 2> $out/harness256.err || exit $?
timeout -k 10 300 python tools/harness_bench.py --n 32 --size 512 > $out/harness512.json 2> $out/harness512.err || exit $?
cat $out/harness256.json $out/harness512.json
