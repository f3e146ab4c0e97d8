# HEAD check: full -m gpu suite, smoke, fp32 headline bench, train bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2h
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r2h/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -8 gpurun_out/r2h/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2h/smoke.log 2>&1 || { cat gpurun_out/r2h/smoke.log; exit 1; }
cat gpurun_out/r2h/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r2h/bench.json 2> gpurun_out/r2h/bench.err || { tail -5 gpurun_out/r2h/bench.err; exit 1; }
cat gpurun_out/r2h/bench.json
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r2h/train.json 2> gpurun_out/r2h/train.err || { tail -5 gpurun_out/r2h/train.err; exit 1; }
cat gpurun_out/r2h/train.json
exit $rc
