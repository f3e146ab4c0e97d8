# round checkpoint: full -m gpu suite, smoke, default bench (traffic + cpu baseline), fp16 preact+ASPP bench
# (traffic + cpu baseline), rocprofv3 kernel stats of both benches
# (the fp16 kernel stats are taken serialised, UPR_MS_STREAMS=0: see DESIGN §3, two streams per forward)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${CK:-ck}
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${CK:-ck}/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/${CK:-ck}/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${CK:-ck}/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/${CK:-ck}/bench_default.json 2> gpurun_out/${CK:-ck}/bench_default.err || exit $?
cat gpurun_out/${CK:-ck}/bench_default.json
timeout -k 10 400 python bench.py --precision fp16 --variant preact_aspp --ceilings --no-nested > gpurun_out/${CK:-ck}/bench_fp16.json 2> gpurun_out/${CK:-ck}/bench_fp16.err || exit $?
cat gpurun_out/${CK:-ck}/bench_fp16.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${CK:-ck}/prof -o p --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-traffic --cpu-seconds 0 --no-nested > gpurun_out/${CK:-ck}/bench_prof.json 2>&1 || exit $?
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --no-nested > gpurun_out/${CK:-ck}/bench_train.json 2> gpurun_out/${CK:-ck}/bench_train.err || exit $?
UPR_MS_STREAMS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${CK:-ck}/prof16 -o p --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --no-nested > gpurun_out/${CK:-ck}/bench_prof16.json 2>&1 || exit $?
exit $rc
