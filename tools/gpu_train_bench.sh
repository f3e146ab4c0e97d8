# training tests + configs[4] training bench + rocprofv3 kernel stats (run on the GPU box)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tb
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -v --timeout 200 --timeout-method thread > gpurun_out/tb/train_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --train --steps 5 --warmup 2 --cpu-seconds 8 > gpurun_out/tb/train_bench.json 2> gpurun_out/tb/train_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tb/rp -o k --output-format csv -- python3 bench.py --train --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/tb/rp.log 2>&1
