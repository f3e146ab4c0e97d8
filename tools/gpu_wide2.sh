cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wide2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "conv2d or fp16 or full_size or batch_indep or ienet" > gpurun_out/wide2/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/wide2/tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 5 > gpurun_out/wide2/bd_pa.json 2> gpurun_out/wide2/bd_pa.err || exit 1
timeout -k 10 200 python bench.py --precision fp16 --cpu-seconds 0 --no-traffic --breakdown --steps 5 > gpurun_out/wide2/bd_plain.json 2> gpurun_out/wide2/bd_plain.err || exit 1
