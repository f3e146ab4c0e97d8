cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/s3/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/s3/gpu_tests.log
grep -q "Fatal\|core dumped\|Aborted" gpurun_out/s3/gpu_tests.log && exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 3 > gpurun_out/s3/bd_fp16pa.json 2> gpurun_out/s3/bd_fp16pa.err && \
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --breakdown --steps 3 > gpurun_out/s3/bd_fp32.json 2> gpurun_out/s3/bd_fp32.err
