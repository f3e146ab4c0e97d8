cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s3b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py::test_full_size_config "tests/test_gpu_train.py::test_train_grads_variants_vs_oracle" -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/s3b/tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/s3b/tests.log
grep -q "Fatal\|core dumped\|Aborted\|Timeout" gpurun_out/s3b/tests.log && exit 1
timeout -k 10 300 python bench.py --size 1024 --variant preact_aspp --precision fp16 --cpu-seconds 0 --no-traffic --steps 5 > gpurun_out/s3b/c4_fp16.json 2> gpurun_out/s3b/c4_fp16.err && \
timeout -k 10 300 python bench.py --size 1024 --variant preact_aspp --cpu-seconds 0 --no-traffic --steps 5 > gpurun_out/s3b/c4_fp32.json 2> gpurun_out/s3b/c4_fp32.err
