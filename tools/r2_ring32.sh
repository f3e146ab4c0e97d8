# fp32 ring: parity + fp32 headline breakdown A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r32
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py -k "conv2d or fp32 or full_size or rect or crop" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r32/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r32/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 0; do
  UPR_CONV_RING=$r timeout -k 10 200 python bench.py --steps 10 --cpu-seconds 0 --no-traffic --breakdown > gpurun_out/r32/b32_$r.json 2> gpurun_out/r32/b32_$r.err || { tail -5 gpurun_out/r32/b32_$r.err; exit 1; }
  echo "ring=$r"; python -c "import json;d=json.load(open('gpurun_out/r32/b32_$r.json'));print(d['value'],d['roofline']['frac'],d['parity']['max_abs_diff'])"
  grep -E "enc1|fusion|branch34|residual_head|dec1" gpurun_out/r32/b32_$r.err
done
