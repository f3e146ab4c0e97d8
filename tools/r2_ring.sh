# row-ring stream kernel: parity + A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ring
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py -k "conv2d or fp16 or full_size" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ring/tests.log 2>&1
rc=$?; tail -5 gpurun_out/ring/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1; do
  UPR_CONV_RING=$r timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes dec1,fam_h,dec2,enc1c2,enc1s2 > gpurun_out/ring/cb_$r.txt 2>&1 || exit 1
  echo "ring=$r"; cat gpurun_out/ring/cb_$r.txt
done
for r in 1; do
  UPR_CONV_RING=$r timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --steps 10 --cpu-seconds 0 --no-traffic --breakdown > gpurun_out/ring/b16_$r.json 2> gpurun_out/ring/b16_$r.err || { tail -5 gpurun_out/ring/b16_$r.err; exit 1; }
  echo "ring=$r"; python -c "import json;d=json.load(open('gpurun_out/ring/b16_$r.json'));print(d['value'],d['roofline']['layer_roofline_frac'])"
  grep -E "enc1|fusion|branch34|residual_head|dec1|dec2" gpurun_out/ring/b16_$r.err
done
