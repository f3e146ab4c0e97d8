# same-box A/B of two builds on the whole model: per-layer breakdown of lib/libupr_prev.so (A) vs lib/libupr.so (B)
# (fp16 preact+ASPP and fp32 plain), after the parity files on B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-mlab}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py tests/test_gpu_modules.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
A=$GRAFT_REPO_ROOT/retinex-image-enhancement_amd/lib/libupr_prev.so
for i in 1 2; do
  for side in A B; do
    if [ $side = A ]; then L=$A; else L=$GRAFT_REPO_ROOT/retinex-image-enhancement_amd/lib/libupr.so; fi
    UPR_LIB=$L timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --no-nested --breakdown --steps 10 > $out/fp16_$side$i.json 2> $out/fp16_$side$i.layers || exit $?
    python3 -c "import json;d=json.load(open('$out/fp16_$side$i.json'));print('$side fp16', round(d['value'],1), round(d['ms_per_step'],4))" | tee -a $out/ab.txt
  done
done
grep -E "spatial_attention|retinex_tail" $out/fp16_A2.layers $out/fp16_B2.layers
