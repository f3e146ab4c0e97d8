# parity file (conv cases + model fp16/fp32 at size) + fp16 preact+ASPP per-layer breakdown
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-dsq}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --no-nested --breakdown --steps 10 > $out/fp16pa.json 2> $out/fp16pa_layers.txt || exit $?
python3 -c "import json;d=json.load(open('$out/fp16pa.json'));print(d['value'],d['ms_per_step'],d['roofline']['layer_roofline_frac'],d['roofline']['mfma_bound_layers'])"
grep -v amdgpu $out/fp16pa_layers.txt | head -28
