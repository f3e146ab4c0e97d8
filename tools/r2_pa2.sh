# fused PreAct second output: model parity (fp16 preact variants, BN parity), fp16 breakdown
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pa2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py tests/test_gpu_modules.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pa2/tests.log 2>&1
rc=$?; tail -3 gpurun_out/pa2/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 20 > gpurun_out/pa2/fp16.json 2> gpurun_out/pa2/fp16.err || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/pa2/fp16.json").read().strip().splitlines()[-1])
print("fp16", round(d["value"], 1), "img/s  layer frac", round(d["roofline"]["layer_roofline_frac"], 4), d["parity"] if "parity" in d else "")
PY
grep -E "bn1_relu|enc1.conv2|enc2.conv2|enc3.conv2|bottleneck.1.fusion" gpurun_out/pa2/fp16.err
