# 64-pixel ring strips for the 32 -> 32 convs: parity (conv ops + models), A/B (UPR_RING_WIDE), fp16 + fp32 breakdowns
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ringw
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ringw/tests.log 2>&1
rc=$?; tail -3 gpurun_out/ringw/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for w in 0 1; do
echo "wide=$w" >> gpurun_out/ringw/cb.log
UPR_RING_WIDE=$w timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes dec1,dec1p --iters 30 2>/dev/null >> gpurun_out/ringw/cb.log || exit 1
done; done
cat gpurun_out/ringw/cb.log
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 10 > gpurun_out/ringw/fp16.json 2> gpurun_out/ringw/fp16.err || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/ringw/fp16.json").read().strip().splitlines()[-1])
print("fp16", round(d["value"], 1), "img/s  layer frac", round(d["roofline"]["layer_roofline_frac"], 4))
PY
grep -E "dec1|residual_head" gpurun_out/ringw/fp16.err
