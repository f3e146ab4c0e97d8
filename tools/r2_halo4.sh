# ring-halo kernel at W 128 (512-pixel tiles, BN 128): parity + A/B vs gathered (UPR_WIDE_HALO 0/2) on dec3 / enc2c2 / bneck
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/halo5
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv2d or full_size or fp16" > gpurun_out/halo5/tests.log 2>&1
rc=$?; tail -3 gpurun_out/halo5/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for h in 0 2; do
echo "halo=$h" >> gpurun_out/halo5/cb.log
UPR_WIDE_HALO=$h timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,dec3,enc2c2 --iters 30 2>/dev/null >> gpurun_out/halo5/cb.log || exit 1
done; done
cat gpurun_out/halo5/cb.log
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 10 > gpurun_out/halo5/fp16.json 2> gpurun_out/halo5/fp16.err || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/halo5/fp16.json").read().strip().splitlines()[-1])
print("fp16", round(d["value"], 1), "img/s  layer frac", round(d["roofline"]["layer_roofline_frac"], 4))
PY
grep -E "dec3|enc2" gpurun_out/halo5/fp16.err
