# ring landing-zone swizzle + occupancy-3 A/B: conv parity, convbench, fp16 and fp32 breakdowns
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ring2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv2d or full_size or fp16" > gpurun_out/ring2/tests.log 2>&1
rc=$?; tail -3 gpurun_out/ring2/tests.log; [ $rc -eq 0 ] || exit $rc
for o in 0 1 0 1; do
echo "occ3=$o" >> gpurun_out/ring2/cb.log
UPR_RING_OCC3=$o timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes dec1,dec1p,dec2,fam_h --iters 30 2>/dev/null >> gpurun_out/ring2/cb.log || exit 1
done
timeout -k 10 120 python tools/convbench.py --dtype fp32 --shapes dec1,dec1p,fam_h --iters 20 2>/dev/null >> gpurun_out/ring2/cb.log || exit 1
cat gpurun_out/ring2/cb.log
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 10 > gpurun_out/ring2/fp16.json 2> gpurun_out/ring2/fp16.err || exit $?
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --breakdown --steps 10 > gpurun_out/ring2/fp32.json 2> gpurun_out/ring2/fp32.err || exit $?
python3 - <<'PY'
import json
for f in ("fp16", "fp32"):
    d = json.loads(open(f"gpurun_out/ring2/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), "img/s  layer frac", round(d["roofline"]["layer_roofline_frac"], 4), "frac", round(d["roofline"]["frac"], 4))
PY
