# parity tests (model + conv kernels), then fp16 preact+ASPP breakdown and the fp32 default bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q
timeout -k 10 400 python -u -m pytest ${QTESTS:-tests/test_gpu_parity.py tests/test_gpu_bn_parity.py} -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/q/tests.log 2>&1
rc=$?; tail -3 gpurun_out/q/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 10 > gpurun_out/q/fp16.json 2> gpurun_out/q/fp16.err || exit $?
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --breakdown --steps 10 > gpurun_out/q/fp32.json 2> gpurun_out/q/fp32.err || exit $?
python - <<'PY'
import json
for f in ("fp16", "fp32"):
    d = json.loads(open(f"gpurun_out/q/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), "img/s  layer frac", round(d["roofline"]["layer_roofline_frac"], 4), "frac", round(d["roofline"]["frac"], 4))
PY
