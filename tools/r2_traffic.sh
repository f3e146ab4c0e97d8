# bench lines with the corrected PMC conv-kernel list (fp32 default + fp16 preact+ASPP)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tr2
timeout -k 10 400 python bench.py --cpu-seconds 0 > gpurun_out/tr2/fp32.json 2> gpurun_out/tr2/fp32.err || exit $?
timeout -k 10 400 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 > gpurun_out/tr2/fp16.json 2> gpurun_out/tr2/fp16.err || exit $?
python3 - <<'PY'
import json
for f in ("fp32", "fp16"):
    d = json.loads(open(f"gpurun_out/tr2/{f}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, round(d["value"], 1), "frac", round(r["frac"], 4), "layer", round(r["layer_roofline_frac"], 4),
          "traffic/img GB", r["traffic_per_img_GB"], "alg GB/img", r["gemm_alg_GB_per_img"])
PY
