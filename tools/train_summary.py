"""Summarise a training bench line + its rocprofv3 kernel stats (per step)."""
import csv
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{d['value']:.1f} img/s  {d['ms_per_step']:.2f} ms/step")
r = d["roofline"]
for k, v in sorted(r["by_pass"].items(), key=lambda kv: -kv[1]["ms"]):
    print(f"  {k:16s} {v['ms']:7.2f} ms {v['gflop']:8.1f} GF {v['calls']:4d} calls {v['TFLOPs'] or 0:7.1f} TF/s")
print(f"  conv {r['conv_ms']:.2f} ms, non-conv {r['non_conv_ms']:.2f} ms")
if len(sys.argv) > 2:
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = list(csv.DictReader(open(sys.argv[2])))
    tot = sum(float(x["TotalDurationNs"]) for x in rows)
    print(f"kernel time per step {tot / 1e6 / steps:.2f} ms")
    for x in sorted(rows, key=lambda x: -float(x["TotalDurationNs"]))[:int(sys.argv[4]) if len(sys.argv) > 4 else 30]:
        print(f"  {float(x['TotalDurationNs']) / 1e6 / steps:6.2f} ms {int(x['Calls']) // steps:4d}/step "
              f"{float(x['AverageNs']) / 1000:8.1f} us  {x['Name'][:90]}")
