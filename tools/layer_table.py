#!/usr/bin/env python3
"""Tabulate tools/layer_sweep.sh output: per-layer ms for each config + best."""
import glob
import os
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for dt in ("fp32", "fp16"):
    files = sorted(glob.glob(os.path.join(d, f"ls_{dt}_*.log")))
    if not files:
        continue
    cfgs = [re.sub(r".*ls_%s_(\d+)_(\d+)\.log" % dt, r"\1,\2", f) for f in files]
    tab, tot = {}, {}
    for c, f in zip(cfgs, files):
        for line in open(f):
            m = re.match(r"(\S+)\s+(\S+)\s+([\d.]+) ms", line)
            if m:
                tab.setdefault(m.group(1), {})[c] = float(m.group(3))
            if line.startswith("{"):
                tot[c] = float(re.search(r'"ms_per_step": ([\d.]+)', line).group(1))
    print(f"== {dt}   " + " ".join(f"{c:>8s}" for c in cfgs))
    print(f"{'step total':40s}" + " ".join(f"{tot.get(c, 0):8.3f}" for c in cfgs))
    rows = sorted(tab.items(), key=lambda kv: -max(kv[1].values()))
    for name, v in rows:
        if max(v.values()) < 0.05:
            continue
        best = min(v, key=v.get)
        print(f"{name:40s}" + " ".join(f"{v.get(c, 0):8.3f}" for c in cfgs) + f"   best {best}")
