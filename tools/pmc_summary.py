#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection.csv files: per kernel instance, the
mean counter value per launch plus derived ratios.

  python tools/pmc_summary.py gpurun_out/pmcm_fp32_a gpurun_out/pmcm_fp32_b [--match conv_halo]
"""
import csv
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("upr::", "")[:90]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args = [a for a in args if a != match]
    vals = defaultdict(lambda: defaultdict(list))
    for d in args:
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    with open(os.path.join(root, f)) as fh:
                        for r in csv.DictReader(fh):
                            k = short(r["Kernel_Name"])
                            if match and match not in k:
                                continue
                            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(vals.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print("==", k)
        for c in sorted(m):
            print(f"     {c:28s} {m[c]:16.1f}")
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            w = m["SQ_WAVE_CYCLES"]
            print(f"     -> wait_any {m.get('SQ_WAIT_ANY', 0) / w:.2f}  wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / w:.2f}"
                  f"  active {m.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}")
        if "SQ_INSTS_MFMA" in m and m["SQ_INSTS_MFMA"]:
            mf = m["SQ_INSTS_MFMA"]
            print(f"     -> per MFMA: valu {m.get('SQ_INSTS_VALU', 0) / mf:.2f} lds {m.get('SQ_INSTS_LDS', 0) / mf:.2f}"
                  f" salu {m.get('SQ_INSTS_SALU', 0) / mf:.2f} vmem {m.get('SQ_INSTS_VMEM', 0) / mf:.3f}")


if __name__ == "__main__":
    main()
