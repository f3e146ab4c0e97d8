#!/usr/bin/env python3
"""Summarise rocprofv3 counter_collection.csv files: mean counter value per kernel launch.

  python tools/pmc_summary.py gpurun_out/pmc_a_fp32_dec1_4_1 gpurun_out/pmc_b_fp32_dec1_4_1
"""
import csv
import os
import sys
from collections import defaultdict


def main():
    for d in sys.argv[1:]:
        vals = defaultdict(lambda: defaultdict(list))
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    with open(os.path.join(root, f)) as fh:
                        for r in csv.DictReader(fh):
                            k = r["Kernel_Name"].split("(")[0][:60]
                            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print("==", d)
        for k, cs in vals.items():
            print("  ", k)
            for c, v in sorted(cs.items()):
                print(f"     {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
