#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: share, ms per step, calls, average.

  python tools/kstats.py gpurun_out/tp/rp/k_kernel_stats.csv [steps] [top]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total {tot / 1e6:.2f} ms, per step {tot / 1e6 / steps:.2f} ms")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        t = float(r["TotalDurationNs"])
        print(f"{t / tot * 100:5.1f}% {t / 1e6 / steps:7.2f} ms/step calls {r['Calls']:>5} "
              f"avg {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:100]}")


if __name__ == "__main__":
    main()
