"""Per-step kernel table from a rocprofv3 kernel trace: the kernels between the
last two launches of a once-per-step kernel (default adam_kernel)."""
import csv, collections, sys
path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 1
step = rows[a:b]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
agg = collections.defaultdict(lambda: [0, 0])
for r in step:
    n = r["Kernel_Name"]
    agg[n][0] += 1
    agg[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
print(f"step: {len(step)} launches, span {(t1-t0)/1e6:.3f} ms, busy {busy/1e6:.3f} ms")
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{t/1e6:7.3f} ms {c:4d}x {t/c/1e3:8.1f} us  {n[:110]}")
