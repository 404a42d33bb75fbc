"""Per-kernel durations and the idle gaps between consecutive kernels of a rocprofv3 kernel trace
(kernel_trace.csv): python tools/trace_gaps.py <dir> [last_n_kernels]."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 400
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-last:]
dur = defaultdict(list)
gap = defaultdict(list)
prev = None
for r in rows:
    name = r["Kernel_Name"].split("(")[0][:60]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[name].append((e - s) / 1e3)
    if prev is not None:
        gap[name].append((s - prev) / 1e3)
    prev = e
for k in dur:
    v = sorted(dur[k]); g = sorted(gap[k]) or [0]
    print(f"{k:60s} n={len(v):4d} dur med {v[len(v)//2]:7.2f} us  gap-before med {g[len(g)//2]:6.2f} us")
