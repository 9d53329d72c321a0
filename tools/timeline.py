#!/usr/bin/env python3
"""Print one frontend step's GPU timeline from a rocprofv3 --kernel-trace
--memory-copy-trace CSV pair (bash tools/gpu.sh trace)."""
import csv
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tr_g1"
rows = []
for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
    n = r["Kernel_Name"]
    m = re.search(r"([a-z_]+kernel)", n)
    short = m.group(1) if m else n.split("(")[0][-32:]
    if short == "lk_multi_kernel":  # the temporal (21x21) and stereo (11x11) calls
        short += "_21" if "21, 21" in n else "_11"
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + short, r.get("Queue_Id", "")))
for r in csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C:" + r["Direction"][:24], r.get("Queue_Id", "")))
rows.sort()
lk = [x for x in rows if x[2].startswith("K:lk_multi_kernel_21")] or [x for x in rows if x[2].startswith("K:lk_")]
# slices of one step launch their LKs together: step starts = LK starts > 100 us apart
starts = [lk[0][0]]
for x in lk[1:]:
    if x[0] - starts[-1] > 100_000:
        starts.append(x[0])
t0, tp = starts[-1], starts[-2]
print(f"step period {(t0 - tp) / 1e3:.1f} us")
for a, b, n, q in rows:
    if tp <= a < t0:
        print(f"{(a - tp) / 1e3:8.1f} {(b - tp) / 1e3:8.1f} {(b - a) / 1e3:7.1f} q{q} {n}")
