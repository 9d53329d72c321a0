#!/usr/bin/env python3
"""GPU timeline of front-end steps from a rocprofv3 --kernel-trace CSV: the
kernels that start between consecutive temporal-LK launches of one batch size.

  python tools/step_timeline.py TRACE_DIR [--seq 256] [--first K] [--steps 2]
(--first: index of the first step among that batch size's LK launches, in launch
order, negative from the end: the headline's come first when the bench's side legs
run after it, the bucketed leg's last)."""
import argparse
import csv
import glob
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--seq", type=int, default=256)
ap.add_argument("--first", type=int, default=12)
ap.add_argument("--steps", type=int, default=2)
a = ap.parse_args()
f = glob.glob(a.trace + "/**/*kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    m = re.search(r"([a-z_0-9]+_kernel)", n)
    s = m.group(1) if m else n[:30]
    if s == "lk_multi_kernel":
        s += "_21" if "21, 21" in n else "_11"
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), s, r["Queue_Id"], int(r["Grid_Size_Y"])))
rows.sort()
lk = [x for x in rows if x[2] == "lk_multi_kernel_21" and x[4] == a.seq]
first = a.first if a.first >= 0 else len(lk) + a.first
for i in range(first, min(first + a.steps, len(lk) - 1)):
    tp, t0 = lk[i][0], lk[i + 1][0]
    print(f"--- step {i}: period {(t0 - tp) / 1e3:.1f} us")
    for s0, e0, n, q, _ in rows:
        if tp <= s0 < t0:
            print(f"{(s0 - tp) / 1e3:8.1f} {(e0 - tp) / 1e3:8.1f} {(e0 - s0) / 1e3:7.1f} q{q} {n}")
