#!/usr/bin/env python3
"""Fold rocprofv3 PMC passes into profiles/pmc_summary.json.

    python tools/pmc_summary.py FETCH_CSV WRITE_CSV [OUT_JSON] [--label TEXT] [--config NAME]

FETCH_CSV / WRITE_CSV are the `*_counter_collection.csv` files of two separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes over the same command
(the two counters do not fit one pass on gfx950). Per kernel: mean FETCH_SIZE
and WRITE_SIZE per dispatch (KiB), and HBM bytes per launch
    = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(gfx950 FETCH_SIZE counts half the bytes of a read: MI355X_MICROARCH.md §HBM).
The summary is stored under configs[NAME] (bench.py --config; default "kitti"),
so each bench config reads only the counters measured on its own workload.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short_name(k: str) -> str:
    k = k.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", k)


def read(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            acc[short_name(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return acc


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    label, cfg = "", "kitti"
    if "--label" in sys.argv:
        label = sys.argv[sys.argv.index("--label") + 1]
        args.remove(label)
    if "--config" in sys.argv:
        cfg = sys.argv[sys.argv.index("--config") + 1]
        args.remove(cfg)
    fetch_csv, write_csv = args[0], args[1]
    out = args[2] if len(args) > 2 else "profiles/pmc_summary.json"
    fe, wr = read(fetch_csv, "FETCH_SIZE"), read(write_csv, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        f = sum(fe[k]) / len(fe[k]) if fe.get(k) else 0.0
        w = sum(wr[k]) / len(wr[k]) if wr.get(k) else 0.0
        kernels[k] = {"dispatches": max(len(fe.get(k, [])), len(wr.get(k, []))),
                      "fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1),
                      "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}
    try:
        with open(out) as fi:
            doc = json.load(fi)
    except (OSError, ValueError):
        doc = {}
    doc = {"correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halves reads)",
           "configs": doc.get("configs", {})}
    doc["configs"][cfg] = {"source": label, "kernels": kernels}
    with open(out, "w") as fo:
        json.dump(doc, fo, indent=1)
    for k, v in kernels.items():
        print(f"{k:60s} {v['dispatches']:6d} {v['hbm_bytes_per_launch'] / 1e6:10.3f} MB/launch")


if __name__ == "__main__":
    main()
