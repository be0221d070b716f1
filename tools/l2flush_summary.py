#!/usr/bin/env python3
"""Per-launch FETCH_SIZE / WRITE_SIZE of one kernel from tools/l2flush.sh's --pmc passes.

    python tools/l2flush_summary.py OUTDIR KERNEL_REGEX [--skip 3]

OUTDIR holds {case}_{prev}_{fetch,write}/ rocprofv3 directories.  Prints one line per (case, prev):
launches, MB fetched (2 x FETCH_SIZE: gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md
"HBM") and MB written per launch, over the matching dispatches after the first --skip (warm-up).
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def per_dispatch(d, counter, rx):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        return []
    vals, names = defaultdict(float), {}
    for r in csv.DictReader(open(paths[0])):
        if r["Counter_Name"] != counter:
            continue
        vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    return [vals[k] for k in sorted(vals) if re.search(rx, names[k])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("kernel")
    ap.add_argument("--skip", type=int, default=3)
    a = ap.parse_args()
    runs = sorted({os.path.basename(p).rsplit("_", 1)[0] for p in glob.glob(os.path.join(a.outdir, "*_fetch"))})
    for r in runs:
        f = per_dispatch(os.path.join(a.outdir, r + "_fetch"), "FETCH_SIZE", a.kernel)[a.skip:]
        w = per_dispatch(os.path.join(a.outdir, r + "_write"), "WRITE_SIZE", a.kernel)[a.skip:]
        fm = 2.0 * sum(f) / max(1, len(f)) * 1024 / 1e6
        wm = sum(w) / max(1, len(w)) * 1024 / 1e6
        wmin = min(w) * 1024 / 1e6 if w else 0.0
        wmax = max(w) * 1024 / 1e6 if w else 0.0
        print(f"{r:40s} launches {len(f):3d}/{len(w):3d}  fetch {fm:8.2f} MB  write {wm:8.2f} MB "
              f"(min {wmin:.2f} max {wmax:.2f})")


if __name__ == "__main__":
    main()
