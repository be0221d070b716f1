#!/usr/bin/env python3
"""Summarise tools/pmc_passes.sh output: per (kernel, grid) median of every counter, plus derived metrics."""
import csv
import glob
import os
import sys
from collections import defaultdict


def _short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return name.split("(")[0][:60]


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            key = (_short(r["Kernel_Name"]), r["Grid_Size"])
            vals[key][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(d, "p1", "pmc_kernel_trace.csv"))):
        for r in csv.DictReader(open(f)):
            key = (_short(r["Kernel_Name"]), str(int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])))
            durs[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for key, dv in vals.items():
        per = defaultdict(list)
        for (disp, cn), v in dv.items():
            per[cn].append(sum(v))          # sum over dimension instances of one dispatch
        med = {cn: sorted(v)[len(v) // 2] for cn, v in per.items()}
        print(f"== {key[0]} grid={key[1]}  dur(us)={sorted(durs.get(key, [0]))[len(durs.get(key, [0])) // 2]:.1f}")
        for cn in sorted(med):
            print(f"   {cn:28s} {med[cn]:16.0f}")
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in med:
                    print(f"   {c + '/WAVE_CYCLES':40s} {med[c] / wc:8.3f}")
        if "TCC_HIT_sum" in med:
            print(f"   L2 hit rate {med['TCC_HIT_sum'] / max(1, med['TCC_HIT_sum'] + med['TCC_MISS_sum']):.3f}")
        if "FETCH_SIZE" in med:
            print(f"   FETCH_SIZE x2 (gfx950 correction) = {2 * med['FETCH_SIZE'] / 1024:.1f} MB")
        if "WRITE_SIZE" in med:
            print(f"   WRITE_SIZE = {med['WRITE_SIZE'] / 1024:.1f} MB")


if __name__ == "__main__":
    main(sys.argv[1])
