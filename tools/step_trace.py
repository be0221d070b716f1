#!/usr/bin/env python3
"""Per-launch breakdown of one graph-replayed denoising step from a rocprofv3 kernel trace.

    python tools/step_trace.py TRACE.csv [--first REGEX] [--top 40] [--csv OUT]

The bench replays the same HIP graph every step, so the trace holds many copies of one launch
sequence.  Steps are cut at every launch of ``--first`` (the step's entry kernel); the most
common sequence of kernel names is taken as the graph step, and every position in it gets the
median duration over its copies, with its grid / workgroup / LDS / register figures.  Unlike the
per-kernel-name stats this separates the shapes one template serves (e.g. every 1x1 GEMM).
"""
import argparse
import csv
import re
import statistics
from collections import Counter


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n)
    n = re.sub(r"unsigned short", "bf16", n)
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", default="conv_in_kernel|nchw_to_nhwc_kernel",
                    help="regex of the step's entry kernel (ldm_conv_in, or the NCHW gather before conv_in)")
    ap.add_argument("--top", type=int, default=0, help="also list the N longest positions")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        if re.search(a.first, r["Kernel_Name"]):
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append(r)
    sig = Counter(tuple(short(r["Kernel_Name"]) for r in s) for s in steps)
    best, n = sig.most_common(1)[0]
    same = [s for s in steps if tuple(short(r["Kernel_Name"]) for r in s) == best]
    print(f"{len(steps)} step candidates, {n} identical sequences of {len(best)} launches")
    out = []
    for i, name in enumerate(best):
        durs = [(int(s[i]["End_Timestamp"]) - int(s[i]["Start_Timestamp"])) / 1e3 for s in same]
        r = same[0][i]
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        out.append(dict(pos=i, kernel=name, blocks=grid // max(wg, 1), wg=wg, lds=int(r["LDS_Block_Size"]),
                        vgpr=int(r["VGPR_Count"]), agpr=int(r["Accum_VGPR_Count"]), us=statistics.median(durs)))
    span = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3 for s in same]
    busy = sum(o["us"] for o in out)
    print(f"step span median {statistics.median(span):.1f} us, kernel busy {busy:.1f} us")
    fam = Counter()
    cnt = Counter()
    for o in out:
        k = re.sub(r"<.*", "", o["kernel"])
        fam[k] += o["us"]
        cnt[k] += 1
    print("\nby kernel template:")
    for k, v in fam.most_common():
        print(f"  {k:40s} {cnt[k]:4d} launches {v:9.1f} us  {100 * v / busy:5.1f} %")
    print("\nper launch:")
    for o in out:
        print(f"  {o['pos']:4d} {o['us']:8.1f}  blocks={o['blocks']:6d} wg={o['wg']:4d} lds={o['lds']:6d} "
              f"v={o['vgpr']:3d}+{o['agpr']:3d}  {o['kernel']}")
    if a.top:
        print(f"\nlongest {a.top}:")
        for o in sorted(out, key=lambda o: -o["us"])[:a.top]:
            print(f"  {o['pos']:4d} {o['us']:8.1f}  blocks={o['blocks']:6d}  {o['kernel']}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0]))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
