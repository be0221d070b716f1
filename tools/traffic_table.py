#!/usr/bin/env python3
"""Per-op HBM traffic of one UNet step: rocprofv3 FETCH_SIZE / WRITE_SIZE per dispatch, aligned
with the op log bench.py writes for the same run (LDM_OPLOG), against each op's algorithmic bytes.

    python tools/traffic_table.py --fetch DIR --write DIR --oplog FETCH_OPLOG.json [--md OUT.md]

The PMC passes run `bench.py --no-graph --profile-steps 1` (tools/profile_bench.sh), whose last
step is the profiled eager step the op log describes.  Each logged op (family, algorithmic bytes,
shape detail) is matched in order to the dispatches of its family at the end of the trace:
primary kernels start an op; split-K reductions attach to the op before them, GroupNorm statistics
and fp8 K/V quantisation to the op after them; torch / copy kernels are skipped.
HBM bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md "HBM": FETCH_SIZE counts
half of a wide streaming read on gfx950; WRITE_SIZE is exact for 16-B stores, see
tools/write_calib.hip for the other store shapes), KB as rocprofv3 reports them.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_families import kind_of  # noqa: E402  (the table shared with rocprof_summary / step_trace)


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", n).replace("unsigned short", "bf16")[:60]


def read_counter(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(float)
    meta = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        did = int(r["Dispatch_Id"])
        per[did] += float(r["Counter_Value"])
        meta[did] = (r["Kernel_Name"], int(r["Grid_Size"]))
    return per, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--oplog", required=True)
    ap.add_argument("--md", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    fetch, meta = read_counter(a.fetch, "FETCH_SIZE")
    write, wmeta = read_counter(a.write, "WRITE_SIZE")
    ops = json.load(open(a.oplog))["ops"]
    disp = sorted(meta)
    # the profiled step is the tail of the trace: walk backwards over the dispatches, matching the
    # op log from its end (so the warmup / timed eager steps before it are never touched)
    assign = {}
    oi = len(ops) - 1
    pending_post = []
    first = None
    for did in reversed(disp):
        if oi < 0:
            break
        fam, role = kind_of(meta[did][0])
        if fam is None:
            continue
        if role == "post":
            pending_post.append(did)
            continue
        if role == "pre":                       # belongs to the op after it (already assigned)
            if oi + 1 < len(ops):
                assign.setdefault(oi + 1, []).append(did)
            continue
        # strict alignment: the dispatch must be the op the log names next (walking back), so a
        # kernel the family table does not know can never shift the kernel column against the ops
        if ops[oi]["family"] != fam:
            raise SystemExit(f"traffic_table: dispatch {did} ({short(meta[did][0])}, family {fam}) does not "
                             f"match op {oi} ({ops[oi]['family']}: {ops[oi]['detail']}); "
                             f"is a kernel missing from tools/kernel_families.py?")
        assign.setdefault(oi, []).extend([did] + pending_post)
        pending_post = []
        first = did
        oi -= 1
    if oi >= 0:
        raise SystemExit(f"traffic_table: {oi + 1} ops of the log have no dispatch")
    nprim = sum(1 for d in disp if d >= first and kind_of(meta[d][0])[1] == "p")
    if nprim != len(ops):
        raise SystemExit(f"traffic_table: {nprim} primary dispatches in the profiled step, {len(ops)} ops logged")
    rows = []
    for i, op in enumerate(ops):
        ds = assign.get(i)
        if not ds:
            continue
        f = sum(fetch.get(d, 0.0) for d in ds) * 1024.0
        w = sum(write.get(d, 0.0) for d in ds) * 1024.0
        hbm = 2.0 * f + w
        rows.append(dict(op=i, family=op["family"], detail=op["detail"] or op["family"],
                         kernels=",".join(sorted({short(meta[d][0]) for d in ds})),
                         alg_mb=op["bytes"] / 1e6, fetch2_mb=2.0 * f / 1e6, write_mb=w / 1e6, hbm_mb=hbm / 1e6,
                         ratio=hbm / op["bytes"] if op["bytes"] else 0.0))
    fam_tot = defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])
    for r in rows:
        t = fam_tot[r["family"]]
        t[0] += 1
        t[1] += r["alg_mb"]
        t[2] += r["fetch2_mb"]
        t[3] += r["write_mb"]
        t[4] += r["hbm_mb"]
    lines = ["| family | ops | algorithmic MB | 2xFETCH MB | WRITE MB | PMC / algorithmic |", "|---|---|---|---|---|---|"]
    for fam, t in sorted(fam_tot.items(), key=lambda kv: -kv[1][4]):
        lines.append(f"| {fam} | {t[0]} | {t[1]:.1f} | {t[2]:.1f} | {t[3]:.1f} | {t[4] / max(t[1], 1e-9):.2f} |")
    lines += ["", "| # | op (shape) | kernel(s) | algorithmic MB | 2xFETCH MB | WRITE MB | PMC / algorithmic |",
              "|---|---|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| {r['op']} | {r['detail']} | {r['kernels']} | {r['alg_mb']:.1f} | {r['fetch2_mb']:.1f} | "
                     f"{r['write_mb']:.1f} | {r['ratio']:.2f} |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out + "\n")
    if a.json:
        json.dump({"families": {k: dict(ops=v[0], alg_mb=v[1], fetch2_mb=v[2], write_mb=v[3], hbm_mb=v[4])
                                for k, v in fam_tot.items()}, "ops": rows}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
