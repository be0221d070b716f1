#!/usr/bin/env python3
"""Turn the rocprofv3 output of tools/profile_bench.sh into the committed profiles/ summary.

    python tools/rocprof_summary.py --stats DIR --fetch DIR --write DIR --tag r01 [--bench LOG]

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of `python bench.py`
  profiles/<tag>_families.json      per kernel family: launches (host-API calls), average duration
                                    per call, and HBM traffic per call from the PMC passes
                                    (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md "HBM [CDNA4]")
  profiles/<tag>_summary.md         human-readable table of the above

A "family" is what one C-ABI call launches: ldm_conv2d = igemm_kernel (+ splitk_epilogue_kernel
when the plan splits K), ldm_attention = attn_kernel, ldm_group_norm = gn_* kernels, ...  The
per-call average is sum(duration of every kernel in the family) / number of primary launches,
which is what bench.py's HIP events bracket.
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_families import kind_of  # noqa: E402  (the table shared with traffic_table / step_trace)


def family_of(name):
    """(family, is_primary): primary kernels count calls; others add time / traffic to their family."""
    fam, role = kind_of(name)
    if fam is None:
        return "other", True
    return fam, role == "p"


def _one(pattern):
    hits = glob.glob(pattern, recursive=True)
    if not hits:
        raise SystemExit(f"no file matches {pattern}")
    return hits[0]


def read_stats(d):
    path = _one(os.path.join(d, "**", "*kernel_stats.csv"))
    rows = list(csv.DictReader(open(path)))
    return path, rows


def read_counter(d, counter):
    """Per-dispatch sum of `counter` (over dimension instances) -> {family: (primary calls, total)}."""
    path = _one(os.path.join(d, "**", "*counter_collection.csv"))
    per_disp = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per_disp[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    fam = defaultdict(lambda: [0, 0.0])
    for disp, v in per_disp.items():
        f, primary = family_of(names[disp])
        fam[f][0] += int(primary)
        fam[f][1] += v
    return fam


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--bench", help="bench.py stdout of the --stats run (its JSON line is embedded)")
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)

    path, rows = read_stats(a.stats)
    shutil.copy(path, os.path.join(out_dir, f"{a.tag}_kernel_stats.csv"))
    fams = defaultdict(lambda: dict(calls=0, total_ns=0.0, kernels=[]))
    for r in rows:
        f, primary = family_of(r["Name"])
        d = fams[f]
        d["calls"] += int(r["Calls"]) if primary else 0
        d["total_ns"] += float(r["TotalDurationNs"])
        d["kernels"].append((r["Name"], int(r["Calls"]), float(r["AverageNs"])))
    fetch = read_counter(a.fetch, "FETCH_SIZE") if a.fetch else {}
    write = read_counter(a.write, "WRITE_SIZE") if a.write else {}

    result = {}
    for f, d in fams.items():
        e = {"calls": d["calls"], "total_ms": round(d["total_ns"] / 1e6, 3),
             "avg_call_ms": round(d["total_ns"] / max(1, d["calls"]) / 1e6, 5)}
        if f in fetch and f in write and fetch[f][0]:
            # FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE reports half of wide streaming reads on gfx950
            fb = 2.0 * fetch[f][1] * 1024 / fetch[f][0]
            wb = write[f][1] * 1024 / max(1, write[f][0])
            e.update(fetch_bytes_per_call=round(fb), write_bytes_per_call=round(wb),
                     traffic_bytes_per_call=round(fb + wb), pmc_calls=fetch[f][0])
        result[f] = e
    bench = None
    if a.bench and os.path.exists(a.bench):
        for line in open(a.bench):
            if line.startswith("{"):
                bench = json.loads(line)
    workload = ((bench or {}).get("roofline") or {}).get("pmc_workload")
    meta = {"tag": a.tag, "command": "python3 bench.py (see tools/profile_bench.sh)", "workload": workload,
            "traffic_method": "2*FETCH_SIZE + WRITE_SIZE (KiB->bytes), separate --pmc passes, eager steps",
            "families": result, "bench": bench}
    json.dump(meta, open(os.path.join(out_dir, f"{a.tag}_families.json"), "w"), indent=1)

    total = sum(d["total_ns"] for d in fams.values())
    lines = [f"# rocprofv3 summary ({a.tag})", "",
             "Source: `tools/profile_bench.sh` (rocprofv3 --kernel-trace --stats over `python3 bench.py`; "
             "FETCH_SIZE and WRITE_SIZE in their own --pmc passes).", "",
             "| family | calls | total ms | avg/call us | share | HBM bytes/call (PMC) |", "|---|---|---|---|---|---|"]
    for f, d in sorted(fams.items(), key=lambda kv: -kv[1]["total_ns"]):
        e = result[f]
        tr = e.get("traffic_bytes_per_call")
        lines.append(f"| {f} | {d['calls']} | {d['total_ns'] / 1e6:.2f} | {e['avg_call_ms'] * 1e3:.1f} | "
                     f"{d['total_ns'] / total:.1%} | {tr / 1e6:.2f} MB |" if tr else
                     f"| {f} | {d['calls']} | {d['total_ns'] / 1e6:.2f} | {e['avg_call_ms'] * 1e3:.1f} | "
                     f"{d['total_ns'] / total:.1%} | - |")
    lines += ["", "## kernels", "", "| kernel | calls | avg us |", "|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        nm = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        lines.append(f"| `{nm}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} |")
    if bench:
        lines += ["", "## bench line of the profiled run", "", "```", json.dumps(bench), "```"]
    open(os.path.join(out_dir, f"{a.tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:14]))


if __name__ == "__main__":
    main()
