#!/usr/bin/env python3
"""Register / LDS / spill summary of every kernel in one HIP source (gfx950), for tuning.

    python tools/kres.py csrc/igemm.hip [name-regex]
"""
import os
import re
import subprocess
import sys
import tempfile


def main(src, filt="."):
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src,
                            "-o", os.path.join(d, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"(SGPRs Spill|VGPRs Spill|VGPRs|AGPRs|ScratchSize|Occupancy|LDS Size)[^:]*: (\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    for c in rows:
        if re.search(filt, c["name"]):
            print(f"{c['name'][:72]:72s} vgpr={c.get('VGPRs')} agpr={c.get('AGPRs')} occ={c.get('Occupancy')} "
                  f"scratch={c.get('ScratchSize')} vspill={c.get('VGPRs Spill')} sspill={c.get('SGPRs Spill')} "
                  f"lds={c.get('LDS Size')}")
    if r.returncode:
        print(r.stderr[-3000:])


if __name__ == "__main__":
    main(*sys.argv[1:])
