"""Same-box A/B of the graph-replayed denoising step under library tuning hooks.

Box-to-box spread on an unchanged tree is several percent, so a change worth ~1 % is measured here
as interleaved windows of two (or more) captured step graphs in ONE process: each variant applies
its hooks, captures its own DenoiseStep graph, and the variants' timed windows alternate.
    python tools/ab_step.py --frames 8 --variant base "" --variant nofa "K.set_conv_fast_addressing(0)"
A variant's hooks are reset by the next variant's setup (pass explicit values in every variant that
touches a hook)."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variant", nargs=2, action="append", metavar=("NAME", "HOOKS"), required=True)
    args = ap.parse_args()
    import bench
    from ldmseg.ops import native as K
    from ldmseg.pipelines import DenoiseStep

    dev = torch.device("cuda", 0)
    unet = bench.build_unet(dev, torch.bfloat16)
    sched = bench.make_scheduler(dev)
    g = torch.Generator().manual_seed(1)
    rgb = torch.randn(args.frames, 4, 64, 64, generator=g).to(dev)
    lat = torch.randn(args.frames, 4, 64, 64, generator=g).to(dev)
    ts = [int(t) for t in sched.timesteps]
    steppers = {}
    for name, hooks in args.variant:
        exec(hooks, {"K": K, "unet": unet})
        st = DenoiseStep(unet, sched, rgb, self_condition=False, use_graph=True)
        st.set_latents(lat.clone())
        for i in range(3):
            st.run(ts[i], last=False)
        steppers[name] = st
    torch.cuda.synchronize()
    times = {n: [] for n in steppers}
    for _ in range(args.rounds):
        for name, st in steppers.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                st.run(ts[k % len(ts)], last=False)
            torch.cuda.synchronize()
            times[name].append((time.perf_counter() - t0) / args.steps * 1e3)
    out = {n: {"median_ms": sorted(v)[len(v) // 2], "windows_ms": [round(x, 4) for x in v]} for n, v in times.items()}
    print(json.dumps({"frames": args.frames, "variants": out}))


if __name__ == "__main__":
    main()
