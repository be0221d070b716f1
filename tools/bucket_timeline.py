"""When each DDP gradient bucket of one config-3 training iteration becomes ready, and how much of a
ring all-reduce of it would stay exposed.  N = 1: no collective runs; the bucketer's
launch points are timed with HIP events on the compute stream (the stream RCCL would wait on), and
the exchange is modelled as a serial queue of ring all-reduces at a given bus bandwidth.
    python tools/bucket_timeline.py [--clips 2] [--bucket-mb 100] [--world 8]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd"))


def ring_ms(nbytes, world, gbs):
    """Ring all-reduce time: 2 (N - 1) / N of the message over the per-rank bus bandwidth."""
    return 2.0 * (world - 1) / world * nbytes / (gbs * 1e9) * 1e3


def exposure(ready, sizes, finish_ms, world, gbs):
    """Serial all-reduce queue in bucket-ready order: (end of the last reduction, exposed ms)."""
    t = 0.0
    for r, s in sorted(zip(ready, sizes)):
        t = max(t, r) + ring_ms(s, world, gbs)
    return t, max(0.0, t - finish_ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=2)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--bucket-mb", type=float, default=100.0)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    from ldmseg.models import UNet
    from ldmseg.schedulers import DDIMNoiseScheduler
    from ldmseg.trainers import LDMTrainStep

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    with torch.device(dev):
        u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero", cond_channels=4,
                     init_mode_cond="zero")
    u.freeze_layers(["time_embedding"])
    u.train()
    sched = DDIMNoiseScheduler(prediction_type="epsilon", beta_schedule="scaled_linear", beta_start=0.00085,
                               beta_end=0.012, steps_offset=1, clip_sample=False, set_alpha_to_one=False,
                               weight="max_clamp_snr", max_snr=2.0, device=dev, verbose=False)
    step = LDMTrainStep(u, sched, lr=1e-4, weight_decay=0.05, clip_grad=1.0, self_condition=True,
                        compute_dtype=torch.bfloat16, seed=1, bucket_mb=args.bucket_mb)
    B, L = args.clips * args.frames, 64
    g = torch.Generator().manual_seed(100)
    lat = torch.randn(B, 4, L, L, generator=g).to(dev)
    rgb = torch.randn(B, 4, L, L, generator=g).to(dev)
    mask = (torch.rand(B, L, L, generator=g) > 0.05).float().to(dev)
    for _ in range(2):
        step.train_step(lat, rgb, mask)
    torch.cuda.synchronize()

    bk = step.bucketer
    marks = {}
    orig_launch, orig_finish = bk._launch, bk.finish

    def launch(b):
        if not bk.launched[b]:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            marks[b] = ev
        orig_launch(b)

    fin = {}

    def finish():
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        fin["ev"] = ev
        orig_finish()

    bk._launch, bk.finish = launch, finish
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        t0.record()
        step.train_step(lat, rgb, mask)
        t1.record()
        torch.cuda.synchronize()
    finally:
        bk._launch, bk.finish = orig_launch, orig_finish
    total = t0.elapsed_time(t1)
    finish_ms = t0.elapsed_time(fin["ev"])
    rows = []
    for b, (s, e, idx) in enumerate(bk.buckets):
        rows.append({"bucket": b, "mb": (e - s) * 4 / 2 ** 20, "params": len(idx),
                     "ready_ms": t0.elapsed_time(marks[b]) if b in marks else finish_ms})
    sizes = [r["mb"] * 2 ** 20 for r in rows]
    ready = [r["ready_ms"] for r in rows]
    first = min(ready)
    print(f"iteration {total:.2f} ms; first bucket ready {first:.2f} ms; backward done (finish) {finish_ms:.2f} ms; "
          f"{len(rows)} buckets, {sum(sizes) / 2 ** 30:.3f} GiB")
    print(f"{'bucket':>6s} {'MiB':>8s} {'params':>6s} {'ready ms':>9s}")
    for r in rows:
        print(f"{r['bucket']:6d} {r['mb']:8.1f} {r['params']:6d} {r['ready_ms']:9.2f}")
    out = {"iteration_ms": total, "finish_ms": finish_ms, "buckets": rows, "model": []}
    for name, gbs in (("one xGMI link (153 GB/s)", 153.0), ("7 xGMI links striped (1071 GB/s)", 1071.0)):
        end, exp = exposure(ready, sizes, finish_ms, args.world, gbs)
        serial = sum(ring_ms(s, args.world, gbs) for s in sizes)
        print(f"{name}: all-reduce total {serial:.2f} ms; last reduction ends {end:.2f} ms; exposed after the "
              f"backward {exp:.2f} ms = {100 * exp / total:.1f} % of the iteration")
        out["model"].append({"link": name, "bus_gbs": gbs, "allreduce_ms": serial, "end_ms": end, "exposed_ms": exp})
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
