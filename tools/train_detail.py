"""Per-op time of one config-3 training iteration (bench.py --mode train's step), by op family and
shape, from the launch profiler's HIP events (each op bracketed, so the sum is a little above
the graph-free iteration time).  python tools/train_detail.py [--clips 2] [--top 50]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=2)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--top", type=int, default=50)
    args = ap.parse_args()
    from ldmseg.models import UNet
    from ldmseg.ops import native as K
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
                        compute_dtype=torch.bfloat16, seed=1)
    B, L = args.clips * args.frames, 64
    g = torch.Generator().manual_seed(100)
    lat = torch.randn(B, 4, L, L, generator=g).to(dev)
    rgb = torch.randn(B, 4, L, L, generator=g).to(dev)
    mask = (torch.rand(B, L, L, generator=g) > 0.05).float().to(dev)
    for _ in range(2):
        step.train_step(lat, rgb, mask)
    torch.cuda.synchronize()
    prof = K.LaunchProfiler()
    K.set_profiler(prof)
    try:
        step.train_step(lat, rgb, mask)
    finally:
        K.set_profiler(None)
    det = prof.summary(by_detail=True)
    fam = prof.summary()
    tot = sum(v["ms"] for v in fam.values())
    print(f"profiled ops: {tot:.2f} ms")
    for f, v in sorted(fam.items(), key=lambda kv: -kv[1]["ms"]):
        print(f"  {f:14s} {v['launches']:5d} {v['ms']:8.3f} ms")
    print(f"{'family':12s} {'shape':56s} {'n':>4s} {'ms':>8s} {'TF/s':>7s}")
    for (f, s), v in sorted(det.items(), key=lambda kv: -kv[1]["ms"])[:args.top]:
        tf = v["flops"] / v["ms"] / 1e9 if v["ms"] else 0.0
        print(f"{f:12s} {s[:56]:56s} {v['launches']:4d} {v['ms']:8.3f} {tf:7.1f}")


if __name__ == "__main__":
    main()
