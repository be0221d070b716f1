#!/usr/bin/env python3
"""Per-parameter gradient error of the bf16 HIP training path vs the fp32 oracle autograd
(diagnostic for tests/test_gpu_train_unet.py::test_unet_grads_bf16_close_to_oracle)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd"))
import torch  # noqa: E402

from test_gpu_train_unet import _oracle_grads, _unet  # noqa: E402

DEV = "cuda"
for dt in (torch.bfloat16, torch.float32):
    u = _unet(seed=3)
    torch.manual_seed(2)
    B, H = 2, 32
    x = torch.randn(B, 8, H, H)
    gy = torch.randn(B, 4, H, H)
    tt = torch.full((B,), 400, dtype=torch.long)
    ref_out, ref_g = _oracle_grads(u, x, tt, gy)
    ud = u.to(DEV, dtype=dt).train()
    out = ud(x.to(DEV, dt), tt.to(DEV)).sample
    print(dt, "out rel err", ((out.float().cpu() - ref_out).norm() / ref_out.norm()).item())
    (out.float() * gy.to(DEV)).sum().backward()
    named = dict(ud.named_parameters())
    errs = []
    for k, g in ref_g.items():
        mine = named[k].grad.float().cpu()
        errs.append((((mine - g).norm() / g.norm().clamp_min(1e-20)).item(), k))
    errs.sort(reverse=True)
    for e, k in errs[:12]:
        print(f"  {e:.4f} {k}")
