#!/usr/bin/env python3
"""Per-parameter gradient error of the native AE training step vs tests/golden/ae.npz (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd")]
import torch  # noqa: E402

from golden_utils import load  # noqa: E402
from test_gpu_train_ae import Replay, _grads, _inputs, _model  # noqa: E402

z = load("ae.npz")
m = _model(z)
bits, targets = _inputs(z)
ce, mask, grads = _grads(m, bits, targets, Replay())
print("ce", ce.item(), float(z["ce"]), "mask", mask.item(), float(z["mask"]))
named = dict(m.named_parameters())
for name in z["names"]:
    name = str(name)
    ref = torch.from_numpy(z[f"g__{name}"])
    got = grads[named[name]].cpu()
    print(f"{name:24s} {((got - ref).norm() / ref.norm()).item():.2e}  |ref| {ref.norm().item():.3e}")
