"""UNet training step on the HIP path: every parameter gradient of the hand-written backward
against torch autograd through the CPU oracle (oracle/unet.py, fp32) — the reference's
``loss.backward()`` (trainers_ldm_cond.py:851-856) over the same graph.

Parity to diffusers is unpinned (diffusers is absent); the oracle restates its
SD-1.x blocks and is itself pinned per op against torch.nn.functional.  Bars: fp32 1e-3 rel
(north star) on the max-abs error of each gradient tensor, relative to its max-abs value;
bf16 8e-2 on the relative L2 error of each gradient tensor: a rounding-noise sanity check, not
the parity gate (the fp32 path is, and is exact to ~1e-6).  The worst bf16 tensors are the bias
gradients of the 4x4 level, sums over 32 positions with heavy cancellation (5-6 % measured,
tools/grad_err_report.py).
"""
import pytest
import torch

from ldmseg.models import UNet
from oracle import unet as ounet

pytestmark = pytest.mark.gpu
DEV = "cuda"
SMALL = dict(block_out_channels=(64, 128, 128, 128), cross_attention_dim=None)


def _unet(seed=0, cond=0):
    torch.manual_seed(seed)
    u = UNet(**SMALL)
    with torch.no_grad():
        for n, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="random", cond_channels=cond,
                     init_mode_cond="random")
    u.freeze_layers(["time_embedding"])          # base.yaml freeze_layers
    return u


def _oracle_grads(u, x, t, gy):
    named = dict(u.named_parameters())
    sd = {k: v.detach().clone() for k, v in u.state_dict().items()}
    leaves = {}
    for k in list(sd):
        if k.startswith("new_conv."):
            sd.pop(k)
            continue
        if named.get(k) is not None and named[k].requires_grad:
            sd[k] = sd[k].requires_grad_(True)
            leaves[k] = sd[k]
    out = ounet.forward(sd, dict(u.config), x, t)
    (out * gy).sum().backward()
    return out.detach(), {k: v.grad for k, v in leaves.items()}


@pytest.mark.parametrize("B,H,cond,t", [(2, 32, 0, 731), (1, 16, 4, 20)])
def test_unet_grads_fp32_match_oracle_autograd(B, H, cond, t):
    u = _unet(cond=cond)
    torch.manual_seed(1)
    x = torch.randn(B, 8 + cond, H, H)
    gy = torch.randn(B, 4, H, H)
    tt = torch.full((B,), t, dtype=torch.long)
    ref_out, ref_g = _oracle_grads(u, x, tt, gy)
    ud = u.to(DEV).train()
    out = ud(x.to(DEV), tt.to(DEV)).sample
    (out * gy.to(DEV)).sum().backward()
    assert ((out.detach().cpu() - ref_out).abs().max() / ref_out.abs().max()).item() < 1e-3
    named = dict(ud.named_parameters())
    assert set(ref_g) == {k for k, p in named.items() if p.requires_grad}
    worst = []
    for k, g in ref_g.items():
        mine = named[k].grad
        assert mine is not None, k
        e = ((mine.cpu() - g).abs().max() / g.abs().max().clamp_min(1e-20)).item()
        worst.append((e, k))
    worst.sort(reverse=True)
    assert worst[0][0] < 1e-3, worst[:5]
    assert all(p.grad is None for p in ud.time_embedding.parameters())


def test_unet_grads_bf16_close_to_oracle():
    u = _unet(seed=3)
    torch.manual_seed(2)
    B, H = 2, 32
    x = torch.randn(B, 8, H, H)
    gy = torch.randn(B, 4, H, H)
    tt = torch.full((B,), 400, dtype=torch.long)
    _, ref_g = _oracle_grads(u, x, tt, gy)
    ud = u.to(DEV, dtype=torch.bfloat16).train()
    out = ud(x.to(DEV, torch.bfloat16), tt.to(DEV)).sample
    (out.float() * gy.to(DEV)).sum().backward()
    named = dict(ud.named_parameters())
    errs = []
    for k, g in ref_g.items():
        mine = named[k].grad.float().cpu()
        errs.append(((mine - g).norm() / g.norm().clamp_min(1e-20)).item())
    assert max(errs) < 8e-2, sorted(errs)[-5:]


def test_unet_grad_accumulates_over_two_backwards():
    u = _unet(seed=4).to(DEV).train()
    torch.manual_seed(3)
    x = torch.randn(1, 8, 16, 16, device=DEV)
    t = torch.tensor([100], device=DEV)
    u(x, t).sample.square().mean().backward()
    g1 = {k: p.grad.clone() for k, p in u.named_parameters() if p.grad is not None}
    u(x, t).sample.square().mean().backward()
    for k, p in u.named_parameters():
        if k in g1:
            assert torch.allclose(p.grad, 2 * g1[k], rtol=1e-5, atol=1e-6), k
