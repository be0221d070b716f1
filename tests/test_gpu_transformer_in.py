"""The fused Transformer2DModel input half (ldm_transformer_in, csrc/transformer_in.hip) vs the
three launches it replaces and torch fp32.

The op is diffusers Transformer2DModel's  h = proj_in(norm(x)); qkv = to_qkv(norm1(h))  (the
reference UNet runs it through /root/reference/ldmseg/models/unet.py:361-425).  The fused kernel
finalises the GroupNorm from the producer's unit accumulators like gn_apply, runs the same MFMA
sequence per output element, sums the LayerNorm row statistics in the row writer's order and rounds
at the same points, so h and qkv must equal group_norm -> linear(row_stats) -> linear(ln) bit for bit;
against torch fp32 (GroupNorm, Linear, LayerNorm, Linear) the bar is the conv tests' 2e-2 of the
tensor scale.  Covered: the headline shape (B = 8 frames of 64x64 tokens, one tile per CU), two tiles
per block (B = 16), a batch whose images have very different means (the fp64 statistics), and the
whole UNet forward with the fused path on and off.
"""
import pytest
import torch
import torch.nn.functional as F

from ldmseg.ops import native as K

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16
C = 320
HW = 64


def rel_err(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _setup(B, seed, spread=1.0):
    g = torch.Generator().manual_seed(seed)
    wc = (torch.randn(C, C, generator=g) * C ** -0.5).to(DEV)             # the producing 1x1 conv
    bc = (torch.randn(C, generator=g) * 0.1).to(DEV)
    w_in = (torch.randn(C, C, generator=g) * C ** -0.5).to(DEV)
    b_in = (torch.randn(C, generator=g) * 0.1).to(DEV)
    wq = (torch.randn(3 * C, C, generator=g) * C ** -0.5).to(DEV)
    gam = (1.0 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    bet = (0.1 * torch.randn(C, generator=g)).to(DEV)
    ln_g = (1.0 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    ln_b = (0.1 * torch.randn(C, generator=g)).to(DEV)
    x_raw = torch.randn(B, HW, HW, C, generator=g)
    x_raw = x_raw * spread + torch.arange(B).view(B, 1, 1, 1) * (spread - 1.0)   # per-image offsets
    x_raw = x_raw.to(DEV).to(BF)
    pcc = K.PackedConv(wc, bc, BF)
    x = K.conv2d(pcc, x_raw, B, HW, HW, gn_stats=True)                  # carries the unit accumulators
    pc_in = K.PackedConv(w_in, b_in, BF)
    pc_q = K.packed_ln_fold(wq, None, ln_g, ln_b, BF)
    return x, pc_in, pc_q, (gam, bet), (w_in, b_in, wq, ln_g, ln_b)


@pytest.mark.parametrize("B,spread", [(8, 1.0), (16, 1.0), (8, 4.0)])
def test_transformer_in_matches_three_launches(B, spread):
    x, pc_in, pc_q, (gam, bet), (w_in, b_in, wq, ln_g, ln_b) = _setup(B, 10 + B, spread)
    N = HW * HW
    assert K.transformer_in_ok(pc_in, pc_q, x, B, N, 32)
    # the three launches
    h_a = K.group_norm(x, B, N, 32, gam, bet, 1e-6)
    rs = torch.zeros(2 * B * N, dtype=torch.float64, device=DEV)
    h_a = K.linear(pc_in, h_a, row_stats=rs)
    q_a = K.linear(pc_q, h_a, ln=(rs, 1e-5))
    # fused
    h_b, q_b = K.transformer_in(pc_in, pc_q, x, B, N, 32, gam, bet, 1e-6, 1e-5)
    torch.cuda.synchronize()
    assert torch.equal(h_a.view(-1), h_b.view(-1)), f"h max |diff| {(h_a.float().view(-1) - h_b.float().view(-1)).abs().max().item()}"
    assert torch.equal(q_a.view(-1), q_b.view(-1)), f"qkv max |diff| {(q_a.float().view(-1) - q_b.float().view(-1)).abs().max().item()}"
    # torch fp32 reference of the same arithmetic
    xf = x.float().view(B, N, C)
    n = F.group_norm(xf.permute(0, 2, 1), 32, gam, bet, 1e-6).permute(0, 2, 1)
    h_ref = n @ w_in.t() + b_in
    q_ref = F.layer_norm(h_ref, (C,), ln_g, ln_b, 1e-5) @ wq.t()
    assert rel_err(h_b.view(B, N, C), h_ref) < 2e-2
    assert rel_err(q_b.view(B, N, 3 * C), q_ref) < 2e-2


def test_transformer_in_scope():
    x, pc_in, pc_q, (gam, bet), _ = _setup(2, 3)
    N = HW * HW
    assert not K.transformer_in_ok(pc_in, pc_q, x, 2, N, 32)                # 64 tiles: three-launch form
    with pytest.raises(ValueError):
        K.transformer_in(pc_in, pc_q, x, 2, N, 32, gam, bet, 1e-6, 1e-5)
    x8, pc_in8, pc_q8, _, _ = _setup(8, 4)
    assert not K.transformer_in_ok(pc_in8, K.PackedConv(torch.randn(3 * C, C, device=DEV), None, BF), x8, 8, N, 32)
    assert not K.transformer_in_ok(pc_in8, pc_q8, x8.clone(), 8, N, 32)      # no producer statistics


def test_unet_forward_tin_fused_equals_unfused():
    from ldmseg.models import UNet
    torch.manual_seed(0)
    with torch.device(DEV):
        u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero")
    u = u.to(BF).eval()
    x = torch.randn(8, 8, 64, 64, device=DEV).to(BF)
    t = torch.full((8,), 500, device=DEV, dtype=torch.long)
    with torch.no_grad():
        u.set_tin_fused(False)
        y0 = u(x, t).sample.clone()
        u.set_tin_fused(True)
        y1 = u(x, t).sample
    torch.cuda.synchronize()
    assert torch.isfinite(y1.float()).all()
    assert torch.equal(y0, y1)
