"""The fused transformer feed-forward (ldm_feedforward, csrc/feedforward.hip) vs the two-launch
form it replaces and torch fp32.

The op is diffusers BasicTransformerBlock's  h = ff.net.2(GEGLU(ff.net.0(norm3(h)))) + h  (the
reference UNet runs it through Transformer2DModel, /root/reference/ldmseg/models/unet.py:361-425).
The fused kernel keeps the GEGLU intermediate on chip but walks K in the same order with the same
MFMA instruction per output element and rounds at the same points (h * gelu(g) to bf16, then
bf16(acc + b2) before the residual), so its output must equal the unfused pair
linear(ff2, linear(ff1, x, GEGLU, ln)) bit for bit; against torch fp32 (LayerNorm, exact-erf GELU)
the bar is the conv tests' 2e-2 of the tensor scale.  Covered: the headline shape (B = 8 frames
of 64x64 tokens, one tile per CU) in place with the LayerNorm fold, a ragged M (partial last
tile), several tiles per block (M > 256 tiles), no LayerNorm / no bias2, F = 640, the output row
statistics (against an fp64 sum of the stored rows: the partials are grouped differently from
the tile path's), and the whole UNet forward with the fused path on and off.
"""
import pytest
import torch
import torch.nn.functional as F

from ldmseg.ops import native as K

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16
C = 320


def rel_err(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _weights(Fh, seed, bias2=True):
    g = torch.Generator().manual_seed(seed)
    w1 = torch.randn(2 * Fh, C, generator=g) * C ** -0.5
    b1 = torch.randn(2 * Fh, generator=g) * 0.1
    w2 = torch.randn(C, Fh, generator=g) * Fh ** -0.5
    b2 = torch.randn(C, generator=g) * 0.1 if bias2 else None
    gamma = 1.0 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    return [t if t is None else t.to(DEV) for t in (w1, b1, w2, b2, gamma, beta)]


def _row_stats(x):
    xd = x.double()
    return torch.stack([xd.sum(-1), (xd * xd).sum(-1)], -1).reshape(-1).contiguous()


def _torch_ref(x, w1, b1, w2, b2, gamma, beta, ln):
    xf = x.float()
    n = F.layer_norm(xf, (C,), gamma, beta, 1e-5) if ln else xf
    hg = n @ w1.t() + b1
    h, gt = hg.chunk(2, dim=-1)
    y = (h * F.gelu(gt)) @ w2.t()
    if b2 is not None:
        y = y + b2
    return y + xf


@pytest.mark.parametrize("M,Fh,ln,bias2,inplace", [
    (32768, 1280, True, True, True),        # the 64x64 level at B = 8: one 128-row tile per CU
    (128 * 5 + 37, 1280, False, True, False),   # ragged last tile
    (128 * 300 + 64, 1280, True, False, True),  # > 256 tiles: blocks walk two tiles
    (2048, 640, True, True, False),
])
def test_feedforward_matches_two_launches(M, Fh, ln, bias2, inplace):
    torch.manual_seed(M)
    w1, b1, w2, b2, gamma, beta = _weights(Fh, M, bias2)
    x = (torch.randn(M, C, device=DEV) * 1.5 + 0.3).to(BF)
    pc1 = K.packed_ln_fold(w1, b1, gamma, beta, BF, geglu=True) if ln else K.PackedConv(w1, b1, BF, geglu=True)
    pc2 = K.PackedConv(w2, b2, BF)
    rs = _row_stats(x) if ln else None
    lnarg = (rs, 1e-5) if ln else None
    # the two-launch form (GEGLU GEMM with the gelu epilogue, then ff.net.2 + residual) on unsplit
    # tiles (a split-K plan would sum K in fp32 slabs: same values, other rounding)
    xa = x.clone()
    stats_a = torch.zeros(2 * M, dtype=torch.float64, device=DEV)
    K.force_conv_plan(128, 128, 1)
    try:
        f = K.linear(pc1, xa, out_layout=K.OUT_GEGLU, ln=lnarg)
        ya = K.linear(pc2, f, residual=xa, out=xa if inplace else None, row_stats=stats_a)
    finally:
        K.force_conv_plan(0, 0, 1)
    # fused
    xb = x.clone()
    stats_b = torch.zeros(2 * M, dtype=torch.float64, device=DEV)
    yb = K.feedforward(pc1, pc2, xb, ln=lnarg, residual=xb, out=xb if inplace else None, row_stats=stats_b)
    torch.cuda.synchronize()
    if inplace:
        assert yb.data_ptr() == xb.data_ptr()
    assert torch.equal(ya, yb), f"max |diff| {(ya.float() - yb.float()).abs().max().item()}"
    # row statistics: the tile path adds one fp32 partial per 128-column tile, the fused kernel one
    # per row (the fp64 sums then differ by the fp32 rounding of the partials only)
    sa, sb = stats_a.view(-1, 2), stats_b.view(-1, 2)
    ref_s = _row_stats(yb).view(-1, 2)
    for s_ in (sa, sb):
        assert torch.allclose(s_[:, 0], ref_s[:, 0], rtol=1e-5, atol=1e-3 * C)
        assert torch.allclose(s_[:, 1], ref_s[:, 1], rtol=1e-5, atol=1e-3 * C)
    ref = _torch_ref(x, w1, b1, w2, b2, gamma, beta, ln)
    assert rel_err(yb, ref) < 2e-2


def test_feedforward_rejects_unsupported():
    w1, b1, w2, b2, gamma, beta = _weights(1280, 1)
    x = torch.randn(256, C, device=DEV).to(BF)
    pc1 = K.PackedConv(w1, b1, BF, geglu=True)
    with pytest.raises(ValueError):
        K.feedforward(K.PackedConv(w1, b1, BF), K.PackedConv(w2, b2, BF), x)      # not the GEGLU pack
    x640 = torch.randn(256, 640, device=DEV).to(BF)
    g = torch.Generator().manual_seed(2)
    w1b = (torch.randn(2560, 640, generator=g) * 0.04).to(DEV)
    w2b = (torch.randn(640, 1280, generator=g) * 0.03).to(DEV)
    with pytest.raises(RuntimeError):                                            # width 640: not covered
        K.feedforward(K.PackedConv(w1b, None, BF, geglu=True), K.PackedConv(w2b, None, BF), x640)
    assert not K.feedforward_ok(pc1, K.PackedConv(w2, b2, BF), x)                # 2 tiles: two-launch form


def test_unet_forward_fused_equals_unfused():
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
        u.set_ff_fused(False)
        y0 = u(x, t).sample.clone()
        u.set_ff_fused(True)
        y1 = u(x, t).sample
    torch.cuda.synchronize()
    assert torch.isfinite(y1.float()).all()
    assert torch.equal(y0, y1)


@pytest.mark.parametrize("B,HW", [(8, 64), (3, 64)])
def test_feedforward_with_proj_out_matches_three_launches(B, HW):
    """ldm_feedforward with Transformer2DModel.proj_out behind it (h never stored) vs the fused
    feed-forward followed by the separate proj_out conv (residual = transformer input, GroupNorm
    partials): the same output bits; the GroupNorm totals per (image, unit) within the rounding of
    their fp32 partials."""
    M = B * HW * HW
    w1, b1, w2, b2, gamma, beta = _weights(1280, 7)
    g = torch.Generator().manual_seed(8)
    wpo = (torch.randn(C, C, generator=g) * C ** -0.5).to(DEV)
    bpo = (torch.randn(C, generator=g) * 0.1).to(DEV)
    pc1 = K.packed_ln_fold(w1, b1, gamma, beta, BF, geglu=True)
    pc2 = K.PackedConv(w2, b2, BF)
    pc3 = K.PackedConv(wpo, bpo, BF)
    h = (torch.randn(M, C, device=DEV) * 1.5 + 0.3).to(BF)
    x_in = torch.randn(B, HW, HW, C, device=DEV).to(BF)
    lnarg = (_row_stats(h), 1e-5)
    ha = h.clone()
    K.feedforward(pc1, pc2, ha, ln=lnarg, residual=ha, out=ha)
    ya = K.conv2d(pc3, ha, B, HW, HW, residual=x_in, gn_stats=True)
    hb = h.clone()
    yb = K.feedforward(pc1, pc2, hb, ln=lnarg, residual=hb, proj_out=(pc3, x_in, B, HW, HW, True))
    torch.cuda.synchronize()
    assert torch.equal(ya.view(-1), yb.view(-1)), f"max |diff| {(ya.float() - yb.float()).abs().max().item()}"
    assert torch.equal(hb, h)                      # the feed-forward's output was not stored
    pa, pb = K.gn_stats_of(ya), K.gn_stats_of(yb)
    assert pa is not None and pb is not None and pa.shape == pb.shape
    # per (batch, unit) totals: the separate conv may plan other row tiles (B = 3: 64-row tiles),
    # which spreads the partials over the slots and groups the fp32 sums differently
    assert torch.allclose(pa.sum(1), pb.sum(1), rtol=1e-6, atol=1e-3)
