"""Training-path kernels (backward + optimizer) against torch autograd / torch.optim in fp32.

Every case runs the HIP kernel through the C-ABI in the exact fp32 mode (tolerance 1e-4 rel
unless stated; the 1e-3 north-star bar with margin) and in bf16 (5e-2 rel, the bf16
storage bar of the forward tests).  Edge cases: ragged M / N, concat inputs, stride 2 and
nearest-2x geometry, GEGLU interleave, odd token counts for attention, partial K tiles.
"""
import pytest
import torch
import torch.nn.functional as F

from ldmseg.models.unet_train import packed_dgrad
from ldmseg.ops import native as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def tol(dt):
    return 1e-4 if dt == torch.float32 else 5e-2


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


# ------------------------------------------------------------------ conv data + weight grads
CONV_CASES = [
    # B, H, W, c0, c1, cout, k, stride, up
    (2, 16, 16, 64, 0, 64, 3, 1, False),
    (2, 12, 10, 32, 48, 40, 3, 1, False),       # concat input, ragged spatial, cout % 16 != 0
    (2, 16, 16, 64, 0, 96, 3, 2, False),        # Downsample2D
    (2, 8, 8, 64, 0, 64, 3, 1, True),           # Upsample2D (nearest-2x + conv)
    (3, 7, 9, 128, 64, 72, 1, 1, False),        # 1x1 shortcut on a concat
    (1, 5, 5, 16, 0, 320, 3, 1, False),         # conv_in-like (few input channels)
    (4, 32, 32, 320, 0, 320, 3, 1, False),      # many 64-pixel stages per split (L2-touch pipeline)
    (2, 32, 32, 128, 64, 160, 3, 1, False),     # the same with a concat source and a ragged tile
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv_grads(case, dt):
    B, H, W, c0, c1, cout, k, stride, up = case
    torch.manual_seed(0)
    x = torch.randn(B, c0 + c1, H, W, device=DEV)
    w = torch.randn(cout, c0 + c1, k, k, device=DEV) * 0.1
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    inp = F.interpolate(xr, scale_factor=2.0, mode="nearest") if up else xr
    y = F.conv2d(inp, wr, stride=stride, padding=k // 2)
    gy = torch.randn_like(y)
    y.backward(gy)
    xq = x.to(dt)
    x0, x1 = nhwc(xq[:, :c0]), (nhwc(xq[:, c0:]) if c1 else None)
    dyq = nhwc(gy.to(dt))
    pc = K.PackedConv(w, None, dt)
    dw = K.conv2d_wgrad(pc, x0, B, H, W, dyq, x1=x1, stride=stride, upsample=up).view_as(w)
    assert rel(dw, wr.grad) < tol(dt)
    # accumulate mode adds
    dw2 = K.conv2d_wgrad(pc, x0, B, H, W, dyq, x1=x1, stride=stride, upsample=up, dw=dw.clone(), accumulate=True)
    assert rel(dw2, 2 * wr.grad) < tol(dt)
    # data gradient through the transposed / flipped packed weight
    pd = packed_dgrad(w, dt)
    Ho, Wo = y.shape[2], y.shape[3]
    if stride == 2:
        dx = K.conv2d(pd, dyq, B, Ho, Wo, upsample=2)
    elif up:
        du = K.conv2d(pd, dyq, B, Ho, Wo)
        dx = K.sum_pool2(du, B, H, W)
    else:
        dx = K.conv2d(pd, dyq, B, Ho, Wo)
    assert rel(nchw(dx.view(B, H, W, c0 + c1)), xr.grad) < tol(dt)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_geglu_linear_grads(dt):
    torch.manual_seed(1)
    rows, C, F4 = 200, 64, 128
    x = torch.randn(rows, C, device=DEV)
    w = torch.randn(2 * F4, C, device=DEV) * 0.1
    b = torch.randn(2 * F4, device=DEV) * 0.1
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    hg = F.linear(xr, wr, br)
    h, g = hg.chunk(2, dim=-1)
    out = h * F.gelu(g)
    go = torch.randn_like(out)
    out.backward(go)
    pc = K.PackedConv(w, b, dt, geglu=True)
    hq = K.linear(pc, x.to(dt))                                  # packed [h16 | g16] interleave
    fq = K.geglu_fwd(hq)
    assert rel(fq, out) < tol(dt) * 2
    dhg = K.geglu_bwd(hq, go.to(dt).contiguous())
    dw = K.conv2d_wgrad(pc, x.to(dt).contiguous(), rows, 1, 1, dhg)
    assert rel(dw, wr.grad) < tol(dt) * 2
    db = K.colsum(dhg, rows, 2 * F4, geglu=True).view(-1)
    assert rel(db, br.grad) < tol(dt) * 2
    dx = K.conv2d(packed_dgrad(w, dt, geglu=True), dhg, rows, 1, 1).view_as(x)
    assert rel(dx, xr.grad) < tol(dt) * 2


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_colsum_segments(dt):
    torch.manual_seed(2)
    x = torch.randn(4, 300, 40, device=DEV).to(dt)
    s = K.colsum(x.contiguous(), 1200, 40, segments=4)
    assert rel(s, x.float().sum(1)) < 1e-5
    s1 = K.colsum(x.contiguous(), 1200, 40, segments=1, out=s.sum(0).clone(), accumulate=True)
    assert rel(s1.view(-1), 2 * x.float().sum((0, 1))) < 1e-5


# ------------------------------------------------------------------ norms
@pytest.mark.parametrize("act", [K.ACT_NONE, K.ACT_SILU])
@pytest.mark.parametrize("c0,c1,G", [(64, 0, 32), (80, 48, 32), (320, 0, 32)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_group_norm_grads(act, c0, c1, G, dt):
    torch.manual_seed(3)
    B, H, W = 2, 8, 12
    C = c0 + c1
    x = torch.randn(B, C, H, W, device=DEV) * 2 + 0.5
    gam = torch.randn(C, device=DEV)
    bet = torch.randn(C, device=DEV)
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, gam, bet))
    y = F.group_norm(xr, G, gr, br, 1e-5)
    if act == K.ACT_SILU:
        y = F.silu(y)
    gy = torch.randn_like(y)
    y.backward(gy)
    xq = x.to(dt)
    x0, x1 = nhwc(xq[:, :c0]), (nhwc(xq[:, c0:]) if c1 else None)
    out, mr = K.group_norm_train(x0, B, H * W, G, gam, bet, 1e-5, act, x1=x1)
    assert rel(nchw(out.view(B, H, W, C)), y) < tol(dt) * 2
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)
    add = torch.randn(B, H, W, C, device=DEV)
    dx0, dx1 = K.group_norm_bwd(x0, B, H * W, G, mr, gam, bet, act, nhwc(gy.to(dt)), x1=x1,
                                add_src=add.to(dt).contiguous(), dgamma=dg, dbeta=db)
    dx = torch.cat([dx0.view(B, H, W, c0)] + ([dx1.view(B, H, W, c1)] if c1 else []), dim=-1)
    assert rel(nchw(dx), xr.grad + nchw(add)) < tol(dt) * 2
    assert rel(dg, gr.grad) < tol(dt) * 2 and rel(db, br.grad) < tol(dt) * 2


@pytest.mark.parametrize("C", [64, 320, 640, 1280])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layer_norm_grads(C, dt):
    torch.manual_seed(4)
    rows = 333
    x = torch.randn(rows, C, device=DEV) + 0.3
    gam, bet = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, gam, bet))
    y = F.layer_norm(xr, (C,), gr, br, 1e-5)
    gy = torch.randn_like(y)
    y.backward(gy)
    add = torch.randn(rows, C, device=DEV)
    dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
    dx = K.layer_norm_bwd(x.to(dt).contiguous(), gy.to(dt).contiguous(), gam, 1e-5, add_src=add.to(dt).contiguous(),
                          dgamma=dg, dbeta=db)
    assert rel(dx, xr.grad + add) < tol(dt) * 2
    assert rel(dg, gr.grad) < tol(dt) * 2 and rel(db, br.grad) < tol(dt) * 2


# ------------------------------------------------------------------ attention
@pytest.mark.parametrize("B,N,heads,d", [(2, 256, 8, 40), (1, 200, 8, 80), (2, 64, 8, 160), (1, 97, 2, 64),
                                         (1, 300, 4, 32), (1, 4096, 8, 40), (1, 130, 2, 48)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_attention_grads(B, N, heads, d, dt):
    torch.manual_seed(5)
    C = heads * d
    qkv = torch.randn(B, N, 3 * C, device=DEV) * 0.5
    qr = qkv.clone().requires_grad_(True)
    q, k, v = qr.split(C, dim=-1)

    def sp(t):
        return t.reshape(B, N, heads, d).permute(0, 2, 1, 3)
    o = F.scaled_dot_product_attention(sp(q), sp(k), sp(v)).permute(0, 2, 1, 3).reshape(B, N, C)
    go = torch.randn_like(o)
    o.backward(go)
    qq = qkv.to(dt).contiguous()
    oo, lse = K.attention_fwd_lse(qq, qq[..., C:], qq[..., 2 * C:], B, heads, d, N, N, 3 * C, 3 * C, 3 * C)
    assert rel(oo, o) < tol(dt) * 2
    dqkv = torch.empty_like(qq)
    K.attention_bwd(qq, qq[..., C:], qq[..., 2 * C:], oo, go.to(dt).contiguous(), lse, B, heads, d, N, N, 3 * C,
                    3 * C, 3 * C, dqkv, dqkv[..., C:], dqkv[..., 2 * C:], 3 * C, 3 * C)
    for i in range(3):
        assert rel(dqkv[..., i * C:(i + 1) * C], qr.grad[..., i * C:(i + 1) * C]) < tol(dt) * 4, i


@pytest.mark.parametrize("N,d", [(4096, 40), (1000, 64), (77, 32)])
def test_attention_bwd32_matches_16x16_kernels(N, d):
    """The 32x32x16-MFMA backward (head_dim <= 64) against the 16x16x16 kernels it replaced, same
    bf16 inputs: both are fp32-accumulated flash-attention backwards of the same P = 2^(S c2 - lse)."""
    torch.manual_seed(9)
    B, heads = 2, 8
    C = heads * d
    qq = (torch.randn(B, N, 3 * C, device=DEV) * 0.5).to(torch.bfloat16)
    go = torch.randn(B, N, C, device=DEV).to(torch.bfloat16)
    oo, lse = K.attention_fwd_lse(qq, qq[..., C:], qq[..., 2 * C:], B, heads, d, N, N, 3 * C, 3 * C, 3 * C)
    outs = []
    for new in (True, False):
        K.set_attention_bwd32(new)
        try:
            dqkv = torch.empty_like(qq)
            K.attention_bwd(qq, qq[..., C:], qq[..., 2 * C:], oo, go, lse, B, heads, d, N, N, 3 * C, 3 * C, 3 * C,
                            dqkv, dqkv[..., C:], dqkv[..., 2 * C:], 3 * C, 3 * C)
            outs.append(dqkv.float())
        finally:
            K.set_attention_bwd32(True)
    for i in range(3):
        assert rel(outs[0][..., i * C:(i + 1) * C], outs[1][..., i * C:(i + 1) * C]) < 1e-2, i


# ------------------------------------------------------------------ loss / optimizer
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_mse_loss_and_grad(dt):
    torch.manual_seed(6)
    B, Cc, H, W = 3, 4, 16, 16
    pred = torch.randn(B, Cc, H, W, device=DEV)
    tgt = torch.randn(B, Cc, H, W, device=DEV)
    mask = (torch.rand(B, H, W, device=DEV) > 0.2).float()
    t = torch.tensor([5, 999, 300], device=DEV)
    wt = torch.rand(1000, device=DEV)
    pr = pred.clone().requires_grad_(True)
    loss = (F.mse_loss(pr, tgt, reduction="none") * mask[:, None] * wt[t][:, None, None, None]).view(-1).mean()
    loss.backward()
    s, dp = K.mse_loss(pred.to(dt), tgt, mask, t, wt, grad_scale=1.0 / pred.numel())
    assert abs(s.item() / pred.numel() - loss.item()) / loss.item() < (1e-6 if dt == torch.float32 else 2e-2)
    assert rel(dp, pr.grad) < tol(dt)


def test_adamw_and_clip_match_torch():
    torch.manual_seed(7)
    shapes = [(300,), (64, 33), (1000,), (7,)]
    ps = [torch.randn(s, device=DEV) for s in shapes]
    gs = [torch.randn(s, device=DEV) * 3 for s in shapes]
    lrs = [1e-3, 2e-3, 1e-3, 5e-4]
    wds = [0.05, 0.0, 0.05, 0.05]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.AdamW([{"params": [r], "lr": lr, "weight_decay": wd} for r, lr, wd in zip(ref, lrs, wds)],
                            betas=(0.9, 0.999), eps=1e-8)
    n = sum(p.numel() for p in ps)
    flat_p = torch.cat([p.view(-1) for p in ps])
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    import struct
    recs, off = b"", 0
    for p, lr, wd in zip(ps, lrs, wds):
        recs += struct.pack("<qqff", off, off + p.numel(), lr, wd)
        off += p.numel()
    segs = torch.frombuffer(bytearray(recs), dtype=torch.uint8).to(DEV)
    for step in (1, 2, 3):
        for r, g in zip(ref, gs):
            r.grad = g.clone() * step
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        opt.step()
        flat_g = torch.cat([g.view(-1) * step for g in gs])
        sq = K.sq_norm(flat_g)
        K.adamw(flat_p, flat_g, m, v, segs, len(ps), step, sqsum=sq, max_norm=1.0)
    assert rel(flat_p, torch.cat([r.detach().view(-1) for r in ref])) < 1e-5
