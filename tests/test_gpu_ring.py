"""The deep-ring 1x1 GEMM (gemm_ring_kernel, csrc/gemm_ring.hip) vs the tile kernel and torch fp32.

It serves the 16x16 / 8x8 / mid levels' 1x1 GEMMs of the reference UNet
(/root/reference/ldmseg/models/unet.py:361-425: Transformer2DModel proj_in / to_out / proj_out,
the norm1-folded QKV, ff.net.2, the up-block shortcuts on the skip concat).  Its fp32 accumulation
order over K (64-deep K steps, two k32 MFMA halves each, in K order) and its bf16 pre-activation
staging + epilogue_fast are those of the unsplit tile kernel, so stored outputs must be
bit-identical to the forced unsplit 64x64 plan (GEGLU: the register epilogue of the same plan).
The GroupNorm partials and LayerNorm row statistics are sums of the same values grouped by a
different tile shape: compared at 1e-6.  Against torch fp32 the bar is the conv tests' 2e-2 of the
tensor scale.  Covered: both configurations (128x80 / 32x80 tiles), ragged M,
K from 128 to 5120 (deep rings: 80 K steps through 5 / 8 slots), the two-source concat, residual
in place, SiLU, no bias.
"""
import pytest
import torch
import torch.nn.functional as F

from ldmseg.ops import native as K

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def rel_err(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


@pytest.fixture
def ring():
    def run(fn):
        K.set_conv_ring(1)
        K.force_conv_plan(64, 64, 1)            # the reference: unsplit 64x64 tiles
        ref = fn()
        K.force_conv_plan(0, 0, 1)
        K.set_conv_ring(2)                      # the ring kernel whenever legal
        got = fn()
        torch.cuda.synchronize()
        return ref, got
    yield run
    K.force_conv_plan(0, 0, 1)
    K.set_conv_ring(0)


@pytest.mark.parametrize("M,C,N,act,bias", [(2048, 1280, 1280, K.ACT_NONE, True), (512, 1280, 1280, K.ACT_NONE, True),
                                            (2048, 5120, 1280, K.ACT_NONE, True), (512, 5120, 1280, K.ACT_SILU, False),
                                            (2048 + 100, 640, 1280, K.ACT_NONE, True), (300, 128, 640, K.ACT_SILU, True),
                                            (1000, 1280, 3840, K.ACT_NONE, False)])
def test_ring_linear(M, C, N, act, bias, ring):
    torch.manual_seed(5)
    x = torch.randn(M, C).to(DEV, BF)
    lin = torch.nn.Linear(C, N, bias=bias)
    pc = K.PackedConv(lin.weight.to(DEV), None if lin.bias is None else lin.bias.to(DEV), BF)
    y0, y1 = ring(lambda: K.linear(pc, x, act=act))
    assert torch.equal(y0, y1)
    with torch.no_grad():
        ref = lin.to(DEV)(x.float())
        if act == K.ACT_SILU:
            ref = F.silu(ref)
    assert rel_err(y1, ref) < 2e-2


@pytest.mark.parametrize("B,HW", [(8, 256), (8, 64), (3, 256)])
def test_ring_residual_gn_stats(B, HW):
    """proj_out / to_out form: + residual (in place for to_out), GroupNorm partials of the output."""
    torch.manual_seed(6)
    C = 1280
    H = W = int(HW ** 0.5)
    x = torch.randn(B, H, W, C).to(DEV, BF)
    res = torch.randn(B, H, W, C).to(DEV, BF)
    conv = torch.nn.Conv2d(C, C, 1)
    pc = K.PackedConv(conv.weight.to(DEV), conv.bias.to(DEV), BF)
    outs = []
    for mode in (1, 2):
        K.set_conv_ring(mode)
        K.force_conv_plan(*((64, 64, 1) if mode == 1 else (0, 0, 1)))
        try:
            y = K.conv2d(pc, x, B, H, W, residual=res, gn_stats=True)
            outs.append((y, K.gn_stats_of(y).sum(1)))
        finally:
            K.force_conv_plan(0, 0, 1)
            K.set_conv_ring(0)
    (y0, s0), (y1, s1) = outs
    assert torch.equal(y0, y1)
    assert torch.allclose(s0, s1, rtol=1e-6, atol=1e-6)
    yf = y1.double().view(B, HW, C)
    unit = K.gn_unit_for(C)
    ref = torch.stack([yf.view(B, HW, C // unit, unit).sum((1, 3)), (yf ** 2).view(B, HW, C // unit, unit).sum((1, 3))], -1)
    assert torch.allclose(s1, ref, rtol=1e-6, atol=1e-6)
    with torch.no_grad():
        ref_y = F.conv2d(x.float().permute(0, 3, 1, 2), conv.weight.to(DEV), conv.bias.to(DEV)).permute(0, 2, 3, 1)
    assert rel_err(y1, ref_y + res.float()) < 2e-2
    # in place: out aliases the residual (Attention.to_out + hidden_states, unet.py _transformer)
    K.set_conv_ring(2)
    try:
        r2 = res.clone()
        y2 = K.conv2d(pc, x, B, H, W, residual=r2, out=r2)
    finally:
        K.set_conv_ring(0)
    assert torch.equal(y2, y1)


@pytest.mark.parametrize("M,C", [(2048, 1280), (512, 1280), (2048 + 64, 640)])
def test_ring_row_stats_and_ln_fold(M, C, ring):
    """proj_in with row statistics -> the norm1-folded QKV (the LayerNorm fold on the raw rows)."""
    torch.manual_seed(7)
    h = (torch.randn(M, C) * 1.5 + 0.7).to(DEV, BF)
    proj = torch.nn.Linear(C, C)
    pp = K.PackedConv(proj.weight.to(DEV), proj.bias.to(DEV), BF)
    stats = []

    def run():
        rs = torch.zeros(2 * M, dtype=torch.float64, device=DEV)
        y = K.linear(pp, h, row_stats=rs)
        stats.append(rs)
        return y
    y0, y1 = ring(run)
    assert torch.equal(y0, y1)
    assert torch.allclose(stats[0], stats[1], rtol=1e-6, atol=1e-6)
    yd = y1.double()
    assert torch.allclose(stats[1].view(M, 2), torch.stack([yd.sum(1), (yd * yd).sum(1)], 1), rtol=1e-6, atol=1e-6)
    ln = torch.nn.LayerNorm(C)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.normal_(0, 0.2)
    qkv = torch.nn.Linear(C, 2 * C, bias=False)           # N = 2C: a multiple of 80 at both widths
    pq = K.packed_ln_fold(qkv.weight.to(DEV), None, ln.weight.to(DEV), ln.bias.to(DEV), BF)
    rows = stats[1].view(M, 2).contiguous()
    q0, q1 = ring(lambda: K.linear(pq, y1, ln=(rows, 1e-5)))
    assert torch.equal(q0, q1)
    with torch.no_grad():
        ref_q = ln.to(DEV)(y1.float()) @ qkv.weight.to(DEV).t()
    assert rel_err(q1, ref_q) < 2e-2


@pytest.mark.parametrize("B,HW,c0,c1", [(8, 256, 1280, 1280), (8, 64, 1280, 1280), (8, 256, 1280, 640)])
def test_ring_conv1x1_concat(B, HW, c0, c1, ring):
    """The up-block shortcut: a 1x1 conv on the two-source channel concat read in place."""
    torch.manual_seed(9)
    H = W = int(HW ** 0.5)
    x0 = torch.randn(B, H, W, c0).to(DEV, BF)
    x1 = torch.randn(B, H, W, c1).to(DEV, BF)
    conv = torch.nn.Conv2d(c0 + c1, 1280, 1)
    pc = K.PackedConv(conv.weight.to(DEV), conv.bias.to(DEV), BF)
    y0, y1 = ring(lambda: K.conv2d(pc, x0, B, H, W, x1=x1))
    assert torch.equal(y0, y1)
    with torch.no_grad():
        xin = torch.cat([x0.float(), x1.float()], -1)
        ref = F.conv2d(xin.permute(0, 3, 1, 2), conv.weight.to(DEV), conv.bias.to(DEV)).permute(0, 2, 3, 1)
    assert rel_err(y1, ref) < 2e-2


def test_ring_planned_at_deep_levels():
    """The planner routes the B = 8 deep-level shapes to the ring kernel."""
    for M, C, N in [(2048, 1280, 1280), (512, 1280, 1280), (2048, 2560, 1280)]:
        assert K.describe_plan(M, 1, 1, C, N, ksize=1)["kind"] == "ring", (M, C, N)


@pytest.mark.parametrize("rows,C,N,act,out_dt,sinusoid", [(8, 320, 1280, K.ACT_SILU, BF, True),
                                                          (8, 1280, 1280, K.ACT_SILU, BF, False),
                                                          (8, 1280, 20160, K.ACT_NONE, torch.float32, False),
                                                          (1, 320, 1280, K.ACT_SILU, BF, True),
                                                          (16, 1280, 1280, K.ACT_NONE, torch.float32, False),
                                                          (3, 96, 64, K.ACT_NONE, BF, False)])
def test_linear_rows(rows, C, N, act, out_dt, sinusoid):
    """ldm_linear_rows (the time-embedding MLP: TimestepEmbedding linear_1 / linear_2 and the batched
    time_emb_proj, unet.py:301-307) vs the ldm_conv2d tile path and torch fp32.  Its K split over four
    waves sums the fp32 partial tiles in a different order than the tile kernel: 1e-3 relative."""
    torch.manual_seed(11)
    lin = torch.nn.Linear(C, N)
    pc = K.PackedConv(lin.weight.to(DEV), lin.bias.to(DEV), BF)
    if sinusoid:
        t = torch.tensor([417.0], device=DEV)
        half = C // 2
        freqs = torch.exp(-torch.log(torch.tensor(10000.0)) * torch.arange(half) / half).to(DEV)
        x = K.timestep_proj(t, rows, freqs, C, True, BF)
        y = K.linear_rows(pc, None, rows, act=act, out_dtype=out_dt, t=t, freqs=freqs, flip_sin_to_cos=True)
    else:
        x = torch.randn(rows, C).to(DEV, BF)
        y = K.linear_rows(pc, x, rows, act=act, out_dtype=out_dt)
    ref_tile = K.linear(pc, x, act=act, out_dtype=out_dt)
    assert rel_err(y, ref_tile) < 1e-3
    with torch.no_grad():
        ref = lin.to(DEV)(x.float())
        if act == K.ACT_SILU:
            ref = F.silu(ref)
    assert rel_err(y, ref) < 2e-2


@pytest.mark.parametrize("B,H,c0,c1,N,stride,ks,temb,res", [
    (8, 8, 1280, 0, 1280, 1, 0, True, False),        # the 8x8 level conv1 (planner: 4 splits)
    (8, 8, 1280, 0, 1280, 1, 0, False, True),        # conv2 + residual
    (8, 8, 1280, 1280, 1280, 1, 0, True, False),     # up-block conv1 on the skip concat
    (8, 16, 1280, 0, 1280, 2, 3, False, False),      # Downsample2D 16 -> 8, 3 splits
    (3, 8, 640, 0, 320, 1, 7, True, True),           # ragged: 192 rows, 7 splits
    (2, 8, 640, 0, 640, 1, 1, False, True),          # unsplit ring conv (no time embedding)
])
def test_ring_conv3x3(B, H, c0, c1, N, stride, ks, temb, res):
    """The deep-ring kernel's implicit-GEMM 3x3 form (tap-major 64-deep K steps, per-row tap masks for
    the zero padding) with K split into fp32 slabs reduced by the split-K kernel (bias, time
    embedding, residual, GroupNorm partials there).  Its K order differs from the tile kernel's, so
    it is compared to torch fp32 at the conv tests' 2e-2 and to the tile plan at bf16 rounding; the
    GroupNorm statistics (fp32 per reduction tile, fp64 across tiles) against the stored output in
    fp64 at 1e-5."""
    torch.manual_seed(21)
    x = torch.randn(B, c0 + c1, H, H)
    w = torch.randn(N, c0 + c1, 3, 3) / (3 * (c0 + c1) ** 0.5)
    b = torch.randn(N)
    ho = H // stride
    te = torch.randn(B, N) if temb else None
    r = torch.randn(B, N, ho, ho) if res else None
    pc = K.PackedConv(w.to(DEV), b.to(DEV), BF)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV, BF)
    x0 = xn[..., :c0].contiguous()
    x1 = xn[..., c0:].contiguous() if c1 else None
    rn = r.permute(0, 2, 3, 1).contiguous().to(DEV, BF) if res else None
    stats = (ho * ho) % 64 == 0

    def run():
        return K.conv2d(pc, x0, B, H, H, x1=x1, stride=stride, temb=te.to(DEV) if temb else None,
                        temb_stride=N, residual=rn, act=K.ACT_SILU if temb else K.ACT_NONE, gn_stats=stats)
    try:
        K.set_conv_ring(1)
        y_tile = run()
        K.set_conv_ring(2)
        K.set_conv_ring_split(ks)
        assert K.describe_plan(B, H, H, c0, N, c1=c1, ksize=3, stride=stride, temb=temb)["kind"] == "ring"
        y = run()
    finally:
        K.set_conv_ring(0)
        K.set_conv_ring_split(0)
    ref = F.conv2d(x, w, b, stride=stride, padding=1)
    if temb:
        ref = F.silu(ref + te[:, :, None, None])
    if res:
        ref = ref + r
    assert rel_err(y.permute(0, 3, 1, 2), ref) < 2e-2
    assert rel_err(y, y_tile) < 2e-2
    if stats:
        unit = K.gn_unit_for(N)
        s1 = K.gn_stats_of(y).sum(1)
        yd = y.double().view(B, ho * ho, N)
        want = torch.stack([yd.view(B, ho * ho, N // unit, unit).sum((1, 3)),
                            (yd ** 2).view(B, ho * ho, N // unit, unit).sum((1, 3))], -1)
        assert torch.allclose(s1, want, rtol=1e-5, atol=1e-5)
