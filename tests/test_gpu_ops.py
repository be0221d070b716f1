"""Per-op parity of the HIP kernels (through the C ABI) on an MI355X.

References: the reference's golden vectors where the op is the reference's (DDIM, codec),
otherwise plain torch fp32 on the CPU (floating-point kernels).
Tolerances (stated per test): fp32 path 1e-4 relative to the tensor scale (exact fp32 MFMA,
only summation order differs); bf16 path 2e-2 (8-bit mantissa storage, fp32 accumulate).
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_utils import DDIM_CONFIGS, load
from ldmseg.ops import native as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def tol(dt):
    return 1e-4 if dt == torch.float32 else 2e-2


DTYPES = [torch.float32, torch.bfloat16]


# ------------------------------------------------------------------------------ conv / gemm
CONV_CASES = [
    # name, B, Cin(a0), Cin(a1), H, W, Cout, k, stride, upsample
    ("3x3", 2, 64, 0, 16, 12, 96, 3, 1, False),
    ("3x3_s2", 2, 64, 0, 15, 17, 64, 3, 2, False),
    ("3x3_up", 1, 128, 0, 8, 6, 64, 3, 1, True),
    ("3x3_concat", 2, 64, 32, 9, 9, 48, 3, 1, False),
    ("1x1", 3, 160, 0, 7, 11, 320, 1, 1, False),
    ("1x1_concat", 2, 128, 64, 8, 8, 64, 1, 1, False),
    ("odd_n", 1, 32, 0, 5, 5, 4, 3, 1, False),
    ("unet_l0", 1, 320, 0, 64, 64, 320, 3, 1, False),
    ("unet_l3_splitk", 8, 1280, 0, 8, 8, 1280, 3, 1, False),       # few tiles, deep K -> split-K
    ("unet_up_concat_splitk", 4, 1280, 640, 16, 16, 1280, 3, 1, False),
    ("concat_unaligned", 2, 40, 24, 6, 6, 16, 3, 1, False),         # per-lane source select
]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("case", CONV_CASES, ids=[c[0] for c in CONV_CASES])
def test_conv2d(case, dt):
    name, B, c0, c1, H, W, Co, k, s, up = case
    torch.manual_seed(0)
    x = torch.randn(B, c0 + c1, H, W)
    w = torch.randn(Co, c0 + c1, k, k) / (k * (c0 + c1) ** 0.5)
    b = torch.randn(Co)
    temb = torch.randn(B, Co + 5)
    res_needed = not up and s == 1
    xr = F.interpolate(x, scale_factor=2.0, mode="nearest") if up else x
    ref = F.conv2d(xr, w, b, stride=s, padding=k // 2) + temb[:, :Co, None, None]
    ref = F.silu(ref)
    resid = torch.randn_like(ref) if res_needed else None
    if res_needed:
        ref = ref + resid
    pc = K.PackedConv(w.to(DEV), b.to(DEV), dt)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV, dt)
    x0 = xn[..., :c0].contiguous()
    x1 = xn[..., c0:].contiguous() if c1 else None
    temb_d = temb.to(DEV)
    r_d = resid.permute(0, 2, 3, 1).contiguous().to(DEV, dt) if res_needed else None
    out = K.conv2d(pc, x0, B, H, W, x1=x1, stride=s, upsample=up, temb=temb_d, temb_stride=temb.shape[1],
                   residual=r_d, act=K.ACT_SILU)
    assert rel_err(out.permute(0, 3, 1, 2), ref) < tol(dt)
    # NCHW epilogue (conv_out): same numbers, NCHW layout, no extras
    out2 = K.conv2d(pc, x0, B, H, W, x1=x1, stride=s, upsample=up, out_layout=K.OUT_NCHW)
    ref2 = F.conv2d(xr, w, b, stride=s, padding=k // 2)
    assert rel_err(out2, ref2) < tol(dt)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,H,C,Co,G,split", [(2, 32, 128, 320, 32, False), (8, 8, 1280, 1280, 32, True),
                                               (1, 16, 64, 64, 16, False),
                                               (2, 16, 64, 320, 64, False)])   # group 5 ch: unit 10 unusable
def test_conv_epilogue_groupnorm_stats(B, H, C, Co, G, split, dt):
    """Producer-epilogue (sum, sumsq) partials feed GroupNorm: no statistics pass, same result.
    Also across a concat whose second half carries its own producer statistics."""
    torch.manual_seed(8)
    x = torch.randn(B, C, H, H)
    w = torch.randn(Co, C, 3, 3) / (3 * C ** 0.5)
    b = torch.randn(Co)
    y_ref = F.conv2d(x, w, b, padding=1)
    pc = K.PackedConv(w.to(DEV), b.to(DEV), dt)
    y = K.conv2d(pc, x.permute(0, 2, 3, 1).contiguous().to(DEV, dt), B, H, H, gn_stats=True)
    assert K.gn_stats_of(y) is not None
    gam, bet = torch.randn(Co), torch.randn(Co)
    out = K.group_norm(y, B, H * H, G, gam.to(DEV), bet.to(DEV), 1e-5, K.ACT_SILU)
    ref = F.silu(F.group_norm(y_ref, G, gam, bet, 1e-5))
    assert rel_err(out.view(B, H, H, -1).permute(0, 3, 1, 2), ref) < (2e-4 if dt == torch.float32 else 3e-2)
    # concat [y || y2] where y2 has producer stats too
    y2 = K.conv2d(pc, x.permute(0, 2, 3, 1).contiguous().to(DEV, dt), B, H, H, act=K.ACT_SILU, gn_stats=True)
    gam2, bet2 = torch.randn(2 * Co), torch.randn(2 * Co)
    out2 = K.group_norm(y, B, H * H, G, gam2.to(DEV), bet2.to(DEV), 1e-6, x1=y2)
    ref2 = F.group_norm(torch.cat([y_ref, F.silu(y_ref)], 1), G, gam2, bet2, 1e-6)
    assert rel_err(out2.view(B, H, H, -1).permute(0, 3, 1, 2), ref2) < (2e-4 if dt == torch.float32 else 3e-2)


@pytest.mark.parametrize("split", [False, True])
def test_conv_groupnorm_accumulators_and_arena(split):
    """The epilogue's fp64 accumulators hold each (batch, unit of gn_unit channels)'s (sum, sumsq)
    of the STORED output; inside K.gn_arena the second forward with the same key takes them from one zeroed
    buffer and gives the same sums."""
    torch.manual_seed(9)
    B, H, C, Co = (8, 8, 1280, 1280) if split else (2, 64, 128, 320)     # 64x64: 8 slots
    x = torch.randn(B, H, H, C).to(DEV, torch.bfloat16)
    pc = K.PackedConv((torch.randn(Co, C, 3, 3) / (3 * C ** 0.5)).to(DEV), torch.randn(Co).to(DEV), torch.bfloat16)
    sums = []
    for it in range(3):
        with K.gn_arena(("test_arena", split), DEV):
            y = K.conv2d(pc, x, B, H, H, gn_stats=True)
            y2 = K.conv2d(pc, x, B, H, H, act=K.ACT_SILU, gn_stats=True)
        a, a2 = K.gn_stats_of(y), K.gn_stats_of(y2)
        U, S = K.gn_unit_for(Co), K.gn_slots_for(H * H)
        assert a.dtype == torch.float64 and a.shape == (B, S, Co // U, 2)
        if it > 0:                                 # arena slices: one storage for both
            assert a.untyped_storage().data_ptr() == a2.untyped_storage().data_ptr()
        yd = y.double().view(B, H * H, Co // U, U)
        ref = torch.stack([yd.sum((1, 3)), (yd * yd).sum((1, 3))], -1)
        assert torch.allclose(a.sum(1), ref, rtol=1e-5, atol=1e-3)
        sums.append(a.clone())
    assert torch.allclose(sums[0], sums[2], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,Kd,N", [(8, 320, 1280), (1, 1280, 20160), (4096, 320, 2560), (333, 640, 5120)])
def test_linear_and_geglu(M, Kd, N, dt):
    torch.manual_seed(1)
    x = torch.randn(M, Kd)
    lin = torch.nn.Linear(Kd, N)
    pc = K.PackedConv(lin.weight.to(DEV), lin.bias.to(DEV), dt)
    y = K.linear(pc, x.to(DEV, dt), out_dtype=torch.float32)
    with torch.no_grad():
        ref = lin(x)
    assert rel_err(y, ref) < tol(dt)
    pg = K.PackedConv(lin.weight.to(DEV), lin.bias.to(DEV), dt, geglu=True)
    g = K.linear(pg, x.to(DEV, dt), out_layout=K.OUT_GEGLU)
    h, gate = ref.chunk(2, dim=-1)
    assert rel_err(g, h * F.gelu(gate)) < tol(dt)


@pytest.mark.parametrize("offset", [0.7, 60.0])
@pytest.mark.parametrize("M,C", [(4096, 320), (1024, 640), (256, 1280), (333, 320)])
def test_linear_layernorm_fold(M, C, offset):
    """norm -> Linear as ONE GEMM on the raw rows: the producer GEMM (with a residual) sums each
    stored row's (sum, sumsq) in its epilogue (row_stats), the consumer applies
    rstd (x W'^T - mean c1) + W beta + b in its epilogue (packed_ln_fold) — NHWC (QKV) and GEGLU
    (ff.net.0) outputs, against torch fp32 LayerNorm + Linear on the same bf16 rows."""
    torch.manual_seed(21)
    # offset 60: rows whose mean is ~40x their spread (the fold's E[x^2] - mean^2 must not cancel:
    # the row statistics and the variance are fp64)
    x = (torch.randn(M, C) * 1.5 + 0.7).to(DEV, torch.bfloat16)
    res = (torch.randn(M, C) + offset).to(DEV, torch.bfloat16)
    prod = torch.nn.Linear(C, C)
    pp = K.PackedConv(prod.weight.to(DEV), prod.bias.to(DEV), torch.bfloat16)
    rows = torch.zeros(M, 2, device=DEV, dtype=torch.float64)
    h = K.linear(pp, x, residual=res, row_stats=rows)
    hf = h.float()
    assert torch.allclose(rows[:, 0], hf.double().sum(1), rtol=1e-4, atol=1e-2)
    assert torch.allclose(rows[:, 1], (hf.double() ** 2).sum(1), rtol=1e-4, atol=1e-1)
    ln = torch.nn.LayerNorm(C)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.normal_(0, 0.2)
    qkv = torch.nn.Linear(C, 3 * C, bias=False)
    pq = K.packed_ln_fold(qkv.weight.to(DEV), None, ln.weight.to(DEV), ln.bias.to(DEV), torch.bfloat16)
    out = K.linear(pq, h, ln=(rows, 1e-5))
    with torch.no_grad():
        n = ln.to(DEV)(hf)
        ref = n @ qkv.weight.to(DEV).t()
    assert rel_err(out, ref) < 2e-2
    ff = torch.nn.Linear(C, 8 * C)
    pf = K.packed_ln_fold(ff.weight.to(DEV), ff.bias.to(DEV), ln.weight.to(DEV), ln.bias.to(DEV), torch.bfloat16,
                          geglu=True)
    g = K.linear(pf, h, out_layout=K.OUT_GEGLU, ln=(rows, 1e-5))
    with torch.no_grad():
        a, gate = (n @ ff.weight.to(DEV).t() + ff.bias.to(DEV)).chunk(2, dim=-1)
    assert rel_err(g, a * F.gelu(gate)) < 2e-2


@pytest.mark.parametrize("dt", DTYPES)
def test_conv_transpose_shuffle(dt):
    torch.manual_seed(2)
    ct = torch.nn.ConvTranspose2d(64, 32, 2, stride=2)
    x = torch.randn(2, 64, 7, 9)
    pc = K.PackedConv(ct.weight.to(DEV), ct.bias.to(DEV), dt, shuffle2=True)
    y = K.conv2d(pc, x.permute(0, 2, 3, 1).contiguous().to(DEV, dt), 2, 7, 9, out_layout=K.OUT_SHUFFLE2)
    with torch.no_grad():
        ref = ct(x)
    assert rel_err(y.permute(0, 3, 1, 2), ref) < tol(dt)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,cin,cout,H,W", [(2, 320, 320, 16, 16), (8, 1280, 1280, 8, 8), (1, 640, 640, 32, 32),
                                             (2, 64, 96, 4, 8), (3, 128, 160, 8, 12)])
def test_upsample_conv_phases(B, cin, cout, H, W, dt):
    """Upsample2D's conv in phase form (four 2x2 convs over the low-res input, ldm_conv2d upsample
    mode 3) vs torch conv3x3(nearest_upsample_2x(x)) in fp32, and its GroupNorm partials through a
    following GroupNorm; the 3x3 gather form of the same conv for comparison."""
    torch.manual_seed(21)
    x = torch.randn(B, cin, H, W)
    w = torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5)
    b = torch.randn(cout)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), w, b, padding=1)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV, dt)
    pcp = K.PackedConv(w.to(DEV), b.to(DEV), dt, upsample_phases=True)
    y = K.conv2d(pcp, xn, B, H, W, upsample=True, gn_stats=True)
    assert rel_err(y.permute(0, 3, 1, 2), ref) < tol(dt)
    y3 = K.conv2d(K.PackedConv(w.to(DEV), b.to(DEV), dt), xn, B, H, W, upsample=True)
    assert rel_err(y, y3) < tol(dt)
    if cout % 32 == 0 and (4 * H * W) % 64 == 0:
        assert K.gn_stats_of(y) is not None
        gam, bet = torch.randn(cout), torch.randn(cout)
        out = K.group_norm(y, B, 4 * H * W, 32, gam.to(DEV), bet.to(DEV), 1e-5, K.ACT_SILU)
        gref = F.silu(F.group_norm(ref, 32, gam, bet, 1e-5))
        assert rel_err(out.view(B, 2 * H, 2 * W, -1).permute(0, 3, 1, 2), gref) < (3e-4 if dt == torch.float32 else 3e-2)


def test_upsample_phases_unet_close_to_gather_form():
    """The whole UNet with the phase-form Upsample2D convs (default) against the 3x3 gather form:
    the same function up to the bf16 rounding of the summed taps."""
    from ldmseg.models import UNet
    torch.manual_seed(0)
    with torch.device(DEV):
        u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero")
    u = u.to(torch.bfloat16).eval()
    x = torch.randn(8, 8, 64, 64, device=DEV).to(torch.bfloat16)
    t = torch.full((8,), 500, device=DEV, dtype=torch.long)
    with torch.no_grad():
        u.set_upsample_phases(False)
        y0 = u(x, t).sample.float().clone()
        u.set_upsample_phases(True)
        y1 = u(x, t).sample.float()
    torch.cuda.synchronize()
    assert rel_err(y1, y0) < 2e-2


# ------------------------------------------------------------------------------ attention
def _attn_ref(q, k, v, heads):
    B, N, C = q.shape
    d = C // heads
    sp = lambda t: t.reshape(B, t.shape[1], heads, d).permute(0, 2, 1, 3)  # noqa: E731
    o = torch.softmax(sp(q) @ sp(k).transpose(-1, -2) * d ** -0.5, -1) @ sp(v)
    return o.permute(0, 2, 1, 3).reshape(B, N, C)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,N,L,C", [(2, 4096, 4096, 320), (2, 1024, 1024, 640), (2, 256, 256, 1280),
                                     (3, 64, 64, 1280), (2, 200, 77, 320), (1, 100, 130, 640)])
def test_attention(B, N, L, C, dt):
    torch.manual_seed(3)
    q, k, v = torch.randn(B, N, C), torch.randn(B, L, C), torch.randn(B, L, C)
    ref = _attn_ref(q, k, v, 8)
    if N == L:   # the UNet layout: q|k|v packed in one [B, N, 3C] buffer
        qkv = torch.cat([q, k, v], -1).to(DEV, dt)
        o = K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, 8, C // 8, N, N, 3 * C, 3 * C, 3 * C)
    else:        # cross-attention layout
        kv = torch.cat([k, v], -1).to(DEV, dt)
        o = K.attention(q.to(DEV, dt), kv, kv[..., C:], B, 8, C // 8, N, L, C, 2 * C, 2 * C)
    assert rel_err(o, ref) < tol(dt)


@pytest.mark.parametrize("waves", [0, 4, 8])
@pytest.mark.parametrize("B,N,C", [(2, 4096, 320), (2, 1024, 640), (1, 300, 320), (2, 520, 640), (16, 1024, 320),
                                   (16, 1000, 320), (1, 4096, 320)])
def test_attention_block_waves(B, N, C, waves):
    """Every block shape of the bf16 kernel (4 or 8 waves sharing each K/V tile; waves=0 lets
    the launcher pick, which at head_dim 40 with >= 512 blocks is two 8-wave blocks per CU of
    2 query subtiles each), ragged N."""
    torch.manual_seed(5)
    q, k, v = torch.randn(B, N, C), torch.randn(B, N, C), torch.randn(B, N, C)
    ref = _attn_ref(q, k, v, 8)
    qkv = torch.cat([q, k, v], -1).to(DEV, torch.bfloat16)
    K.set_attention_waves(waves)
    try:
        o = K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, 8, C // 8, N, N, 3 * C, 3 * C, 3 * C)
    finally:
        K.set_attention_waves(0)
    assert rel_err(o, ref) < tol(torch.bfloat16)


@pytest.mark.parametrize("B,N", [(8, 1024), (1, 300), (2, 64)])
def test_attention_d80_forms_agree(B, N):
    """head_dim 80 on the 32x32x16 kernel (the default: the d = 40 kernel's form with a 96-wide
    Q.K^T and three 32-row P.V blocks) and on the 16x16x32 kernel: both within the bf16 bar of the
    fp32 reference, and close to each other; the log-sum-exp the training backward reads agrees."""
    torch.manual_seed(6)
    C = 640
    q, k, v = torch.randn(B, N, C), torch.randn(B, N, C), torch.randn(B, N, C)
    ref = _attn_ref(q, k, v, 8)
    qkv = torch.cat([q, k, v], -1).to(DEV, torch.bfloat16)
    outs = []
    try:
        for on in (True, False):
            K.set_attention_d80(on)
            o, lse = K.attention_fwd_lse(qkv, qkv[..., C:], qkv[..., 2 * C:], B, 8, 80, N, N, 3 * C, 3 * C, 3 * C)
            outs.append((o.float(), lse.float()))
    finally:
        K.set_attention_d80(True)
    for o, _ in outs:
        assert rel_err(o, ref) < tol(torch.bfloat16)
    assert (outs[0][0] - outs[1][0]).abs().max().item() < 0.05
    assert torch.allclose(outs[0][1], outs[1][1], atol=2e-2)


@pytest.mark.parametrize("B,N", [(4, 4096), (4, 4096 + 37), (4, 64 * 3 + 5), (8, 4096 + 37)])
def test_attention_d40_qs2_close_to_default(B, N):
    """head_dim 40 under the alternative kernels of ldm_attention_set_qs2 against the default and a
    torch fp32 reference on the device: mode 1 (two 32-query subtiles per wave; the shared rescale
    decision moves m by different bf16 steps, so within bf16 rounding, not bit-identical) and mode 2
    (the software-pipelined tile loop: the same operations per query, bit-identical), and the default
    two-subtile interleaved kernel (ldm_attention_set_il, each subtile with its own rescale decision:
    the 32-query kernel's arithmetic, bit-identical; taken from 256 blocks, B = 4 / 8 at N = 4096)
    against the 32-query kernel it replaces, on 128-key tiles by default and on 64- / 256-key tiles
    (one / four 64-key halves per barrier, ldm_attention_set_il(2 / 3): the same halves in the same
    order, bit-identical).  Ragged N exercises the masked last key tile and the partial query block; N = 197 gives 4 key tiles (the
    pipeline's two-tile unroll with an odd tail)."""
    torch.manual_seed(9)
    C, H = 320, 8
    qkv = torch.randn(B, N, 3 * C, device=DEV).to(torch.bfloat16)
    x = qkv.float().view(B, N, 3, H, 40).permute(2, 0, 3, 1, 4)
    ref = torch.cat([torch.softmax(x[0][b:b + 1] @ x[1][b:b + 1].transpose(-1, -2) * 40 ** -0.5, -1) @ x[2][b:b + 1]
                     for b in range(B)]).permute(0, 2, 1, 3).reshape(B, N, C)
    outs = []
    try:
        K.set_attention_kvsplit(0)          # unsplit kernels only
        K.set_attention_il(False)           # mode 0 = the 32-query kernel
        for mode in (0, 1, 2):
            K.set_attention_qs2(mode)
            outs.append(K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, 40, N, N, 3 * C, 3 * C, 3 * C).float())
        K.set_attention_qs2(0)
        K.set_attention_il(True)
        outs.append(K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, 40, N, N, 3 * C, 3 * C, 3 * C).float())
        for kt_mode in (2, 3):              # the interleaved kernel on 64- / 256-key tiles (default 128)
            K.set_attention_il(kt_mode)
            outs.append(K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, 40, N, N, 3 * C, 3 * C, 3 * C).float())
    finally:
        K.set_attention_qs2(0)
        K.set_attention_il(True)
        K.set_attention_kvsplit(-1)
    for o in outs:
        assert ((o - ref).norm() / ref.norm()).item() < 1e-2
    assert (outs[0] - outs[1]).abs().max().item() < 0.05
    assert torch.equal(outs[0], outs[2])
    assert torch.equal(outs[0], outs[3])
    assert torch.equal(outs[0], outs[4]) and torch.equal(outs[0], outs[5])


@pytest.mark.parametrize("B,N,hd", [(4, 4096, 40), (4, 4096 + 37, 40), (4, 64 * 3 + 5, 40), (4, 64, 40), (4, 40, 40),
                                    (8, 1024, 80), (8, 1024 + 19, 80)])
def test_attention_skew_bit_identical(B, N, hd):
    """ldm_attention_set_skew(2): the 32x32x16 head_dim 40 / 80 kernel with the block's upper waves one
    half-iteration behind (softmax + P.V of tile t - 1 before Q.K^T of tile t).  Every wave runs the
    same operations in the same order, so output and log-sum-exp are bit-identical to the default
    form; N covers 0, 1, 3 and 64 full key tiles plus ragged tails."""
    torch.manual_seed(10)
    C, H = 8 * hd, 8
    qkv = torch.randn(B, N, 3 * C, device=DEV).to(torch.bfloat16)
    outs = []
    try:
        if hd == 40:
            K.set_attention_waves(8)        # the 8-wave two-blocks-per-CU kernel at every N
        for mode in (1, 2):
            K.set_attention_skew(mode)
            o, lse = K.attention_fwd_lse(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, hd, N, N, 3 * C, 3 * C, 3 * C)
            outs.append((o, lse))
    finally:
        K.set_attention_skew(0)
        K.set_attention_waves(0)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    x = qkv.float().view(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(x[0] @ x[1].transpose(-1, -2) * hd ** -0.5, -1) @ x[2]).permute(0, 2, 1, 3).reshape(B, N, C)
    assert ((outs[1][0].float() - ref).norm() / ref.norm()).item() < 1e-2


# planner cases at each head dim's UNet level (d = 40: 64x64, N = 4096; d = 80: 32x32, N = 1024)
KVSPLIT_CASES = [(B, N * (4 if hd == 40 else 1) + r, sp, hd) for hd in (40, 80) for B, N, r, sp in
                 [(1, 1024, 0, -1), (1, 1024, 37, -1), (1, 0, 64 * 5 + 3, 3), (1, 0, 300, 2), (2, 0, 1024, 8),
                  (1, 1024, 0, 3), (1, 0, 256 + 1, 2)]] + [(1, 256, -1, 160), (1, 64, -1, 160), (1, 1024 + 5, 4, 160),
                                                          (2, 300, 2, 160), (8, 256, -1, 160), (1, 200, 4, 160)]
# head_dim 160 runs on the 16x16x32 kernel by default and on the 32x32x16 one under ldm_attention_set_d160
KVSPLIT_CASES = [c + (False,) for c in KVSPLIT_CASES] + [c + (True,) for c in KVSPLIT_CASES if c[3] == 160]


@pytest.mark.parametrize("B,N,splits,hd,route32", KVSPLIT_CASES)
def test_attention_kvsplit(B, N, splits, hd, route32):
    """ldm_attention_ws: head_dim 40 with the keys split over blocks (fp32 partials + log-sum-exp,
    merged by attn_kv_combine) against torch fp32 and against the unsplit kernel; a large logit sits
    in the last key tile so the merge's rescale is exercised."""
    torch.manual_seed(12)
    H = 8
    C = H * hd
    K.set_attention_d160(route32)
    q, k, v = torch.randn(B, N, C), torch.randn(B, N, C), torch.randn(B, N, C)
    k[0, N - 2] = q[0, 5] * 4.0
    qkv = torch.cat([q, k, v], -1).to(DEV).to(torch.bfloat16)
    try:
        K.set_attention_kvsplit(0)
        o0 = K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, hd, N, N, 3 * C, 3 * C, 3 * C)
        K.set_attention_kvsplit(splits)
        p = K.AttnParams(0, 0, 0, 0, 3 * C, 3 * C, 3 * C, C, B, H, hd, N, N, hd ** -0.5, K.dtype_code(torch.bfloat16))
        p.q = p.k = p.v = p.o = 1 << 20              # any 16-byte-aligned address: sizing only
        if N > 128 and not (B == 8 and hd == 160 and not route32):   # (N = 64: one key tile; B = 8 fills)
            assert K.load_library().ldm_attention_workspace_bytes(ctypes.byref(p)) > 0
        o1 = K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, hd, N, N, 3 * C, 3 * C, 3 * C)
    finally:
        K.set_attention_kvsplit(-1)
        K.set_attention_d160(False)
    x = qkv.float().view(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(x[0] @ x[1].transpose(-1, -2) * hd ** -0.5, -1) @ x[2]).permute(0, 2, 1, 3).reshape(B, N, C)
    assert rel_err(o1, ref) < 1e-2
    assert rel_err(o1, o0.float()) < 1e-2
    # P is rounded to bf16 against a different running max per split, so not bit-identical to the
    # one-pass kernel: the same bound as the qs2 form, and no worse against fp32 than the one pass
    assert (o1.float() - o0.float()).abs().max().item() < 0.05
    assert rel_err(o1, ref) <= 1.2 * rel_err(o0, ref) + 1e-4


@pytest.mark.parametrize("B,N", [(8, 256), (1, 256), (8, 64), (2, 200)])
def test_attention_d160_forms(B, N):
    """head_dim 160 (the 16x16 / 8x8 levels) on the 32x32x16 kernel (ldm_attention_set_d160(True)) and
    on the 16x16x32 one (default), both against torch fp32; unsplit (kvsplit 0)."""
    torch.manual_seed(13)
    H, hd = 8, 160
    C = H * hd
    qkv = torch.randn(B, N, 3 * C, device=DEV).to(torch.bfloat16)
    x = qkv.float().view(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax(x[0] @ x[1].transpose(-1, -2) * hd ** -0.5, -1) @ x[2]).permute(0, 2, 1, 3).reshape(B, N, C)
    outs = []
    try:
        K.set_attention_kvsplit(0)
        for on in (True, False):
            K.set_attention_d160(on)
            o, lse = K.attention_fwd_lse(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, hd, N, N, 3 * C, 3 * C, 3 * C)
            outs.append((o.float(), lse.float()))
    finally:
        K.set_attention_d160(False)
        K.set_attention_kvsplit(-1)
    for o, _ in outs:
        assert ((o - ref).norm() / ref.norm()).item() < 1e-2
    assert (outs[0][0] - outs[1][0]).abs().max().item() < 0.05
    assert torch.allclose(outs[0][1], outs[1][1], atol=2e-2)


def test_attention_kvsplit_planner():
    """The planner splits only the under-occupied single-frame head_dim-40 case."""
    lib = K.load_library()

    def ws(B, N, hd=40, H=8):
        p = K.AttnParams(1 << 20, 1 << 20, 1 << 20, 1 << 20, 3 * H * hd, 3 * H * hd, 3 * H * hd, H * hd, B, H, hd, N, N,
                         hd ** -0.5, K.dtype_code(torch.bfloat16))
        return int(lib.ldm_attention_workspace_bytes(ctypes.byref(p)))

    assert ws(1, 4096) > 0
    assert ws(8, 4096) == 0            # 1024 query blocks already
    assert ws(1, 1024, hd=80) > 0      # 32 eight-wave blocks at the 32x32 level
    assert ws(8, 1024, hd=80) == 0     # 256 already
    assert ws(1, 256, hd=160) > 0      # 32 four-wave blocks of the 16x16x32 kernel at the 16x16 level
    assert ws(8, 256, hd=160) == 0     # 256 already
    assert ws(1, 64, hd=160) == 0      # the 8x8 level: one key tile
    try:
        K.set_attention_d160(True)
        assert ws(1, 256, hd=160) > 0  # 16 four-wave blocks at the 16x16 level
        assert ws(1, 64, hd=160) == 0  # the 8x8 level: one key tile
    finally:
        K.set_attention_d160(False)
    assert ws(1, 77) == 0              # a single key tile
    assert ws(4, 197) == 0             # 32 query blocks but only 4 key tiles


@pytest.mark.parametrize("B,N,hd,splits", [(8, 4096, 40, 0), (4, 64 * 7 + 5, 40, 0), (8, 1024, 80, 0), (2, 1024 + 9, 80, 0),
                                            (1, 4096, 40, -1), (1, 64 * 9 + 3, 40, 3), (1, 1024, 80, -1)])
def test_attention_pair_bit_identical(B, N, hd, splits):
    """ldm_attention_set_pair(1) (the head_dim-80 default): the key-tile loop unrolled by two runs the
    same operations in the same order, so output and log-sum-exp are bit-identical to the one-tile
    loop (odd and even tile counts, ragged tails; at head_dim 40 both settings run one kernel); modes 2 / 3
    run 128-key tiles (two 64-key halves per barrier) without / with the unroll: the same halves in the
    same order, bit-identical too."""
    torch.manual_seed(14)
    H = 8
    C = H * hd
    qkv = torch.randn(B, N, 3 * C, device=DEV).to(torch.bfloat16)
    outs = []
    try:
        K.set_attention_kvsplit(splits)
        for mode in (0, 1, 2, 3):
            K.set_attention_pair(mode)
            outs.append([K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, hd, N, N, 3 * C, 3 * C, 3 * C)])
            if splits == 0:
                outs[-1].append(K.attention_fwd_lse(qkv, qkv[..., C:], qkv[..., 2 * C:], B, H, hd, N, N, 3 * C,
                                                    3 * C, 3 * C)[1])
    finally:
        K.set_attention_pair(True)
        K.set_attention_kvsplit(-1)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def test_attention_softmax_spike():
    """Force the online-softmax rescale: a huge logit in the LAST kv tile of some rows."""
    torch.manual_seed(4)
    B, N, C = 1, 512, 320
    q, k, v = torch.randn(B, N, C), torch.randn(B, N, C), torch.randn(B, N, C)
    k[0, 500] = q[0, 7] * 4.0
    k[0, 3] = -q[0, 9] * 4.0
    ref = _attn_ref(q, k, v, 8)
    qkv = torch.cat([q, k, v], -1).to(DEV)
    o = K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, 8, 40, N, N, 3 * C, 3 * C, 3 * C)
    assert rel_err(o, ref) < 1e-4


@pytest.mark.parametrize("maxcol", [2, 1, 0])
@pytest.mark.parametrize("C,N", [(320, 520), (640, 300), (320, 4096), (320, 77)])
def test_attention_softmax_spike_bf16(C, N, maxcol):
    """bf16 kernel under forced rescales, with and without the max column (scale and running max
    carried in the Q.K^T head-dim padding): a huge logit in the last kv tile, a first kv tile
    whose logits are all very negative for some rows (the first-tile max must still be taken),
    and a row whose max grows tile after tile.  maxcol 2: the 32x32x16 head_dim-40 kernel."""
    torch.manual_seed(14)
    B = 1
    q, k, v = torch.randn(B, N, C), torch.randn(B, N, C), torch.randn(B, N, C)
    k[0, N - 3] = q[0, 7] * 4.0                      # spike in the last tile
    k[0, :64] -= q[0, 11] * 3.0                      # row 11: first tile far below the rest
    for t in range(1, N // 64):                      # row 5: max grows every tile
        k[0, 64 * t + 1] = q[0, 5] * (0.5 * t / (N // 64))
    ref = _attn_ref(q, k, v, 8)
    qkv = torch.cat([q, k, v], -1).to(DEV, torch.bfloat16)
    K.set_attention_maxcol(maxcol)
    try:
        o = K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, 8, C // 8, N, N, 3 * C, 3 * C, 3 * C)
    finally:
        K.set_attention_maxcol(2)
    assert rel_err(o, ref) < 2e-2
    assert (o.float() - ref.to(DEV)).abs().max().item() < 0.05


# ------------------------------------------------------------------------------ norms
@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,HW,c0,c1,G,eps,act", [(2, 4096, 320, 0, 32, 1e-5, True), (2, 256, 1280, 1280, 32, 1e-5, True),
                                                  (3, 100, 640, 320, 32, 1e-6, False), (1, 64, 64, 0, 16, 1e-6, True),
                                                  # single-block small-image kernel (gn_small): config 5's 4x8 level,
                                                  # an in-place concat, 10-channel groups straddling 16-B vectors
                                                  (16, 32, 1280, 0, 32, 1e-5, True), (4, 32, 640, 640, 32, 1e-5, True),
                                                  (2, 8, 320, 0, 32, 1e-6, False)])
def test_group_norm(B, HW, c0, c1, G, eps, act, dt):
    torch.manual_seed(5)
    x = torch.randn(B, HW, c0 + c1) * 3 + 1.5
    gam, bet = torch.randn(c0 + c1), torch.randn(c0 + c1)
    ref = F.group_norm(x.permute(0, 2, 1), G, gam, bet, eps).permute(0, 2, 1)
    if act:
        ref = F.silu(ref)
    xd = x.to(DEV, dt)
    y = K.group_norm(xd[..., :c0].contiguous(), B, HW, G, gam.to(DEV), bet.to(DEV), eps,
                     K.ACT_SILU if act else K.ACT_NONE, x1=xd[..., c0:].contiguous() if c1 else None)
    assert rel_err(y, ref) < tol(dt)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("rows,C,eps,act", [(4096, 320, 1e-5, False), (333, 1280, 1e-5, False),
                                            (1000, 256, 1e-6, True), (17, 2560, 1e-5, False),
                                            (8191, 640, 1e-5, False), (5, 40, 1e-5, True),
                                            (140001, 320, 1e-5, False)])   # > one grid-stride sweep
def test_layer_norm(rows, C, eps, act, dt):
    torch.manual_seed(6)
    x = torch.randn(rows, C) * 2 - 0.5
    gam, bet = torch.randn(C), torch.randn(C)
    ref = F.layer_norm(x, (C,), gam, bet, eps)
    if act:
        ref = F.silu(ref)
    y = K.layer_norm(x.to(DEV, dt), gam.to(DEV), bet.to(DEV), eps, K.ACT_SILU if act else K.ACT_NONE)
    assert rel_err(y, ref) < tol(dt)


# ------------------------------------------------------------------------------ timestep / DDIM
def test_timestep_proj():
    import math
    t = torch.tensor([999.0, 0.0, 421.0, 19.0])
    half = 160
    freqs = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32) / half)
    emb = t[:, None] * freqs[None]
    ref = torch.cat([torch.cos(emb), torch.sin(emb)], -1)
    y = K.timestep_proj(t.to(DEV), 4, freqs.to(DEV), 320, True, torch.float32)
    assert (y.cpu() - ref).abs().max().item() < 2e-5
    y1 = K.timestep_proj(t[:1].to(DEV), 4, freqs.to(DEV), 320, False, torch.float32)
    ref1 = torch.cat([torch.sin(emb[:1]), torch.cos(emb[:1])], -1).expand(4, -1)
    assert (y1.cpu() - ref1).abs().max().item() < 2e-5


@pytest.mark.parametrize("cname", list(DDIM_CONFIGS))
def test_ddim_against_reference_golden(cname):
    from ldmseg.schedulers import DDIMNoiseScheduler
    z = load("ddim.npz")
    s = DDIMNoiseScheduler(**DDIM_CONFIGS[cname], device=DEV, verbose=False)
    s.set_timesteps_inference(50)
    mo = torch.from_numpy(z[f"{cname}__step_model_output"]).to(DEV)
    x = torch.from_numpy(z[f"{cname}__step_sample"]).to(DEV)
    for t in z[f"{cname}__step_t"]:
        for clipped in (0, 1):
            for tt in (int(t), torch.tensor(int(t), device=DEV)):      # host int and device scalar
                r = s.step(mo, tt, x, use_clipped_model_output=bool(clipped))
                np.testing.assert_allclose(r.prev_sample.cpu().numpy(), z[f"{cname}__step_{t}_{clipped}__prev"],
                                           rtol=1e-5, atol=1e-6)
                np.testing.assert_allclose(r.pred_original_sample.cpu().numpy(),
                                           z[f"{cname}__step_{t}_{clipped}__x0"], rtol=1e-5, atol=1e-6)
    tb = torch.from_numpy(z[f"{cname}__an_t"]).to(DEV)
    x0 = torch.from_numpy(z[f"{cname}__an_x0"]).to(DEV)
    eps = torch.from_numpy(z[f"{cname}__an_eps"]).to(DEV)
    np.testing.assert_allclose(s.add_noise(x0, eps.clone(), tb).cpu().numpy(), z[f"{cname}__an_out"], rtol=1e-5,
                               atol=1e-6)
    np.testing.assert_allclose(s.add_noise(x0, eps.clone(), tb, scale=2.0).cpu().numpy(), z[f"{cname}__an_out_s2"],
                               rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(s.remove_noise(x, eps, tb).cpu().numpy(), z[f"{cname}__rn_out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(s.remove_noise(x, eps, tb, 0.5).cpu().numpy(), z[f"{cname}__rn_out_s2"], rtol=1e-5,
                               atol=1e-5)


# ------------------------------------------------------------------------------ bit codec (bit-exact)
def test_bit_codec_known_answer_pngs():
    from ldmseg.data import decode_bitmap, encode_bitmap
    z = load("codec.npz")
    sem = torch.from_numpy(z["fixture_semseg"].astype(np.int64)).to(DEV)
    planes, _ = encode_bitmap(sem, n=16, fill_value=0.5, ignore_label=0)
    assert np.array_equal((planes.cpu().numpy() * 255).astype(np.uint8), z["fixture_bits_u8"])
    assert np.array_equal(decode_bitmap(2 * planes - 1).cpu().numpy(), z["fixture_decode"])


@pytest.mark.parametrize("case", list(load("codec.npz")["cases"]))
def test_bit_codec_cases(case):
    from ldmseg.data import decode_bitmap, encode_bitmap
    z = load("codec.npz")
    i = list(z["cases"]).index(case)
    n, ign = int(z["cases_n"][i]), int(z["cases_ignore"][i])
    ids = torch.from_numpy(z[f"{case}__ids"]).to(DEV)
    planes, mask = encode_bitmap(ids, n=n, fill_value=0.5, ignore_label=ign)
    assert np.array_equal(planes.cpu().numpy(), z[f"{case}__enc"])
    assert np.array_equal(mask.cpu().numpy(), z[f"{case}__ignore_mask"])
    assert np.array_equal(decode_bitmap(2 * planes - 1).cpu().numpy(), z[f"{case}__dec_clean"])
    noisy = torch.from_numpy(z[f"{case}__noisy"]).to(DEV)
    assert np.array_equal(decode_bitmap(noisy).cpu().numpy(), z[f"{case}__dec_noisy"])


def test_bit_codec_batched_roundtrip_full_size():
    """Size-independent property at the KITTI frame size: decode(2*encode-1) == ids (31 -> 0)."""
    from ldmseg.data import decode_bitmap, encode_bitmap
    g = torch.Generator(device=DEV).manual_seed(0)
    ids = torch.randint(0, 32, (8, 192, 640), generator=g, device=DEV)
    planes, mask = encode_bitmap(ids, n=5, fill_value=0.5, ignore_label=255)
    assert planes.shape == (8, 5, 192, 640) and not mask.any()
    dec = decode_bitmap(2 * planes - 1)
    exp = ids.clone()
    exp[exp == 31] = 0
    assert torch.equal(dec, exp)


# ------------------------------------------------------------------------------ resize / layout
@pytest.mark.parametrize("size,sf", [((64, 64), None), (None, 2), ((192, 640), None), (None, 4)])
def test_resize_bilinear(size, sf):
    torch.manual_seed(7)
    x = torch.randn(2, 5, 24, 80)
    ref = F.interpolate(x, size=size, scale_factor=sf, mode="bilinear", align_corners=False)
    y = K.resize_bilinear(x.to(DEV), size=size, scale_factor=sf)
    assert rel_err(y, ref) < 1e-5
    y2 = K.resize_bilinear(x.to(DEV), size=size, scale_factor=sf, mul=2.0, add=-1.0)
    assert rel_err(y2, 2 * ref - 1) < 1e-5


def test_nchw_to_nhwc_concat():
    a, b, c = torch.randn(2, 4, 8, 8), torch.randn(2, 4, 8, 8), torch.randn(2, 4, 8, 8)
    y = K.nchw_to_nhwc([a.to(DEV), b.to(DEV, torch.bfloat16), c.to(DEV)], 16, torch.float32)
    ref = torch.cat([a, b.bfloat16().float(), c, torch.zeros(2, 4, 8, 8)], 1).permute(0, 2, 3, 1)
    assert torch.equal(y.cpu(), ref)
