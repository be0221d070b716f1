"""The A-register-stationary short-K 1x1 GEMM (gemm_ars_kernel, csrc/gemm_ars.h) vs the tile
kernels and torch fp32.

It serves the K = 320 projections of the 64x64 UNet level (proj_in with row statistics, the
LayerNorm-folded QKV, to_out with an in-place residual, the LayerNorm-folded GEGLU).  Its fp32
accumulation order over K and its epilogue arithmetic are those of the 2-blocks-per-CU tile
kernel, so the stored bf16 outputs must be bit-identical to the planner's tile path
(ldm_conv2d_set_ars(1)); row statistics are atomically summed (order differs: allclose).  Against
torch fp32 the bar is the conv tests' 2e-2 of the tensor scale.  Ragged M (rows past the last
full 256-row panel, panels split over N ranges) and the minimum one-panel launch are covered.
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
def ars_mode():
    yield lambda m: K.set_conv_ars(m)
    K.set_conv_ars(0)


def both(fn, ars_mode):
    ars_mode(1)
    ref = fn()
    ars_mode(2)
    got = fn()
    torch.cuda.synchronize()
    return ref, got


@pytest.mark.parametrize("M", [256, 4096, 4000, 32768 + 96])
@pytest.mark.parametrize("N,act", [(320, K.ACT_NONE), (960, K.ACT_NONE), (480, K.ACT_SILU)])
def test_ars_linear_residual_rowstats(M, N, act, ars_mode):
    torch.manual_seed(5)
    x = torch.randn(M, 320).to(DEV, BF)
    lin = torch.nn.Linear(320, N)
    pc = K.PackedConv(lin.weight.to(DEV), lin.bias.to(DEV), BF)
    res = torch.randn(M, N).to(DEV, BF)

    def run():
        rows = torch.zeros(M, 2, device=DEV, dtype=torch.float64)
        y = K.linear(pc, x, residual=res, row_stats=rows, act=act)
        return y, rows
    (y0, r0), (y1, r1) = both(run, ars_mode)
    assert torch.equal(y0, y1)
    assert torch.allclose(r0, r1, rtol=1e-5, atol=1e-2)
    with torch.no_grad():
        ref = lin.to(DEV)(x.float())
        if act == K.ACT_SILU:
            ref = F.silu(ref)
        ref = ref + res.float()
    assert rel_err(y1, ref) < 2e-2
    hf = y1.float()
    assert torch.allclose(r1[:, 0], hf.double().sum(1), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("M", [512, 8192 + 256 + 13])
def test_ars_in_place_residual(M, ars_mode):
    """to_out: out aliases the residual (h = to_out(attn) + h written over h)."""
    torch.manual_seed(6)
    a = torch.randn(M, 320).to(DEV, BF)
    lin = torch.nn.Linear(320, 320)
    pc = K.PackedConv(lin.weight.to(DEV), lin.bias.to(DEV), BF)
    h0 = torch.randn(M, 320).to(DEV, BF)

    def run():
        h = h0.clone()
        rows = torch.zeros(M, 2, device=DEV, dtype=torch.float64)
        K.linear(pc, a, residual=h, out=h, row_stats=rows)
        return h, rows
    (y0, r0), (y1, r1) = both(run, ars_mode)
    assert torch.equal(y0, y1)
    assert torch.allclose(r0, r1, rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("M", [4096, 1000, 32768])
def test_ars_layernorm_fold_qkv_geglu(M, ars_mode):
    torch.manual_seed(7)
    C = 320
    h = (torch.randn(M, C) * 1.5 + 0.7).to(DEV, BF)
    hf = h.float()
    rows = torch.stack([hf.double().sum(1), (hf.double() ** 2).sum(1)], 1).contiguous()
    ln = torch.nn.LayerNorm(C)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.normal_(0, 0.2)
    qkv = torch.nn.Linear(C, 3 * C, bias=False)
    ff = torch.nn.Linear(C, 8 * C)
    pq = K.packed_ln_fold(qkv.weight.to(DEV), None, ln.weight.to(DEV), ln.bias.to(DEV), BF)
    pf = K.packed_ln_fold(ff.weight.to(DEV), ff.bias.to(DEV), ln.weight.to(DEV), ln.bias.to(DEV), BF, geglu=True)
    q0, q1 = both(lambda: K.linear(pq, h, ln=(rows, 1e-5)), ars_mode)
    g0, g1 = both(lambda: K.linear(pf, h, out_layout=K.OUT_GEGLU, ln=(rows, 1e-5)), ars_mode)
    assert torch.equal(q0, q1)
    assert torch.equal(g0, g1)
    with torch.no_grad():
        n = ln.to(DEV)(hf)
        ref_q = n @ qkv.weight.to(DEV).t()
        a, gate = (n @ ff.weight.to(DEV).t() + ff.bias.to(DEV)).chunk(2, dim=-1)
    assert rel_err(q1, ref_q) < 2e-2
    assert rel_err(g1, a * F.gelu(gate)) < 2e-2


def test_ars_plain_geglu(ars_mode):
    torch.manual_seed(8)
    M = 2048 + 40
    x = torch.randn(M, 320).to(DEV, BF)
    ff = torch.nn.Linear(320, 2560)
    pg = K.PackedConv(ff.weight.to(DEV), ff.bias.to(DEV), BF, geglu=True)
    g0, g1 = both(lambda: K.linear(pg, x, out_layout=K.OUT_GEGLU), ars_mode)
    assert torch.equal(g0, g1)
    with torch.no_grad():
        a, gate = ff.to(DEV)(x.float()).chunk(2, dim=-1)
    assert rel_err(g1, a * F.gelu(gate)) < 2e-2
