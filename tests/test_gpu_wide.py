"""The wide-tile persistent 1x1 GEMM (gemm_wide_kernel, csrc/gemm_wide.hip) vs the tile kernels
and torch fp32.

It serves the large-N projections of diffusers' BasicTransformerBlock (the reference's UNet,
/root/reference/ldmseg/models/unet.py:361-425, runs them through Transformer2DModel): the
LayerNorm-folded QKV and GEGLU ff.net.0.  Its fp32 accumulation order over K (64-deep K tiles,
two k32 MFMA steps each, in K order) and its epilogue arithmetic are those of the 2-blocks-per-CU tile
kernel, so stored bf16 outputs must be bit-identical to the unsplit 128x128 tile path (forced plan:
no split-K, no A-stationary kernel).  Against torch fp32 the bar is the conv tests' 2e-2 of the
tensor scale.  Covered: ragged M (partial last tile, rows dropped by the store range check),
several tiles per block (the persistent walk and its cross-tile prefetch, double-buffered
per-tile scratch), K from 128 to 5120, the two-source concat, SiLU, no bias.
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
def wide():
    def run(fn):
        K.force_conv_plan(128, 128, 1)          # the reference: unsplit 128x128 tiles
        ref = fn()
        K.force_conv_plan(0, 0, 1)
        K.set_conv_wide(2)                      # the wide kernel whenever legal
        got = fn()
        torch.cuda.synchronize()
        return ref, got
    yield run
    K.force_conv_plan(0, 0, 1)
    K.set_conv_wide(0)


@pytest.mark.parametrize("M,C,N,act,bias", [(256, 320, 320, K.ACT_NONE, True), (4096 + 64 + 5, 320, 960, K.ACT_NONE, True),
                                            (32768, 320, 960, K.ACT_NONE, False), (8192, 640, 1920, K.ACT_SILU, True),
                                            (2048 + 100, 1280, 3840, K.ACT_NONE, True), (2048, 5120, 1280, K.ACT_NONE, True),
                                            (1000, 128, 640, K.ACT_SILU, False)])
def test_wide_linear(M, C, N, act, bias, wide):
    torch.manual_seed(5)
    x = torch.randn(M, C).to(DEV, BF)
    lin = torch.nn.Linear(C, N, bias=bias)
    pc = K.PackedConv(lin.weight.to(DEV), None if lin.bias is None else lin.bias.to(DEV), BF)
    y0, y1 = wide(lambda: K.linear(pc, x, act=act))
    assert torch.equal(y0, y1)
    with torch.no_grad():
        ref = lin.to(DEV)(x.float())
        if act == K.ACT_SILU:
            ref = F.silu(ref)
    assert rel_err(y1, ref) < 2e-2


@pytest.mark.parametrize("M,C", [(4096, 320), (1000, 320), (32768, 320), (8192, 640), (2048 + 64, 1280)])
def test_wide_layernorm_fold_qkv_geglu(M, C, wide):
    torch.manual_seed(7)
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
    q0, q1 = wide(lambda: K.linear(pq, h, ln=(rows, 1e-5)))
    g0, g1 = wide(lambda: K.linear(pf, h, out_layout=K.OUT_GEGLU, ln=(rows, 1e-5)))
    assert torch.equal(q0, q1)
    assert torch.equal(g0, g1)
    with torch.no_grad():
        n = ln.to(DEV)(hf)
        ref_q = n @ qkv.weight.to(DEV).t()
        a, gate = (n @ ff.weight.to(DEV).t() + ff.bias.to(DEV)).chunk(2, dim=-1)
    assert rel_err(q1, ref_q) < 2e-2
    assert rel_err(g1, a * F.gelu(gate)) < 2e-2


@pytest.mark.parametrize("M,C,N", [(2048 + 40, 640, 5120), (32768, 320, 2560), (300, 1280, 10240)])
def test_wide_plain_geglu(M, C, N, wide):
    torch.manual_seed(8)
    x = torch.randn(M, C).to(DEV, BF)
    ff = torch.nn.Linear(C, N)
    pg = K.PackedConv(ff.weight.to(DEV), ff.bias.to(DEV), BF, geglu=True)
    g0, g1 = wide(lambda: K.linear(pg, x, out_layout=K.OUT_GEGLU))
    assert torch.equal(g0, g1)
    with torch.no_grad():
        a, gate = ff.to(DEV)(x.float()).chunk(2, dim=-1)
    assert rel_err(g1, a * F.gelu(gate)) < 2e-2


@pytest.mark.parametrize("B,HW,c0,c1,N", [(8, 1024, 640, 0, 640), (8, 4096, 320, 320, 320), (8, 256, 1280, 1280, 1280)])
def test_wide_conv1x1_concat(B, HW, c0, c1, N, wide):
    """NHWC 1x1 conv on a two-source channel concat read in place (the up-block shortcut)."""
    torch.manual_seed(9)
    H = W = int(HW ** 0.5)
    x0 = torch.randn(B, H, W, c0).to(DEV, BF)
    x1 = torch.randn(B, H, W, c1).to(DEV, BF) if c1 else None
    conv = torch.nn.Conv2d(c0 + c1, N, 1)
    pc = K.PackedConv(conv.weight.to(DEV), conv.bias.to(DEV), BF)
    y0, y1 = wide(lambda: K.conv2d(pc, x0, B, H, W, x1=x1))
    assert torch.equal(y0, y1)
    with torch.no_grad():
        xin = x0.float() if x1 is None else torch.cat([x0.float(), x1.float()], -1)
        ref = F.conv2d(xin.permute(0, 3, 1, 2), conv.weight.to(DEV), conv.bias.to(DEV)).permute(0, 2, 3, 1)
    assert rel_err(y1, ref) < 2e-2


def test_wide_not_used_with_residual():
    """Calls with a residual (or statistics) stay on the tile kernels even with the wide kernel
    forced on (its epilogue has no residual read); they must still be correct."""
    torch.manual_seed(10)
    M, C, N = 32768, 320, 960
    x = torch.randn(M, C).to(DEV, BF)
    lin = torch.nn.Linear(C, N)
    pc = K.PackedConv(lin.weight.to(DEV), lin.bias.to(DEV), BF)
    res = torch.randn(M, N).to(DEV, BF)
    K.set_conv_wide(2)
    try:
        y = K.linear(pc, x, residual=res)
    finally:
        K.set_conv_wide(0)
    with torch.no_grad():
        ref = lin.to(DEV)(x.float()) + res.float()
    assert rel_err(y, ref) < 2e-2
