"""ldm_conv2d under every tile plan (forced through ldm_conv2d_force_plan) vs torch fp32.

The built-in planner picks one plan per shape; these tests run the SAME shapes through each
kernel variant — the 256x160 three-stage bf16 kernel (with and without split-K) and the
128/64/32 tile kernels — so a variant the planner does not pick for the test sizes is still
covered.  Tolerance: bf16 storage, fp32 accumulate -> 2e-2 of the tensor scale (the same bar
as tests/test_gpu_ops.py); fp32 -> 1e-4.
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
def plan():
    def set_plan(bm, bn, ks, stages=0):
        K.force_conv_plan(bm, bn, ks)
        K.force_conv_stages(stages)
    yield set_plan
    K.force_conv_plan(0, 0, 1)
    K.force_conv_stages(0)
    K.set_conv_splitk_cols(0)


SKC = [64, 128]     # split-K reduction tile widths (ldm_conv2d_set_splitk_cols; both forced)


PLANS = [(256, 160, 1, 0), (256, 160, 3, 0), (128, 160, 1, 0), (128, 160, 1, 3), (128, 160, 3, 4), (64, 160, 2, 0),
         (128, 128, 1, 0), (128, 32, 2, 0), (64, 64, 1, 0), (32, 128, 3, 0), (64, 160, 3, 4), (64, 64, 2, 4)]
SHAPES = [
    # name, B, c0, c1, H, W, Cout, k, stride, upsample
    ("l0", 1, 320, 0, 32, 32, 320, 3, 1, False),
    ("ragged_m_n", 1, 64, 0, 20, 20, 200, 3, 1, False),
    ("concat", 2, 128, 64, 9, 9, 160, 3, 1, False),
    ("upsample", 1, 128, 0, 8, 6, 192, 3, 1, True),
    ("stride2", 2, 64, 0, 17, 15, 96, 3, 2, False),
    ("pointwise", 3, 320, 0, 10, 10, 960, 1, 1, False),
    ("deep_k", 2, 1280, 0, 8, 8, 320, 3, 1, False),
]


@pytest.mark.parametrize("skc", SKC)
@pytest.mark.parametrize("pl", PLANS, ids=[f"{a}x{b}_k{c}_s{d}" for a, b, c, d in PLANS])
@pytest.mark.parametrize("case", SHAPES, ids=[s[0] for s in SHAPES])
def test_conv_plan(case, pl, skc, plan):
    if pl[2] == 1 and skc != SKC[0]:
        pytest.skip("unsplit plan: no split-K reduction")
    name, B, c0, c1, H, W, Co, k, s, up = case
    torch.manual_seed(3)
    x = torch.randn(B, c0 + c1, H, W)
    w = torch.randn(Co, c0 + c1, k, k) / (k * (c0 + c1) ** 0.5)
    b = torch.randn(Co)
    temb = torch.randn(B, Co)
    xr = F.interpolate(x, scale_factor=2.0, mode="nearest") if up else x
    ref = F.silu(F.conv2d(xr, w, b, stride=s, padding=k // 2) + temb[:, :, None, None])
    resid = torch.randn_like(ref)
    ref = ref + resid
    pc = K.PackedConv(w.to(DEV), b.to(DEV), BF)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV, BF)
    x0 = xn[..., :c0].contiguous()
    x1 = xn[..., c0:].contiguous() if c1 else None
    plan(*pl)
    K.set_conv_splitk_cols(skc)
    out = K.conv2d(pc, x0, B, H, W, x1=x1, stride=s, upsample=up, temb=temb.to(DEV), temb_stride=Co,
                   residual=resid.permute(0, 2, 3, 1).contiguous().to(DEV, BF), act=K.ACT_SILU)
    assert rel_err(out.permute(0, 3, 1, 2), ref) < 2e-2


@pytest.mark.parametrize("skc", SKC)
@pytest.mark.parametrize("pl", PLANS, ids=[f"{a}x{b}_k{c}_s{d}" for a, b, c, d in PLANS])
def test_plan_groupnorm_stats(pl, skc, plan):
    """Epilogue GroupNorm partials (two 128-row halves in the large kernel, split-K reduce)."""
    B, H, C, Co, G = 2, 16, 192, 320, 32
    torch.manual_seed(4)
    x = torch.randn(B, C, H, H)
    w = torch.randn(Co, C, 3, 3) / (3 * C ** 0.5)
    b = torch.randn(Co)
    y_ref = F.conv2d(x, w, b, padding=1)
    pc = K.PackedConv(w.to(DEV), b.to(DEV), BF)
    plan(*pl)
    K.set_conv_splitk_cols(skc)
    y = K.conv2d(pc, x.permute(0, 2, 3, 1).contiguous().to(DEV, BF), B, H, H, gn_stats=True)
    assert K.gn_stats_of(y) is not None
    gam, bet = torch.randn(Co), torch.randn(Co)
    out = K.group_norm(y, B, H * H, G, gam.to(DEV), bet.to(DEV), 1e-5, K.ACT_SILU)
    ref = F.silu(F.group_norm(y_ref, G, gam, bet, 1e-5))
    assert rel_err(out.view(B, H, H, -1).permute(0, 3, 1, 2), ref) < 3e-2


@pytest.mark.parametrize("pl", [(256, 160, 1), (128, 160, 1), (128, 128, 1), (64, 64, 1)],
                         ids=["256x160", "128x160", "128x128", "64x64"])
@pytest.mark.parametrize("M,Kd,N", [(300, 320, 2560), (1024, 640, 640)])
def test_plan_geglu(M, Kd, N, pl, plan):
    torch.manual_seed(5)
    x = torch.randn(M, Kd)
    lin = torch.nn.Linear(Kd, N)
    with torch.no_grad():
        h, gate = lin(x).chunk(2, dim=-1)
    pg = K.PackedConv(lin.weight.to(DEV), lin.bias.to(DEV), BF, geglu=True)
    plan(*pl)
    g = K.linear(pg, x.to(DEV, BF), out_layout=K.OUT_GEGLU)
    assert rel_err(g, h * F.gelu(gate)) < 2e-2


@pytest.mark.parametrize("pl", [(256, 160, 1), (128, 128, 1)], ids=["256x160", "128x128"])
def test_plan_shuffle2(pl, plan):
    """ConvTranspose2d(k2, s2) as GEMM + pixel-shuffle epilogue (seg-VAE decoder)."""
    torch.manual_seed(6)
    B, C, H, W, Co = 2, 256, 12, 20, 80
    x = torch.randn(B, C, H, W)
    ct = torch.nn.ConvTranspose2d(C, Co, 2, stride=2)
    with torch.no_grad():
        ref = ct(x)
    pc = K.PackedConv(ct.weight.to(DEV), ct.bias.to(DEV), BF, shuffle2=True)
    plan(*pl)
    y = K.conv2d(pc, x.permute(0, 2, 3, 1).contiguous().to(DEV, BF), B, H, W, out_layout=K.OUT_SHUFFLE2)
    assert rel_err(y.permute(0, 3, 1, 2), ref) < 2e-2


def test_planner_picks_halo_for_level0(plan):
    """With no override the level-0 UNet conv (64 wide, 320 channels) goes to the halo-tiled
    kernel: identical output to the forced halo plan, a different summation order from the
    tap-major igemm (so not bit-equal to it), and close to both."""
    torch.manual_seed(7)
    B, C, H = 8, 320, 64
    x = torch.randn(B, H, H, C, device=DEV).to(BF)
    w = torch.randn(C, C, 3, 3, device=DEV) * 0.02
    pc = K.PackedConv(w, torch.zeros(C, device=DEV), BF)
    try:
        y_auto = K.conv2d(pc, x, B, H, H)
        K.set_conv_halo(2)
        y_halo = K.conv2d(pc, x, B, H, H)
        K.set_conv_halo(1)
        y_igemm = K.conv2d(pc, x, B, H, H)
    finally:
        K.set_conv_halo(0)
    assert torch.equal(y_auto, y_halo)
    assert rel_err(y_halo, y_igemm) < 1e-2


HALO_SHAPES = [
    # name, B, c0, c1, H, W, Cout
    ("w64_320", 2, 320, 0, 8, 64, 320),
    ("w64_concat_640_320", 1, 640, 320, 4, 64, 320),
    ("w64_ragged_n200", 1, 128, 0, 8, 64, 200),
    ("w32_640", 2, 640, 0, 8, 32, 640),
    ("w32_concat_1280_640", 1, 1280, 640, 4, 32, 640),
    ("w32_64ch", 1, 64, 0, 12, 32, 160),
    # 256-row tiles at width 32 (8 rows), K split over channel blocks (the wide up-block concats)
    ("w32_r8_concat_1280_640_split2", 1, 1280, 640, 8, 32, 640),
    ("w32_r8_concat_640_640_split3", 2, 640, 640, 16, 32, 320),
    ("w32_r8_640_one_split", 1, 640, 0, 16, 32, 160),
    # whole 16x16 images, K split over channel blocks (fp32 slab + reduction)
    ("w16_1280_split4", 2, 1280, 0, 16, 16, 320),
    ("w16_concat_640_640_split3", 1, 640, 640, 16, 16, 320),
    ("w16_640_one_split", 1, 640, 0, 16, 16, 160),
]


@pytest.fixture
def halo_on():
    K.set_conv_halo(2)
    yield
    K.set_conv_halo(0)
    K.set_conv_halo_split(0)
    K.set_conv_halo_rows32(0)


@pytest.mark.parametrize("case", HALO_SHAPES, ids=[c[0] for c in HALO_SHAPES])
@pytest.mark.parametrize("epi", ["temb_silu_res", "plain", "stats"])
def test_halo_conv(case, epi, halo_on):
    """The halo-tiled 3x3 kernel (every channel block's input rows staged once, 9 taps read from
    LDS) vs torch fp32: time embedding + SiLU + residual epilogue, plain, and the GroupNorm
    partials through a following GroupNorm.  Bar 2e-2 (bf16 storage) / 3e-2 after GroupNorm."""
    name, B, c0, c1, H, W, Co = case
    if W == 32:
        K.set_conv_halo_rows32(8 if "_r8" in name else 4)
    if W == 16 or "_r8" in name:
        K.set_conv_halo_split(int(name.split("split")[-1]) if name[-1].isdigit() else 1)
    torch.manual_seed(11)
    x = torch.randn(B, c0 + c1, H, W)
    w = torch.randn(Co, c0 + c1, 3, 3) / (3 * (c0 + c1) ** 0.5)
    b = torch.randn(Co)
    pc = K.PackedConv(w.to(DEV), b.to(DEV), BF)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV, BF)
    x0 = xn[..., :c0].contiguous()
    x1 = xn[..., c0:].contiguous() if c1 else None
    y_ref = F.conv2d(x, w, b, padding=1)
    if epi == "temb_silu_res":
        temb = torch.randn(B, Co)
        resid = torch.randn(B, Co, H, W)
        ref = F.silu(y_ref + temb[:, :, None, None]) + resid
        out = K.conv2d(pc, x0, B, H, W, x1=x1, temb=temb.to(DEV), temb_stride=Co, act=K.ACT_SILU,
                       residual=resid.permute(0, 2, 3, 1).contiguous().to(DEV, BF))
        assert rel_err(out.permute(0, 3, 1, 2), ref) < 2e-2
    elif epi == "plain":
        out = K.conv2d(pc, x0, B, H, W, x1=x1)
        assert rel_err(out.permute(0, 3, 1, 2), y_ref) < 2e-2
    else:
        if Co % 32 or (H * W) % 64:
            pytest.skip("GroupNorm(32) partials need Cout % 32 == 0 and HW % 64 == 0")
        y = K.conv2d(pc, x0, B, H, W, x1=x1, gn_stats=True)
        assert K.gn_stats_of(y) is not None
        gam, bet = torch.randn(Co), torch.randn(Co)
        out = K.group_norm(y, B, H * W, 32, gam.to(DEV), bet.to(DEV), 1e-5, K.ACT_SILU)
        ref = F.silu(F.group_norm(y_ref, 32, gam, bet, 1e-5))
        assert rel_err(out.view(B, H, W, -1).permute(0, 3, 1, 2), ref) < 3e-2


@pytest.mark.parametrize("ks", [2, 3, 5, 16, 20])
@pytest.mark.parametrize("B,H,C,Co", [(1, 8, 1280, 1280), (2, 16, 192, 320), (1, 10, 64, 200)])
def test_splitk_reduction_tiles(B, H, C, Co, ks, plan):
    """The split-K reduction on every tile shape (rows 16 / 32 / 64 x columns 64 / 128): the splits
    are summed in index order whatever the tile, so outputs are bit-identical across shapes and the
    GroupNorm partials (the same values grouped per tile) agree to 1e-6; vs torch fp32 at 2e-2."""
    torch.manual_seed(12)
    x = torch.randn(B, C, H, H)
    w = torch.randn(Co, C, 3, 3) / (3 * C ** 0.5)
    b = torch.randn(Co)
    temb = torch.randn(B, Co)
    resid = torch.randn(B, Co, H, H)
    pc = K.PackedConv(w.to(DEV), b.to(DEV), BF)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV, BF)
    rn = resid.permute(0, 2, 3, 1).contiguous().to(DEV, BF)
    stats = (H * H) % 64 == 0
    outs = []
    try:
        for rows, cols in [(64, 128), (64, 64), (32, 64), (16, 64), (32, 128)]:
            plan(64, 160, ks)
            K.set_conv_splitk_cols(cols)
            K.set_conv_splitk_rows(rows)
            y = K.conv2d(pc, xn, B, H, H, temb=temb.to(DEV), temb_stride=Co, residual=rn, act=K.ACT_SILU,
                         gn_stats=stats)
            outs.append((y, K.gn_stats_of(y).sum(1) if stats else None))
    finally:
        K.set_conv_splitk_rows(0)
    y0, s0 = outs[0]
    for y, s in outs[1:]:
        assert torch.equal(y, y0)
        if stats:
            assert torch.allclose(s, s0, rtol=1e-6, atol=1e-6)
    ref = F.silu(F.conv2d(x, w, b, padding=1) + temb[:, :, None, None]) + resid
    assert rel_err(y0.permute(0, 3, 1, 2), ref) < 2e-2


FA_CASES = [
    # name, B, c0, c1, H, W, Cout, k, stride, up, plan
    ("3x3", 2, 320, 0, 16, 16, 320, 3, 1, False, (128, 160, 1)),
    ("3x3_split", 1, 1280, 0, 8, 8, 1280, 3, 1, False, (64, 160, 8)),
    ("3x3_ring3", 2, 640, 0, 16, 16, 640, 3, 1, False, (128, 160, 4, 3)),
    ("stride2", 2, 320, 0, 17, 15, 320, 3, 2, False, (64, 160, 2)),
    ("concat", 2, 640, 320, 16, 16, 320, 3, 1, False, (128, 160, 1)),
    ("ragged", 1, 64, 0, 20, 20, 200, 3, 1, False, (64, 64, 1)),
    ("1x1", 3, 640, 0, 10, 10, 960, 1, 1, False, (64, 160, 1)),
    ("1x1_concat_split", 2, 640, 640, 8, 8, 1280, 1, 1, False, (64, 64, 4)),
    ("phase_up", 2, 640, 0, 16, 16, 640, 3, 1, True, (0, 0, 1)),
]


@pytest.mark.parametrize("case", FA_CASES, ids=[c[0] for c in FA_CASES])
def test_fast_addressing_bit_identical(case, plan):
    """ldm_conv2d_set_fast_addressing: the per-row offsets + wave-uniform K position fetch the same
    bytes into the same LDS places as the general address walk, so outputs are bit-identical (3x3
    stride 1 / 2, two-source concat, ragged M / N, 1x1, split K, the 3-stage ring, the phase-form
    upsample)."""
    name, B, c0, c1, H, W, Co, k, s, up, pl = case
    torch.manual_seed(13)
    x = torch.randn(B, c0 + c1, H, W)
    w = torch.randn(Co, c0 + c1, k, k) / (k * (c0 + c1) ** 0.5)
    b = torch.randn(Co)
    pc = K.PackedConv(w.to(DEV), b.to(DEV), BF, upsample_phases=up)
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV, BF)
    x0 = xn[..., :c0].contiguous()
    x1 = xn[..., c0:].contiguous() if c1 else None
    outs = []
    try:
        for fa in (False, True):
            K.set_conv_fast_addressing(fa)
            if pl[0]:
                plan(*pl)
            outs.append(K.conv2d(pc, x0, B, H, W, x1=x1, stride=s, upsample=up, act=K.ACT_SILU))
    finally:
        K.set_conv_fast_addressing(4)
    assert torch.equal(outs[0], outs[1])
    xr = F.interpolate(x, scale_factor=2.0, mode="nearest") if up else x
    ref = F.silu(F.conv2d(xr, w, b, stride=s, padding=k // 2))
    assert rel_err(outs[1].permute(0, 3, 1, 2), ref) < 2e-2
