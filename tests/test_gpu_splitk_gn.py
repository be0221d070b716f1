"""Split-K reduction + GroupNorm(+SiLU) in one launch (ldm_conv2d gn_out, csrc/igemm.hip
splitk_gn_kernel): the deep levels' ResnetBlock2D conv1 -> norm2, conv2 -> the next norm1 /
Transformer2DModel.norm and Downsample2D -> norm1 (/root/reference/ldmseg/models/unet.py:361-425 ->
diffusers ResnetBlock2D / Transformer2DModel).

Bars:
  - the pre-norm output equals the two-launch path (splitk_epilogue_kernel) bit for bit: same slab
    sums in split order, same epilogue arithmetic;
  - the GroupNorm unit accumulators it emits are the exact fp64 sums of the stored bf16 values;
  - the normalised tensor equals ldm_group_norm run on that output with those accumulators bit for
    bit (same (mean, rstd) formation and apply arithmetic);
  - against the two-launch path (whose statistics are fp32 tile partials) within 1e-2 of the
    tensor scale, and against torch fp32 F.group_norm (+ F.silu) of the same output within 1e-2;
  - gn_skip_out (the pre-norm tensor dead) gives the same normalised bits.
Shapes: every deep-level shape of the headline B = 8 step, of config 2 (B = 1: 16-32 blocks) and
of config 5 (B = 16, 8x16 / 4x8), incl. time embedding, residual, stride-2 Downsample2D, 20-channel groups.
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


def _case(B, H, W, cin, cout, k, stride, temb, res, gact, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = (torch.randn(B, H, W, cin, device=DEV, generator=g)).to(BF)
    w = torch.randn(cout, cin, k, k, device=DEV, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    b = torch.randn(cout, device=DEV, generator=g) * 0.1
    pc = K.PackedConv(w, b, BF)
    Ho, Wo = (H // stride, W // stride)
    te = torch.randn(B, cout + 64, device=DEV, generator=g) if temb else None
    r = torch.randn(B, Ho, Wo, cout, device=DEV, generator=g).to(BF) if res else None
    gamma = torch.rand(cout, device=DEV, generator=g) + 0.5
    beta = torch.randn(cout, device=DEV, generator=g) * 0.2
    kw = dict(stride=stride, residual=r, gn_stats=True)          # (Downsample2D: padding 1)
    if temb:
        kw.update(temb=te[:, 64:], temb_stride=te.shape[1])
    return pc, x, kw, (Ho, Wo), gamma, beta


# (B, H, W, cin, cout, ksize, stride, temb, residual, gn act): the deep levels of the UNet step
SHAPES = [
    (8, 8, 8, 1280, 1280, 3, 1, True, False, K.ACT_SILU),       # 8x8 conv1 -> norm2
    (8, 8, 8, 1280, 1280, 3, 1, False, True, K.ACT_SILU),       # 8x8 conv2 -> next norm1
    (8, 8, 8, 1280, 1280, 3, 1, False, True, K.ACT_NONE),       # mid conv2 -> transformer norm
    (8, 16, 16, 640, 1280, 3, 1, True, False, K.ACT_SILU),      # 16x16 conv1 of the 640 -> 1280 block
    (8, 16, 16, 1280, 1280, 3, 1, False, True, K.ACT_NONE),     # 16x16 conv2 -> transformer norm
    (8, 32, 32, 640, 640, 3, 2, False, False, K.ACT_SILU),      # Downsample2D 32 -> 16, 20-ch groups
    (8, 16, 16, 1280, 1280, 3, 2, False, False, K.ACT_SILU),    # Downsample2D 16 -> 8
    (1, 8, 8, 1280, 1280, 3, 1, True, False, K.ACT_SILU),       # config 2 (B = 1): 32 blocks
    (1, 16, 16, 1280, 1280, 3, 1, False, True, K.ACT_NONE),
    (1, 32, 32, 640, 640, 3, 2, False, False, K.ACT_SILU),      # 16 blocks
    (16, 8, 16, 1280, 1280, 3, 1, True, False, K.ACT_SILU),     # config 5 (T = 16, 32x64 latents)
    (16, 4, 8, 1280, 1280, 3, 1, False, True, K.ACT_SILU),
]


@pytest.mark.parametrize("B,H,W,cin,cout,k,stride,temb,res,gact", SHAPES)
def test_splitk_gn_fused(B, H, W, cin, cout, k, stride, temb, res, gact):
    G, eps = 32, 1e-5
    pc, x, kw, (Ho, Wo), gamma, beta = _case(B, H, W, cin, cout, k, stride, temb, res, gact, seed=B * H + cin)
    hw = Ho * Wo
    K.set_gn_fuse(False)
    try:
        ref = K.conv2d(pc, x, B, H, W, gn_next=(G, gamma, beta, eps, gact, True), **kw)
        assert getattr(ref, K.GN_DONE_ATTR) is None
        ref_n = K.group_norm(ref, B, hw, G, gamma, beta, eps, gact)
    finally:
        K.set_gn_fuse(True)
    out = K.conv2d(pc, x, B, H, W, gn_next=(G, gamma, beta, eps, gact, True), **kw)
    done = getattr(out, K.GN_DONE_ATTR)
    assert done is not None, "the deep-level plan should split K and take the fused GroupNorm"
    gout = K.group_norm(out, B, hw, G, gamma, beta, eps, gact)
    assert gout is done[1]                                  # no second launch
    assert torch.equal(out, ref)                            # pre-norm output bit for bit
    part = getattr(out, K.GN_PART_ATTR)
    if part is not None:          # (hw = 32, config 5's 4x8 level: no producer statistics, gn_small)
        unit = cout // part.shape[2]
        o64 = out.double().view(B, hw, cout // unit, unit)
        assert torch.allclose(part.sum(1)[..., 0], o64.sum((1, 3)), rtol=1e-12, atol=1e-9)
        assert torch.allclose(part.sum(1)[..., 1], (o64 * o64).sum((1, 3)), rtol=1e-12, atol=1e-9)
        c = out.clone()
        setattr(c, K.GN_PART_ATTR, part)
        g2 = K.group_norm(c, B, hw, G, gamma, beta, eps, gact)
        assert torch.equal(gout.reshape(-1), g2.reshape(-1))     # = gn_apply on it
    assert rel_err(gout.reshape(-1), ref_n.reshape(-1)) < 1e-2
    with torch.no_grad():
        t = F.group_norm(out.float().permute(0, 3, 1, 2), G, gamma, beta, eps)
        if gact == K.ACT_SILU:
            t = F.silu(t)
    assert rel_err(gout.reshape(B, Ho, Wo, cout).permute(0, 3, 1, 2), t) < 1e-2
    dead = K.conv2d(pc, x, B, H, W, gn_next=(G, gamma, beta, eps, gact, False), **kw)
    assert K.group_norm(dead, B, hw, G, gamma, beta, eps, gact) is dead
    assert torch.equal(dead.reshape(-1), gout.reshape(-1))


def test_splitk_gn_out_of_scope_falls_back():
    """An unsplit plan (the 64x64 level) or a grid below the hook's minimum does not take gn_out: the conv stores its statistics and the
    GroupNorm runs as its own launch; a different GroupNorm than the one announced never reuses the
    fused result."""
    B, H, W, C, G = 2, 64, 64, 320, 32
    pc, x, kw, _, gamma, beta = _case(B, H, W, C, C, 3, 1, True, False, K.ACT_SILU, seed=7)
    out = K.conv2d(pc, x, B, H, W, gn_next=(G, gamma, beta, 1e-5, K.ACT_SILU, True), **kw)
    assert getattr(out, K.GN_DONE_ATTR) is None
    y = K.group_norm(out, B, H * W, G, gamma, beta, 1e-5, K.ACT_SILU)
    with torch.no_grad():
        t = F.silu(F.group_norm(out.float().permute(0, 3, 1, 2), G, gamma, beta, 1e-5))
    assert rel_err(y.reshape(B, H, W, C).permute(0, 3, 1, 2), t) < 1e-2
    # grids below the min-blocks hook keep the two launches
    pc, x, kw, _, gamma, beta = _case(1, 8, 8, 1280, 1280, 3, 1, True, False, K.ACT_SILU, seed=9)
    K.set_gn_fuse_min_blocks(64)
    try:
        out = K.conv2d(pc, x, 1, 8, 8, gn_next=(32, gamma, beta, 1e-5, K.ACT_SILU, True), **kw)
    finally:
        K.set_gn_fuse_min_blocks(16)
    assert getattr(out, K.GN_DONE_ATTR) is None
    pc, x, kw, _, gamma, beta = _case(8, 8, 8, 1280, 1280, 3, 1, True, False, K.ACT_SILU, seed=8)
    out = K.conv2d(pc, x, 8, 8, 8, gn_next=(32, gamma, beta, 1e-5, K.ACT_SILU, True), **kw)
    assert getattr(out, K.GN_DONE_ATTR) is not None
    other = K.group_norm(out, 8, 64, 32, gamma, beta, 1e-5, K.ACT_NONE)    # another activation: a launch
    assert other is not getattr(out, K.GN_DONE_ATTR)[1]
    with torch.no_grad():
        t = F.group_norm(out.float().permute(0, 3, 1, 2), 32, gamma, beta, 1e-5)
    assert rel_err(other.reshape(8, 8, 8, 1280).permute(0, 3, 1, 2), t) < 1e-2


@pytest.mark.parametrize("B", [1, 8])
def test_unet_sd14_gn_fuse_vs_unfused(B):
    """The SD-1.4 UNet (random init, bf16, 64x64 latents) with the deep levels' GroupNorms in the
    split-K reductions vs the two-launch path: the same model output within the bf16 bar, and the
    fused step issues fewer GroupNorm launches."""
    from ldmseg.models import UNet
    torch.manual_seed(0)
    u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="random")
    with torch.no_grad():
        for _, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    u = u.eval().to(DEV, BF)
    x = torch.randn(B, 8, 64, 64, device=DEV).to(BF)
    t = torch.tensor(501, device=DEV)
    prof = K.LaunchProfiler()
    K.set_profiler(prof)
    try:
        y1 = u(x, t).sample
    finally:
        K.set_profiler(None)
    n_fused = prof.summary()["group_norm"]["launches"]
    K.set_gn_fuse(False)
    prof = K.LaunchProfiler()
    K.set_profiler(prof)
    try:
        y0 = u(x, t).sample
    finally:
        K.set_profiler(None)
        K.set_gn_fuse(True)
    n_plain = prof.summary()["group_norm"]["launches"]
    assert torch.isfinite(y1.float()).all()
    assert rel_err(y1, y0) < 2e-2
    assert n_fused <= n_plain - 20, (n_fused, n_plain)
