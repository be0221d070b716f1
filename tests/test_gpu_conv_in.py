"""ldm_conv_in (csrc/conv_in.hip): the UNet's conv_in (/root/reference/ldmseg/models/unet.py:357, the
8 / 12-channel conv of modify_encoder :178-233) read straight from the sampler's NCHW sources
[x_t || rgb (|| cond)] (trainers_ldm_cond.py:1134-1141) in one launch.

Against the two launches it replaces (ldm_nchw_to_nhwc + ldm_conv2d): the same bf16 inputs and the
same k32 chunks of the tap-major K in the same order, so the outputs agree to a bf16 ulp at most (the
test reports whether they are bit-identical); against torch fp32 F.conv2d on the bf16-rounded inputs
within the conv tests' 1e-2; its GroupNorm unit accumulators equal the fp64 sums of the stored values
to fp32 rounding; and the UNet with it on / off (8 and 12 input channels) within the bf16 bar.
Shapes: the headline (B = 8, 64x64), config 2 (B = 1), config 5 (B = 16, 32x64), self-conditioning.
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


@pytest.mark.parametrize("B,H,W,nsrc", [(8, 64, 64, 2), (1, 64, 64, 2), (16, 32, 64, 2), (2, 64, 64, 3),
                                        (3, 16, 32, 1)])
def test_conv_in_matches_two_launches_and_torch(B, H, W, nsrc):
    g = torch.Generator(device=DEV).manual_seed(B * H + nsrc)
    srcs = [torch.randn(B, 4, H, W, device=DEV, generator=g) * (1.0 + i) for i in range(nsrc)]
    cin = 4 * nsrc
    conv = torch.nn.Conv2d(cin, 320, 3, padding=1).to(DEV)
    with torch.no_grad():
        conv.bias.normal_(0.0, 0.2, generator=g)
    pc = K.PackedConv(conv.weight, conv.bias, BF, cin_pad=16)
    assert K.conv_in_ok(pc, srcs, B, H, W) == (B * H >= K.CONV_IN_MIN_ROWS)
    out = K.conv_in(pc, srcs, B, H, W)          # (the kernel itself takes every size)
    x = K.nchw_to_nhwc(srcs, 16, BF)
    ref = K.conv2d(pc, x, B, H, W, gn_stats=True)
    assert out.shape == ref.shape == (B, H, W, 320) and out.dtype == BF
    d = (out.float() - ref.float()).abs()
    ulp = ref.float().abs().clamp_min(2.0 ** -100) * 2.0 ** -7
    assert bool((d <= ulp).all()), d.max().item()
    print(f"B={B} {H}x{W} sources={nsrc}: bit-identical to the two launches: {torch.equal(out, ref)}")
    with torch.no_grad():
        xin = torch.cat(srcs, 1).to(BF).float()
        t = F.conv2d(xin, conv.weight.to(BF).float(), conv.bias, padding=1).permute(0, 2, 3, 1)
    assert rel_err(out, t) < 1e-2
    part = getattr(out, K.GN_PART_ATTR)
    if (H * W) % 64 == 0:
        unit = 320 // part.shape[2]
        o64 = out.double().view(B, H * W, 320 // unit, unit)
        assert torch.allclose(part.sum(1)[..., 0], o64.sum((1, 3)), rtol=1e-5, atol=1e-3)
        assert torch.allclose(part.sum(1)[..., 1], (o64 * o64).sum((1, 3)), rtol=1e-5, atol=1e-3)
        # the GroupNorm it feeds, from these accumulators, against torch on the same output
        gam, bet = torch.rand(320, device=DEV) + 0.5, torch.randn(320, device=DEV) * 0.1
        y = K.group_norm(out, B, H * W, 32, gam, bet, 1e-5, K.ACT_SILU)
        with torch.no_grad():
            ty = F.silu(F.group_norm(out.float().permute(0, 3, 1, 2), 32, gam, bet, 1e-5))
        assert rel_err(y.view(B, H, W, 320).permute(0, 3, 1, 2), ty) < 1e-2
    else:
        assert part is None


@pytest.mark.parametrize("cond", [0, 4])
def test_unet_conv_in_fused_vs_two_launches(cond):
    from ldmseg.models import UNet
    torch.manual_seed(0)
    u = UNet(block_out_channels=(64, 128, 128, 128), cross_attention_dim=None)
    with torch.no_grad():
        for _, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="random", cond_channels=cond,
                     init_mode_cond="random")
    u = u.eval().to(DEV, BF)
    srcs = [torch.randn(8, 4, 32, 32, device=DEV) for _ in range(2 + cond // 4)]   # 256 rows: fused
    t = torch.tensor([377.0], device=DEV)
    y1 = u.forward_sources(srcs, t)
    u.set_conv_in_fused(False)
    try:
        y0 = u.forward_sources(srcs, t)
    finally:
        u.set_conv_in_fused(True)
    assert torch.isfinite(y1.float()).all()
    assert rel_err(y1, y0) < 2e-2
