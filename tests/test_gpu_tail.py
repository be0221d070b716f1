"""The fused UNet tail (ldm_unet_tail, csrc/tail.hip): conv_norm_out -> SiLU -> conv_out (-> DDIM step)
in one launch, /root/reference/ldmseg/models/unet.py:428-431 and ddim_scheduler.py:218-269.

Against the unfused launches (ldm_group_norm + ldm_conv2d NCHW + ldm_ddim_step): the GroupNorm-SiLU
values are the same bf16 numbers (gn_apply's arithmetic), the conv sums them in a different K order, so
the bf16 model outputs agree to a few bf16 ulps (bar 1e-2 of the tensor scale) and against torch fp32 to
the conv tests' 2e-2; the fused DDIM step on the fused model output is the ldm_ddim_step arithmetic and
must equal ldm_ddim_step run on that output bit for bit.  Covered: the UNet's 64x64 (headline) and 32x64
(config 5) latents, B = 1 and 8, the 12-channel-input variant's same tail, epsilon and v prediction,
clipping, an odd group count of the statistics slots.
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


def _producer(B, H, W, C, seed):
    """An NHWC bf16 tensor with the producer GroupNorm accumulators a conv epilogue attaches."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = (torch.randn(B, H, W, C, device=DEV, generator=g) * 1.3 + 0.2).to(BF)
    pc = K.PackedConv(torch.eye(C, device=DEV)[:, :, None, None], torch.zeros(C, device=DEV), BF)
    return K.conv2d(pc, x, B, H, W, gn_stats=True)                   # identity 1x1: same values + stats


@pytest.mark.parametrize("B,H,W", [(8, 64, 64), (1, 64, 64), (2, 32, 64), (1, 16, 32)])
def test_tail_matches_unfused_and_torch(B, H, W):
    torch.manual_seed(3)
    C, G = 320, 32
    x = _producer(B, H, W, C, 5)
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    conv = torch.nn.Conv2d(C, 4, 3, padding=1).to(DEV)
    pc = K.PackedConv(conv.weight, conv.bias, BF)
    eps = K.unet_tail(x, B, H, W, G, gamma, beta, 1e-5, pc, BF)
    h = K.group_norm(x, B, H * W, G, gamma, beta, 1e-5, K.ACT_SILU)
    ref = K.conv2d(pc, h, B, H, W, out_layout=K.OUT_NCHW)
    assert eps.shape == ref.shape == (B, 4, H, W) and eps.dtype == BF
    assert rel_err(eps, ref) < 1e-2
    with torch.no_grad():
        xf = x.float().permute(0, 3, 1, 2)
        t = F.silu(F.group_norm(xf, G, gamma, beta, 1e-5))
        ref32 = conv(t)
    assert rel_err(eps, ref32) < 2e-2


@pytest.mark.parametrize("pred,clip", [("epsilon", False), ("v_prediction", True)])
def test_tail_fused_ddim_step_equals_ddim_kernel(pred, clip):
    torch.manual_seed(4)
    B, H, W, C, G = 8, 64, 64, 320, 32
    x = _producer(B, H, W, C, 6)
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    conv = torch.nn.Conv2d(C, 4, 3, padding=1).to(DEV)
    pc = K.PackedConv(conv.weight, conv.bias, BF)
    sample = torch.randn(B, 4, H, W, device=DEV)
    ac = torch.linspace(0.9999, 0.005, 1000, device=DEV)
    t = torch.tensor([741], dtype=torch.int64, device=DEV)
    d = dict(sample=sample, t=t, alphas_cumprod=ac, final_alpha=1.0, step_ratio=20, prediction_type=pred,
             clip_sample=clip, clip_range=1.0, use_clipped=False, out_dtype=torch.float32)
    eps, prev, x0 = K.unet_tail(x, B, H, W, G, gamma, beta, 1e-5, pc, BF, ddim=d, want_eps=True)
    p2, x2 = K.ddim_step(eps, sample, t, ac, 1.0, 20, pred, clip, 1.0, False, torch.float32)
    assert torch.equal(prev, p2) and torch.equal(x0, x2)
    _, prev3, x03 = K.unet_tail(x, B, H, W, G, gamma, beta, 1e-5, pc, BF, ddim=d, want_eps=False)
    assert torch.equal(prev3, prev) and torch.equal(x03, x0)


def test_unet_forward_ddim_step_fused_vs_unfused():
    """UNet.forward_ddim_step with the tail fused vs the separate GroupNorm / conv_out / DDIM launches on
    a small bf16 UNet (same module, same inputs)."""
    from ldmseg.models import UNet
    from ldmseg.schedulers import DDIMNoiseScheduler
    torch.manual_seed(0)
    u = UNet(block_out_channels=(64, 128, 128, 128), cross_attention_dim=None)
    with torch.no_grad():
        for _, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="random")
    u = u.eval().to(DEV, BF)
    sch = DDIMNoiseScheduler()
    sch.set_timesteps_inference(50)
    B = 2
    lat = torch.randn(B, 4, 32, 32, device=DEV)
    rgb = torch.randn(B, 4, 32, 32, device=DEV)
    t_f = torch.tensor([501.0], device=DEV)
    t_i = torch.tensor([501], dtype=torch.int64, device=DEV)
    p1, x1 = u.forward_ddim_step([lat, rgb], t_f, sch, t_i, lat)
    u.set_tail_fused(False)
    try:
        p2, x2 = u.forward_ddim_step([lat, rgb], t_f, sch, t_i, lat)
    finally:
        u.set_tail_fused(True)
    assert p1.dtype == p2.dtype == torch.float32
    assert rel_err(p1, p2) < 2e-2 and rel_err(x1, x2) < 2e-2


def _small_bf16_unet(cond_channels):
    from ldmseg.models import UNet
    torch.manual_seed(0)
    u = UNet(block_out_channels=(64, 128, 128, 128), cross_attention_dim=None)
    with torch.no_grad():
        for _, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="random", cond_channels=cond_channels,
                     init_mode_cond="random")
    return u.eval().to(DEV, BF)


@pytest.mark.parametrize("self_condition", [False, True])
def test_sample_latents_bf16_inplace_tail(self_condition):
    """The headline sampling path: DenoiseStep passes prev_out = its latents, so the fused
    bf16 tail writes prev_sample over the latents it reads, inside the captured step graph; with
    self-conditioning the x0 of each step is copied into the third conv_in source, and the last step
    returns x0.  Graph replay must equal eager bit for bit, and both must match the unfused tail
    (ldm_group_norm + ldm_conv2d + ldm_ddim_step into fresh tensors, then copied) within the tail's
    bf16 bar at every step."""
    from ldmseg.pipelines import sample_latents
    from ldmseg.schedulers import DDIMNoiseScheduler
    u = _small_bf16_unet(4 if self_condition else 0)
    sch = DDIMNoiseScheduler()
    g = torch.Generator(device=DEV).manual_seed(11)
    rgb = torch.randn(2, 4, 32, 32, device=DEV, generator=g)
    kw = dict(num_inference_steps=6, seed=3, self_condition=self_condition, return_all_latents=True)
    eager = sample_latents(u, sch, rgb, use_graph=False, **kw)
    graph = sample_latents(u, sch, rgb, use_graph=True, **kw)
    assert eager.shape == (6 * 2, 4, 32, 32) and torch.isfinite(eager).all()
    assert torch.equal(eager, graph)
    u.set_tail_fused(False)
    try:
        unfused = sample_latents(u, sch, rgb, use_graph=False, **kw)
    finally:
        u.set_tail_fused(True)
    for s in range(6):
        assert rel_err(eager[2 * s:2 * s + 2], unfused[2 * s:2 * s + 2]) < 3e-2, s
