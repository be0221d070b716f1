#!/usr/bin/env python3
"""Micro-benchmark single HIP ops at UNet shapes (for A/B of kernel variants and rocprofv3).

    python tools/opbench.py [--iters N] [--only NAME ...]

Prints one line per case: mean launch time (HIP events, current stream) and achieved
TFLOP/s or GB/s.  All variants run interleaved in ONE process (MI355X_MICROARCH §5.4 rule 24).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd"))

import torch  # noqa: E402

from ldmseg.ops import native as K  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16
BATCH = 8          # --batch: the conv / GEMM cases' B (their shapes are written for the bench's B = 8)


def conv_case(B, H, W, Cin, Cout, k=3, stride=1, up=False, layout=K.OUT_NHWC, geglu=False, residual=False,
              temb=False, stats=False, c1=0, phases=False, rows32=0):
    B = max(1, B * BATCH // 8)
    g = torch.Generator(device=DEV).manual_seed(0)
    x0 = torch.randn(B, H, W, Cin - c1, device=DEV, generator=g).to(BF)
    x1 = torch.randn(B, H, W, c1, device=DEV, generator=g).to(BF) if c1 else None
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) * 0.05
    pc = K.PackedConv(w, torch.randn(Cout, device=DEV), BF, geglu=geglu, upsample_phases=phases)
    ho, wo = (2 * H, 2 * W) if up else ((H - 1) // stride + 1, (W - 1) // stride + 1)
    res = torch.randn(B, ho, wo, Cout, device=DEV).to(BF) if residual else None
    te = torch.randn(B, Cout, device=DEV) if temb else None
    out_layout = K.OUT_GEGLU if geglu else layout

    def run():
        K.set_conv_halo_rows32(rows32)
        return K.conv2d(pc, x0, B, H, W, x1=x1, stride=stride, upsample=up, residual=res, temb=te,
                        temb_stride=Cout if temb else 0, out_layout=out_layout, gn_stats=stats)
    flops = 2.0 * B * ho * wo * Cout * (4 if phases else k * k) * Cin     # executed (phase form: 4 taps)
    return run, flops, None


def ln_gemm_case(rows, C, N, geglu=False):
    """A LayerNorm-folded 1x1 GEMM as the transformer runs it (norm1 -> QKV, norm3 -> GEGLU): the packed
    W diag(gamma) weight, the producer's fp64 row statistics."""
    rows = max(1, rows * BATCH // 8)
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(rows, C, device=DEV, generator=g).to(BF)
    w = torch.randn(N, C, device=DEV, generator=g) * 0.05
    pc = K.packed_ln_fold(w, torch.randn(N, device=DEV, generator=g), torch.rand(C, device=DEV, generator=g) + 0.5,
                          torch.randn(C, device=DEV, generator=g) * 0.1, BF, geglu=geglu)
    xf = x.double()
    rs = torch.stack([xf.sum(1), (xf * xf).sum(1)], 1).contiguous()
    lay = K.OUT_GEGLU if geglu else K.OUT_NHWC
    return (lambda: K.linear(pc, x, ln=(rs, 1e-5), out_layout=lay)), 2.0 * rows * N * C, None


def conv_in_case(B, H=64, W=64, fused=True, stats=True):
    """The UNet's conv_in from the sampler's two fp32 NCHW sources: ldm_conv_in, or nchw_to_nhwc +
    ldm_conv2d (gn_stats on, as the UNet runs it)."""
    B = max(1, B * BATCH // 8)
    g = torch.Generator(device=DEV).manual_seed(0)
    srcs = [torch.randn(B, 4, H, W, device=DEV, generator=g) for _ in range(2)]
    pc = K.PackedConv(torch.randn(320, 8, 3, 3, device=DEV, generator=g) * 0.1, torch.randn(320, device=DEV), BF,
                      cin_pad=16)

    def run():
        if fused:
            return K.conv_in(pc, srcs, B, H, W, gn_stats=stats)
        return K.conv2d(pc, K.nchw_to_nhwc(srcs, 16, BF), B, H, W, gn_stats=stats)
    return run, 2.0 * B * H * W * 320 * 72, None


def mm_case(M, K, N):
    """torch.mm (hipBLASLt) on the same GEMM shape: the library reference point, no epilogue."""
    a = torch.randn(M, K, device=DEV).to(BF)
    b = torch.randn(K, N, device=DEV).to(BF)
    return (lambda: torch.mm(a, b)), 2.0 * M * K * N, None


def attn_case(B, N, C, heads=8, legacy=False, waves=0, maxcol=2, fp8=False, scaled=True, d80=True, qs2=0, skew=0,
              pair=True, il=True):
    qkv = torch.randn(B, N, 3 * C, device=DEV).to(BF)

    def run():
        K.set_attention_d80(d80)
        K.set_attention_qs2(qs2)
        K.set_attention_il(il)
        K.set_attention_skew(skew)
        K.set_attention_pair(pair)
        K.force_attention_legacy(legacy)
        K.set_attention_waves(waves)
        K.set_attention_maxcol(maxcol)
        K.set_attention_fp8_scaled(scaled)
        return K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, heads, C // heads, N, N, 3 * C, 3 * C, 3 * C,
                           fp8=fp8)
    return run, 4.0 * B * heads * N * N * (C // heads), None


def wgrad_case(B, H, W, Cin, Cout, k=3, geglu=False, ring=True, fast=True, r3=True):
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(B, H, W, Cin, device=DEV, generator=g).to(BF)
    dy = torch.randn(B, H, W, Cout, device=DEV, generator=g).to(BF)
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) * 0.05
    pc = K.PackedConv(w, None, BF, geglu=geglu)
    dw = torch.empty(Cout, Cin, k, k, device=DEV) if k == 3 else torch.empty(Cout, Cin, device=DEV)

    def run():
        K.set_wgrad_ring(ring)
        K.set_wgrad_fast_loader(fast)
        K.set_wgrad_reduce3(r3)
        return K.conv2d_wgrad(pc, x, B, H, W, dy, dw=dw)
    return run, 2.0 * B * H * W * Cout * k * k * Cin, None


def colsum_case(rows, C, segments=1, geglu=False):
    x = torch.randn(rows, C, device=DEV).to(BF)
    out = torch.empty(segments, C, device=DEV)

    def run():
        return K.colsum(x, rows, C, segments, geglu=geglu, out=out)
    return run, 0.0, 2.0 * rows * C


def gn_bwd_case(B, HW, C, silu=True, add=True):
    x = torch.randn(B, HW, C, device=DEV).to(BF)
    dy = torch.randn(B, HW, C, device=DEV).to(BF)
    gamma = torch.randn(C, device=DEV)
    beta = torch.randn(C, device=DEV)
    act = K.ACT_SILU if silu else K.ACT_NONE
    _, mr = K.group_norm_train(x, B, HW, 32, gamma, beta, 1e-5, act=act)
    a = torch.randn(B, HW, C, device=DEV).to(BF) if add else None
    dx = torch.empty_like(x)
    dg = torch.zeros(C, device=DEV)
    db = torch.zeros(C, device=DEV)

    def run():
        return K.group_norm_bwd(x, B, HW, 32, mr, gamma, beta, act, dy, add_src=a, dx0=dx, dgamma=dg, dbeta=db)
    # algorithmic bytes: the partial pass reads x, dy; the apply pass reads x, dy (, add) and writes dx
    return run, 0.0, (6 if add else 5) * x.numel() * 2.0


def attn_bwd_case(B, N, C, heads=8, new=True):
    d = C // heads
    qkv = (torch.randn(B, N, 3 * C, device=DEV) * 0.5).to(BF)
    go = torch.randn(B, N, C, device=DEV).to(BF)
    o, lse = K.attention_fwd_lse(qkv, qkv[..., C:], qkv[..., 2 * C:], B, heads, d, N, N, 3 * C, 3 * C, 3 * C)
    dqkv = torch.empty_like(qkv)

    def run():
        K.set_attention_bwd32(new)
        return K.attention_bwd(qkv, qkv[..., C:], qkv[..., 2 * C:], o, go, lse, B, heads, d, N, N, 3 * C, 3 * C,
                               3 * C, dqkv, dqkv[..., C:], dqkv[..., 2 * C:], 3 * C, 3 * C)
    return run, 10.0 * B * heads * N * N * d, None     # five N x N x d matmuls (S, dP, dV, dK, dQ)


def ff_case(rows, fused=True, Fh=1280, proj_out=False):
    """The transformer FeedForward at width 320 (LayerNorm-folded GEGLU + ff.net.2 + residual): the
    fused ldm_feedforward or the two ldm_conv2d launches it replaces."""
    C = 320
    rows = max(128, rows * BATCH // 8)
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(rows, C, device=DEV, generator=g).to(BF)
    w1 = torch.randn(2 * Fh, C, device=DEV, generator=g) * 0.05
    w2 = torch.randn(C, Fh, device=DEV, generator=g) * 0.03
    pc1 = K.packed_ln_fold(w1, torch.randn(2 * Fh, device=DEV), torch.ones(C, device=DEV), torch.zeros(C, device=DEV),
                           BF, geglu=True)
    pc2 = K.PackedConv(w2, torch.randn(C, device=DEV), BF)
    xd = x.double()
    rs = torch.stack([xd.sum(-1), (xd * xd).sum(-1)], -1).reshape(-1).contiguous()
    res = torch.randn(rows, C, device=DEV).to(BF)

    pc3 = K.PackedConv(torch.randn(C, C, device=DEV, generator=g) * 0.05, torch.randn(C, device=DEV), BF)
    B, HW = rows // 4096, 64

    def run():
        if proj_out:
            if fused:
                return K.feedforward(pc1, pc2, x, ln=(rs, 1e-5), residual=res, proj_out=(pc3, res, B, HW, HW, True))
            h = K.feedforward(pc1, pc2, x, ln=(rs, 1e-5), residual=res)
            return K.conv2d(pc3, h, B, HW, HW, residual=res, gn_stats=True)
        if fused:
            return K.feedforward(pc1, pc2, x, ln=(rs, 1e-5), residual=res)
        f = K.linear(pc1, x, out_layout=K.OUT_GEGLU, ln=(rs, 1e-5))
        return K.linear(pc2, f, residual=res)
    return run, 2.0 * rows * 3 * Fh * C, None


def tin_case(B, fused=True, mode=1):
    """Transformer2DModel input half at the 64x64 level: GroupNorm -> proj_in -> LN-folded QKV, as
    ldm_transformer_in or the three launches it replaces."""
    C, HW = 320, 64
    B = max(1, B * BATCH // 8)
    g = torch.Generator(device=DEV).manual_seed(0)
    x_raw = torch.randn(B, HW, HW, C, device=DEV, generator=g).to(BF)
    pcc = K.PackedConv(torch.randn(C, C, device=DEV, generator=g) * 0.05, None, BF)
    pc_in = K.PackedConv(torch.randn(C, C, device=DEV, generator=g) * 0.05, torch.randn(C, device=DEV), BF)
    pc_q = K.packed_ln_fold(torch.randn(3 * C, C, device=DEV, generator=g) * 0.05, None,
                            torch.ones(C, device=DEV), torch.zeros(C, device=DEV), BF)
    x = K.conv2d(pcc, x_raw, B, HW, HW, gn_stats=True)
    gam, bet = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    N = HW * HW

    def run():
        if fused:
            K.set_transformer_in_mode(mode)
            return K.transformer_in(pc_in, pc_q, x, B, N, 32, gam, bet, 1e-6, 1e-5)
        h = K.group_norm(x, B, N, 32, gam, bet, 1e-6)
        rs = torch.zeros(2 * B * N, dtype=torch.float64, device=DEV)
        h = K.linear(pc_in, h, row_stats=rs)
        return K.linear(pc_q, h, ln=(rs, 1e-5))
    return run, 2.0 * B * N * C * 4 * C, None


def gn_case(B, HW, C, stats):
    x = torch.randn(B, HW, C, device=DEV).to(BF)
    if stats:
        setattr(x, K.GN_PART_ATTR, torch.zeros(B, K.gn_slots_for(HW), C // K.gn_unit_for(C), 2, dtype=torch.float64,
                                               device=DEV))
    gam, bet = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)

    def run():
        return K.group_norm(x, B, HW, 32, gam, bet, 1e-5, K.ACT_SILU)
    return run, None, (2 + (0 if stats else 1)) * x.numel() * 2


def copy_case(n):
    """Bandwidth reference: a device copy of n bf16 elements (read + write)."""
    x = torch.randn(n, device=DEV).to(BF)
    y = torch.empty_like(x)

    def run():
        y.copy_(x)
        return y
    return run, None, 2 * n * 2


def tail_case(B, fused=True, ddim=True):
    """The UNet tail at the 64x64 level: GroupNorm -> SiLU -> conv_out (320 -> 4) (-> DDIM), as one
    ldm_unet_tail launch or the group_norm + conv2d (NCHW) + ddim_step launches it replaces."""
    C, H, G = 320, 64, 32
    B = max(1, B * BATCH // 8)
    g = torch.Generator(device=DEV).manual_seed(0)
    xr = torch.randn(B, H, H, C, device=DEV, generator=g).to(BF)
    pid = K.PackedConv(torch.eye(C, device=DEV)[:, :, None, None], torch.zeros(C, device=DEV), BF)
    x = K.conv2d(pid, xr, B, H, H, gn_stats=True)
    gam, bet = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1
    pc = K.PackedConv(torch.randn(4, C, 3, 3, device=DEV, generator=g) * 0.02, torch.randn(4, device=DEV), BF)
    smp = torch.randn(B, 4, H, H, device=DEV)
    ac = torch.linspace(0.9999, 0.005, 1000, device=DEV)
    t = torch.tensor([741], dtype=torch.int64, device=DEV)
    d = dict(sample=smp, t=t, alphas_cumprod=ac, final_alpha=1.0, step_ratio=20, prediction_type="epsilon",
             clip_sample=False, clip_range=1.0, use_clipped=False, out_dtype=torch.float32)

    def run():
        if fused:
            return K.unet_tail(x, B, H, H, G, gam, bet, 1e-5, pc, BF, ddim=d if ddim else None, want_eps=not ddim)
        h = K.group_norm(x, B, H * H, G, gam, bet, 1e-5, K.ACT_SILU)
        e = K.conv2d(pc, h, B, H, H, out_layout=K.OUT_NCHW)
        return K.ddim_step(e, smp, t, ac, 1.0, 20, "epsilon", False, 1.0, False, torch.float32) if ddim else e
    return run, None, x.numel() * 2


def temb_case(B, fused=True):
    """The time-embedding MLP: sinusoid -> linear_1 + SiLU -> linear_2 + SiLU -> the 22 batched
    time_emb_proj (1280 -> 20160), as ldm_linear_rows launches or the tproj + tile-GEMM path."""
    g = torch.Generator(device=DEV).manual_seed(0)
    l1 = K.PackedConv(torch.randn(1280, 320, device=DEV, generator=g) * 0.05, torch.randn(1280, device=DEV), BF)
    l2 = K.PackedConv(torch.randn(1280, 1280, device=DEV, generator=g) * 0.03, torch.randn(1280, device=DEV), BF)
    tp = K.PackedConv(torch.randn(20160, 1280, device=DEV, generator=g) * 0.03, torch.randn(20160, device=DEV), BF)
    freqs = torch.exp(-torch.log(torch.tensor(10000.0)) * torch.arange(160) / 160).to(DEV)
    t = torch.tensor([741.0], device=DEV)

    def run():
        if fused:
            e = K.linear_rows(l1, None, B, act=K.ACT_SILU, t=t, freqs=freqs)
            e = K.linear_rows(l2, e, B, act=K.ACT_SILU)
            return K.linear_rows(tp, e, B, out_dtype=torch.float32)
        e = K.timestep_proj(t, B, freqs, 320, True, BF)
        e = K.linear(l1, e, act=K.ACT_SILU)
        e = K.linear(l2, e, act=K.ACT_SILU)
        return K.linear(tp, e, out_dtype=torch.float32)
    return run, None, (tp.w.numel() + l1.w.numel() + l2.w.numel()) * 2


def ln_case(rows, C):
    x = torch.randn(rows, C, device=DEV).to(BF)
    gam, bet = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    return (lambda: K.layer_norm(x, gam, bet, 1e-5)), None, 2 * x.numel() * 2


def panoptic_case(B, Kc, H, W):
    x = torch.randn(B, Kc, H, W, device=DEV)

    def run():
        pred, cnt, mc = K.panoptic_pixels(x, 0.5, 255, "max")
        return K.panoptic_finalize(pred, cnt, mc, 512, 0.5, 255)
    # two reads of the logits + pred write/read + out write
    return run, None, 2 * x.numel() * 4 + 3 * B * H * W * 4


CASES = {
    "conv3_l0_320": lambda: conv_case(8, 64, 64, 320, 320, temb=True, stats=True),
    "conv3_l0_320_ns": lambda: conv_case(8, 64, 64, 320, 320, temb=True),
    "conv3_up_l0_960_ns": lambda: conv_case(8, 64, 64, 960, 320, c1=320, residual=True),
    "conv3_l1_640_ns": lambda: conv_case(8, 32, 32, 640, 640, temb=True),
    "conv3_l1_640": lambda: conv_case(8, 32, 32, 640, 640, temb=True, stats=True),
    "conv3_l2_1280": lambda: conv_case(8, 16, 16, 1280, 1280, temb=True, stats=True),
    "conv3_l3_1280": lambda: conv_case(8, 8, 8, 1280, 1280, temb=True, stats=True),
    "conv_in_16": lambda: conv_case(8, 64, 64, 16, 320, stats=True),
    "cin_fused": lambda: conv_in_case(8),
    "cin_two": lambda: conv_in_case(8, fused=False),
    "cin_fused_nostats": lambda: conv_in_case(8, stats=False),
    "cin_two_nostats": lambda: conv_in_case(8, fused=False, stats=False),
    "conv_in_16_nostats": lambda: conv_case(8, 64, 64, 16, 320),
    "conv_in_64_nostats": lambda: conv_case(8, 64, 64, 64, 320),
    "gemm_320_k64": lambda: conv_case(8, 64, 64, 64, 320, k=1),
    "conv3_l3_1280_res": lambda: conv_case(8, 8, 8, 1280, 1280, residual=True, stats=True),
    "conv3_l3_up_2560": lambda: conv_case(8, 8, 8, 2560, 1280, c1=1280, temb=True, stats=True),
    "conv3_down_l2": lambda: conv_case(8, 16, 16, 1280, 1280, stride=2, stats=True),
    "conv3_up_l0_960": lambda: conv_case(8, 64, 64, 960, 320, c1=320, residual=True, stats=True),
    "conv3_upsample_640": lambda: conv_case(8, 32, 32, 640, 640, up=True, stats=True),
    "gemm_proj_320": lambda: conv_case(8, 64, 64, 320, 320, k=1, residual=True),
    "gemm_qkv_320": lambda: conv_case(8, 64, 64, 320, 960, k=1),
    "gemm_geglu_320": lambda: conv_case(8, 64, 64, 320, 2560, k=1, geglu=True),
    "gemm_plain_2560_320": lambda: conv_case(8, 64, 64, 320, 2560, k=1),
    "gemm_ff2_1280": lambda: conv_case(8, 64, 64, 1280, 320, k=1, residual=True),
    "gemm_geglu_1280": lambda: conv_case(8, 16, 16, 1280, 10240, k=1, geglu=True),
    "gemm_qkv_640": lambda: conv_case(8, 32, 32, 640, 1920, k=1),
    "gemm_ln_qkv_640": lambda: ln_gemm_case(8192, 640, 1920),
    "gemm_ln_geglu_640": lambda: ln_gemm_case(8192, 640, 5120, geglu=True),
    "gemm_ln_qkv_1280": lambda: ln_gemm_case(2048, 1280, 3840),
    "gemm_ln_geglu_1280": lambda: ln_gemm_case(2048, 1280, 10240, geglu=True),
    "gemm_geglu_640": lambda: conv_case(8, 32, 32, 640, 5120, k=1, geglu=True),
    "gemm_ff2_2560": lambda: conv_case(8, 32, 32, 2560, 640, k=1, residual=True),
    "gemm_proj_640": lambda: conv_case(8, 32, 32, 640, 640, k=1, residual=True),
    "conv3_up_l1_1920": lambda: conv_case(8, 32, 32, 1920, 640, c1=640, residual=True, stats=True),
    "conv3_up_l1_1920_r8": lambda: conv_case(8, 32, 32, 1920, 640, c1=640, residual=True, stats=True, rows32=8),
    "conv3_up_l1_1280": lambda: conv_case(8, 32, 32, 1280, 640, c1=640, temb=True, stats=True),
    "conv3_up_l1_1280_r8": lambda: conv_case(8, 32, 32, 1280, 640, c1=640, temb=True, stats=True, rows32=8),
    "conv3_up_l1_960": lambda: conv_case(8, 32, 32, 960, 640, c1=320, temb=True, stats=True),
    "conv3_up_l1_960_r8": lambda: conv_case(8, 32, 32, 960, 640, c1=320, temb=True, stats=True, rows32=8),
    "conv3_l1_640_r8": lambda: conv_case(8, 32, 32, 640, 640, temb=True, stats=True, rows32=8),
    "conv3_l1_in_320_r8": lambda: conv_case(8, 32, 32, 320, 640, temb=True, stats=True, rows32=8),
    "conv3_upsample_320": lambda: conv_case(8, 32, 32, 640, 640, up=True, stats=True),
    "conv3_upsample_640_ph": lambda: conv_case(8, 32, 32, 640, 640, up=True, stats=True, phases=True),
    "conv3_upsample_1280": lambda: conv_case(8, 16, 16, 1280, 1280, up=True, stats=True),
    "conv3_upsample_1280_ph": lambda: conv_case(8, 16, 16, 1280, 1280, up=True, stats=True, phases=True),
    "conv3_upsample_l3": lambda: conv_case(8, 8, 8, 1280, 1280, up=True, stats=True),
    "conv3_upsample_l3_ph": lambda: conv_case(8, 8, 8, 1280, 1280, up=True, stats=True, phases=True),
    "conv3_l2_up_2560": lambda: conv_case(8, 16, 16, 2560, 1280, c1=1280, residual=True, stats=True),
    "gemm_short_l1_1920": lambda: conv_case(8, 32, 32, 1920, 640, k=1, c1=640, residual=True),
    "gemm_short_l1_1280": lambda: conv_case(8, 32, 32, 1280, 640, k=1, c1=640, residual=True),
    "gemm_short_l1_960": lambda: conv_case(8, 32, 32, 960, 640, k=1, c1=320, residual=True),
    "gemm_short_l1_in": lambda: conv_case(8, 32, 32, 320, 640, k=1, residual=True),
    "gemm_short_l0_960": lambda: conv_case(8, 64, 64, 960, 320, k=1, c1=320, residual=True),
    "gemm_short_l0_640": lambda: conv_case(8, 64, 64, 640, 320, k=1, c1=320, residual=True),
    "gemm_proj_1280_l2": lambda: conv_case(8, 16, 16, 1280, 1280, k=1, residual=True),
    "gemm_proj_1280_l3": lambda: conv_case(8, 8, 8, 1280, 1280, k=1, residual=True),
    "gemm_short_l3_2560": lambda: conv_case(8, 8, 8, 2560, 1280, k=1, c1=1280, residual=True),
    "gemm_short_l2_2560": lambda: conv_case(8, 16, 16, 2560, 1280, k=1, c1=1280, residual=True),
    "gemm_short_l2_1920": lambda: conv_case(8, 16, 16, 1920, 1280, k=1, c1=640, residual=True),
    "gemm_qkv_1280": lambda: conv_case(8, 16, 16, 1280, 3840, k=1),
    "gemm_qkv_1280_l3": lambda: conv_case(8, 8, 8, 1280, 3840, k=1),
    "gemm_geglu_1280_l3": lambda: conv_case(8, 8, 8, 1280, 10240, k=1, geglu=True),
    "gemm_ff2_5120_l3": lambda: conv_case(8, 8, 8, 5120, 1280, k=1, residual=True),
    "gemm_ff2_5120": lambda: conv_case(8, 16, 16, 5120, 1280, k=1, residual=True),
    "gemm_geglu_1280_l2": lambda: conv_case(8, 16, 16, 1280, 10240, k=1, geglu=True),
    "conv3_l3_2560": lambda: conv_case(8, 8, 8, 2560, 1280, c1=1280, residual=True, stats=True),
    "conv3_s2_l2": lambda: conv_case(8, 16, 16, 1280, 1280, stride=2, stats=True),
    "conv3_s2_l0": lambda: conv_case(8, 64, 64, 320, 320, stride=2, stats=True),
    "conv3_s2_l1": lambda: conv_case(8, 32, 32, 640, 640, stride=2, stats=True),
    "conv3_l1_in_320": lambda: conv_case(8, 32, 32, 320, 640, temb=True, stats=True),
    "conv3_l1_res_640": lambda: conv_case(8, 32, 32, 640, 640, residual=True, stats=True),
    "conv3_l2_in_640": lambda: conv_case(8, 16, 16, 640, 1280, temb=True, stats=True),
    "tin_l0": lambda: tin_case(8),
    "tin_l0_unfused": lambda: tin_case(8, fused=False),
    "tin_l0_m0": lambda: tin_case(8, mode=0),
    "tin_l0_noload": lambda: tin_case(8, mode=9),
    "tin_l0_nomfma": lambda: tin_case(8, mode=17),
    "ff_l0": lambda: ff_case(8 * 4096),
    "ff_l0_unfused": lambda: ff_case(8 * 4096, fused=False),
    "ff_po_l0": lambda: ff_case(8 * 4096, proj_out=True),
    "ff_po_l0_separate": lambda: ff_case(8 * 4096, fused=False, proj_out=True),
    "mm_8192": lambda: mm_case(8192, 8192, 8192),
    "mm_4096": lambda: mm_case(4096, 4096, 4096),
    "mm_geglu_320": lambda: mm_case(32768, 320, 2560),
    "mm_qkv_320": lambda: mm_case(32768, 320, 960),
    "mm_proj_320": lambda: mm_case(32768, 320, 320),
    "mm_ff2_1280": lambda: mm_case(32768, 1280, 320),
    "mm_geglu_640": lambda: mm_case(8192, 640, 5120),
    "mm_proj_640": lambda: mm_case(8192, 640, 640),
    "mm_ff2_2560": lambda: mm_case(8192, 2560, 640),
    "mm_geglu_1280": lambda: mm_case(2048, 1280, 10240),
    "mm_proj_1280": lambda: mm_case(2048, 1280, 1280),
    "mm_qkv_1280": lambda: mm_case(2048, 1280, 3840),
    "mm_ff2_5120": lambda: mm_case(2048, 5120, 1280),
    "mm_proj_1280_l3": lambda: mm_case(512, 1280, 1280),
    "mm_qkv_1280_l3": lambda: mm_case(512, 1280, 3840),
    "mm_geglu_1280_l3": lambda: mm_case(512, 1280, 10240),
    "mm_conv_l0_320": lambda: mm_case(32768, 2880, 320),
    "mm_conv_l1_640": lambda: mm_case(8192, 5760, 640),
    "mm_conv_l2_1280": lambda: mm_case(2048, 11520, 1280),
    "mm_conv_l3_1280": lambda: mm_case(512, 11520, 1280),
    "attn_4096_d40": lambda: attn_case(8, 4096, 320),
    "attn_c5_2048_d40": lambda: attn_case(16, 2048, 320),
    "attn_c5_2048_d40_fp8": lambda: attn_case(16, 2048, 320, fp8=True),
    "attn_c5_2048_d40_fp8pv": lambda: attn_case(16, 2048, 320, fp8=True, scaled=False),
    "attn_4096_d40_fp8": lambda: attn_case(8, 4096, 320, fp8=True),
    "attn_4096_d40_qs2": lambda: attn_case(8, 4096, 320, qs2=1),
    "attn_4096_d40_noskew": lambda: attn_case(8, 4096, 320, skew=1),
    "attn_1024_d80_nopair": lambda: attn_case(8, 1024, 640, pair=False),
    "attn_1024_d80": lambda: attn_case(8, 1024, 640),
    "attn_1024_d80_kt128": lambda: attn_case(8, 1024, 640, pair=2),
    "attn_1024_d80_kt128p": lambda: attn_case(8, 1024, 640, pair=3),
    "attn_4096_d40_skew": lambda: attn_case(8, 4096, 320, skew=2),
    "attn_4096_d40_occ1": lambda: attn_case(8, 4096, 320, skew=3),
    "attn_1024_d80_noskew": lambda: attn_case(8, 1024, 640, skew=1),
    "attn_1024_d80_skew": lambda: attn_case(8, 1024, 640, skew=2),
    "attn_c5_2048_d40_noskew": lambda: attn_case(16, 2048, 320, skew=1),
    "attn_c5_2048_d40_skew": lambda: attn_case(16, 2048, 320, skew=2),
    "attn_4096_d40_pipe": lambda: attn_case(8, 4096, 320, qs2=2),
    "attn_4096_d40_noil": lambda: attn_case(8, 4096, 320, il=False),
    "attn_4096_d40_kt64": lambda: attn_case(8, 4096, 320, il=2),
    "attn_c5_2048_d40_kt64": lambda: attn_case(16, 2048, 320, il=2),
    "attn_4096_d40_kt256": lambda: attn_case(8, 4096, 320, il=3),
    "attn_c5_2048_d40_kt256": lambda: attn_case(16, 2048, 320, il=3),
    "attn_c5_2048_d40_noil": lambda: attn_case(16, 2048, 320, il=False),
    "attn_c5_2048_d40_qs2": lambda: attn_case(16, 2048, 320, qs2=1),
    "attn_c5_2048_d40_pipe": lambda: attn_case(16, 2048, 320, qs2=2),
    "attn_c5_2048_d40_fp8_qs2": lambda: attn_case(16, 2048, 320, fp8=True, qs2=1),
    "attn_4096_d40_fma": lambda: attn_case(8, 4096, 320, maxcol=0),
    "attn_4096_d40_mc16": lambda: attn_case(8, 4096, 320, maxcol=1),
    "attn_1024_d80_fma": lambda: attn_case(8, 1024, 640, maxcol=0),
    "attn_4096_d40_legacy": lambda: attn_case(8, 4096, 320, legacy=True),
    "attn_1024_d80_legacy": lambda: attn_case(8, 1024, 640, legacy=True),
    "attn_256_d160_legacy": lambda: attn_case(8, 256, 1280, legacy=True),
    "attn_1024_d80": lambda: attn_case(8, 1024, 640),
    "attn_1024_d80_kt128": lambda: attn_case(8, 1024, 640, pair=2),
    "attn_1024_d80_kt128p": lambda: attn_case(8, 1024, 640, pair=3),
    "attn_1024_d80_x16": lambda: attn_case(8, 1024, 640, d80=False),
    "attn_4096_d40_w8": lambda: attn_case(8, 4096, 320, waves=8),
    "attn_1024_d80_w8": lambda: attn_case(8, 1024, 640, waves=8),
    "attn_4096_d40_w4": lambda: attn_case(8, 4096, 320, waves=4),
    "attn_256_d160": lambda: attn_case(8, 256, 1280),
    "colsum_l0_320": lambda: colsum_case(65536, 320),
    "colsum_l0_320_seg16": lambda: colsum_case(65536, 320, 16),
    "colsum_geglu_2560": lambda: colsum_case(65536, 2560, geglu=True),
    "colsum_l2_1280": lambda: colsum_case(4096, 1280),
    "gnb_l0_320": lambda: gn_bwd_case(16, 4096, 320),
    "gnb_l0_960_noadd": lambda: gn_bwd_case(16, 4096, 960, add=False),
    "gnb_l2_1280": lambda: gn_bwd_case(16, 256, 1280),
    "wgrad_l0_320": lambda: wgrad_case(16, 64, 64, 320, 320),
    "wgrad_l1_640": lambda: wgrad_case(16, 32, 32, 640, 640),
    "wgrad_l2_1280": lambda: wgrad_case(16, 16, 16, 1280, 1280),
    "wgrad_l3_1280": lambda: wgrad_case(16, 8, 8, 1280, 1280),
    "wgrad_up_960": lambda: wgrad_case(16, 64, 64, 960, 320),
    "wgrad_geglu_320": lambda: wgrad_case(16, 64, 64, 320, 2560, k=1, geglu=True),
    "wgrad_ff2_1280": lambda: wgrad_case(16, 64, 64, 1280, 320, k=1),
    "wgrad_proj_320": lambda: wgrad_case(16, 64, 64, 320, 320, k=1),
    "wgrad_qkv_320": lambda: wgrad_case(16, 64, 64, 320, 960, k=1),
    "wgrad_l0_320_gen": lambda: wgrad_case(16, 64, 64, 320, 320, fast=False),
    "wgrad_l1_640_gen": lambda: wgrad_case(16, 32, 32, 640, 640, fast=False),
    "wgrad_l2_1280_gen": lambda: wgrad_case(16, 16, 16, 1280, 1280, fast=False),
    "wgrad_l3_1280_gen": lambda: wgrad_case(16, 8, 8, 1280, 1280, fast=False),
    "wgrad_up_960_gen": lambda: wgrad_case(16, 64, 64, 960, 320, fast=False),
    "wgrad_geglu_320_gen": lambda: wgrad_case(16, 64, 64, 320, 2560, k=1, geglu=True, fast=False),
    "wgrad_ff2_1280_gen": lambda: wgrad_case(16, 64, 64, 1280, 320, k=1, fast=False),
    "wgrad_proj_320_gen": lambda: wgrad_case(16, 64, 64, 320, 320, k=1, fast=False),
    "wgrad_qkv_320_gen": lambda: wgrad_case(16, 64, 64, 320, 960, k=1, fast=False),
    "wgrad_l0_320_ns5": lambda: wgrad_case(16, 64, 64, 320, 320, ring=2),
    "wgrad_l1_640_ns5": lambda: wgrad_case(16, 32, 32, 640, 640, ring=2),
    "wgrad_l2_1280_ns5": lambda: wgrad_case(16, 16, 16, 1280, 1280, ring=2),
    "wgrad_up_960_ns5": lambda: wgrad_case(16, 64, 64, 960, 320, ring=2),
    "wgrad_geglu_320_ns5": lambda: wgrad_case(16, 64, 64, 320, 2560, k=1, geglu=True, ring=2),
    "wgrad_qkv_320_ns5": lambda: wgrad_case(16, 64, 64, 320, 960, k=1, ring=2),
    "wgrad_l0_320_r1": lambda: wgrad_case(16, 64, 64, 320, 320, r3=False),
    "wgrad_l2_1280_r1": lambda: wgrad_case(16, 16, 16, 1280, 1280, r3=False),
    "wgrad_l3_1280_r1": lambda: wgrad_case(16, 8, 8, 1280, 1280, r3=False),
    "wgrad_up_960_r1": lambda: wgrad_case(16, 64, 64, 960, 320, r3=False),
    "wgrad_l0_320_old": lambda: wgrad_case(16, 64, 64, 320, 320, ring=False),
    "wgrad_l1_640_old": lambda: wgrad_case(16, 32, 32, 640, 640, ring=False),
    "wgrad_l2_1280_old": lambda: wgrad_case(16, 16, 16, 1280, 1280, ring=False),
    "wgrad_up_960_old": lambda: wgrad_case(16, 64, 64, 960, 320, ring=False),
    "wgrad_geglu_320_old": lambda: wgrad_case(16, 64, 64, 320, 2560, k=1, geglu=True, ring=False),
    "wgrad_qkv_320_old": lambda: wgrad_case(16, 64, 64, 320, 960, k=1, ring=False),
    "attn_bwd_4096_d40": lambda: attn_bwd_case(16, 4096, 320),
    "attn_bwd_4096_d40_old": lambda: attn_bwd_case(16, 4096, 320, new=False),
    "attn_bwd_1024_d80": lambda: attn_bwd_case(16, 1024, 640),
    "gn_l0_fused": lambda: gn_case(8, 4096, 320, True),
    "copy_l0": lambda: copy_case(8 * 4096 * 320),
    "gn_l0_unfused": lambda: gn_case(8, 4096, 320, False),
    "gn_l1_fused": lambda: gn_case(8, 1024, 640, True),
    "gn_l2_fused": lambda: gn_case(8, 256, 1280, True),
    "gn_l3_fused": lambda: gn_case(8, 64, 1280, True),
    "gn_up0_fused": lambda: gn_case(8, 4096, 960, True),
    "ln_l0": lambda: ln_case(32768, 320),
    "tail_l0": lambda: tail_case(8),
    "tail_l0_eps": lambda: tail_case(8, ddim=False),
    "tail_l0_unfused": lambda: tail_case(8, fused=False),
    "temb_mlp": lambda: temb_case(8),
    "temb_mlp_unfused": lambda: temb_case(8, fused=False),
    "panoptic_k128_512": lambda: panoptic_case(8, 128, 512, 512),
    "panoptic_k30_512": lambda: panoptic_case(8, 30, 512, 512),
    "ln_l1": lambda: ln_case(8192, 640),
    "ln_l2": lambda: ln_case(2048, 1280),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--plans", nargs="*", default=["auto"],
                    help="conv tile plans to compare: 'auto' or 'bm,bn,ksplit[,stages]' (e.g. 256,160,1 or 128,160,8,4)")
    ap.add_argument("--groups", nargs="*", type=int, default=[8], help="conv tile-raster groups to compare")
    ap.add_argument("--lib", default=None, help="load this library build instead (e.g. exp/libabl1.so)")
    ap.add_argument("--epi", type=int, default=0, help="conv epilogue mode (ldm_conv2d_set_epilogue)")
    ap.add_argument("--ars", nargs="*", type=int, default=[0],
                    help="short-K 1x1 GEMM modes to compare (ldm_conv2d_set_ars: 0 planner, 1 never, 2 when legal)")
    ap.add_argument("--wide", nargs="*", type=int, default=[0],
                    help="wide-tile persistent 1x1 GEMM modes (ldm_conv2d_set_wide: 0 planner, 1 never, 2 BM 256, 3 BM 128)")
    ap.add_argument("--ring", nargs="*", type=int, default=[0],
                    help="deep-ring 1x1 GEMM modes to compare (ldm_conv2d_set_ring: 0 planner, 1 never, 2 when legal)")
    ap.add_argument("--rsplit", type=int, default=0, help="ldm_conv2d_set_ring_split for every case")
    ap.add_argument("--fa", nargs="*", type=int, default=[1],
                    help="tile-kernel fast operand addressing to compare (ldm_conv2d_set_fast_addressing: 0 off, 1 on)")
    ap.add_argument("--skcols", nargs="*", type=int, default=[0],
                    help="split-K reduction tile widths to compare (ldm_conv2d_set_splitk_cols: 0 planner, 64, 128)")
    ap.add_argument("--graph", action="store_true",
                    help="time each case as a captured HIP graph of --iters launches (device time: the eager loop "
                         "is host-bound below ~20 us per launch)")
    ap.add_argument("--batch", type=int, default=8, help="B of the conv / GEMM cases (config 2: 1)")
    a = ap.parse_args()
    global BATCH
    BATCH = a.batch
    if a.lib:
        K.load_library(os.path.abspath(a.lib))
    K.set_conv_epilogue(a.epi)
    K.set_conv_ring_split(a.rsplit)
    names = a.only or list(CASES)
    built = {}
    for n in names:
        if not n.startswith(("conv", "gemm")) or n.startswith("wgrad"):
            built[n] = CASES[n]()
            continue
        for pl in a.plans:
            for gm in a.groups:
                for am, sk, wd, rg, fa in [(x, y, z, r, f) for x in a.ars for y in a.skcols for z in a.wide for r in a.ring
                                           for f in a.fa]:
                    run, fl, nb = CASES[n]()
                    f = [0, 0, 1, 0] if pl == "auto" else [int(v) for v in pl.split(",")] + [0]
                    bm, bn, ks, st = f[:4]

                    def run_pl(run=run, bm=bm, bn=bn, ks=ks, st=st, gm=gm, am=am, sk=sk, wd=wd, rg=rg, fa=fa):
                        K.set_conv_fast_addressing(fa)
                        K.set_conv_splitk_cols(sk)
                        K.force_conv_plan(bm, bn, ks)
                        K.force_conv_stages(st)
                        K.set_conv_raster_group(gm)
                        K.set_conv_ars(am)
                        K.set_conv_wide(wd)
                        K.set_conv_ring(rg)
                        return run()
                    name = n if pl == "auto" else f"{n}@{pl}"
                    name = name if len(a.groups) == 1 else f"{name}/g{gm}"
                    name = name if len(a.ars) == 1 else f"{name}/ars{am}"
                    name = name if len(a.skcols) == 1 else f"{name}/skc{sk}"
                    name = name if len(a.wide) == 1 else f"{name}/w{wd}"
                    name = name if len(a.ring) == 1 else f"{name}/ring{rg}"
                    built[name if len(a.fa) == 1 else f"{name}/fa{fa}"] = (run_pl, fl, nb)
    for n, (run, _, _) in built.items():
        run()
    torch.cuda.synchronize()
    graphs = {}
    if a.graph:
        for n, (run, _, _) in built.items():
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                run()
            torch.cuda.current_stream().wait_stream(side)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                for _ in range(a.iters):
                    run()
            graphs[n] = gr
        torch.cuda.synchronize()
    res = {n: [] for n in built}
    for rnd in range(3):
        for n, (run, _, _) in built.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if a.graph:
                graphs[n].replay()
            else:
                for _ in range(a.iters):
                    run()
            e1.record()
            torch.cuda.synchronize()
            res[n].append(e0.elapsed_time(e1) / a.iters)
    for n, (run, flops, nbytes) in built.items():
        ms = min(res[n])
        perf = f"{flops / ms / 1e9:8.1f} TF/s" if flops else f"{nbytes / ms / 1e6:8.1f} GB/s"
        print(f"{n:22s} {ms * 1e3:9.1f} us  {perf}", flush=True)


if __name__ == "__main__":
    main()
