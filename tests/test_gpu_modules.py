"""Module-level parity of the drop-in modules on an MI355X.

* GeneralVAESeg  vs the REFERENCE's golden outputs (tests/golden/vae.npz), fp32 1e-4 rel.
* UNet           vs the CPU oracle (oracle/unet.py; parity with diffusers unpinned), fp32 at
                 the north-star tolerance 1e-3 rel, bf16 5e-2 rel.
* Denoising loop (TrainerDiffusion.sample semantics) vs the oracle loop.
"""
import numpy as np
import pytest
import torch

from golden_utils import VAE_CONFIGS, load, vae_state_dict
from ldmseg.models import GeneralVAESeg, UNet
from ldmseg.schedulers import DDIMNoiseScheduler
from oracle import ddim as oddim
from oracle import unet as ounet

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


# ------------------------------------------------------------------------------ VAE
@pytest.mark.parametrize("cname", list(VAE_CONFIGS))
def test_vae_matches_reference_golden(cname):
    z = load("vae.npz")
    v = GeneralVAESeg(**VAE_CONFIGS[cname])
    v.load_state_dict(vae_state_dict(z, cname), strict=True)
    v = v.to(DEV).eval()
    x = torch.from_numpy(z[f"{cname}__x"]).to(DEV)
    post = v.encode(x).latent_dist
    for name, t in (("moments", post.parameters), ("mean", post.mean), ("logvar", post.logvar), ("std", post.std)):
        assert rel_err(t, torch.from_numpy(z[f"{cname}__{name}"])) < 1e-4, name
    dec_i = v.decode(post.mode(), interpolate=True)
    dec_n = v.decode(post.mode(), interpolate=False)
    assert rel_err(dec_i, torch.from_numpy(z[f"{cname}__dec_interp"])) < 1e-4
    assert rel_err(dec_n, torch.from_numpy(z[f"{cname}__dec_nointerp"])) < 1e-4
    fwd = v(x, sample_posterior=False).sample
    assert rel_err(fwd, torch.from_numpy(z[f"{cname}__forward"])) < 1e-4
    # bf16 path against the same reference outputs
    vb = v.to(torch.bfloat16)
    db = vb.decode(vb.encode(x.bfloat16()).latent_dist.mode(), interpolate=True)
    assert rel_err(db, torch.from_numpy(z[f"{cname}__dec_interp"])) < 5e-2


# ------------------------------------------------------------------------------ UNet
SMALL = dict(block_out_channels=(64, 128, 128, 128), cross_attention_dim=None)


def _unet(cfg, seed=0, in_ch=8, cond=0):
    torch.manual_seed(seed)
    u = UNet(**cfg)
    # non-trivial norm affines / biases (default init makes GN gamma = 1, beta = 0)
    with torch.no_grad():
        for n, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    u.modify_encoder(in_channels=in_ch, init_mode_seg="copy", init_mode_image="random", cond_channels=cond,
                     init_mode_cond="random")
    return u.eval()


def _oracle_cfg(u):
    return dict(u.config)


@pytest.mark.parametrize("B,H,cond", [(2, 32, 0), (1, 24, 4)])
def test_unet_small_fp32_matches_oracle(B, H, cond):
    u = _unet(SMALL, cond=cond)
    sd = {k: v.detach().clone() for k, v in u.state_dict().items()}
    torch.manual_seed(1)
    x = torch.randn(B, 8 + cond, H, H)
    t = torch.tensor(731)
    with torch.no_grad():
        ref = ounet.forward(sd, _oracle_cfg(u), x, t)
    ud = u.to(DEV)
    out = ud(x.to(DEV), t.to(DEV)).sample
    assert out.shape == ref.shape and out.dtype == torch.float32
    assert rel_err(out, ref) < 1e-3
    # per-frame timesteps [B]
    tb = torch.tensor([999, 19][:B])
    with torch.no_grad():
        ref_b = ounet.forward(sd, _oracle_cfg(u), x, tb)
    assert rel_err(ud(x.to(DEV), tb.to(DEV)).sample, ref_b) < 1e-3


def test_unet_small_with_cross_attention():
    cfg = dict(block_out_channels=(64, 128, 128, 128), cross_attention_dim=96)
    torch.manual_seed(0)
    u = UNet(**cfg).eval()
    sd = {k: v.detach().clone() for k, v in u.state_dict().items()}
    x = torch.randn(2, 4, 16, 16)
    ehs = torch.randn(2, 77, 96)
    with torch.no_grad():
        ref = ounet.forward(sd, _oracle_cfg(u), x, torch.tensor(500), ehs)
    out = u.to(DEV)(x.to(DEV), torch.tensor(500, device=DEV), ehs.to(DEV)).sample
    assert rel_err(out, ref) < 1e-3


def test_unet_sd14_fullsize_fp32_matches_oracle():
    """The real SD-1.4 graph (815.5 M params, cross-attn removed, 8-ch conv_in) at 64x64, B=1."""
    torch.manual_seed(0)
    u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero")
    u.eval()
    sd = u.state_dict()
    x = torch.randn(1, 8, 64, 64)
    with torch.no_grad():
        torch.set_num_threads(16)
        ref = ounet.forward(sd, _oracle_cfg(u), x, torch.tensor(979))
    ud = u.to(DEV)
    out = ud(x.to(DEV), torch.tensor(979, device=DEV)).sample
    assert rel_err(out, ref) < 1e-3
    ub = ud.to(torch.bfloat16)
    outb = ub(x.to(DEV, torch.bfloat16), torch.tensor(979, device=DEV)).sample
    assert outb.dtype == torch.bfloat16
    assert rel_err(outb, ref) < 5e-2


def test_unet_bf16_small_matches_oracle():
    u = _unet(SMALL)
    sd = {k: v.detach().clone() for k, v in u.state_dict().items()}
    x = torch.randn(2, 8, 32, 32)
    with torch.no_grad():
        ref = ounet.forward(sd, _oracle_cfg(u), x, torch.tensor(100))
    ub = u.to(DEV, torch.bfloat16)
    out = ub(x.to(DEV, torch.bfloat16), torch.tensor(100, device=DEV)).sample
    assert rel_err(out, ref) < 5e-2


# ------------------------------------------------------------------------------ sampler
def test_denoise_loop_matches_oracle():
    from ldmseg.pipelines import sample_latents
    u = _unet(SMALL, cond=4)
    sd = {k: v.detach().clone() for k, v in u.state_dict().items()}
    sched_kw = dict(prediction_type="epsilon", beta_schedule="scaled_linear", beta_start=0.00085, beta_end=0.012,
                    clip_sample=False, set_alpha_to_one=False)
    s = DDIMNoiseScheduler(**sched_kw, device=DEV, verbose=False)
    torch.manual_seed(3)
    rgb = torch.randn(2, 4, 16, 16)
    steps = 5
    lat = sample_latents(u.to(DEV), s, rgb.to(DEV), num_inference_steps=steps, seed=0, self_condition=True)
    # oracle loop (trainers_ldm_cond.py:1091-1166)
    _, ac, final = oddim.tables("scaled_linear", 1000, 0.00085, 0.012, False)
    lat_o = torch.randn((2, 4, 16, 16), generator=torch.Generator().manual_seed(0))
    cond = torch.zeros_like(rgb)
    ts = oddim.inference_timesteps(1000, steps)
    with torch.no_grad():
        for i, t in enumerate(ts):
            eps = ounet.forward(sd, _oracle_cfg(u), torch.cat([lat_o, rgb, cond], 1), torch.tensor(int(t)))
            _, cond = oddim.step(ac, final, 1000, steps, eps, int(t), lat_o)
            prev, x0 = oddim.step(ac, final, 1000, steps, eps, int(t), lat_o)
            lat_o = x0 if i == len(ts) - 1 else prev
    assert rel_err(lat, lat_o) < 1e-3
    # the same loop replayed through one captured HIP graph per step gives identical results
    lat_g = sample_latents(u, s, rgb.to(DEV), num_inference_steps=steps, seed=0, self_condition=True, use_graph=True)
    assert torch.equal(lat_g, lat)


def test_unet_sd14_headline_batch_matches_single_frames():
    """The headline workload's B = 8 bf16 forward (the exact plans of the benchmarked step: unsplit
    64x64 / 32x32 tiles, fused split-K GroupNorm at the deep levels, the interleaved two-subtile
    attention) against the same UNet run frame by frame at B = 1 (a different plan for nearly every
    launch: split-K everywhere, split-KV attention), whose arithmetic test_unet_sd14_fullsize_fp32_matches_oracle
    pins to the oracle.  Frames are independent (T folded into the batch), so every frame of the B = 8
    output must agree with its B = 1 run within the bf16 bar (5e-2, as bf16 against the oracle)."""
    torch.manual_seed(0)
    u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="random")
    with torch.no_grad():
        for _, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    u = u.eval().to(DEV, torch.bfloat16)
    x = torch.randn(8, 8, 64, 64, device=DEV).to(torch.bfloat16)
    t = torch.tensor(613, device=DEV)
    y8 = u(x, t).sample
    assert torch.isfinite(y8.float()).all()
    for i in range(8):
        y1 = u(x[i:i + 1], t).sample
        assert rel_err(y8[i:i + 1], y1) < 5e-2, i      # (the bf16-vs-oracle bar)
