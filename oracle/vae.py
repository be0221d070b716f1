"""GeneralVAESeg encode/decode — torch fp32 CPU restatement (test infrastructure only).

Follows ldmseg/models/vae.py:
  encoder stack  define_encoder :175-245 (resize_input=False, num_mid_blocks=0)
  decoder stack  define_decoder :124-173
  posterior      DiagonalGaussianDistribution :371-425 (split, clamp logvar [-30,20], std)
  decode         :268-272 (bilinear x interpolation_factor, align_corners=False)
  LayerNorm2d    :310-323 (normalise over C, eps 1e-6)
Weights come from a state_dict with the reference's nn.Sequential keys
(encoder.<i>.weight, decoder.<i>.weight).
"""
import torch
import torch.nn.functional as F


def encoder_spec(in_channels, block_out_channels, int_channels, latent_channels, num_latents):
    """List of (kind, args) mirroring the nn.Sequential indices of define_encoder."""
    spec = [("conv", dict(stride=1)), ("silu", {})]
    for _ in range(len(block_out_channels) - 1):
        spec += [("conv", dict(stride=1)), ("conv", dict(stride=2)), ("silu", {})]
    spec += [("conv", dict(stride=1)), ("identity", {}), ("gn", dict(eps=1e-6)), ("silu", {}),
             ("conv", dict(stride=1))]
    return spec


def decoder_spec(num_upscalers):
    spec = [("conv", dict(stride=1)), ("identity", {})]
    for _ in range(num_upscalers):
        spec += [("convT", {}), ("ln2d", dict(eps=1e-6)), ("silu", {})]
    spec += [("gn", dict(eps=1e-5)), ("silu", {}), ("conv", dict(stride=1))]
    return spec


def run_sequential(x, spec, sd, prefix, groups):
    for i, (kind, a) in enumerate(spec):
        w = sd.get(f"{prefix}.{i}.weight")
        b = sd.get(f"{prefix}.{i}.bias")
        if kind == "conv":
            x = F.conv2d(x, w, b, stride=a["stride"], padding=w.shape[-1] // 2)
        elif kind == "convT":
            x = F.conv_transpose2d(x, w, b, stride=2)
        elif kind == "silu":
            x = F.silu(x)
        elif kind == "gn":
            x = F.group_norm(x, groups, w, b, eps=a["eps"])
        elif kind == "ln2d":
            u = x.mean(1, keepdim=True)
            s = (x - u).pow(2).mean(1, keepdim=True)
            x = (x - u) / torch.sqrt(s + a["eps"])
            x = w[:, None, None] * x + b[:, None, None]
    return x


def encode(sd, x, cfg):
    """Returns (moments, mean, logvar, std) of the gaussian posterior."""
    spec = encoder_spec(cfg["in_channels"], cfg["block_out_channels"], cfg["int_channels"],
                        cfg["latent_channels"], cfg.get("num_latents", 2))
    moments = run_sequential(x, spec, sd, "encoder", cfg["norm_num_groups"])
    p = moments.clamp(-5.0, 5.0) if cfg.get("clamp_output", False) else moments
    mean, logvar = torch.chunk(p, 2, dim=1)
    act = cfg.get("act_fn", "none")
    if act == "tanh":
        mean = torch.tanh(mean)
    elif act == "sigmoid":
        mean = 2 * torch.sigmoid(mean) - 1
    elif act == "clip":
        mean = mean.clamp(-1, 1)
    logvar = logvar.clamp(-30.0, 20.0)
    return moments, mean, logvar, torch.exp(0.5 * logvar)


def decode(sd, z, cfg, interpolate=True):
    nu = cfg.get("num_upscalers", 1)
    x = run_sequential(z, decoder_spec(nu), sd, "decoder", cfg["norm_num_groups"])
    factor = 2 ** (len(cfg["block_out_channels"]) - 1) // (2 ** nu)
    if interpolate:
        x = F.interpolate(x, scale_factor=factor, mode="bilinear", align_corners=False)
    return x
