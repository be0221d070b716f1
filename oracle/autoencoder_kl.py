"""diffusers AutoencoderKL encoder (GeneralVAEImage.encode, ldmseg/models/vae.py:36-39, with the
decoder removed as in tools/main_ldm.py:139) — torch fp32 functional restatement (test
infrastructure only, see oracle/__init__.py).

PARITY UNPINNED: the arithmetic lives in the un-vendored ``diffusers`` package (version not
pinned by the reference) and no reference file holds an output of it.  This
restates the published SD-1.x VAE encoder: conv_in; DownEncoderBlock2D x4 (2 ResnetBlock2D each,
GroupNorm(32, eps 1e-6) + SiLU, no time embedding; Downsample2D = F.pad (0,1,0,1) + 3x3 stride-2
conv without padding, on all but the last block); UNetMidBlock2D (resnet, single-head attention
with GroupNorm, q/k/v/out linears with bias, softmax(q k^T / sqrt(C)), residual; resnet);
GroupNorm + SiLU + conv_out (2 x latent channels); quant_conv 1x1.  latent_dist.mode() = mean.
"""
import torch
import torch.nn.functional as F


GROUPS = [32]   # norm_num_groups of the model under test (set by encode_moments)


def _gn(sd, pre, x, eps=1e-6):
    return F.group_norm(x, GROUPS[0], sd[pre + ".weight"], sd[pre + ".bias"], eps)


def _conv(sd, pre, x, stride=1, padding=1):
    return F.conv2d(x, sd[pre + ".weight"], sd[pre + ".bias"], stride=stride, padding=padding)


def _resnet(sd, pre, x):
    h = _conv(sd, pre + ".conv1", F.silu(_gn(sd, pre + ".norm1", x)))
    h = _conv(sd, pre + ".conv2", F.silu(_gn(sd, pre + ".norm2", h)))
    sc = _conv(sd, pre + ".conv_shortcut", x, padding=0) if pre + ".conv_shortcut.weight" in sd else x
    return sc + h


def _attention(sd, pre, x):
    B, C, H, W = x.shape
    h = _gn(sd, pre + ".group_norm", x).view(B, C, H * W).transpose(1, 2)        # [B, N, C]
    lin = lambda n, t: F.linear(t, sd[f"{pre}.{n}.weight"], sd[f"{pre}.{n}.bias"])  # noqa: E731
    q, k, v = lin("to_q", h), lin("to_k", h), lin("to_v", h)
    p = torch.softmax(q @ k.transpose(1, 2) * C ** -0.5, dim=-1)
    o = lin("to_out.0", p @ v)
    return o.transpose(1, 2).reshape(B, C, H, W) + x


def encode_moments(sd, x, n_blocks=4, layers_per_block=2, groups=32):
    """x [B, 3, H, W] fp32 in [-1, 1] -> moments [B, 2L, H/8, W/8] (after quant_conv)."""
    GROUPS[0] = groups
    h = _conv(sd, "encoder.conv_in", x)
    for i in range(n_blocks):
        for j in range(layers_per_block):
            h = _resnet(sd, f"encoder.down_blocks.{i}.resnets.{j}", h)
        if f"encoder.down_blocks.{i}.downsamplers.0.conv.weight" in sd:
            h = _conv(sd, f"encoder.down_blocks.{i}.downsamplers.0.conv", F.pad(h, (0, 1, 0, 1)), stride=2, padding=0)
    h = _resnet(sd, "encoder.mid_block.resnets.0", h)
    h = _attention(sd, "encoder.mid_block.attentions.0", h)
    h = _resnet(sd, "encoder.mid_block.resnets.1", h)
    h = _conv(sd, "encoder.conv_out", F.silu(_gn(sd, "encoder.conv_norm_out", h)))
    return _conv(sd, "quant_conv", h, padding=0)
