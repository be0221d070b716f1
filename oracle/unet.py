"""SD-1.x UNet2DConditionModel forward — torch fp32 CPU restatement (test infrastructure only).

PARITY UNPINNED w.r.t. the reference: ldmseg/models/unet.py:24 subclasses the
un-vendored diffusers.UNet2DConditionModel, so no reference output
exists in this container.  This module restates the graph the reference configures
(reference orchestration ldmseg/models/unet.py:281-436) from the
public diffusers block semantics, operating on a state_dict with diffusers key names:

  time_proj       sinusoid(320, flip_sin_to_cos=True, shift 0)          unet.py:305
  time_embedding  linear_1 -> SiLU -> linear_2                          unet.py:307
  conv_in         3x3                                                    unet.py:357
  down/mid/up     ResnetBlock2D / Transformer2DModel / Down/Upsample2D   unet.py:361-425
  out             GN(eps 1e-5) -> SiLU -> conv_out 3x3                   unet.py:428-431

It is the checker for the HIP path at reduced widths and the CPU baseline in bench.py.
"""
import math

import torch
import torch.nn.functional as F


def timestep_proj(t, dim=320, flip_sin_to_cos=True, shift=0.0, max_period=10000):
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32) / (half - shift)
    emb = t[:, None].float() * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


def _lin(sd, p, x):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))


def _conv(sd, p, x, stride=1):
    w = sd[p + ".weight"]
    return F.conv2d(x, w, sd.get(p + ".bias"), stride=stride, padding=w.shape[-1] // 2)


def resnet(sd, p, x, temb, groups, eps):
    h = F.silu(F.group_norm(x, groups, sd[p + ".norm1.weight"], sd[p + ".norm1.bias"], eps))
    h = _conv(sd, p + ".conv1", h)
    h = h + _lin(sd, p + ".time_emb_proj", F.silu(temb))[:, :, None, None]
    h = F.silu(F.group_norm(h, groups, sd[p + ".norm2.weight"], sd[p + ".norm2.bias"], eps))
    h = _conv(sd, p + ".conv2", h)
    if p + ".conv_shortcut.weight" in sd:
        x = _conv(sd, p + ".conv_shortcut", x)
    return x + h


def attention(sd, p, x, ctx, heads):
    q = _lin(sd, p + ".to_q", x)
    k = _lin(sd, p + ".to_k", ctx)
    v = _lin(sd, p + ".to_v", ctx)
    B, N, C = q.shape
    d = C // heads

    def split(t):
        return t.reshape(B, t.shape[1], heads, d).permute(0, 2, 1, 3)

    s = torch.matmul(split(q), split(k).transpose(-1, -2)) * (d ** -0.5)
    o = torch.matmul(s.softmax(dim=-1), split(v))
    o = o.permute(0, 2, 1, 3).reshape(B, N, C)
    return _lin(sd, p + ".to_out.0", o)


def transformer(sd, p, x, ehs, groups, heads):
    B, C, H, W = x.shape
    res = x
    h = F.group_norm(x, groups, sd[p + ".norm.weight"], sd[p + ".norm.bias"], 1e-6)
    h = _conv(sd, p + ".proj_in", h)
    h = h.permute(0, 2, 3, 1).reshape(B, H * W, C)
    tb = p + ".transformer_blocks.0"
    n = F.layer_norm(h, (C,), sd[tb + ".norm1.weight"], sd[tb + ".norm1.bias"], 1e-5)
    h = attention(sd, tb + ".attn1", n, n, heads) + h
    if tb + ".attn2.to_q.weight" in sd and ehs is not None:
        n = F.layer_norm(h, (C,), sd[tb + ".norm2.weight"], sd[tb + ".norm2.bias"], 1e-5)
        h = attention(sd, tb + ".attn2", n, ehs, heads) + h
    n = F.layer_norm(h, (C,), sd[tb + ".norm3.weight"], sd[tb + ".norm3.bias"], 1e-5)
    hid, gate = _lin(sd, tb + ".ff.net.0.proj", n).chunk(2, dim=-1)
    h = _lin(sd, tb + ".ff.net.2", hid * F.gelu(gate)) + h
    h = h.reshape(B, H, W, C).permute(0, 3, 1, 2)
    return _conv(sd, p + ".proj_out", h) + res


def forward(sd, cfg, sample, timesteps, encoder_hidden_states=None):
    """sample [B,Cin,H,W] fp32, timesteps [B] (or scalar) -> noise prediction [B,4,H,W]."""
    G = cfg.get("norm_num_groups", 32)
    eps = cfg.get("norm_eps", 1e-5)
    heads = cfg.get("attention_head_dim", 8)
    boc = list(cfg["block_out_channels"])
    lpb = cfg.get("layers_per_block", 2)
    down_types = cfg["down_block_types"]
    up_types = cfg["up_block_types"]
    B = sample.shape[0]
    t = torch.as_tensor(timesteps).reshape(-1).expand(B)
    temb = timestep_proj(t, boc[0], cfg.get("flip_sin_to_cos", True), cfg.get("freq_shift", 0))
    temb = _lin(sd, "time_embedding.linear_2", F.silu(_lin(sd, "time_embedding.linear_1", temb)))

    x = _conv(sd, "conv_in", sample)
    skips = [x]
    for i, bt in enumerate(down_types):
        for j in range(lpb):
            x = resnet(sd, f"down_blocks.{i}.resnets.{j}", x, temb, G, eps)
            if "CrossAttn" in bt:
                x = transformer(sd, f"down_blocks.{i}.attentions.{j}", x, encoder_hidden_states, G, heads)
            skips.append(x)
        if i < len(down_types) - 1:
            x = _conv(sd, f"down_blocks.{i}.downsamplers.0.conv", x, stride=2)
            skips.append(x)
    x = resnet(sd, "mid_block.resnets.0", x, temb, G, eps)
    x = transformer(sd, "mid_block.attentions.0", x, encoder_hidden_states, G, heads)
    x = resnet(sd, "mid_block.resnets.1", x, temb, G, eps)
    for i, bt in enumerate(up_types):
        for j in range(lpb + 1):
            x = torch.cat([x, skips.pop()], dim=1)
            x = resnet(sd, f"up_blocks.{i}.resnets.{j}", x, temb, G, eps)
            if "CrossAttn" in bt:
                x = transformer(sd, f"up_blocks.{i}.attentions.{j}", x, encoder_hidden_states, G, heads)
        if i < len(up_types) - 1:
            x = F.interpolate(x, scale_factor=2.0, mode="nearest")
            x = _conv(sd, f"up_blocks.{i}.upsamplers.0.conv", x)
    x = F.silu(F.group_norm(x, G, sd["conv_norm_out.weight"], sd["conv_norm_out.bias"], eps))
    return _conv(sd, "conv_out", x)
