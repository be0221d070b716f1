"""GeneralVAEImage — the RGB image encoder of the LDM on the HIP kernels.

The reference's GeneralVAEImage (ldmseg/models/vae.py:36-39) is diffusers' AutoencoderKL with
``set_scaling_factor``; tools/main_ldm.py:137-140 loads the SD-1.4 ``vae`` subfolder, replaces the
decoder with nn.Identity and uses only ``encode(x).latent_dist.mode()`` (encode_inputs,
trainers_ldm_cond.py:336-396).  This module keeps that surface and diffusers' parameter names
(``encoder.*``, ``quant_conv.*``, ``post_quant_conv.*``) so checkpoints load unchanged.

HIP path (NHWC activations): every conv is ldm_conv2d (the Downsample2D convs with pad_mode 1 =
F.pad (0, 1, 0, 1) + unpadded stride-2 conv), GroupNorm(+SiLU) consumes the producing conv's
statistics, shortcut/residual adds are conv epilogues.  The mid-block attention has a single
head of dim 512 (beyond the flash kernel's 160), so it runs as GEMM -> row softmax -> GEMM per
image: S = Q K^T (fp32), P = softmax(S / sqrt(C)) (ldm_softmax_rows), O = P V with V produced
transposed by a GEMM of W_v against the normalised tokens and its bias added in the P.V epilogue
(softmax rows sum to one).  Parity is unpinned (diffusers is absent): tested against
oracle/autoencoder_kl.py, a torch fp32 restatement.
"""
import json
import os
from typing import Optional, Tuple

import torch
import torch.nn as nn

from ..ops import native as K
from ..utils import OutputDict
from .vae import DiagonalGaussianDistribution


class EncoderOutput(OutputDict):
    latent_dist: torch.Tensor


class ResnetBlock2D(nn.Module):
    """diffusers ResnetBlock2D with temb_channels=None (no time embedding)."""

    def __init__(self, in_channels, out_channels, groups=32, eps=1e-6):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, padding=1)
        self.norm2 = nn.GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, padding=1)
        self.nonlinearity = nn.SiLU()
        self.conv_shortcut = nn.Conv2d(in_channels, out_channels, 1) if in_channels != out_channels else None
        self.groups, self.eps = groups, eps


class Downsample2D(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=0)


class DownEncoderBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels, num_layers, groups, add_downsample):
        super().__init__()
        self.resnets = nn.ModuleList(
            [ResnetBlock2D(in_channels if i == 0 else out_channels, out_channels, groups) for i in range(num_layers)])
        self.downsamplers = nn.ModuleList([Downsample2D(out_channels)]) if add_downsample else None


class Attention(nn.Module):
    """diffusers Attention as built by UNetMidBlock2D for the VAE (one head, GroupNorm, biases)."""

    def __init__(self, channels, groups=32, eps=1e-6):
        super().__init__()
        self.group_norm = nn.GroupNorm(groups, channels, eps=eps, affine=True)
        self.to_q = nn.Linear(channels, channels)
        self.to_k = nn.Linear(channels, channels)
        self.to_v = nn.Linear(channels, channels)
        self.to_out = nn.ModuleList([nn.Linear(channels, channels), nn.Dropout(0.0)])
        self.groups, self.eps = groups, eps


class UNetMidBlock2D(nn.Module):
    def __init__(self, channels, groups):
        super().__init__()
        self.attentions = nn.ModuleList([Attention(channels, groups)])
        self.resnets = nn.ModuleList([ResnetBlock2D(channels, channels, groups),
                                      ResnetBlock2D(channels, channels, groups)])


class Encoder(nn.Module):
    def __init__(self, in_channels, block_out_channels, layers_per_block, groups, latent_channels):
        super().__init__()
        self.conv_in = nn.Conv2d(in_channels, block_out_channels[0], 3, padding=1)
        self.down_blocks = nn.ModuleList()
        c = block_out_channels[0]
        for i, co in enumerate(block_out_channels):
            self.down_blocks.append(DownEncoderBlock2D(c, co, layers_per_block, groups,
                                                       add_downsample=i < len(block_out_channels) - 1))
            c = co
        self.mid_block = UNetMidBlock2D(c, groups)
        self.conv_norm_out = nn.GroupNorm(groups, c, eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(c, 2 * latent_channels, 3, padding=1)


# pre-0.14 diffusers names of the VAE attention (the SD-1.4 checkpoint's)
_LEGACY = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.", ".proj_attn.": ".to_out.0."}


class GeneralVAEImage(nn.Module):
    def __init__(self, in_channels: int = 3, out_channels: int = 3,
                 block_out_channels: Tuple[int, ...] = (128, 256, 512, 512), layers_per_block: int = 2,
                 latent_channels: int = 4, norm_num_groups: int = 32, scaling_factor: float = 0.18215, **_unused):
        super().__init__()
        self.config = dict(in_channels=in_channels, out_channels=out_channels,
                           block_out_channels=tuple(block_out_channels), layers_per_block=layers_per_block,
                           latent_channels=latent_channels, norm_num_groups=norm_num_groups,
                           scaling_factor=scaling_factor)
        self.encoder = Encoder(in_channels, block_out_channels, layers_per_block, norm_num_groups, latent_channels)
        self.quant_conv = nn.Conv2d(2 * latent_channels, 2 * latent_channels, 1)
        self.post_quant_conv = nn.Conv2d(latent_channels, latent_channels, 1)
        self.decoder = nn.Identity()        # tools/main_ldm.py:139
        self.scaling_factor = scaling_factor
        self._plan, self._plan_key = None, None

    def set_scaling_factor(self, scaling_factor):                  # vae.py:38-39
        self.scaling_factor = scaling_factor

    @property
    def dtype(self):
        return next(self.parameters()).dtype

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, subfolder=None, cache_dir=None, **kwargs):
        """Local diffusers layout: <path>/<subfolder>/config.json + diffusion_pytorch_model
        .safetensors (or .bin, read with weights_only=True).  The decoder weights are skipped."""
        root = os.path.join(pretrained_model_name_or_path, subfolder or "")
        with open(os.path.join(root, "config.json")) as f:
            cfg = json.load(f)
        model = cls(**{**cfg, **kwargs})
        st = os.path.join(root, "diffusion_pytorch_model.safetensors")
        if os.path.exists(st):
            from safetensors.torch import load_file
            sd = load_file(st)
        else:
            sd = torch.load(os.path.join(root, "diffusion_pytorch_model.bin"), map_location="cpu", weights_only=True)
        model.load_state_dict(remap_legacy_keys(sd), strict=True)
        return model

    def load_state_dict(self, state_dict, strict=True, **kw):
        sd = {k: v for k, v in remap_legacy_keys(state_dict).items() if not k.startswith("decoder.")}
        self._plan = None
        return super().load_state_dict(sd, strict=strict, **kw)

    # ------------------------------------------------------------------ HIP plan
    def prepare(self):
        key = (self.dtype, next(self.parameters()).device) + tuple((p.data_ptr(), p._version)
                                                                   for p in self.parameters())
        if self._plan is not None and self._plan_key == key:
            return self._plan
        dt = self.dtype
        if dt not in (torch.float32, torch.bfloat16):
            raise TypeError(f"GeneralVAEImage HIP path runs in float32 or bfloat16, not {dt}")
        pk = lambda m, **kw: K.PackedConv(m.weight, m.bias, dt, **kw)      # noqa: E731
        gnp = lambda m: (m.weight.detach().float().contiguous(), m.bias.detach().float().contiguous())  # noqa: E731
        P = {}
        e = self.encoder
        cin_pad = (e.conv_in.in_channels + 7) // 8 * 8
        P["cin_pad"] = cin_pad
        P["conv_in"] = pk(e.conv_in, cin_pad=cin_pad)
        for r in [m for m in self.modules() if isinstance(m, ResnetBlock2D)]:
            P[id(r)] = dict(n1=gnp(r.norm1), c1=pk(r.conv1), n2=gnp(r.norm2), c2=pk(r.conv2),
                            sc=None if r.conv_shortcut is None else pk(r.conv_shortcut))
        for blk in e.down_blocks:
            if blk.downsamplers is not None:
                P[id(blk.downsamplers[0])] = pk(blk.downsamplers[0].conv)
        a = e.mid_block.attentions[0]
        P["attn"] = dict(norm=gnp(a.group_norm), q=pk(a.to_q), k=pk(a.to_k),
                         wv=a.to_v.weight.detach().to(dt).contiguous(), bv=a.to_v.bias.detach().float().contiguous(),
                         out=pk(a.to_out[0]))
        P["out_norm"] = gnp(e.conv_norm_out)
        P["conv_out"] = pk(e.conv_out)
        P["quant"] = pk(self.quant_conv)
        self._plan, self._plan_key = P, key
        return P

    def _resnet(self, P, r, x, B, H, W):
        p = P[id(r)]
        h = K.group_norm(x, B, H * W, r.groups, *p["n1"], r.eps, K.ACT_SILU)
        h = K.conv2d(p["c1"], h, B, H, W, gn_stats=True)
        h = K.group_norm(h, B, H * W, r.groups, *p["n2"], r.eps, K.ACT_SILU)
        res = x if p["sc"] is None else K.conv2d(p["sc"], x, B, H, W)
        return K.conv2d(p["c2"], h, B, H, W, residual=res, gn_stats=True)

    def _attention(self, P, a, x, B, H, W):
        p = P["attn"]
        N, C = H * W, x.shape[-1]
        Np = (N + 63) // 64 * 64
        h = K.group_norm(x, B, N, a.groups, *p["norm"], a.eps)                    # [B, N, C]
        q = K.linear(p["q"], h)
        k = K.linear(p["k"], h)
        out = torch.empty_like(x)
        for b in range(B):
            hb, kb = h[b], k[b]
            if Np != N:                                # zero rows: S[:, N:] = 0, V^T[:, N:] = 0
                hb = torch.cat([hb, hb.new_zeros(Np - N, C)])
                kb = torch.cat([kb, kb.new_zeros(Np - N, C)])
            s = K.conv2d(K.packed_rows(kb.contiguous()), q[b], 1, 1, N, out_dtype=torch.float32)       # [N, Np]
            pm = K.softmax_rows(s.view(N, Np), N, C ** -0.5, self.dtype)                              # [N, Np]
            vt = K.conv2d(K.packed_rows(hb.contiguous()), p["wv"], 1, 1, C)                          # [C, Np]
            o = K.conv2d(K.packed_rows(vt.view(C, Np), bias=p["bv"]), pm, 1, 1, N)                   # [N, C]
            K.linear(p["out"], o, residual=x[b], out=out[b])
        return out

    @torch.no_grad()
    def encode_moments(self, x):
        """x [B, 3, H, W] in [-1, 1] -> moments fp32 [B, 2L, H/8, W/8] (encoder + quant_conv)."""
        with K.gn_arena(("vae_image", id(self), tuple(x.shape), self.dtype), x.device):
            return self._encode_moments(x)

    def _encode_moments(self, x):
        P = self.prepare()
        B, _, H, W = x.shape
        if H % 8 or W % 8:
            raise ValueError("GeneralVAEImage expects H and W divisible by 8")
        e = self.encoder
        h = K.nchw_to_nhwc([x], P["cin_pad"], self.dtype)
        h = K.conv2d(P["conv_in"], h, B, H, W)
        for blk in e.down_blocks:
            for r in blk.resnets:
                h = self._resnet(P, r, h, B, H, W)
            if blk.downsamplers is not None:
                h = K.conv2d(P[id(blk.downsamplers[0])], h, B, H, W, stride=2, pad_mode=1, gn_stats=True)
                H, W = H // 2, W // 2
        mb = e.mid_block
        h = self._resnet(P, mb.resnets[0], h, B, H, W)
        h = self._attention(P, mb.attentions[0], h, B, H, W)
        h = self._resnet(P, mb.resnets[1], h, B, H, W)
        h = K.group_norm(h, B, H * W, e.conv_norm_out.num_groups, *P["out_norm"], e.conv_norm_out.eps, K.ACT_SILU)
        h = K.conv2d(P["conv_out"], h, B, H, W)
        return K.conv2d(P["quant"], h, B, H, W, out_layout=K.OUT_NCHW, out_dtype=torch.float32)

    def encode(self, x, return_dict: bool = True):
        post = DiagonalGaussianDistribution(self.encode_moments(x))
        if not return_dict:
            return (post,)
        return EncoderOutput(latent_dist=post)

    def forward(self, sample, sample_posterior: bool = False, return_dict: bool = True,
                generator: Optional[torch.Generator] = None):
        """The decoder is nn.Identity (tools/main_ldm.py:139): forward returns the latent."""
        post = self.encode(sample).latent_dist
        z = post.sample(generator=generator) if sample_posterior else post.mode()
        return OutputDict(sample=z) if return_dict else (z,)


def remap_legacy_keys(sd):
    out = {}
    for k, v in sd.items():
        for old, new in _LEGACY.items():
            if old in k and ".attentions." in k:
                k = k.replace(old, new)
        out[k] = v
    return out
