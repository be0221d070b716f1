"""Drop-in ``UNet`` for ldmseg/models/unet.py:24 (an SD-1.x UNet2DConditionModel subclass).

The module tree and parameter names are diffusers' (so ``state_dict`` / ``load_state_dict``
stay checkpoint-compatible, trainers_ldm_cond.py:1846-1848,1891-1894); the arithmetic of
``forward`` (unet.py:281-436) runs entirely through the gfx950 HIP library:

  NCHW sample --nchw_to_nhwc--> NHWC activations (channels contiguous) for the whole graph
  timestep    --timestep_proj / linear(+SiLU) x2--> emb; every ResNet's time_emb_proj is
              ONE batched GEMM whose per-(b, n) output is added in the conv1 epilogue
  ResNet      GN+SiLU -> conv3x3 (+bias +temb) -> GN+SiLU -> conv3x3 (+bias +shortcut residual)
              up-block skip concats are read in place by GN and the convs (never copied)
  Transformer GN -> proj_in -> LN -> fused QKV GEMM -> flash attention -> to_out (+residual)
              -> LN -> GEGLU GEMM (gelu epilogue) -> net.2 (+residual) -> proj_out (+residual)
  Down/Up     stride-2 conv / conv reading the input through a nearest-2x upsample
  out         GN+SiLU -> conv_out written straight to NCHW

In train mode with grad enabled, ``forward`` goes through ``_UNetTrainFn``: the same HIP
forward keeping its activations, and the hand-written HIP backward of models/unet_train.py
(gradients flow to every trainable parameter, as under torch autograd; not to the input
sample, which the reference's training never needs).
"""
import contextlib
import json
import math
import os
from typing import Any, Dict, Optional, Tuple, Union

import torch
import torch.nn as nn

from ..ops import native as K
from ..utils import OutputDict


class UNetOutput(OutputDict):
    sample: torch.FloatTensor


# --------------------------------------------------------------------------------------
# module tree with diffusers parameter names
# --------------------------------------------------------------------------------------
class Timesteps(nn.Module):
    def __init__(self, num_channels, flip_sin_to_cos=True, downscale_freq_shift=0.0):
        super().__init__()
        self.num_channels = num_channels
        self.flip_sin_to_cos = flip_sin_to_cos
        self.downscale_freq_shift = downscale_freq_shift

    def frequencies(self, device):
        half = self.num_channels // 2
        exponent = -math.log(10000) * torch.arange(half, dtype=torch.float32) / (half - self.downscale_freq_shift)
        return torch.exp(exponent).to(device)


class TimestepEmbedding(nn.Module):
    def __init__(self, in_channels, time_embed_dim):
        super().__init__()
        self.linear_1 = nn.Linear(in_channels, time_embed_dim)
        self.act = nn.SiLU()
        self.linear_2 = nn.Linear(time_embed_dim, time_embed_dim)


class ResnetBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels, temb_channels, groups=32, eps=1e-5):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.groups, self.eps = groups, eps
        self.norm1 = nn.GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, padding=1)
        self.time_emb_proj = nn.Linear(temb_channels, out_channels)
        self.norm2 = nn.GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, padding=1)
        self.nonlinearity = nn.SiLU()
        self.conv_shortcut = nn.Conv2d(in_channels, out_channels, 1) if in_channels != out_channels else None


class Attention(nn.Module):
    def __init__(self, query_dim, heads, dim_head, cross_attention_dim=None):
        super().__init__()
        inner = heads * dim_head
        self.heads, self.dim_head = heads, dim_head
        self.is_cross = cross_attention_dim is not None
        kv_dim = cross_attention_dim or query_dim
        self.to_q = nn.Linear(query_dim, inner, bias=False)
        self.to_k = nn.Linear(kv_dim, inner, bias=False)
        self.to_v = nn.Linear(kv_dim, inner, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim), nn.Dropout(0.0)])


class GEGLU(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)


class FeedForward(nn.Module):
    def __init__(self, dim, mult=4):
        super().__init__()
        self.net = nn.ModuleList([GEGLU(dim, dim * mult), nn.Dropout(0.0), nn.Linear(dim * mult, dim)])


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, heads, dim_head, cross_attention_dim=None):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim)
        self.attn1 = Attention(dim, heads, dim_head)
        if cross_attention_dim is not None:
            self.norm2 = nn.LayerNorm(dim)
            self.attn2 = Attention(dim, heads, dim_head, cross_attention_dim)
        else:
            self.norm2 = None
            self.attn2 = None
        self.norm3 = nn.LayerNorm(dim)
        self.ff = FeedForward(dim)


class Transformer2DModel(nn.Module):
    def __init__(self, heads, dim_head, in_channels, groups=32, cross_attention_dim=None):
        super().__init__()
        inner = heads * dim_head
        self.groups = groups
        self.norm = nn.GroupNorm(groups, in_channels, eps=1e-6, affine=True)
        self.proj_in = nn.Conv2d(in_channels, inner, 1)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(inner, heads, dim_head, cross_attention_dim)])
        self.proj_out = nn.Conv2d(inner, in_channels, 1)


class Downsample2D(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=1)


class Upsample2D(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, padding=1)


class DownBlock(nn.Module):
    """CrossAttnDownBlock2D (has_cross_attention) or DownBlock2D."""

    def __init__(self, cin, cout, temb, layers, groups, eps, heads, attn, cross_dim, add_down):
        super().__init__()
        self.has_cross_attention = attn
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, temb, groups, eps)
                                      for i in range(layers)])
        if attn:
            self.attentions = nn.ModuleList([Transformer2DModel(heads, cout // heads, cout, groups, cross_dim)
                                             for _ in range(layers)])
        self.downsamplers = nn.ModuleList([Downsample2D(cout)]) if add_down else None


class UpBlock(nn.Module):
    """CrossAttnUpBlock2D (has_cross_attention) or UpBlock2D."""

    def __init__(self, cin, cprev, cout, temb, layers, groups, eps, heads, attn, cross_dim, add_up):
        super().__init__()
        self.has_cross_attention = attn
        res = []
        for i in range(layers):
            skip = cin if i == layers - 1 else cout
            rin = cprev if i == 0 else cout
            res.append(ResnetBlock2D(rin + skip, cout, temb, groups, eps))
        self.resnets = nn.ModuleList(res)
        if attn:
            self.attentions = nn.ModuleList([Transformer2DModel(heads, cout // heads, cout, groups, cross_dim)
                                             for _ in range(layers)])
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if add_up else None


class UNetMidBlock2DCrossAttn(nn.Module):
    def __init__(self, c, temb, groups, eps, heads, cross_dim):
        super().__init__()
        self.has_cross_attention = True
        self.resnets = nn.ModuleList([ResnetBlock2D(c, c, temb, groups, eps), ResnetBlock2D(c, c, temb, groups, eps)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, c // heads, c, groups, cross_dim)])


class _Config(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


SD_V1_CONFIG = dict(
    sample_size=64, in_channels=4, out_channels=4, center_input_sample=False, flip_sin_to_cos=True, freq_shift=0,
    down_block_types=("CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "DownBlock2D"),
    up_block_types=("UpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D"),
    block_out_channels=(320, 640, 1280, 1280), layers_per_block=2, downsample_padding=1, mid_block_scale_factor=1,
    act_fn="silu", norm_num_groups=32, norm_eps=1e-5, cross_attention_dim=768, attention_head_dim=8,
)


# --------------------------------------------------------------------------------------
# the drop-in UNet
# --------------------------------------------------------------------------------------
class UNet(nn.Module):
    """UNet2DConditionModel-compatible module whose forward runs on the HIP kernels."""

    config_name = "config.json"

    def __init__(self, **kwargs):
        super().__init__()
        cfg = dict(SD_V1_CONFIG)
        cfg.update({k: v for k, v in kwargs.items() if not k.startswith("_")})
        self.config = _Config(cfg)
        boc = list(cfg["block_out_channels"])
        lpb = cfg["layers_per_block"]
        G, eps = cfg["norm_num_groups"], cfg["norm_eps"]
        heads = cfg["attention_head_dim"]
        cross = cfg.get("cross_attention_dim")
        temb = boc[0] * 4
        self.conv_in = nn.Conv2d(cfg["in_channels"], boc[0], 3, padding=1)
        self.time_proj = Timesteps(boc[0], cfg["flip_sin_to_cos"], cfg["freq_shift"])
        self.time_embedding = TimestepEmbedding(boc[0], temb)
        self.encoder_hid_proj = None
        down = []
        c = boc[0]
        for i, bt in enumerate(cfg["down_block_types"]):
            cin, c = c, boc[i]
            down.append(DownBlock(cin, c, temb, lpb, G, eps, heads, "CrossAttn" in bt, cross, i < len(boc) - 1))
        self.down_blocks = nn.ModuleList(down)
        self.mid_block = UNetMidBlock2DCrossAttn(boc[-1], temb, G, eps, heads, cross)
        rev = list(reversed(boc))
        up = []
        cprev = rev[0]
        for i, bt in enumerate(cfg["up_block_types"]):
            cout = rev[i]
            cin = rev[min(i + 1, len(boc) - 1)]
            up.append(UpBlock(cin, cprev, cout, temb, lpb + 1, G, eps, heads, "CrossAttn" in bt, cross,
                              i < len(boc) - 1))
            cprev = cout
        self.up_blocks = nn.ModuleList(up)
        self.conv_norm_out = nn.GroupNorm(G, boc[0], eps=eps)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(boc[0], cfg["out_channels"], 3, padding=1)
        self.gradient_checkpointing = False
        self._plan = None
        self._plan_key = None
        self._dplan = None
        self._compute_dtype = None

    # ------------------------------------------------------------ diffusers-style API
    @property
    def dtype(self) -> torch.dtype:
        return next(self.parameters()).dtype

    @property
    def compute_dtype(self) -> torch.dtype:
        """dtype the HIP kernels compute in: the parameters' dtype, unless set_compute_dtype()
        chose another (fp32 master weights computing in bf16 — the role of the reference's
        fp16 autocast, trainers_ldm_cond.py:831,836)."""
        return self._compute_dtype or self.dtype

    def set_compute_dtype(self, dtype=None):
        self._compute_dtype = dtype
        self._plan = self._plan_key = self._dplan = None

    @property
    def device(self) -> torch.device:
        return next(self.parameters()).device

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, subfolder=None, cache_dir=None, **kwargs):
        """Load a local diffusers UNet folder (config.json + weights), tools/main_ldm.py:147.

        Only local paths are supported (no hub download); weights are read with loaders that
        execute nothing from the file (safetensors, or torch.load(weights_only=True)).
        """
        path = pretrained_model_name_or_path if subfolder is None else os.path.join(pretrained_model_name_or_path,
                                                                                    subfolder)
        with open(os.path.join(path, cls.config_name)) as f:
            cfg = json.load(f)
        keep = set(SD_V1_CONFIG) | {"sample_size"}
        model = cls(**{k: (tuple(v) if isinstance(v, list) else v) for k, v in cfg.items() if k in keep})
        st = os.path.join(path, "diffusion_pytorch_model.safetensors")
        if os.path.exists(st):
            from safetensors.torch import load_file
            sd = load_file(st)
        else:
            sd = torch.load(os.path.join(path, "diffusion_pytorch_model.bin"), map_location="cpu", weights_only=True)
        sd = _remap_legacy_keys(sd)
        model.load_state_dict(sd, strict=True)
        return model

    def enable_gradient_checkpointing(self):
        self.gradient_checkpointing = True

    def get_lr_func(self, name: str, lr_decay_rate: float = 1.0) -> float:   # unet.py:107-119
        if name.startswith("module."):
            name = name[len("module."):]
        if name.startswith("conv_in.") or name.startswith("down_blocks."):
            return lr_decay_rate
        return 1.0

    def remove_cross_attention(self):                                        # unet.py:83-105
        blocks = list(self.down_blocks) + [self.mid_block] + list(self.up_blocks)
        for blk in blocks:
            if getattr(blk, "has_cross_attention", False):
                for attn in blk.attentions:
                    for tb in attn.transformer_blocks:
                        tb.attn2 = None
                        tb.norm2 = None
        self._plan = None

    def modify_encoder(self, in_channels: int = 4, init_mode_seg: str = "copy", init_mode_image: str = "copy",
                       cond_channels: int = 0, init_mode_cond: str = "zero", separate_conv: bool = False,
                       separate_encoder: bool = False, add_adaptor: bool = False,
                       init_mode_adaptor: str = "random") -> None:
        """unet.py:124-233.  The 8(+cond)-channel conv_in branch, including its quirks: the
        'div' modes are no-ops (the quotient of ``.copy_(w) / 2.`` is discarded, :188,202) and
        the cond 'mean' branch tests init_mode_image (:225)."""
        assert in_channels in [4, 8], "in_channels must be 4 or 8"
        assert separate_conv + separate_encoder <= 1
        if separate_conv or separate_encoder:
            raise NotImplementedError("separate_conv / separate_encoder are non-default variants, not on the "
                                      "accelerated path (SURVEY.md §2 row 1)")
        if in_channels != 8:
            return
        old = self.conv_in
        w_old, b_old = old.weight.data, old.bias.data
        self.new_conv = nn.Conv2d(in_channels + cond_channels, old.out_channels, kernel_size=old.kernel_size,
                                  stride=old.stride, padding=old.padding, bias=old.bias is not None)
        self.new_conv.to(device=w_old.device, dtype=w_old.dtype)
        W = self.new_conv.weight.data
        mean4 = torch.mean(w_old, dim=1, keepdim=True).repeat(1, 4, 1, 1)
        for sl, mode, what in ((slice(0, 4), init_mode_seg, "seg"), (slice(4, 8), init_mode_image, "image")):
            if mode in ("copy", "div"):
                W[:, sl].copy_(w_old)
            elif mode == "mean":
                W[:, sl].copy_(mean4)
            elif mode == "zero":
                W[:, sl].zero_()
            elif mode != "random":
                raise NotImplementedError(f"init_mode {what} {mode} not implemented")
        self.new_conv.bias.data.copy_(b_old)
        assert W.shape == torch.Size([old.out_channels, 8 + cond_channels, 3, 3])
        if cond_channels > 0:
            if init_mode_cond == "zero":
                W[:, 8:].zero_()
            elif init_mode_image == "mean":
                W[:, 8:].copy_(mean4)
            elif init_mode_cond != "random":
                raise NotImplementedError(f"init_mode cond {init_mode_cond} not implemented")
        self.conv_in = self.new_conv          # aliased: state_dict holds conv_in.* AND new_conv.*
        self._plan = None

    def freeze_layers(self, layers=("norm", "time_embedding")) -> None:      # unet.py:235-279
        for layer in layers:
            if layer == "norm":
                for m in self.modules():
                    if isinstance(m, (nn.GroupNorm, nn.LayerNorm, nn.BatchNorm2d)):
                        m.requires_grad_(False)
            elif layer == "time_embedding":
                self.time_embedding.requires_grad_(False)
            elif layer in ("conv_in", "down_blocks"):
                pass                                 # only acts with separate_encoder (not built)
            else:
                raise NotImplementedError(f"layer {layer} not implemented")

    # ------------------------------------------------------------ packed-weight plan
    def _signature(self):
        return (self.compute_dtype, self.device, self.ln_fold, self.upsample_phases) + tuple((p.data_ptr(), p._version)
                                                                       for p in self.parameters())

    @staticmethod
    def _pk(weights, biases, dt, **kw):
        """PackedConv of the row-concatenation of ``weights`` (+ concatenated ``biases``), recording
        its source parameters so models.repack.PackRefresher can rewrite it in place after an
        optimizer update (ldm_repack) instead of re-running this packing."""
        w = weights[0] if len(weights) == 1 else torch.cat(weights)
        bs = [b for b in biases if b is not None]
        b = None if not bs else (bs[0] if len(bs) == 1 else torch.cat(bs))
        pc = K.PackedConv(w, b, dt, **kw)
        pc.src_w, pc.src_b = list(weights), bs
        return pc

    def prepare(self, force=False):
        """(Re)pack every weight for the HIP kernels; cached until a parameter changes."""
        key = self._signature()
        if not force and self._plan is not None and self._plan_key == key:
            return self._plan
        dt = self.compute_dtype
        if dt not in (torch.float32, torch.bfloat16):
            raise TypeError(f"UNet HIP path runs in float32 or bfloat16, not {dt}")
        f32 = lambda t: None if t is None else t.detach().float().contiguous()  # noqa: E731
        P = {}
        cin = self.conv_in.in_channels
        cin_pad = (cin + 15) // 16 * 16
        P["conv_in"] = self._pk([self.conv_in.weight], [self.conv_in.bias], dt, cin_pad=cin_pad)
        P["cin_pad"] = cin_pad
        P["freqs"] = self.time_proj.frequencies(self.device)
        te = self.time_embedding
        P["lin1"] = K.PackedConv(te.linear_1.weight, te.linear_1.bias, dt)
        P["lin2"] = K.PackedConv(te.linear_2.weight, te.linear_2.bias, dt)
        # all ResNets' time_emb_proj as one GEMM [sum Cout, 1280]
        resnets = [m for m in self.modules() if isinstance(m, ResnetBlock2D)]
        ws, bs, off = [], [], 0
        for r in resnets:
            ws.append(r.time_emb_proj.weight)
            bs.append(r.time_emb_proj.bias)
            P[id(r), "temb_off"] = off
            off += r.out_channels
        P["temb_proj"] = self._pk(ws, bs, dt)
        P["temb_total"] = off
        for r in resnets:
            P[id(r)] = dict(
                n1=(f32(r.norm1.weight), f32(r.norm1.bias)), n2=(f32(r.norm2.weight), f32(r.norm2.bias)),
                c1=self._pk([r.conv1.weight], [r.conv1.bias], dt), c2=self._pk([r.conv2.weight], [r.conv2.bias], dt),
                sc=None if r.conv_shortcut is None else self._pk([r.conv_shortcut.weight], [r.conv_shortcut.bias], dt),
                off=P[id(r), "temb_off"])
        for t in [m for m in self.modules() if isinstance(m, Transformer2DModel)]:
            tb = t.transformer_blocks[0]
            a1 = tb.attn1
            d = dict(norm=(f32(t.norm.weight), f32(t.norm.bias)),
                     proj_in=self._pk([t.proj_in.weight], [t.proj_in.bias], dt),
                     proj_out=self._pk([t.proj_out.weight], [t.proj_out.bias], dt),
                     ln1=(f32(tb.norm1.weight), f32(tb.norm1.bias)), ln3=(f32(tb.norm3.weight), f32(tb.norm3.bias)),
                     qkv=self._pk([a1.to_q.weight, a1.to_k.weight, a1.to_v.weight], [], dt),
                     out1=self._pk([a1.to_out[0].weight], [a1.to_out[0].bias], dt),
                     heads=a1.heads, dim_head=a1.dim_head,
                     ff1=self._pk([tb.ff.net[0].proj.weight], [tb.ff.net[0].proj.bias], dt, geglu=True),
                     ff2=self._pk([tb.ff.net[2].weight], [tb.ff.net[2].bias], dt), attn2=None)
            if dt == torch.bfloat16 and self.ln_fold:
                # norm1 -> QKV and norm3 -> ff.net.0 as single GEMMs on the raw rows (the producers,
                # proj_in and to_out, sum each row's statistics in their epilogues)
                d["qkv_ln"] = K.packed_ln_fold(torch.cat([a1.to_q.weight, a1.to_k.weight, a1.to_v.weight]), None,
                                               tb.norm1.weight, tb.norm1.bias, dt)
                d["ff1_ln"] = K.packed_ln_fold(tb.ff.net[0].proj.weight, tb.ff.net[0].proj.bias, tb.norm3.weight,
                                               tb.norm3.bias, dt, geglu=True)
                d["ln_eps"] = (tb.norm1.eps, tb.norm3.eps)
            if tb.attn2 is not None:
                a2 = tb.attn2
                d["attn2"] = dict(ln2=(f32(tb.norm2.weight), f32(tb.norm2.bias)),
                                  q=K.PackedConv(a2.to_q.weight, None, dt),
                                  kv=K.PackedConv(torch.cat([a2.to_k.weight, a2.to_v.weight]), None, dt),
                                  out=K.PackedConv(a2.to_out[0].weight, a2.to_out[0].bias, dt))
            P[id(t)] = d
        for m in self.modules():
            if isinstance(m, Upsample2D) and self.upsample_phases:
                # nearest-2x upsample + 3x3 conv as four 2x2 phase convs over the low-res input
                # (4/9 of the FLOPs; ldm_conv2d upsample mode 3)
                # (no src_w: ldm_repack has no phase layout — training runs with the phases off)
                P[id(m)] = K.PackedConv(m.conv.weight, m.conv.bias, dt, upsample_phases=True)
            elif isinstance(m, (Downsample2D, Upsample2D)):
                P[id(m)] = self._pk([m.conv.weight], [m.conv.bias], dt)
        P["out_norm"] = (f32(self.conv_norm_out.weight), f32(self.conv_norm_out.bias))
        P["conv_out"] = self._pk([self.conv_out.weight], [self.conv_out.bias], dt)
        P["resnets"] = resnets
        self._plan, self._plan_key = P, key
        self._dplan = None
        return P

    def prepare_dgrad(self):
        """Packed weights of the backward: the data-gradient (transposed, flipped) weight of every
        conv / linear, keyed by id(module), plus conv_out padded to 8 output channels for its
        weight gradient (the 4-channel output gradient is padded to 8 for 16-byte rows)."""
        P = self.prepare()
        if self._dplan is not None:
            return self._dplan
        from .unet_train import packed_dgrad
        dt = self.compute_dtype
        D = {}
        for r in P["resnets"]:
            D[id(r.conv1)] = packed_dgrad(r.conv1.weight, dt)
            D[id(r.conv2)] = packed_dgrad(r.conv2.weight, dt)
            if r.conv_shortcut is not None:
                D[id(r.conv_shortcut)] = packed_dgrad(r.conv_shortcut.weight, dt)
        for t in [m for m in self.modules() if isinstance(m, Transformer2DModel)]:
            tb = t.transformer_blocks[0]
            a1 = tb.attn1
            D[id(t.proj_in)] = packed_dgrad(t.proj_in.weight, dt)
            D[id(t.proj_out)] = packed_dgrad(t.proj_out.weight, dt)
            D[id(a1)] = packed_dgrad(torch.cat([a1.to_q.weight, a1.to_k.weight, a1.to_v.weight]), dt)
            D[id(a1)].dg_src = ([a1.to_q.weight, a1.to_k.weight, a1.to_v.weight], False)
            D[id(a1.to_out[0])] = packed_dgrad(a1.to_out[0].weight, dt)
            D[id(tb.ff.net[0].proj)] = packed_dgrad(tb.ff.net[0].proj.weight, dt, geglu=True)
            D[id(tb.ff.net[2])] = packed_dgrad(tb.ff.net[2].weight, dt)
        for m in self.modules():
            if isinstance(m, (Downsample2D, Upsample2D)):
                D[id(m)] = packed_dgrad(m.conv.weight, dt)
        co = self.conv_out.out_channels
        D["conv_out"] = packed_dgrad(self.conv_out.weight, dt, cin_pad=8)
        wpad = torch.zeros(8, *self.conv_out.weight.shape[1:], dtype=self.conv_out.weight.dtype,
                           device=self.conv_out.weight.device)
        wpad[:co] = self.conv_out.weight.detach()
        P["conv_out_t"] = K.PackedConv(wpad, None, dt)
        P["conv_out_t"].src_w, P["conv_out_t"].src_b = [self.conv_out.weight], []   # rows co..7 stay zero
        self._dplan = D
        return D

    @property
    def attention_fp8(self):
        return getattr(self, "_attention_fp8", False)

    def set_attention_fp8(self, enabled=True):
        """BASELINE config 5: self-attention on the block-scaled e4m3 MFMA (ldm_attention_fp8: Q.K^T
        and P.V in fp8) at the head dims that kernel covers (K.FP8_SCALED_HEAD_DIMS) when the compute
        dtype is bf16; an inference option (the training path keeps bf16)."""
        self._attention_fp8 = bool(enabled)

    def invalidate_packed(self):
        """Drop the packed weights (call after an in-place optimizer update that bypasses
        torch's version counter, e.g. the fused AdamW of ldmseg.trainers)."""
        self._plan = self._plan_key = self._dplan = None

    # ------------------------------------------------------------ HIP forward pieces
    def _gn_next(self, P, m):
        """conv2d(gn_next=...) spec of the GroupNorm that consumes a block output next: a ResnetBlock2D's
        norm1 (+SiLU) or a Transformer2DModel's norm (no activation); None when the consumer reads a
        concat or no GroupNorm (the split-K reduction then only emits the statistics)."""
        if m is None:
            return None
        if isinstance(m, ResnetBlock2D):
            return (m.groups, *P[id(m)]["n1"], m.eps, K.ACT_SILU, True)
        return (m.groups, *P[id(m)]["norm"], 1e-6, K.ACT_NONE, True)

    def _resnet(self, P, r, xs, B, H, W, temb_all, gn_next=None):
        """gn_next: the GroupNorm consuming this block's output (see _gn_next); the deep levels' split
        convs apply it (and norm2 after conv1) in their split-K reduction's launch."""
        p = P[id(r)]
        x0, x1 = xs
        side = None
        if p["sc"] is not None and self.sc_concurrent:
            # the 1x1 shortcut reads only the block input: it runs on a side stream beside
            # GroupNorm -> conv1 -> GroupNorm (captured as a parallel branch of the step graph) and
            # joins before conv2 adds it; x0 / x1 stay referenced here until the join
            main = torch.cuda.current_stream(x0.device)
            side = self._side_stream(x0.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                res = K.conv2d(p["sc"], x0, B, H, W, x1=x1)
        h = K.group_norm(x0, B, H * W, r.groups, *p["n1"], r.eps, K.ACT_SILU, x1=x1)
        h = K.conv2d(p["c1"], h, B, H, W, temb=temb_all[:, p["off"]:], temb_stride=temb_all.shape[1], gn_stats=True,
                     gn_next=(r.groups, *p["n2"], r.eps, K.ACT_SILU, False))
        h = K.group_norm(h, B, H * W, r.groups, *p["n2"], r.eps, K.ACT_SILU)
        if side is not None:
            main.wait_stream(side)
            res.record_stream(main)
        elif p["sc"] is not None:
            res = K.conv2d(p["sc"], x0, B, H, W, x1=x1)
        else:
            assert x1 is None
            res = x0
        return K.conv2d(p["c2"], h, B, H, W, residual=res, gn_stats=True, gn_next=gn_next)

    def _side_stream(self, dev):
        st = getattr(self, "_side", None)
        if st is None or st.device != dev:
            st = self._side = torch.cuda.Stream(device=dev)
        return st

    @property
    def sc_concurrent(self):
        return getattr(self, "_sc_concurrent", False)

    def set_sc_concurrent(self, enabled=True):
        """Run the ResnetBlock2D 1x1 shortcuts (and the time-embedding MLP) on a side stream beside
        GroupNorm -> conv1 -> GroupNorm (conv_in): the same kernels and results, as parallel branches
        of the step graph.  Default off: same-box A/B of the captured step (tools/ab_step.py) measured
        9.27 -> 9.44 ms at B = 8 and 4.25 -> 4.45 ms at B = 1 — each fork / join of graph branches costs
        more than the overlap returns."""
        self._sc_concurrent = bool(enabled)

    @property
    def ln_fold(self):
        return getattr(self, "_ln_fold", True)

    def set_ln_fold(self, enabled=True):
        """bf16 inference: fold norm1 / norm3 into the QKV / ff.net.0 GEMMs (default on); off runs
        the separate LayerNorm kernels (A/B, and the form the training path differentiates — the
        training step turns it off, so its packs can be refreshed in place by ldm_repack)."""
        self._ln_fold = bool(enabled)
        self._plan = self._plan_key = self._dplan = None

    @property
    def ff_fused(self):
        return getattr(self, "_ff_fused", True)

    def set_ff_fused(self, enabled=True):
        """bf16 inference with the LayerNorm fold: run the 64x64 level's FeedForward as one
        ldm_feedforward launch (default on; K.feedforward_ok decides per call); off runs the GEGLU
        and ff.net.2 GEMMs separately (A/B — the results are the same bit for bit)."""
        self._ff_fused = bool(enabled)

    @property
    def upsample_phases(self):
        # inference only: the autograd drop-in (train mode) differentiates the 3x3 gather form
        return getattr(self, "_up_phases", True) and not self.training

    def set_upsample_phases(self, enabled=True):
        """Run every Upsample2D conv as four 2x2 phase convs over its low-res input (default on:
        4/9 of the 3x3 conv's FLOPs, the taps that read the same source pixel summed in fp32 before
        the bf16 rounding); off runs the 3x3 conv through the nearest-2x gather (the form the
        training backward differentiates: LDMTrainStep turns it off with the LayerNorm fold)."""
        self._up_phases = bool(enabled)
        self._plan = self._plan_key = self._dplan = None

    @property
    def tin_fused(self):
        return getattr(self, "_tin_fused", True)

    def set_tin_fused(self, enabled=True):
        """bf16 inference with the LayerNorm fold: run the 64x64 level's GroupNorm -> proj_in ->
        norm1-folded QKV as one ldm_transformer_in launch (default on; K.transformer_in_ok decides
        per call); off runs the three launches (A/B — the results are the same bit for bit)."""
        self._tin_fused = bool(enabled)

    @property
    def ff_proj_out_fused(self):
        return getattr(self, "_ff_po_fused", True)

    def set_ff_proj_out_fused(self, enabled=True):
        """With the fused feed-forward: also run Transformer2DModel.proj_out in the same launch
        (default on; results identical to the separate proj_out call)."""
        self._ff_po_fused = bool(enabled)

    def _transformer(self, P, t, x, B, H, W, ehs):
        p = P[id(t)]
        C = x.shape[-1]
        N = H * W
        cross = p["attn2"] is not None and ehs is not None
        if self.ln_fold and "qkv_ln" in p:
            rs3 = None if cross else K.zeroed_f64(2 * B * N, x.device)
            if self.tin_fused and K.transformer_in_ok(p["proj_in"], p["qkv_ln"], x, B, N, t.groups):
                # norm -> proj_in -> norm1-folded QKV in one launch (h and its row statistics on chip)
                h, qkv = K.transformer_in(p["proj_in"], p["qkv_ln"], x, B, N, t.groups, *p["norm"], 1e-6,
                                          p["ln_eps"][0])
            else:
                h = K.group_norm(x, B, N, t.groups, *p["norm"], 1e-6)
                rs1 = K.zeroed_f64(2 * B * N, x.device)
                h = K.linear(p["proj_in"], h, row_stats=rs1)             # [B, N, C] + row (sum, sumsq)
                qkv = K.linear(p["qkv_ln"], h, ln=(rs1, p["ln_eps"][0]))  # = to_qkv(norm1(h))
        else:
            rs3 = None
            h = K.group_norm(x, B, N, t.groups, *p["norm"], 1e-6)
            h = K.linear(p["proj_in"], h)                                # [B, N, C]
            n = K.layer_norm(h, *p["ln1"], 1e-5)
            qkv = K.linear(p["qkv"], n)                                  # [B, N, 3C]
        heads, dh = p["heads"], p["dim_head"]
        # fp8 where the block-scaled MFMA kernel exists (head_dim 40: the top level, ~87 % of config
        # 5's attention FLOPs); the non-scaled fp8 MFMA of the other head dims runs at the bf16 rate,
        # so those levels stay bf16
        fp8 = self.attention_fp8 and qkv.dtype == torch.bfloat16 and dh in K.FP8_SCALED_HEAD_DIMS
        a = K.attention(qkv, qkv[..., C:], qkv[..., 2 * C:], B, heads, dh, N, N, 3 * C, 3 * C, 3 * C, fp8=fp8)
        h = K.linear(p["out1"], a, residual=h, out=h, row_stats=rs3)
        if cross:
            q2 = p["attn2"]
            n = K.layer_norm(h, *q2["ln2"], 1e-5)
            q = K.linear(q2["q"], n)
            e = ehs.to(self.compute_dtype).contiguous()
            kv = K.linear(q2["kv"], e)                                   # [B, L, 2C]
            L = e.shape[1]
            a = K.attention(q, kv, kv[..., C:], B, heads, dh, N, L, C, 2 * C, 2 * C)
            h = K.linear(q2["out"], a, residual=h, out=h)
        if rs3 is not None and self.ff_fused and K.feedforward_ok(p["ff1_ln"], p["ff2"], h):
            # ff.net.2(GEGLU(ff.net.0(norm3(h)))) + h in one launch, the 4C intermediate on chip
            if self.ff_proj_out_fused:     # + proj_out in the same launch (h never stored)
                return K.feedforward(p["ff1_ln"], p["ff2"], h, ln=(rs3, p["ln_eps"][1]), residual=h,
                                     proj_out=(p["proj_out"], x, B, H, W, True))
            h = K.feedforward(p["ff1_ln"], p["ff2"], h, ln=(rs3, p["ln_eps"][1]), residual=h, out=h)
            return K.conv2d(p["proj_out"], h, B, H, W, residual=x, gn_stats=True)
        if rs3 is not None:
            f = K.linear(p["ff1_ln"], h, out_layout=K.OUT_GEGLU, ln=(rs3, p["ln_eps"][1]))   # ff.net.0(norm3(h))
        else:
            n = K.layer_norm(h, *p["ln3"], 1e-5)
            f = K.linear(p["ff1"], n, out_layout=K.OUT_GEGLU)            # [B, N, 4C]
        h = K.linear(p["ff2"], f, residual=h, out=h)
        return K.conv2d(p["proj_out"], h, B, H, W, residual=x, gn_stats=True)

    def _trainable(self):
        return [p for p in self.parameters() if p.requires_grad]

    def forward(
        self,
        sample: torch.FloatTensor,
        timestep: Union[torch.Tensor, float, int],
        encoder_hidden_states: Optional[torch.Tensor] = None,
        class_labels: Optional[torch.Tensor] = None,
        timestep_cond: Optional[torch.Tensor] = None,
        attention_mask: Optional[torch.Tensor] = None,
        cross_attention_kwargs: Optional[Dict[str, Any]] = None,
        down_block_additional_residuals: Optional[Tuple[torch.Tensor]] = None,
        mid_block_additional_residual: Optional[torch.Tensor] = None,
        return_dict: bool = True,
        timestep_img: Optional[Union[torch.Tensor, float, int]] = None,
    ) -> Union[UNetOutput, Tuple]:
        if class_labels is not None or timestep_cond is not None or attention_mask is not None:
            raise NotImplementedError("class_labels / timestep_cond / attention_mask are not on the reference path")
        if down_block_additional_residuals is not None or mid_block_additional_residual is not None:
            raise NotImplementedError("additional residuals belong to the separate_encoder variant")
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            out = _UNetTrainFn.apply(self, timestep, sample, *self._trainable())
        else:
            out = self.forward_sources([sample], timestep, encoder_hidden_states)
        if not return_dict:
            return (out,)
        return UNetOutput(sample=out)

    @torch.no_grad()
    def forward_sources(self, sources, timestep, encoder_hidden_states=None):
        """forward() on the channel concatenation of up to three NCHW tensors without
        materialising it (the sampler's ``torch.cat([x_t, rgb, cond], 1)``,
        trainers_ldm_cond.py:1134-1141, is folded into the NCHW->NHWC gather of conv_in).
        All GroupNorm accumulators of the pass come from one zeroed arena (K.gn_arena)."""
        s0 = sources[0]
        with K.gn_arena(("unet", id(self), tuple(s0.shape), self.compute_dtype), s0.device):
            return self._forward_sources(sources, timestep, encoder_hidden_states)

    @torch.no_grad()
    def forward_ddim_step(self, sources, timestep, scheduler, t_int, sample, encoder_hidden_states=None,
                          prev_out=None):
        """One sampler step, trainers_ldm_cond.py:1144-1162: eps = unet(cat(sources), t) and
        scheduler.step(eps, t, sample) -> (prev_sample, pred_original_sample).  On the bf16 path the
        step runs inside the UNet tail's launch (ldm_unet_tail: GroupNorm -> SiLU -> conv_out -> DDIM
        on the same device arithmetic as ldm_ddim_step, the model output rounded to bf16 first, as the
        unfused conv stores it); otherwise the two calls.  prev_out (fused path only): the tensor
        prev_sample is written to — the sampler passes the latent buffer itself (an in-place update).
        Callers must use the returned prev_sample, which is a new tensor on the unfused path."""
        s0 = sources[0]
        ddim = scheduler.fused_step_args(t_int, sample, self.compute_dtype, prev_out=prev_out)
        with K.gn_arena(("unet", id(self), tuple(s0.shape), self.compute_dtype), s0.device):
            r = self._forward_sources(sources, timestep, encoder_hidden_states, ddim=ddim)
        if isinstance(r, tuple):
            return r[1], r[2]
        out = scheduler.step(r, t_int, sample)
        return out.prev_sample, out.pred_original_sample

    def _time_embedding(self, P, t, B, dt):
        """Timesteps -> TimestepEmbedding -> SiLU -> the batched time_emb_proj of every ResnetBlock2D
        (unet.py:301-307): fp32 [B, sum of their out channels]."""
        if dt == torch.bfloat16 and P["lin1"].cin == self.time_proj.num_channels and \
                K.linear_rows_ok(P["lin1"], B, sinusoid=True) and all(K.linear_rows_ok(P[k], B) for k in ("lin2", "temb_proj")):
            # few-row GEMMs that stream each weight once (ldm_linear_rows); the sinusoid is formed
            # inside linear_1's launch
            emb = K.linear_rows(P["lin1"], None, B, act=K.ACT_SILU, t=t, freqs=P["freqs"],
                                flip_sin_to_cos=self.time_proj.flip_sin_to_cos)
            emb = K.linear_rows(P["lin2"], emb, B, act=K.ACT_SILU)     # = SiLU(time_embedding(t))
            temb_all = K.linear_rows(P["temb_proj"], emb, B, out_dtype=torch.float32)
        else:
            emb = K.timestep_proj(t, B, P["freqs"], self.time_proj.num_channels, self.time_proj.flip_sin_to_cos, dt)
            emb = K.linear(P["lin1"], emb, act=K.ACT_SILU)
            emb = K.linear(P["lin2"], emb, act=K.ACT_SILU)               # = SiLU(time_embedding(t))
            temb_all = K.linear(P["temb_proj"], emb, out_dtype=torch.float32)  # [B, sum Cout]
        return temb_all

    def _forward_sources(self, sources, timestep, encoder_hidden_states=None, ddim=None):
        P = self.prepare()
        dt = self.compute_dtype
        sample = sources[0]
        dev = sample.device
        B, _, H, W = sample.shape
        Cin = sum(s.shape[1] for s in sources)
        if Cin != self.conv_in.in_channels:
            raise ValueError(f"UNet expects {self.conv_in.in_channels} input channels, got {Cin}")
        # 1. time (unet.py:301-307): timesteps.expand(B) -> sinusoid -> MLP; SiLU(emb) feeds
        #    the batched time_emb_proj GEMM (fp32 out, added in the conv1 epilogues)
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep], device=dev)
        t = timestep.reshape(-1).to(device=dev, dtype=torch.float32)
        # the time-embedding MLP is independent of conv_in: with sc_concurrent it runs on the side
        # stream beside the input conversion and conv_in, joined before the first ResnetBlock2D
        side = self._side_stream(dev) if self.sc_concurrent and dev.type == "cuda" else None
        if side is not None:
            main = torch.cuda.current_stream(dev)
            side.wait_stream(main)
        with (torch.cuda.stream(side) if side is not None else contextlib.nullcontext()):
            temb_all = self._time_embedding(P, t, B, dt)
        # 3. conv_in (unet.py:357)
        if self.conv_in_fused and K.conv_in_ok(P["conv_in"], sources, B, H, W):
            x = K.conv_in(P["conv_in"], sources, B, H, W)                  # gather + conv in one launch
        else:
            x = K.nchw_to_nhwc(sources, P["cin_pad"], dt)
            x = K.conv2d(P["conv_in"], x, B, H, W, gn_stats=True)
        if side is not None:
            main.wait_stream(side)
            temb_all.record_stream(main)
        skips = [(x, H, W)]
        mb = self.mid_block
        nb = len(self.down_blocks)
        for bi, blk in enumerate(self.down_blocks):
            for j, r in enumerate(blk.resnets):
                # the GroupNorm that reads this resnet's output next (applied in its conv2's split-K
                # reduction where the plan splits: the 16x16 / 8x8 levels)
                if blk.has_cross_attention:
                    nxt = blk.attentions[j]
                elif j + 1 < len(blk.resnets):
                    nxt = blk.resnets[j + 1]
                elif blk.downsamplers is None:
                    nxt = mb.resnets[0] if bi + 1 == nb else self.down_blocks[bi + 1].resnets[0]
                else:
                    nxt = None
                x = self._resnet(P, r, (x, None), B, H, W, temb_all, gn_next=self._gn_next(P, nxt))
                if blk.has_cross_attention:
                    x = self._transformer(P, blk.attentions[j], x, B, H, W, encoder_hidden_states)
                skips.append((x, H, W))
            if blk.downsamplers is not None:
                nxt = self.down_blocks[bi + 1].resnets[0] if bi + 1 < nb else mb.resnets[0]
                x = K.conv2d(P[id(blk.downsamplers[0])], x, B, H, W, stride=2, gn_stats=True,
                             gn_next=self._gn_next(P, nxt))
                H, W = (H + 1) // 2, (W + 1) // 2
                skips.append((x, H, W))
        x = self._resnet(P, mb.resnets[0], (x, None), B, H, W, temb_all, gn_next=self._gn_next(P, mb.attentions[0]))
        x = self._transformer(P, mb.attentions[0], x, B, H, W, encoder_hidden_states)
        x = self._resnet(P, mb.resnets[1], (x, None), B, H, W, temb_all)
        for blk in self.up_blocks:
            for j, r in enumerate(blk.resnets):
                s, sh, sw = skips.pop()
                assert (sh, sw) == (H, W)
                # (the next resnet's norm1 reads [x || skip]: only a transformer's norm is applied early)
                nxt = blk.attentions[j] if blk.has_cross_attention else None
                x = self._resnet(P, r, (x, s), B, H, W, temb_all, gn_next=self._gn_next(P, nxt))  # cat read in place
                if blk.has_cross_attention:
                    x = self._transformer(P, blk.attentions[j], x, B, H, W, encoder_hidden_states)
            if blk.upsamplers is not None:
                x = K.conv2d(P[id(blk.upsamplers[0])], x, B, H, W, upsample=True, gn_stats=True)
                H, W = 2 * H, 2 * W
        G = self.conv_norm_out.num_groups
        if self.tail_fused and K.unet_tail_ok(x, B, H, W, G, P["conv_out"]):
            # conv_norm_out -> SiLU -> conv_out (-> the sampler's DDIM step) in one launch
            return K.unet_tail(x, B, H, W, G, *P["out_norm"], self.conv_norm_out.eps, P["conv_out"], dt, ddim=ddim,
                               want_eps=False)
        x = K.group_norm(x, B, H * W, G, *P["out_norm"], self.conv_norm_out.eps, K.ACT_SILU)
        return K.conv2d(P["conv_out"], x, B, H, W, out_layout=K.OUT_NCHW)

    @property
    def conv_in_fused(self):
        return getattr(self, "_conv_in_fused", True)

    def set_conv_in_fused(self, enabled=True):
        """bf16: run conv_in as one ldm_conv_in launch straight from the NCHW sources (default on); off
        runs ldm_nchw_to_nhwc + ldm_conv2d (A/B: same bf16 inputs, the conv within bf16 rounding)."""
        self._conv_in_fused = bool(enabled)

    @property
    def tail_fused(self):
        return getattr(self, "_tail_fused", True)

    def set_tail_fused(self, enabled=True):
        """bf16: run conv_norm_out -> SiLU -> conv_out (and, in forward_ddim_step, the DDIM step) as
        one ldm_unet_tail launch (default on); off runs ldm_group_norm + ldm_conv2d (+ ldm_ddim_step)."""
        self._tail_fused = bool(enabled)


class _UNetTrainFn(torch.autograd.Function):
    """Autograd node of one UNet forward (the drop-in path for the reference's
    ``loss.backward()``, trainers_ldm_cond.py:851-856): forward on the HIP kernels keeping the
    activations the hand-written backward (unet_train.UNetTrainGraph) needs; backward returns
    fp32 gradients for every trainable parameter."""

    @staticmethod
    def forward(ctx, unet, timestep, sample, *params):
        from .unet_train import UNetTrainGraph
        grads = {}

        def sink(p):
            g = grads.get(p)
            if g is None:
                g = grads[p] = torch.empty(p.shape, dtype=torch.float32, device=p.device)
                return g, False
            return g, True

        with torch.no_grad():
            graph = UNetTrainGraph(unet, sink)
            out = graph.forward([sample.detach()], timestep)
        ctx.graph, ctx.grads, ctx.params = graph, grads, params
        return out

    @staticmethod
    def backward(ctx, d_out):
        with torch.no_grad():
            ctx.graph.backward(d_out.to(ctx.graph.u.compute_dtype).contiguous())
        gs = []
        for p in ctx.params:
            g = ctx.grads.get(p)
            gs.append(None if g is None else g.to(p.dtype))
        ctx.graph = None
        return (None, None, None, *gs)


def _remap_legacy_keys(sd):
    """Older diffusers checkpoints name the attention output projection ``to_out.0`` already;
    the pre-0.14 ``attentions.*.query/key/value/proj_attn`` names only occur in VAE mid blocks,
    which are not part of this UNet.  Kept as the single place to add remaps."""
    return sd
