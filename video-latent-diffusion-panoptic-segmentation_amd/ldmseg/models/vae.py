"""Drop-in ``GeneralVAESeg`` (ldmseg/models/vae.py:42-307) on the HIP kernels.

Module tree = the reference's nn.Sequential indices (encoder.<i>, decoder.<i>), so AE
checkpoints load strictly (vae.py:117-122).  encode/decode run NHWC through ldm_conv2d
(implicit GEMM; the SiLU after a conv is fused into its epilogue, the ConvTranspose k2s2 is a
GEMM with a pixel-shuffle epilogue), ldm_layer_norm (LayerNorm2d + SiLU), ldm_group_norm
(+SiLU), ldm_gaussian_posterior and ldm_resize_bilinear.  Supported: parametrization
'gaussian' / 'auto', resize_input=False, num_mid_blocks=0, skip_encoder=False (the
configurations of base.yaml and the KITTI AE); the codebook/gumbel posteriors
(vae.py:428-570) are off the path.
"""
from typing import Optional, Tuple, Union

import torch
import torch.nn as nn

from ..ops import native as K
from ..utils import OutputDict


class RangeDict(OutputDict):
    min: torch.Tensor
    max: torch.Tensor


class VAEOutput(OutputDict):
    sample: torch.Tensor
    posterior: torch.Tensor


class EncoderOutput(OutputDict):
    latent_dist: torch.Tensor


class LayerNorm2d(nn.Module):
    """Channel LayerNorm on NCHW (vae.py:310-323); executed by ldm_layer_norm on NHWC rows."""

    def __init__(self, num_channels: int, eps: float = 1e-6) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.ones(num_channels))
        self.bias = nn.Parameter(torch.zeros(num_channels))
        self.eps = eps


class DiagonalGaussianDistribution(object):
    """vae.py:371-425, with mean/logvar/std/var produced by one HIP kernel from the moments."""

    def __init__(self, parameters: torch.Tensor, clamp_output: bool = False, act_fn: str = "none"):
        self.parameters = parameters
        self.mean, self.logvar, self.std, self.var = K.gaussian_posterior(parameters, clamp_output, act_fn)
        if parameters.dtype != torch.float32:
            self.mean, self.logvar, self.std, self.var = (t.to(parameters.dtype) for t in
                                                          (self.mean, self.logvar, self.std, self.var))
        self.clamp_output = clamp_output
        self.act_fn = act_fn

    def mode(self):
        return self.mean

    def sample(self, generator: Optional[torch.Generator] = None) -> torch.FloatTensor:
        noise = torch.randn(self.mean.shape, generator=generator, device=self.parameters.device,
                            dtype=self.parameters.dtype)
        return self.mean + self.std * noise

    def kl(self):
        return 0.5 * torch.sum(torch.pow(self.mean, 2) + self.var - 1.0 - self.logvar, dim=[1, 2, 3])

    def get_range(self):
        return RangeDict(min=self.mean.min(), max=self.mean.max())


class Bottleneck(object):
    """parametrization='auto' (vae.py:326-368)."""

    def __init__(self, parameters: torch.Tensor, act_fn: str = "none"):
        self.parameters = parameters
        self.mean, _, _, _ = K.gaussian_posterior(torch.cat([parameters, parameters], 1), False,
                                                  act_fn if act_fn != "clip" else "none")
        if act_fn == "clip":
            self.mean = self.mean.clamp(-5.0, 5.0)
        self.mean = self.mean.to(parameters.dtype)
        self.act_fn = act_fn

    def mode(self):
        return self.mean

    def sample(self, generator=None):
        return self.mean

    def kl(self):
        return torch.sum(torch.pow(self.mean, 2), dim=[1, 2, 3])


class GeneralVAESeg(nn.Module):
    def __init__(self, in_channels: int = 3, int_channels: int = 256, out_channels: int = 19,
                 block_out_channels: Tuple[int] = (32, 64, 128, 256), latent_channels: int = 4,
                 norm_num_groups: int = 32, scaling_factor: float = 0.18215, pretrained_path: Optional[str] = None,
                 encoder: Optional[nn.Module] = None, num_mid_blocks: int = 0, num_latents: int = 2,
                 num_upscalers: int = 1, upscale_channels: int = 256, parametrization: str = "gaussian",
                 fuse_rgb: bool = False, resize_input: bool = False, act_fn: str = "none",
                 clamp_output: bool = False, freeze_codebook: bool = False, skip_encoder: bool = False) -> None:
        super().__init__()
        if num_mid_blocks > 0 or resize_input or skip_encoder or "discrete" in parametrization:
            raise NotImplementedError("mid blocks / resize_input / skip_encoder / discrete posteriors are not on "
                                      "the accelerated path (base.yaml uses none of them)")
        assert parametrization in ["gaussian", "auto"]
        if parametrization == "auto":
            num_latents = 1
        self.enable_mid_block = False
        self.num_mid_blocks = 0
        self.downsample_factor = 2 ** (len(block_out_channels) - 1)
        self.norm_num_groups = norm_num_groups
        self.latent_channels = latent_channels
        if encoder is None:
            if fuse_rgb:
                in_channels += 3
            self.define_encoder(in_channels, block_out_channels, int_channels, norm_num_groups, latent_channels,
                                num_latents)
        else:
            self.encoder = encoder
            self.encoder.requires_grad_(False)
        self.define_decoder(out_channels, int_channels, norm_num_groups, latent_channels, num_upscalers,
                            upscale_channels)
        self.scaling_factor = scaling_factor
        self.gradient_checkpoint = False
        self.parametrization = parametrization
        self.interpolation_factor = self.downsample_factor // (2 ** num_upscalers)
        self.num_latents = num_latents
        self.act_fn = act_fn
        self.clamp_output = clamp_output
        self.in_channels = in_channels
        self._plan = None
        self._plan_key = None
        if pretrained_path is not None:
            self.load_pretrained(pretrained_path)

    # ------------------------------------------------------------ structure (reference indices)
    def define_decoder(self, num_classes, int_channels=256, norm_num_groups=32, latent_channels=4,
                       num_upscalers=1, upscale_channels=256):
        dim = upscale_channels
        ups = []
        for i in range(num_upscalers):
            ups += [nn.ConvTranspose2d(int_channels if i == 0 else dim, dim, kernel_size=2, stride=2),
                    LayerNorm2d(dim), nn.SiLU()]
        ups += [nn.GroupNorm(norm_num_groups, dim), nn.SiLU(), nn.Conv2d(dim, num_classes, 3, padding=1)]
        self.decoder = nn.Sequential(nn.Conv2d(latent_channels, int_channels, kernel_size=3, padding=1),
                                     nn.Identity(), *ups)

    def define_encoder(self, in_channels, block_out_channels, int_channels=256, norm_num_groups=32,
                       latent_channels=4, num_latents=2):
        layers = [nn.Conv2d(in_channels, block_out_channels[0], kernel_size=3, padding=1), nn.SiLU()]
        for i in range(len(block_out_channels) - 1):
            ci, co = block_out_channels[i], block_out_channels[i + 1]
            layers += [nn.Conv2d(ci, ci, kernel_size=3, padding=1),
                       nn.Conv2d(ci, co, kernel_size=3, padding=1, stride=2), nn.SiLU()]
        layers += [nn.Conv2d(block_out_channels[-1], int_channels, kernel_size=3, padding=1), nn.Identity(),
                   nn.GroupNorm(num_channels=int_channels, num_groups=norm_num_groups, eps=1e-6), nn.SiLU(),
                   nn.Conv2d(int_channels, latent_channels * num_latents, 3, padding=1)]
        self.encoder = nn.Sequential(*layers)

    def enable_gradient_checkpointing(self):
        raise NotImplementedError("Gradient checkpointing not implemented for a shallow VAE")

    def load_pretrained(self, pretrained_path):
        data = torch.load(pretrained_path, map_location="cpu", weights_only=True)
        sd = {k.replace("module.", ""): v for k, v in data["vae"].items()}
        self.load_state_dict(sd, strict=True)

    def freeze_layers(self):
        raise NotImplementedError

    def freeze_encoder(self):
        self.encoder.requires_grad_(False)

    @property
    def dtype(self):
        return next(self.parameters()).dtype

    # ------------------------------------------------------------ HIP plans
    @staticmethod
    def _fuse(seq, dt, cin_pad):
        """Turn an nn.Sequential into fused HIP steps: conv(+SiLU) / convT+LN2d(+SiLU) / GN(+SiLU)."""
        steps, mods, i = [], list(seq), 0
        first = True
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            silu = isinstance(nxt, nn.SiLU)
            if isinstance(m, nn.Conv2d):
                pc = K.PackedConv(m.weight, m.bias, dt, cin_pad=cin_pad if first else None)
                steps.append(("conv", pc, m.stride[0], K.ACT_SILU if silu else K.ACT_NONE))
                first = False
            elif isinstance(m, nn.ConvTranspose2d):
                steps.append(("convT", K.PackedConv(m.weight, m.bias, dt, shuffle2=True)))
                silu = False
            elif isinstance(m, LayerNorm2d):
                steps.append(("ln", m.weight.detach().float().contiguous(), m.bias.detach().float().contiguous(),
                              m.eps, K.ACT_SILU if silu else K.ACT_NONE))
            elif isinstance(m, nn.GroupNorm):
                steps.append(("gn", m.num_groups, m.weight.detach().float().contiguous(),
                              m.bias.detach().float().contiguous(), m.eps, K.ACT_SILU if silu else K.ACT_NONE))
            elif isinstance(m, (nn.Identity, nn.SiLU)):
                silu = False
            else:
                raise NotImplementedError(f"{type(m).__name__} in the VAE stack")
            i += 2 if silu else 1
        return steps

    def prepare(self, force=False):
        key = (self.dtype, next(self.parameters()).device) + tuple((p.data_ptr(), p._version)
                                                                   for p in self.parameters())
        if not force and self._plan is not None and self._plan_key == key:
            return self._plan
        dt = self.dtype
        if dt not in (torch.float32, torch.bfloat16):
            raise TypeError(f"GeneralVAESeg HIP path runs in float32 or bfloat16, not {dt}")
        enc_in = self.encoder[0].in_channels
        dec_in = self.decoder[0].in_channels
        self._enc_pad = (enc_in + 7) // 8 * 8
        self._dec_pad = (dec_in + 7) // 8 * 8
        self._plan = (self._fuse(self.encoder, dt, self._enc_pad), self._fuse(self.decoder, dt, self._dec_pad))
        self._plan_key = key
        return self._plan

    @staticmethod
    def _run(steps, x, B, H, W, last_nchw):
        for si, st in enumerate(steps):
            last = si == len(steps) - 1
            if st[0] == "conv":
                _, pc, stride, act = st
                layout = K.OUT_NCHW if (last and last_nchw) else K.OUT_NHWC
                x = K.conv2d(pc, x, B, H, W, stride=stride, act=act, out_layout=layout)
                if stride == 2:
                    H, W = (H + 1) // 2, (W + 1) // 2
            elif st[0] == "convT":
                x = K.conv2d(st[1], x, B, H, W, out_layout=K.OUT_SHUFFLE2)
                H, W = 2 * H, 2 * W
            elif st[0] == "ln":
                x = K.layer_norm(x, st[1], st[2], st[3], st[4])
            elif st[0] == "gn":
                x = K.group_norm(x, B, H * W, st[1], st[2], st[3], st[4], st[5])
        return x, H, W

    @torch.no_grad()
    def encode_moments(self, semseg):
        enc, _ = self.prepare()
        B, C, H, W = semseg.shape
        x = K.nchw_to_nhwc([semseg], self._enc_pad, self.dtype)
        moments, _, _ = self._run(enc, x, B, H, W, last_nchw=True)
        return moments

    def encode(self, semseg):                                                # vae.py:253-266
        moments = self.encode_moments(semseg)
        if self.parametrization == "gaussian":
            post = DiagonalGaussianDistribution(moments, clamp_output=self.clamp_output, act_fn=self.act_fn)
        else:
            post = Bottleneck(moments, act_fn=self.act_fn)
        return EncoderOutput(latent_dist=post)

    @torch.no_grad()
    def decode(self, z, interpolate=True):                                   # vae.py:268-272
        _, dec = self.prepare()
        B, C, H, W = z.shape
        x = K.nchw_to_nhwc([z], self._dec_pad, self.dtype)
        logits, _, _ = self._run(dec, x, B, H, W, last_nchw=True)
        if interpolate:
            logits = K.resize_bilinear(logits, scale_factor=self.interpolation_factor)
        return logits

    def forward(self, sample: torch.FloatTensor, sample_posterior: bool = True, return_dict: bool = True,
                generator: Optional[torch.Generator] = None, rgb_sample: Optional[torch.FloatTensor] = None,
                valid_mask: Optional[torch.FloatTensor] = None) -> Union[VAEOutput, torch.FloatTensor]:
        x = sample if rgb_sample is None else torch.cat([sample, rgb_sample], dim=1)
        posterior = self.encode(x).latent_dist
        z = posterior.sample(generator=generator) if sample_posterior else posterior.mode()
        if valid_mask is not None:
            z = z * valid_mask[:, None]
        dec = self.decode(z, interpolate=False)
        if not return_dict:
            return (dec,)
        return VAEOutput(sample=dec, posterior=posterior)
