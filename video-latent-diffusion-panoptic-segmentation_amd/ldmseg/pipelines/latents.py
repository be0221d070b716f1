"""encode_inputs / decode_latents of TrainerDiffusion on the HIP path (rows a12, a13, f3).

encode_inputs (trainers_ldm_cond.py:336-396): bilinear resize of the input (align_corners=False)
fused with the ``2x - 1`` affine (one ldm_resize_bilinear launch), encode, mode() (or
sample()), bilinear resize of the latent to L x L fused with the ``* scaling_factor``.
decode_latents (:398-444): z / scaling_factor, the seg-VAE decode (with its x2 bilinear), and
either the logits or the argmax / confidence-thresholded predictions (ldm_panoptic_pixels).
The RGB latents come from GeneralVAEImage.encode, the segmentation latents from
GeneralVAESeg.encode — the same encode_func contract as the reference.
"""
import torch

from ..ops import native as K
from .panoptic import threshold_predictions


@torch.no_grad()
def encode_inputs(images, encode_func, scaling_factor, latent_size, resize=(192, 640), sample_posterior=False,
                  weight_dtype=torch.float32, generator=None):
    """images fp32 NCHW in [0, 1] (GPU) -> (latents, latents_mean) fp32 [B, Lc, L, L]."""
    if isinstance(resize, int):
        resize = (resize, resize)
    x = K.resize_bilinear(images.float(), size=tuple(resize), mul=2.0, add=-1.0, out_dtype=weight_dtype) \
        if resize is not None else (2.0 * images - 1.0).to(weight_dtype)
    dist = encode_func(x).latent_dist
    mean = dist.mode().float()
    lat = dist.sample(generator=generator).float() if sample_posterior else mean
    ls = (latent_size, latent_size) if isinstance(latent_size, int) else tuple(latent_size)
    if resize is not None:
        latents = K.resize_bilinear(lat, size=ls, mul=scaling_factor)
        means = latents if not sample_posterior else K.resize_bilinear(mean, size=ls, mul=scaling_factor)
    else:
        latents = K.resize_bilinear(lat, size=tuple(lat.shape[-2:]), mul=scaling_factor)
        means = latents if not sample_posterior else K.resize_bilinear(mean, size=tuple(mean.shape[-2:]),
                                                                        mul=scaling_factor)
    return latents, (latents.clone() if not sample_posterior else means)


@torch.no_grad()
def decode_latents(vae_semseg, latents, return_logits=False, threshold_output=False, mask_th=0.5, ignore_label=255,
                   weight_dtype=torch.float32):
    """-> logits fp32 [B, K, H, W] (return_logits) or int64 predictions [B, H, W] (the input of
    the reference's encode_seg colour map, :433-437)."""
    z = K.resize_bilinear(latents.float(), size=tuple(latents.shape[-2:]), mul=1.0 / vae_semseg.scaling_factor,
                          out_dtype=weight_dtype)
    images = vae_semseg.decode(z).float()
    if return_logits:
        return images
    return threshold_predictions(images, mask_th, ignore_label, threshold_output)
