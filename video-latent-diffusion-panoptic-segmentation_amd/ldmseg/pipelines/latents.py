"""encode_inputs / decode_latents of TrainerDiffusion on the HIP path (rows a12, a13, f3).

encode_inputs (trainers_ldm_cond.py:336-396): bilinear resize of the input (align_corners=False)
fused with the ``2x - 1`` affine (one ldm_resize_bilinear launch), encode, mode() (or
sample()), bilinear resize of the latent to L x L fused with the ``* scaling_factor``.
decode_latents (:398-444): z / scaling_factor, the seg-VAE decode (with its x2 bilinear), and
either the logits or the argmax / confidence-thresholded predictions (ldm_panoptic_pixels).
The RGB latents come from GeneralVAEImage.encode, the segmentation latents from
GeneralVAESeg.encode — the same encode_func contract as the reference.
"""
import numpy as np
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


def color_map(N=256, normalized=False):
    """The PASCAL colour map of ldmseg/utils/utils.py:240-258 (bit i of the label goes to bit
    7 - i//3 of channel i % 3)."""
    ids = np.arange(N)
    cmap = np.zeros((N, 3), dtype=np.int64)
    c = ids.copy()
    for j in range(8):
        for ch in range(3):
            cmap[:, ch] |= ((c >> ch) & 1) << (7 - j)
        c = c >> 3
    return cmap.astype(np.float32) / 255 if normalized else cmap.astype(np.uint8)


_CMAP = {}


def encode_seg(predictions):
    """TrainerDiffusion.encode_seg (trainers_ldm_cond.py:326-334): int label maps [B, H, W]
    -> colour images uint8 [B, H, W, 3] (labels taken mod 256, as ``astype(np.uint8)``).  The
    table lookup runs on the predictions' device; the result is a host numpy array, as the
    reference returns."""
    dev = predictions.device
    if dev not in _CMAP:
        _CMAP[dev] = torch.from_numpy(color_map()).to(dev)
    return _CMAP[dev][(predictions & 255).long()].cpu().numpy()


@torch.no_grad()
def decode_latents(vae_semseg, latents, return_logits=False, threshold_output=False, mask_th=0.5, ignore_label=255,
                   weight_dtype=torch.float32, return_predictions=False):
    """decode_latents (trainers_ldm_cond.py:398-444).  return_logits: fp32 logits [B, K, H, W]
    (GPU).  Otherwise the reference's output: argmax (+ ignore_label where the max softmax
    probability < mask_th when threshold_output) colour-mapped to uint8 numpy [B, H, W, 3]; a
    3-channel decoder gives the (x/2 + 0.5) uint8 image.  return_predictions=True (an opt-in
    this build adds) returns the int64 label map [B, H, W] on the GPU instead of its colours."""
    z = K.resize_bilinear(latents.float(), size=tuple(latents.shape[-2:]), mul=1.0 / vae_semseg.scaling_factor,
                          out_dtype=weight_dtype)
    images = vae_semseg.decode(z).float()
    if return_logits:
        return images
    if images.shape[1] == 3:
        img = (images / 2 + 0.5).clamp(0, 1)
        return (img.cpu().permute(0, 2, 3, 1).numpy() * 255).astype(np.uint8)
    pred = threshold_predictions(images, mask_th, ignore_label, threshold_output)
    if return_predictions:
        return pred
    return encode_seg(pred)
