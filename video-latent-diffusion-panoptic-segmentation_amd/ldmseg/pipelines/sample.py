"""Full sampling for one clip (BASELINE config 4; TrainerDiffusion.compute_pq's per-batch body,
trainers_ldm_cond.py:1222-1330): RGB encode -> DDIM denoise -> seg-VAE decode -> panoptic head,
every stage on the HIP kernels, nothing leaving the GPU but each frame's surviving segment ids."""
import torch

from . import sample_latents
from .latents import decode_latents, encode_inputs
from .panoptic import postprocess_panoptic


@torch.no_grad()
def sample_panoptic(rgb_images, vae_image, vae_semseg, unet, scheduler, *, rgb_size=192, latent_size=64,
                    num_inference_steps=50, seed=0, self_condition=False, mask_th=0.5, count_th=512,
                    overlap_th=0.5, ignore_label=255, threshold_output=True, threshold_mode="max",
                    padding_masks=None, orig_sizes=None, use_graph=True, stepper=None):
    """rgb_images fp32 [B, 3, H, W] in [0, 1] (GPU; B = the T frames of a clip) -> per frame
    {"panoptic_seg": (ids [h, w] int64, segments_info), "cleaned_pred": ...}.
    ``stepper``: a prepared DenoiseStep to reuse (its HIP graph) across clips of one shape."""
    B, _, H, W = rgb_images.shape
    rgb_latents, _ = encode_inputs(rgb_images, vae_image.encode, vae_image.scaling_factor, latent_size,
                                   resize=rgb_size, weight_dtype=vae_image.dtype)          # :1230-1236
    if stepper is not None:
        stepper.rgb.copy_(rgb_latents)
    latents = sample_latents(unet, scheduler, rgb_latents, num_inference_steps, seed, self_condition,
                             use_graph=use_graph, stepper=stepper)                        # :1240-1250
    logits = decode_latents(vae_semseg, latents, return_logits=True, weight_dtype=vae_semseg.dtype)  # :1253-1259
    if padding_masks is None:
        padding_masks = torch.ones(B, H, W, dtype=torch.bool, device=rgb_images.device)
    if orig_sizes is None:
        orig_sizes = [(H, W)] * B
    return postprocess_panoptic(logits, (H, W), padding_masks, orig_sizes, mask_th, count_th, overlap_th,
                                ignore_label, threshold_output, threshold_mode)          # :1262-1330
