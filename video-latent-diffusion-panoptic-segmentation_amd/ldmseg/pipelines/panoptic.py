"""Panoptic head of the sampling path on the HIP kernels.

Drop-in for the per-image CPU loop of TrainerDiffusion.compute_pq
(ldmseg/trainers/trainers_ldm_cond.py:1276-1330) and for the argmax / confidence threshold
of decode_latents (:426-435).  Everything stays on the GPU: the two bilinear resamples
(ldm_resize_bilinear), the argmax + confidence threshold + per-label histograms
(ldm_panoptic_pixels) and the segment filter + relabel (ldm_panoptic_finalize); only the
per-image list of surviving segment ids crosses to the host.
"""
import torch

from ..ops import native as K


def panoptic_head(logits, mask_th, count_th, overlap_th, ignore_label, threshold_output=True,
                  threshold_mode="max"):
    """logits fp32 [B, K, H, W] (GPU) -> (cleaned int64 [B, H, W] with -1 = dropped, keep bool [B, K]).

    ``cleaned`` is the reference's ``cleaned_pred`` (:1302-1317) for every image; ``cleaned + 1``
    is its ``panoptic_seg`` and ``keep`` lists the labels of ``segments_info``."""
    if threshold_mode not in ("max", "topk_diff"):
        raise ValueError(f"threshold_mode {threshold_mode!r}")
    mode = threshold_mode if threshold_output else "none"
    pred, counts, mcounts = K.panoptic_pixels(logits.float(), mask_th, ignore_label, mode)
    out, keep = K.panoptic_finalize(pred, counts, mcounts, count_th, overlap_th, ignore_label)
    return out.long() - 1, keep.bool()


def segments_info(keep_row):
    """[K] bool -> the reference's segments_info list (:1320-1326), ids ascending."""
    return [{"id": int(k) + 1, "category_id": 1, "isthing": True}
            for k in torch.nonzero(keep_row).flatten().tolist()]


def _crop_box(padding_mask):
    """crop_padding's bounding box (:1175-1181) of the nonzero padding-mask pixels."""
    rows = torch.nonzero(padding_mask.any(1)).flatten()
    cols = torch.nonzero(padding_mask.any(0)).flatten()
    return int(rows[0]), int(rows[-1]) + 1, int(cols[0]), int(cols[-1]) + 1


def postprocess_panoptic(masks_logits, image_hw, padding_masks, orig_sizes, mask_th, count_th, overlap_th,
                         ignore_label, threshold_output=True, threshold_mode="max"):
    """compute_pq's per-batch post-processing (:1276-1330) on the GPU.

    masks_logits fp32 [B, K, Hd, Wd] (decode_latents(return_logits=True)); image_hw = the RGB
    input size; padding_masks [B, Hi, Wi]; orig_sizes [(h, w)] per image.  Returns, per image,
    ``{"panoptic_seg": (cleaned + 1, segments_info), "cleaned_pred": cleaned}`` (GPU int64)."""
    x = K.resize_bilinear(masks_logits.float(), size=tuple(image_hw))
    results = []
    for i in range(x.shape[0]):
        y0, y1, x0, x1 = _crop_box(padding_masks[i])
        m = x[i:i + 1, :, y0:y1, x0:x1]
        m = K.resize_bilinear(m, size=tuple(orig_sizes[i]))
        cleaned, keep = panoptic_head(m, mask_th, count_th, overlap_th, ignore_label, threshold_output,
                                      threshold_mode)
        results.append({"panoptic_seg": (cleaned[0] + 1, segments_info(keep[0])), "cleaned_pred": cleaned[0]})
    return results


def threshold_predictions(images, mask_th, ignore_label, threshold_output=True):
    """decode_latents' non-logit branch (:426-435): argmax over channels, ignore_label where the
    max softmax probability is < mask_th.  images fp32 [B, K, H, W] (GPU) -> int64 [B, H, W]."""
    pred, _, _ = K.panoptic_pixels(images.float(), mask_th, ignore_label, "max" if threshold_output else "none")
    return pred.long()
