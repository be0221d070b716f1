"""Panoptic head of TrainerDiffusion.compute_pq — numpy/torch-CPU restatement (test infrastructure
only, see oracle/__init__.py).

Follows ldmseg/trainers/trainers_ldm_cond.py:
  :1276-1281  F.interpolate(masks_logits, size=image size, bilinear, align_corners=False)
  :1287-1296  crop_padding (:1175-1181: bounding box of the padding mask), interpolate to the
              original size, argmax, softmax-max (or top1 - top2) < mask_th -> ignore_label
  :1299-1330  sigmoid; per unique label: drop (-> -1) if count < count_th or label in
              {-1, ignore_label}, or count / #(sigmoid >= mask_th) < overlap_th; keep otherwise
Pinned by tests/golden/panoptic.npz (the reference method run on a stand-in trainer).
"""
import numpy as np
import torch
import torch.nn.functional as F


def head(logits, mask_th, count_th, overlap_th, ignore_label, threshold_output=True, threshold_mode="max"):
    """logits fp32 [K, H, W] (torch CPU) -> cleaned_pred int64 [H, W] (-1 = dropped)."""
    pred = torch.argmax(logits, dim=0)
    if threshold_output:
        probs = F.softmax(logits, dim=0)
        if threshold_mode == "topk_diff":
            tk = torch.topk(probs, k=2, dim=0)
            probs = tk.values[0] - tk.values[1]
        else:
            probs = probs.max(dim=0)[0]
        pred[probs < mask_th] = ignore_label
    pred = pred.numpy()
    sig = torch.sigmoid(logits).numpy()
    cleaned = pred.copy()
    for lab, cnt in zip(*np.unique(pred, return_counts=True)):
        if cnt < count_th or lab in {-1, ignore_label}:
            cleaned[cleaned == lab] = -1
            continue
        with np.errstate(divide="ignore", invalid="ignore"):
            ratio = (pred == lab).sum() / (sig[lab] >= mask_th).sum()
        if ratio < overlap_th:
            cleaned[cleaned == lab] = -1
    return cleaned


def postprocess(masks_logits, image_hw, padding_masks, orig_sizes, **kw):
    """[B, K, Hd, Wd] decoder logits -> list of cleaned_pred [h, w] per image (:1276-1330)."""
    x = F.interpolate(masks_logits, size=tuple(image_hw), mode="bilinear", align_corners=False)
    outs = []
    for i in range(x.shape[0]):
        co = padding_masks[i].nonzero()
        y0, y1 = co[:, 0].min(), co[:, 0].max()
        x0, x1 = co[:, 1].min(), co[:, 1].max()
        m = x[i][:, y0:y1 + 1, x0:x1 + 1]
        m = F.interpolate(m[None].float(), size=tuple(orig_sizes[i]), mode="bilinear", align_corners=False)[0]
        outs.append(head(m, **kw))
    return outs
