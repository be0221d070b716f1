"""DVPQ output format and multi-rank accumulation.

- ``write_dvpq_frame`` writes the two PNGs per frame that eval/eval_dvpq.py consumes unchanged:
  ``<pan_dir>/<stem>cat.png`` (category ids, 255 = void) and ``<pan_dir>/<stem>ins.png``
  (instance ids); the script sorts both lists lexicographically (:170-176) and pairs them with
  the sorted ``video_sequence/val/*gtFine_class*`` files, and reads id = cat * 2**20 + ins
  (:105-110).  Choose stems that sort in frame order (e.g. ``f"{seq:06d}_{frame:06d}_"``).
- ``reduce_pq_accumulators`` is the one collective of the sampling path: the per-class
  (iou, tp, fn, fp) sums of eval_dvpq.py:186-189, all-reduced over the ranks that each
  evaluated their own clips (the reference has no such step; it evaluates on one process).
- ``dvpq_summary`` is the script's final formula (:190-205).
"""
import os

import numpy as np
import torch


def write_dvpq_frame(pan_dir, stem, cat, ins):
    """cat / ins: integer [H, W] arrays or tensors (cat in [0, 255], ins >= 0)."""
    from PIL import Image

    cat = cat.cpu().numpy() if torch.is_tensor(cat) else np.asarray(cat)
    ins = ins.cpu().numpy() if torch.is_tensor(ins) else np.asarray(ins)
    if cat.shape != ins.shape or cat.ndim != 2:
        raise ValueError("cat and ins must be [H, W] of one shape")
    if cat.min() < 0 or cat.max() > 255:
        raise ValueError("category ids must lie in [0, 255] (uint8 PNG)")
    if ins.min() < 0 or ins.max() >= 2 ** 16:
        raise ValueError("instance ids must lie in [0, 65535]")
    os.makedirs(pan_dir, exist_ok=True)
    Image.fromarray(cat.astype(np.uint8)).save(os.path.join(pan_dir, f"{stem}cat.png"))
    ins_img = Image.fromarray(ins.astype(np.uint8)) if ins.max() < 256 else Image.fromarray(ins.astype(np.uint16))
    ins_img.save(os.path.join(pan_dir, f"{stem}ins.png"))


def panoptic_to_dvpq(cleaned, category=0, dropped_category=19):
    """compute_pq's class-agnostic output (cleaned_pred: segment label >= 0, -1 = dropped,
    trainers_ldm_cond.py:1302-1326, every segment ``category_id`` 1) -> the (cat, ins) pair of a
    DVPQ prediction: kept pixels get ``category`` and instance = label + 1 (its panoptic id);
    dropped pixels get ``dropped_category`` with instance 0 — 19, the category eval_dvpq.py
    itself gives predictions it discards (:143), since a predicted category 255 would index past
    its 20 per-class accumulators (:98-99)."""
    c = cleaned.cpu().numpy() if torch.is_tensor(cleaned) else np.asarray(cleaned)
    keep = c >= 0
    return np.where(keep, category, dropped_category), np.where(keep, c + 1, 0)


def reduce_pq_accumulators(iou, tp, fn, fp, group=None):
    """Sum the per-class accumulators over all ranks (float64; returns four numpy arrays).
    Uses the process group's device: CUDA tensors for nccl (RCCL), host tensors for gloo."""
    import torch.distributed as dist

    acc = torch.from_numpy(np.stack([np.asarray(a, np.float64) for a in (iou, tp, fn, fp)]))
    if dist.is_available() and dist.is_initialized():
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
        t = acc.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        acc = t.cpu()
    a = acc.numpy()
    return a[0], a[1], a[2], a[3]


def dvpq_summary(iou, tp, fn, fp, num_things=8, num_classes=19, eps=1e-10):
    """(PQ, things PQ, stuff PQ) in percent, exactly as eval_dvpq.py:190-205 prints them."""
    iou, tp, fn, fp = (np.asarray(a, np.float64)[:num_classes] for a in (iou, tp, fn, fp))
    sq = iou / (tp + eps)
    rq = tp / (tp + 0.5 * fn + 0.5 * fp + eps)
    pq = sq * rq
    mean = lambda a: a.mean() * 100 if a.size else float("nan")     # noqa: E731
    return mean(pq), mean(pq[:num_things]), mean(pq[num_things:])
