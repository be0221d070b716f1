"""Bit-channel mask codec — numpy restatement (test infrastructure only, see oracle/__init__.py).

Follows ldmseg/data/cityscapes.py:256-270 (identical copies: kitti.py:292-306,
dataset/semKITTI_dataset.py:152-166; coco.py:378-391 lacks the 31 -> 0 quirk).
"""
import numpy as np


def encode_bitmap(ids: np.ndarray, n: int, ignore_label: int, fill_value: float = 0.5):
    """ids [H,W] int -> (planes [n,H,W] float32, ignore_mask [H,W] bool).

    plane_i = (ids >> i) mod 2 (floor-mod, so negative ids give 1 bits like torch.remainder);
    every plane is set to ``fill_value`` where ids == ignore_label   (cityscapes.py:257-260).
    """
    ids = np.asarray(ids, dtype=np.int64)
    ignore = ids == ignore_label
    shifts = np.arange(n, dtype=np.int64)[:, None, None]
    planes = np.mod(np.right_shift(ids[None], shifts), 2).astype(np.float32)
    planes[:, ignore] = np.float32(fill_value)
    return planes, ignore


def decode_bitmap(planes: np.ndarray, drop_31: bool = True):
    """planes [n,H,W] float -> ids [H,W] int64:  sum_i [x_i > 0] 2^i, then 31 -> 0
    (cityscapes.py:263-270; ``drop_31=False`` gives the coco.py:386-391 variant)."""
    planes = np.asarray(planes)
    n = planes.shape[0]
    weights = (2 ** np.arange(n, dtype=np.int64))[:, None, None]
    v = ((planes > 0).astype(np.int64) * weights).sum(axis=0).astype(np.int64)
    if drop_31:
        v[v == 31] = 0
    return v
