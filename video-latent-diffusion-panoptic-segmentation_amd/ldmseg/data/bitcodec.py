"""Bit-channel mask codec on the GPU (bit-exact with the reference).

Reference: Cityscapes.encode_bitmap / decode_bitmap, ldmseg/data/cityscapes.py:256-270
(identical copies kitti.py:292-306, dataset/semKITTI_dataset.py:152-166; coco.py:378-391
without the 31 -> 0 quirk).  The reference runs it per sample in DataLoader workers on the
CPU; here it is one HIP kernel over a whole [B, H, W] batch already in HBM.
"""
import torch

from ..ops import native as K


def encode_bitmap(x: torch.Tensor, n: int = 5, fill_value: float = 0.5, ignore_label: int = 255):
    """ids [..., H, W] -> (planes fp32 [..., n, H, W], ignore_mask bool [..., H, W])."""
    return K.bit_encode(x.to(torch.int64), n, ignore_label, fill_value)


def decode_bitmap(x: torch.Tensor, n: int = 5, drop_31: bool = True):
    """planes [..., n, H, W] -> ids int64 [..., H, W]: sum_i [x_i > 0] 2^i (then 31 -> 0).

    Like the reference, the bit count is taken from the planes tensor, not from ``n``."""
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return K.bit_decode(x, drop_31=drop_31)


class BitmapCodecMixin:
    """Gives a dataset the reference's method signatures (self.ignore_label is used)."""

    decode_drops_31 = True

    def encode_bitmap(self, x: torch.Tensor, n: int = 5, fill_value: float = 0.5):
        return encode_bitmap(x, n, fill_value, self.ignore_label)

    def decode_bitmap(self, x: torch.Tensor, n: int = 5):
        return decode_bitmap(x, n, self.decode_drops_31)
