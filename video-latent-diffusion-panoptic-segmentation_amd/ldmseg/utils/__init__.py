"""Utilities the reference's trainers touch on the hot path (ldmseg/utils/utils.py)."""
from collections import OrderedDict

import torch
import torch.distributed as dist


class OutputDict(OrderedDict):
    """OrderedDict whose items are also attributes (ldmseg/utils/utils.py:26-31)."""

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        super().__setattr__(key, value)

    def __setattr__(self, key, value):
        super().__setitem__(key, value)
        super().__setattr__(key, value)


def is_dist_avail_and_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_world_size() -> int:
    return dist.get_world_size() if is_dist_avail_and_initialized() else 1


def get_rank() -> int:
    return dist.get_rank() if is_dist_avail_and_initialized() else 0


def is_main_process() -> bool:
    return get_rank() == 0


def gpu_gather(tensor: torch.Tensor) -> torch.Tensor:
    """all_gather along dim 0 (ldmseg/utils/utils.py:76-81)."""
    if tensor.ndim == 0:
        tensor = tensor.clone()[None]
    out = [torch.empty_like(tensor) for _ in range(get_world_size())]
    dist.all_gather(out, tensor.contiguous())
    return torch.cat(out, dim=0)
