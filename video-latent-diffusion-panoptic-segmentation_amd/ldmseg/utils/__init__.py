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


# ------------------------------------------------------------------ multi-GPU sampling
# Denoising shards with no exchange: each rank samples its own clips, the
# way the reference's DistributedSampler splits the validation set
# (trainers_ldm_cond.py:245-247); the only collectives are the timing max and the final sum
# of per-class PQ accumulators.
def distributed_sampler_indices(n: int, rank: int, world: int, shuffle: bool = True, seed: int = 0,
                                epoch: int = 0):
    """Indices torch.utils.data.DistributedSampler(drop_last=False) yields on `rank`:
    optional seeded permutation, padded by wrap-around to a multiple of `world`, then
    every world-th index from `rank`."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    per = -(-n // world)
    total = per * world
    pad = total - n
    if pad > 0:
        idx += (idx * (-(-pad // max(1, len(idx)))))[:pad]
    return idx[rank:total:world]


def max_over_ranks(x: float, device=None) -> float:
    """Max of a host scalar over all ranks (bench timing); identity when not distributed."""
    if not is_dist_avail_and_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def sum_over_ranks(t: torch.Tensor) -> torch.Tensor:
    """In-place sum of an accumulator tensor (e.g. per-class TP/FP/FN/IoU) over all ranks."""
    if is_dist_avail_and_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t
