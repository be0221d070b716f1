"""World-size-2 gloo tests of the multi-rank control flow (CPU).

bench.py --gpus N and distributed sampling run one independent clip shard per rank and only
exchange the timing max and the PQ accumulator sums; these check that logic on CPU ranks.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ldmseg.utils import distributed_sampler_indices, gpu_gather, max_over_ranks, sum_over_ranks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard = distributed_sampler_indices(n, rank, world, shuffle=True, seed=3)
        gathered = gpu_gather(torch.tensor(shard))
        elapsed = max_over_ranks(1.0 + rank)
        acc = sum_over_ranks(torch.tensor([float(rank + 1), 2.0]))
        q.put((rank, shard, gathered.tolist(), elapsed, acc.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [10, 7])
def test_world2_sharding_and_reductions(n):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from torch.utils.data import DistributedSampler
    for rank, shard, gathered, elapsed, acc in res:
        ref = list(DistributedSampler(list(range(n)), num_replicas=world, rank=rank, shuffle=True, seed=3))
        assert shard == ref
        assert elapsed == 2.0                      # max over ranks of 1.0 + rank
        assert acc == [3.0, 4.0]
    union = res[0][2]
    assert sorted(set(union)) == list(range(n))    # every clip is sampled by some rank
    assert len(union) == 2 * (-(-n // 2))
