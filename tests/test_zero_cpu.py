"""ZeRO stage 1 bookkeeping of LDMTrainStep on CPU ranks (gloo, world 2; row f1).

The reference wraps AdamW in ZeroRedundancyOptimizer when optimizer_zero_redundancy is set
(optim.py:71-78, tools/scripts/train_diffusion.sh:27) and consolidates the state before saving
(trainers_ldm_cond.py:1844-1866).  Here: the two ranks' shards are disjoint and cover the flat
buffer, every AdamW segment is split between them without loss, and a torch AdamW state loaded
into the sharded optimizer comes back bit-identical from consolidate_state_dict() (collective) +
state_dict() (local; it refuses an unconsolidated sharded state), through checkpoint.save called
on every rank (rank 0 writes) and a resume on every rank.  The
update arithmetic itself runs on the GPU (tests/test_gpu_train_full.py, ZeRO vs unsharded).
"""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_checkpoint import _reference_adamw, _unet


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, tmp):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ldmseg.schedulers import DDIMNoiseScheduler
        from ldmseg.trainers.ldm import LDMTrainStep
        lr_func = lambda name: 0.1 if "conv_in" in name else 1.0      # noqa: E731
        ref = _reference_adamw(_unet(2), 1e-4, 0.01, 0.0, lr_func)
        for p in (p for g in ref.param_groups for p in g["params"]):
            p.grad = torch.randn_like(p)
        ref.step()
        ts = LDMTrainStep(_unet(2 + rank), DDIMNoiseScheduler(), lr=1e-4, weight_decay=0.01, weight_decay_norm=0.0,
                          lr_factor_func=lr_func, zero_redundancy=True)
        ts.load_state_dict(ref.state_dict())
        try:                                  # sharded state: state_dict() alone must refuse
            ts.state_dict()
            refused = False
        except RuntimeError:
            refused = True
        ts.consolidate_state_dict()           # collective: every rank; only rank 0 keeps the moments
        kept_on_host = rank != 0 or all(t.device.type == "cpu" for t in ts._consolidated[1:])
        if rank != 0:                         # not the consolidating rank: nothing kept, state_dict refuses
            try:
                ts.state_dict()
                refused = False
            except RuntimeError:
                pass
        for dst in range(world):              # each rank's own consolidation (collective per call)
            ts.consolidate_state_dict(to=dst)
            if rank == dst:
                mine = ts.state_dict()
        # torch semantics: the consolidated copy serves repeated state_dict() calls on its rank
        #  until the next optimizer step
        released = rank != world - 1 or ts.state_dict()["state"].keys() == mine["state"].keys()
        theirs = ref.state_dict()
        # checkpoint.save on every rank: consolidated collectively, written by rank 0 only
        from ldmseg.utils import checkpoint
        path = os.path.join(tmp, "model.pt")
        checkpoint.save(path, unet=ts.unet, vae_semseg=torch.nn.Linear(1, 1), step=1, epoch=0, opt=ts)
        dist.barrier()
        saved = checkpoint.read(path)["opt"]
        same_saved = all(torch.equal(saved["state"][i][k], theirs["state"][i][k])
                         for i in theirs["state"] for k in ("exp_avg", "exp_avg_sq"))
        # resume on every rank: a local load (no collective), same moments back
        ts2 = LDMTrainStep(_unet(2), DDIMNoiseScheduler(), lr=1e-4, weight_decay=0.01, weight_decay_norm=0.0,
                           lr_factor_func=lr_func, zero_redundancy=True)
        ts2.load_state_dict(saved)
        for dst in range(world):
            ts2.consolidate_state_dict(to=dst)
            if rank == dst:
                back = ts2.state_dict()
        same_resumed = all(torch.equal(back["state"][i][k], theirs["state"][i][k])
                           for i in theirs["state"] for k in ("exp_avg", "exp_avg_sq"))
        same = mine["state"].keys() == theirs["state"].keys() and all(
            torch.equal(mine["state"][i][k], theirs["state"][i][k])
            for i in theirs["state"] for k in ("exp_avg", "exp_avg_sq"))
        q.put((rank, ts.shard, ts.exp_avg.numel(), ts.flat.numel, [list(s[:2]) for s in ts.seg_hp],
               [s[:2] for s in ts.shard_segments()], same and refused and same_saved and same_resumed and kept_on_host and released, ts.step_count,
               ts.flat.data.numpy().copy()))   # by value
    finally:
        dist.destroy_process_group()


def test_zero1_shards_and_consolidated_state_world2(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, sh0, m0, n, segs, loc0, same0, st0, d0), (r1, sh1, m1, _, _, loc1, same1, st1, d1) = res
    assert sh0[0] == 0 and sh0[1] == sh1[0] and sh1[1] == n and sh0[1] % 64 == 0
    assert m0 == sh0[1] - sh0[0] and m1 == sh1[1] - sh1[0] and max(m0, m1) < n
    # every segment's elements land in exactly one shard, re-based to the shard start
    covered = [(s + sh0[0], e + sh0[0]) for s, e in loc0] + [(s + sh1[0], e + sh1[0]) for s, e in loc1]
    total = sum(e - s for s, e in covered)
    assert total == sum(e - s for s, e in segs)
    merged = sorted(covered)
    assert all(a[1] <= b[0] for a, b in zip(merged, merged[1:]))
    assert same0 and same1 and st0 == st1 == 1
    assert (d0 == d1).all()                         # rank 0's weights broadcast at construction


def _subgroup_worker(rank, world, port, q, tmp):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from torch.distributed.optim import ZeroRedundancyOptimizer
        from ldmseg.utils import checkpoint as ck
        groups = [dist.new_group([r]) for r in range(world)]      # every rank creates every group
        torch.manual_seed(rank)
        lin = torch.nn.Linear(8, 8)
        opt = ZeroRedundancyOptimizer(lin.parameters(), optimizer_class=torch.optim.AdamW, lr=1e-3,
                                      process_group=groups[rank])
        lin(torch.randn(4, 8)).square().sum().backward()
        opt.step()
        path = os.path.join(tmp, f"model_{rank}.pt")
        ck.save(path, unet=lin, vae_semseg=torch.nn.Identity(), opt=opt)
        sd = ck.read(path)["opt"] if os.path.exists(path) else None
        q.put((rank, sd is not None and len(sd["state"]) == 2 and sd["state"][0]["step"].item() == 1))
    finally:
        dist.destroy_process_group()


def test_save_torch_zero_over_subgroup_without_rank0(tmp_path):
    """a torch ZeroRedundancyOptimizer keeps its group in `process_group`.  Over a
    subgroup that excludes global rank 0 the state is consolidated to that group's first rank, and
    that rank (not global rank 0, which holds none of it) must write the file."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_worker, args=(r, world, port, q, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, True), (1, True)]
