"""CPU (gloo) tests of the data-parallel gradient exchange (ldmseg/trainers/ddp.py): flat buffer
views, bucket cutting, out-of-order readiness, and the sum over world_size 2 — the reference's
DDP reducer semantics (tools/main_ldm.py:184-197) on the flat-buffer design."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ldmseg.trainers import FlatParams, GradBucketer


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_flat_params_views_and_buckets():
    ps = [torch.nn.Parameter(torch.randn(s)) for s in [(10, 3), (7,), (100,), (5, 5)]]
    vals = [p.detach().clone() for p in ps]
    fp = FlatParams(ps)
    # offsets at 16-byte boundaries (ldm_repack / AdamW vector loads): 7 floats are followed by a gap of 1
    assert fp.offsets == [0, 32, 40, 140] and fp.numel == 30 + 2 + 7 + 1 + 100 + 25
    for p, v in zip(ps, vals):
        assert torch.equal(p.detach(), v)
        assert p.data.data_ptr() % 16 == 0
        assert p.data.data_ptr() >= fp.data.data_ptr()
        assert p.grad.shape == p.shape
    fp.data.add_(1.0)
    assert torch.equal(ps[2].detach(), vals[2] + 1)
    b = GradBucketer(fp, bucket_bytes=150)      # 37.5 floats -> cuts after params 0, 2 and 3
    spans = [(s, e) for s, e, _ in b.buckets]
    assert spans[0][0] == 0 and spans[-1][1] == fp.numel
    assert all(spans[i][1] == spans[i + 1][0] for i in range(len(spans) - 1))
    b.ready(ps[:1])
    b.finish()                                   # world 1: no collective, state reset
    assert b.pending == [len(i) for _, _, i in b.buckets]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        ps = [torch.nn.Parameter(torch.randn(s)) for s in [(64, 8), (33,), (500,), (9, 9)]]
        fp = FlatParams(ps)
        b = GradBucketer(fp, bucket_bytes=1024)
        for i, p in enumerate(ps):
            p.grad.copy_(torch.full(p.shape, float(rank + 1) * (i + 1)))
        b.ready([ps[3], ps[1]])          # out of order, partial
        b.ready([ps[0], ps[2], ps[1]])   # duplicates are ignored
        b.finish()
        ok = all(torch.allclose(p.grad, torch.full(p.shape, 3.0 * (i + 1))) for i, p in enumerate(ps))
        q.put((rank, ok, len(b.buckets)))
    finally:
        dist.destroy_process_group()


def test_bucketed_allreduce_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(n >= 2 for _, _, n in res)
