"""DVPQ output format + the multi-rank accumulator all-reduce (CPU).

The PNG pair written by ldmseg.evaluations.write_dvpq_frame is read back exactly the way
eval/eval_dvpq.py:105-110 reads predictions (np.array(Image.open(...)), id = cat * 2**20 + ins)
and scored with the golden-pinned oracle vpq_eval; the per-rank accumulators summed over a
world-2 gloo group must equal the single-process sums (eval_dvpq.py:186-189)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from golden_utils import load
from ldmseg.evaluations import dvpq_summary, reduce_pq_accumulators, write_dvpq_frame
from oracle import dvpq as odvpq

MAX_INS = 2 ** 20


def _read_pred(pan_dir, stem):
    from PIL import Image
    cat = np.array(Image.open(os.path.join(pan_dir, f"{stem}cat.png")))
    ins = np.array(Image.open(os.path.join(pan_dir, f"{stem}ins.png")))
    return cat.astype(np.int32) * MAX_INS + ins.astype(np.int32)


@pytest.mark.parametrize("ins_max", [200, 3000])
def test_write_dvpq_frame_round_trip(tmp_path, ins_max):
    rng = np.random.default_rng(0)
    cat = rng.integers(0, 19, size=(24, 40))
    cat[rng.random(cat.shape) < 0.1] = 255
    ins = rng.integers(0, ins_max, size=cat.shape)
    write_dvpq_frame(str(tmp_path), "000000_000001_", cat, torch.from_numpy(ins))
    got = _read_pred(str(tmp_path), "000000_000001_")
    np.testing.assert_array_equal(got, cat.astype(np.int32) * MAX_INS + ins.astype(np.int32))
    names = sorted(os.listdir(tmp_path))
    assert names == ["000000_000001_cat.png", "000000_000001_ins.png"]


def test_write_dvpq_frame_rejects_bad_ids(tmp_path):
    with pytest.raises(ValueError):
        write_dvpq_frame(str(tmp_path), "a_", np.full((2, 2), 300), np.zeros((2, 2)))
    with pytest.raises(ValueError):
        write_dvpq_frame(str(tmp_path), "a_", np.zeros((2, 2)), np.zeros((3, 2)))


def test_written_frames_score_like_the_golden_vpq(tmp_path):
    """Golden vpq cases -> PNGs -> read back -> oracle vpq_eval == the reference's numbers."""
    z = load("vpq.npz")
    for c in range(int(z["n_cases"])):
        pred = z[f"c{c}__pred"]
        write_dvpq_frame(str(tmp_path), f"c{c}_", pred // MAX_INS, pred % MAX_INS)
        back = _read_pred(str(tmp_path), f"c{c}_")
        np.testing.assert_array_equal(back, pred)
        iou, tp, fn, fp = odvpq.vpq_eval(back, z[f"c{c}__gt"])
        np.testing.assert_allclose(iou, z[f"c{c}__iou"])
        np.testing.assert_array_equal(tp, z[f"c{c}__tp"])
        np.testing.assert_array_equal(fn, z[f"c{c}__fn"])
        np.testing.assert_array_equal(fp, z[f"c{c}__fp"])


def test_dvpq_summary_formula():
    rng = np.random.default_rng(1)
    iou, tp, fn, fp = (rng.random(20) * 10 for _ in range(4))
    pq, tpq, spq = dvpq_summary(iou, tp, fn, fp)
    eps = 1e-10
    sq = iou[:19] / (tp[:19] + eps)
    rq = tp[:19] / (tp[:19] + 0.5 * fn[:19] + 0.5 * fp[:19] + eps)
    ref = sq * rq
    assert pq == pytest.approx(ref.mean() * 100) and tpq == pytest.approx(ref[:8].mean() * 100)
    assert spq == pytest.approx(ref[8:].mean() * 100)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = load("vpq.npz")
        acc = [np.zeros(20) for _ in range(4)]
        for c in range(rank, int(z["n_cases"]), world):          # each rank scores its own frames
            for a, v in zip(acc, odvpq.vpq_eval(z[f"c{c}__pred"], z[f"c{c}__gt"])):
                a += v
        q.put((rank, [a.tolist() for a in reduce_pq_accumulators(*acc)]))
    finally:
        dist.destroy_process_group()


def test_world2_pq_accumulator_all_reduce():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    z = load("vpq.npz")
    tot = [np.zeros(20) for _ in range(4)]
    for c in range(int(z["n_cases"])):
        for a, key in zip(tot, ("iou", "tp", "fn", "fp")):
            a += z[f"c{c}__{key}"]
    for _, acc in res:
        for a, t in zip(acc, tot):
            np.testing.assert_allclose(a, t, rtol=1e-12)
