"""Data-parallel gradient exchange for the native training step.

The reference wraps the UNet in torch DDP (tools/main_ldm.py:184-197) whose reducer
all-reduces fp32 gradient buckets over NCCL.  Here the trainable parameters live in ONE flat
fp32 buffer (their ``.data`` / ``.grad`` are views into it), laid out in the order the
hand-written backward finishes them, and cut into buckets of whole parameters.  The backward
reports each block's parameters as they complete (UNetTrainGraph ``on_ready``); a bucket whose
last parameter completes is all-reduced right away with ``async_op=True`` — on RCCL that runs
on the communicator's stream after the compute already queued, so the exchange of early buckets
overlaps the rest of the backward.  ``finish()`` joins the outstanding reductions.

Bucket size: xGMI is point-to-point (7 links per MI355X), so a ring all-reduce is per-link
bound and wants few, large messages; 100 MB buckets put ~33 collectives on a 3.25 GB fp32
gradient, each long enough to reach the ring's bus bandwidth, while the first buckets still
finish early in the backward.
"""
import torch
import torch.distributed as dist


class FlatParams:
    """Re-home ``params`` (in the given order) into one flat fp32 data buffer and one flat fp32
    grad buffer; every parameter's ``.data`` and ``.grad`` become views into them.

    ``pad_to`` (>= the parameters' total) sizes the data storage: ``self.storage`` holds
    ``pad_to`` elements (the tail zero) and ``self.data`` is its first ``numel``, so a ZeRO-1
    all-gather of equal shards can write straight into it.

    Every offset is a multiple of ``ALIGN`` floats (16 bytes): the packed-weight refresh
    (ldm_repack) and the fused AdamW read their sources with 16-byte vector loads.  A parameter
    whose numel is not a multiple of 4 is followed by a zero gap (never written by the backward,
    so the gradient there stays 0 and the gap adds nothing to the clip norm)."""

    ALIGN = 4

    def __init__(self, params, device=None, pad_to=None):
        params = list(params)
        if not params:
            raise ValueError("no trainable parameters")
        device = device or params[0].device
        self.params = params
        self.offsets, n = self.layout(params)
        self.numel = n
        self.storage = torch.zeros(max(n, pad_to or 0), dtype=torch.float32, device=device)
        self.data = self.storage[:n]
        self.grad = torch.zeros(n, dtype=torch.float32, device=device)
        for p, o in zip(params, self.offsets):
            k = p.numel()
            self.data[o:o + k].copy_(p.detach().reshape(-1).float())
            p.data = self.data[o:o + k].view(p.shape)
            p.grad = self.grad[o:o + k].view(p.shape)
        self.index = {id(p): i for i, p in enumerate(params)}

    @classmethod
    def layout(cls, params):
        """(offsets, total) of ``params`` laid out back to back at ALIGN-float boundaries."""
        offsets, n = [], 0
        for p in params:
            n = -(-n // cls.ALIGN) * cls.ALIGN
            offsets.append(n)
            n += p.numel()
        return offsets, n

    def view_of(self, p, flat):
        i = self.index[id(p)]
        o = self.offsets[i]
        return flat[o:o + p.numel()].view(p.shape)


class GradBucketer:
    """Bucketed, overlapped all-reduce (sum) of a FlatParams grad buffer."""

    def __init__(self, flat: FlatParams, bucket_bytes=100 * 2 ** 20, group=None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.buckets = []           # (start, end, param indices)
        cur, start, size = [], 0, 0
        for i, p in enumerate(flat.params):
            cur.append(i)
            size += p.numel() * 4
            if size >= bucket_bytes:
                end = flat.offsets[i] + p.numel()
                self.buckets.append((start, end, cur))
                cur, start, size = [], end, 0
        if cur:
            self.buckets.append((start, flat.numel, cur))
        self.bucket_of = {}
        for b, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self.bucket_of[i] = b
        self.reset()

    def reset(self):
        self.pending = [len(idx) for _, _, idx in self.buckets]
        self.seen = set()
        self.works = []
        self.launched = [False] * len(self.buckets)

    def _launch(self, b):
        if self.launched[b]:
            return
        self.launched[b] = True
        if self.world > 1:
            s, e, _ = self.buckets[b]
            self.works.append(dist.all_reduce(self.flat.grad[s:e], group=self.group, async_op=True))

    def ready(self, params):
        """Mark parameters whose gradients are final (enqueued on the current stream)."""
        for p in params:
            i = self.flat.index.get(id(p))
            if i is None or i in self.seen:
                continue
            self.seen.add(i)
            b = self.bucket_of[i]
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self._launch(b)

    def finish(self):
        """Launch any bucket not yet reduced (parameters the backward never reported, e.g.
        unused) and wait for every reduction (the current stream waits on the RCCL stream)."""
        for b in range(len(self.buckets)):
            self._launch(b)
        for w in self.works:
            w.wait()
        self.reset()
