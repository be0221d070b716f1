"""In-place refresh of the UNet's packed weights after an optimizer update (ldm_repack).

The HIP kernels read weights packed as bf16 ``[n][kpad]`` (UNet.prepare) and, in the backward,
as flipped / transposed data-gradient packs (UNet.prepare_dgrad).  The reference's optimizer
updates the torch parameters in place (trainers_ldm_cond.py:769-781); here the fused AdamW updates
the fp32 master buffer, after which every pack built from a trainable parameter is stale.
Rebuilding them with torch ops costs ~1200 small kernels per iteration (~15 ms of the 148 ms
training iteration, profiles/r02d_train_kernel_stats.csv).  PackRefresher instead describes every
pack once — destination tensor, source parameter(s), layout mode — in a device table, and one
ldm_repack launch rewrites all of them from the current fp32 weights.
"""
import ctypes
import struct

import torch

from ..ops import native as K

_DESC = struct.Struct("<QQqiiiiiiiiii")      # ldm_repack_desc (include/ldmseg_hip.h), 64 bytes


def _iter_packs(obj):
    if isinstance(obj, K.PackedConv):
        yield obj
    elif isinstance(obj, dict):
        for v in obj.values():
            yield from _iter_packs(v)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            yield from _iter_packs(v)


def _contiguous_run(params):
    """The params as one row-concatenated fp32 source: they must lie back to back in memory (the
    flat master buffer keeps a module's parameters adjacent); returns the first or None."""
    p0 = params[0]
    addr = p0.data_ptr() + p0.numel() * 4
    for q in params[1:]:
        if q.data_ptr() != addr or q.dtype != torch.float32:
            return None
        addr += q.numel() * 4
    return p0


class PackRefresher:
    """Rewrites every pack of ``unet``'s current plans that depends on a trainable parameter."""

    def __init__(self, unet):
        self.u = unet
        self._for = None           # (plan, dplan) objects the table was built for
        self.table = None
        self.ndesc = 0
        self.total = 0
        self.fallback = []         # packs ldm_repack cannot express (rebuilt by torch: none in the SD UNet)

    def _descs(self, P, D):
        recs = []

        def add(src, dst, rows, row0, kpad, co, ci, ks, cpad, mode, geglu):
            f32 = int(dst.dtype == torch.float32 and mode != 2)
            if dst.dtype not in (torch.float32, torch.bfloat16):
                raise TypeError(f"ldm_repack writes bf16 / fp32 packs, not {dst.dtype}")
            if mode != 2 and (ks > 3 or cpad % 8):
                raise ValueError("ldm_repack packs ks <= 3 with 8-aligned channel padding")
            ntiles = -(-rows // 2048) if mode == 2 else -(-rows // 16) * -(-cpad // 64)
            recs.append((src.data_ptr(), dst.data_ptr(), ntiles, rows, row0, kpad, co, ci, ks, cpad, mode, geglu,
                         f32))

        for pc in _iter_packs(P):
            ws = getattr(pc, "src_w", None)
            if not ws or not any(w.requires_grad for w in ws):
                continue
            if any(w.dtype != torch.float32 or not w.is_contiguous() for w in ws):
                self.fallback.append(pc)
                continue
            row0 = 0
            for w in ws:
                co, ci = w.shape[0], w.shape[1]
                ks = w.shape[2] if w.ndim == 4 else 1
                rows = pc.n if len(ws) == 1 else co         # a single source may be row-padded (conv_out_t)
                add(w, pc.w, rows, row0, pc.kpad, co, ci, ks, pc.cin, 0, int(pc.geglu))
                row0 += rows
            bs = pc.src_b
            if pc.bias is not None and bs and not (len(bs) == 1 and pc.bias.data_ptr() == bs[0].data_ptr()):
                j0 = 0
                for b in bs:                                # concatenated / interleaved copy: refresh it
                    add(b, pc.bias, b.numel(), j0, 0, b.numel(), 0, 1, 1, 2, int(pc.geglu))
                    j0 += b.numel()
        for pc in _iter_packs(D):
            src = getattr(pc, "dg_src", None)
            if src is None:
                continue
            ws, geglu = src
            ws = ws if isinstance(ws, (list, tuple)) else [ws]
            if not any(w.requires_grad for w in ws):
                continue
            w0 = _contiguous_run(ws)
            if w0 is None:
                self.fallback.append(pc)
                continue
            co = sum(w.shape[0] for w in ws)
            ci = w0.shape[1]
            ks = w0.shape[2] if w0.ndim == 4 else 1
            add(w0, pc.w, pc.n, 0, pc.kpad, co, ci, ks, pc.cin, 1, int(geglu))
        return recs

    def _build(self):
        P, D = self.u._plan, self.u._dplan
        self.fallback = []
        recs = self._descs(P, D or {})
        blob, c0 = bytearray(), 0
        for (src, dst, ntiles, rows, row0, kpad, co, ci, ks, cpad, mode, geglu, f32) in recs:
            blob += _DESC.pack(src, dst, c0, rows, row0, kpad, co, ci, ks, cpad, mode, geglu, f32)
            c0 += ntiles
        self.ndesc, self.total = len(recs), c0
        dev = self.u.device
        self.table = torch.frombuffer(blob, dtype=torch.uint8).to(dev) if recs else None
        self._for = (P, D)

    def run(self):
        """Refresh after an in-place update of the trainable parameters (no torch version bump)."""
        u = self.u
        if u._plan is None:                                 # nothing packed yet: prepare() packs fresh
            return
        if self._for is None or self._for[0] is not u._plan or self._for[1] is not u._dplan:
            self._build()
        if self.fallback:                                   # cannot be expressed: rebuild everything
            u.invalidate_packed()
            return
        if self.ndesc:
            K.repack(self.table, self.ndesc, self.total, u.device)
        u._plan_key = u._signature()                        # the plan is current again
