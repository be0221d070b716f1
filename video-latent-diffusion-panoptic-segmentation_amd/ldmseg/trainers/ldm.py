"""One LDM training iteration on the HIP path (SURVEY.md §8 row a15, row f1 for N > 1).

Follows TrainerDiffusion.train_single_epoch for one batch with gradient_accumulate_every = 1
(trainers_ldm_cond.py:792-900):
  noise = randn_like(latents); t = randint(min_noise_level, T, (B,))              :816-821
  noisy = scheduler.add_noise(latents, noise, t)                                   :822
  self_condition: cond = remove_noise(noisy, unet([noisy || rgb || 0], t), t)      :824-833 (no grad)
  compute_loss: pred = unet([noisy || rgb (|| cond)], t); target = noise (epsilon) or latents
                loss = mean((pred - target)^2 * mask * weights[t])                 :530-619 (l2, ohem 1)
  loss.backward(); clip_grad_norm_(clip_grad); AdamW step; zero_grad                :851-862, :769-781
with the optimizer of trainers/optim.py get_optim_unet: per-parameter lr = base_lr *
lr_factor_func(name), weight decay = weight_decay_norm for norm layers, else weight_decay.

Native pieces: the concatenations are never materialised (the conv_in gather reads the
sources), the forward keeps activations for the hand-written backward (models/unet_train.py),
the loss and its gradient are one kernel, the clip coefficient is computed on the device, and
AdamW is one fused kernel over the flat fp32 master buffer — no host synchronisation inside
the step.  With torch.distributed initialised, gradients are summed by bucketed all-reduces
that start while the backward is still running (trainers/ddp.py); the loss gradient carries
the 1/world factor so the sum is DDP's average.

ZeRO stage 1 (``zero_redundancy=True``; optim.py:71-78 wraps AdamW in
ZeroRedundancyOptimizer when ``optimizer_zero_redundancy`` is set, tools/scripts/
train_diffusion.sh:27): the AdamW moments exist only for this rank's contiguous shard of the
flat buffer; gradients are still all-reduced whole (DDP), the clip norm is taken over the whole
reduced gradient, each rank updates its shard, and the shards are all-gathered back into every
rank's parameters — the same arithmetic, element for element, as the unsharded step.

Not native (raises): ohem_ratio < 1, rgb/cond noise levels > 0, inpainting masks,
prob_train_on_pred > 0 — all off in base.yaml / train_diffusion.sh.
"""
import contextlib
import struct

import torch
import torch.distributed as dist
import torch.nn as nn

from ..models.repack import PackRefresher
from ..models.unet import ResnetBlock2D
from ..models.unet_train import UNetTrainGraph
from ..ops import native as K
from .ddp import FlatParams, GradBucketer

NORM_TYPES = (nn.GroupNorm, nn.LayerNorm, nn.BatchNorm2d)


def unet_backward_order(unet):
    """Trainable parameters in the order the native backward finishes them: reverse forward
    order of the blocks, every ResNet's time_emb_proj last (its batched GEMM backward runs
    after the whole graph)."""
    fwd = [unet.conv_in]
    for blk in unet.down_blocks:
        for j, r in enumerate(blk.resnets):
            fwd.append(r)
            if blk.has_cross_attention:
                fwd.append(blk.attentions[j])
        if blk.downsamplers is not None:
            fwd.append(blk.downsamplers[0])
    mb = unet.mid_block
    fwd += [mb.resnets[0], mb.attentions[0], mb.resnets[1]]
    for blk in unet.up_blocks:
        for j, r in enumerate(blk.resnets):
            fwd.append(r)
            if blk.has_cross_attention:
                fwd.append(blk.attentions[j])
        if blk.upsamplers is not None:
            fwd.append(blk.upsamplers[0])
    fwd += [unet.conv_norm_out, unet.conv_out]
    temb = [q for m in unet.modules() if isinstance(m, ResnetBlock2D) for q in m.time_emb_proj.parameters()]
    temb_ids = {id(q) for q in temb}
    order, seen = [], set()
    for m in reversed(fwd):
        for q in m.parameters():
            if q.requires_grad and id(q) not in temb_ids and id(q) not in seen:
                order.append(q)
                seen.add(id(q))
    order += [q for q in temb if q.requires_grad]
    rest = [q for q in unet.parameters() if q.requires_grad and id(q) not in seen and id(q) not in temb_ids]
    return order + rest


class LDMTrainStep:
    def __init__(self, unet, scheduler, lr=1e-4, weight_decay=0.0, weight_decay_norm=0.0, betas=(0.9, 0.999),
                 eps=1e-8, clip_grad=3.0, lr_factor_func=None, self_condition=False, min_noise_level=0,
                 compute_dtype=torch.bfloat16, bucket_mb=100, group=None, seed=None, zero_redundancy=False,
                 inplace_gather=False):
        self.unet, self.sched = unet, scheduler
        # the training forward differentiates separate LayerNorms; with the fold off every pack is a
        # plain layout of its parameters, refreshed in place after each update (models/repack.py).
        # The module's inference setting is restored inside ``for_inference()`` (validation sampling)
        self._inference_fold = unet.ln_fold
        self._inference_phases = getattr(unet, "_up_phases", True)   # the setting, not its train-mode value
        unet.set_ln_fold(False)
        unet.set_upsample_phases(False)           # the backward differentiates the 3x3 upsample conv
        self.refresher = PackRefresher(unet)
        self.self_condition = self_condition
        self.min_noise_level = min_noise_level
        self.clip_grad = float(clip_grad)
        self.betas, self.eps = betas, eps
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        unet.set_compute_dtype(compute_dtype)
        names = {id(p): n for n, p in unet.named_parameters()}
        norm_ids = {id(q) for m in unet.modules() if isinstance(m, NORM_TYPES) for q in m.parameters(recurse=False)}
        order = unet_backward_order(unet)
        dev = order[0].device
        # ZeRO-1 shards are S elements (a multiple of 64) so the all-gather moves equal pieces;
        # the flat storage is padded to S x world once, so the gather writes straight into it
        self.zero = bool(zero_redundancy) and self.world > 1
        # RCCL in-place all-gather straight into the padded flat storage (no 3.26 GB temporary);
        # opt-in until a multi-GPU RCCL run has checked it against the out-of-place form
        self.inplace_gather = bool(inplace_gather)
        n = FlatParams.layout(order)[1]
        self.shard_len = -(-n // (64 * self.world)) * 64 if self.zero else n
        self.flat = FlatParams(order, dev, pad_to=self.shard_len * self.world if self.zero else None)
        self.bucketer = GradBucketer(self.flat, bucket_mb * 2 ** 20, group)
        lr_factor_func = lr_factor_func or unet.get_lr_func
        self.base_lr = lr
        self.seg_hp = []
        # get_optim_unet's grouping key (optim.py:196-243): the construction-time lr, plus the
        # weight decay only for norm layers — other parameters carry no per-group weight_decay,
        # so a norm group stays separate even when weight_decay_norm == weight_decay
        self.seg_key = []
        for p, o in zip(self.flat.params, self.flat.offsets):
            plr = lr * lr_factor_func(names[id(p)])
            wd = weight_decay_norm if id(p) in norm_ids else weight_decay
            self.seg_hp.append([o, o + p.numel(), plr, wd])
            self.seg_key.append((plr, wd if id(p) in norm_ids else None))
        # ZeRO-1 shard [lo, hi) of the flat buffer (the whole buffer without it)
        self._consolidated = None
        if self.zero:
            self.rank = dist.get_rank(group)
            lo = min(self.rank * self.shard_len, n)
            self.shard = (lo, min(lo + self.shard_len, n))
        else:
            self.shard = (0, n)
        self._upload_segments()
        self.exp_avg = torch.zeros(self.shard[1] - self.shard[0], dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros_like(self.exp_avg)
        self.step_count = 0
        # DistributedDataParallel(...) broadcasts rank 0's module state — every parameter, the
        # frozen time_embedding included, and every buffer — when it is constructed
        # (tools/main_ldm.py:184-197): every rank starts from the same weights even when their
        # init seeds differ or a checkpoint was loaded on rank 0 only.
        self.broadcast_parameters()
        self.sqsum = torch.zeros((), dtype=torch.float64, device=dev)
        self.gen = None
        if seed is not None:
            self.gen = torch.Generator(device=dev)
            self.gen.manual_seed(seed)
        unet.invalidate_packed()

    def _src(self):
        return dist.get_global_rank(self.group, 0) if self.group is not None else 0

    def _broadcast(self, *tensors):
        if self.world > 1:
            for t in tensors:
                dist.broadcast(t, self._src(), group=self.group)

    def shard_segments(self):
        """The AdamW segment records of this rank's shard: every segment that intersects
        [lo, hi), clipped to it and re-based to lo (all of them without ZeRO)."""
        lo, hi = self.shard
        return [(max(s, lo) - lo, min(e, hi) - lo, lr, wd) for s, e, lr, wd in self.seg_hp if e > lo and s < hi]

    def _upload_segments(self):
        segs = self.shard_segments()
        self.nseg = len(segs)
        recs = b"".join(struct.pack("<qqff", s, e, lr, wd) for s, e, lr, wd in segs) or bytes(24)
        self.segs = torch.frombuffer(bytearray(recs), dtype=torch.uint8).to(self.flat.data.device)

    def _full(self, shard_buf):
        """The whole-buffer tensor of a sharded one (collective under ZeRO; the buffer itself
        otherwise).  Gathered by an all-reduce of zero-padded copies when the backend is not
        RCCL (gloo has no CUDA all-gather); x + 0 is exact."""
        if not self.zero:
            return shard_buf
        S, w, r = self.shard_len, self.world, self.rank
        buf = torch.zeros(S * w, dtype=shard_buf.dtype, device=shard_buf.device)
        buf[r * S:r * S + shard_buf.numel()].copy_(shard_buf)
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(buf, buf[r * S:(r + 1) * S].clone(), group=self.group)
        else:
            dist.all_reduce(buf, group=self.group)
        return buf[:self.flat.numel]

    def _gather_parameters(self):
        """ZeroRedundancyOptimizer.step's parameter sync: every rank's updated shard to all.  By
        default through _full (an out-of-place all-gather on RCCL, a sum of zero-padded copies on
        gloo, which has no CUDA all-gather).  With ``inplace_gather`` (RCCL only) the all-gather
        writes straight into the padded flat storage, whose own shard is already in place."""
        S, r = self.shard_len, self.rank
        st = self.flat.storage
        if self.inplace_gather and dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(st, st[r * S:(r + 1) * S], group=self.group)
        else:
            lo, hi = self.shard
            self.flat.data.copy_(self._full(self.flat.data[lo:hi]))

    def set_lr(self, lr):
        """update_scheduler (trainers_ldm_cond.py:783-790): the scheduled lr replaces EVERY
        group's lr (the per-parameter lr factors of the first step are not re-applied)."""
        for s in self.seg_hp:
            s[2] = lr
        self._upload_segments()

    # ---- optimizer state in torch.optim.AdamW's format (checkpoint layout, utils/checkpoint.py)
    def reference_param_groups(self):
        """get_optim_unet's parameter groups (trainers/optim.py:196-217 + reduce_param_groups):
        parameters in named_modules order, grouped by their (lr, weight_decay) in order of first
        appearance.  Returns [((lr, wd), [param, ...]), ...]."""
        memo, groups = set(), {}
        for _, m in self.unet.named_modules():
            for _, q in m.named_parameters(recurse=False):
                if not q.requires_grad or id(q) in memo or id(q) not in self.flat.index:
                    continue
                memo.add(id(q))
                # grouped by the construction-time key, not the scheduled lr: after set_lr every
                # group has the same lr, but the reference optimizer keeps its groups
                groups.setdefault(self.seg_key[self.flat.index[id(q)]], []).append(q)
        return list(groups.items())

    def _group_defaults(self, lr, wd):
        g = torch.optim.AdamW([torch.zeros(1)], lr=lr, betas=self.betas, eps=self.eps, weight_decay=wd)
        d = dict(g.param_groups[0])
        d.pop("params")
        return d

    def consolidate_state_dict(self, to=0):
        """ZeroRedundancyOptimizer.consolidate_state_dict(to): COLLECTIVE under ZeRO (every rank
        of the group must call it); gathers the sharded AdamW moments.  Only rank ``to`` (a rank of
        the group) keeps them, in host memory, so that state_dict() can then be called there alone
        (rank 0 inside checkpoint.save); the other ranks keep nothing, and the GPU temporaries of
        the gather are released before this returns.  The host copy stays valid (state_dict() may be
        called on it any number of times, as with torch's ZeroRedundancyOptimizer) until the next
        optimizer step.  No-op without ZeRO."""
        if not self.zero:
            return
        keep = self.rank == to
        moments = []
        for m in (self.exp_avg, self.exp_avg_sq):
            full = self._full(m)
            moments.append(full.cpu() if keep else None)
            del full
        self._consolidated = (self.step_count, *moments) if keep else None

    def state_dict(self):
        """torch.optim.AdamW.state_dict() of the same optimizer (fp32 moments, ``step``).  Local
        (never a collective).  Under ZeRO it needs consolidate_state_dict(to=this rank) on every
        rank first, as torch's ZeroRedundancyOptimizer does, and raises otherwise — a rank-0-only
        save can then never block inside a collective the other ranks do not join.  The
        consolidated host copy serves every call until the next step() releases it."""
        if self.zero:
            c = self._consolidated
            if c is None or c[0] != self.step_count:
                raise RuntimeError("ZeRO optimizer state is sharded: call consolidate_state_dict(to=rank) on every "
                                   "rank (checkpoint.save does) before state_dict() on that rank")
            exp_avg, exp_avg_sq = c[1], c[2]
        else:
            exp_avg, exp_avg_sq = self.exp_avg, self.exp_avg_sq
        state, pgs, idx = {}, [], 0
        for _, ps in self.reference_param_groups():
            _, _, lr, wd = self.seg_hp[self.flat.index[id(ps[0])]]        # the group's current lr
            ids = []
            for q in ps:
                if self.step_count > 0:
                    state[idx] = {"step": torch.tensor(float(self.step_count)),
                                  "exp_avg": self.flat.view_of(q, exp_avg).detach().clone(),
                                  "exp_avg_sq": self.flat.view_of(q, exp_avg_sq).detach().clone()}
                ids.append(idx)
                idx += 1
            pgs.append({**self._group_defaults(lr, wd), "params": ids})
        return {"state": state, "param_groups": pgs}

    def load_state_dict(self, sd, broadcast=False):
        """Inverse of state_dict(); also accepts a reference run's AdamW state_dict when its
        parameter grouping matches (same lr factors / weight decays).  Local by default: every
        rank loads the same checkpoint, as the reference's resume does on all ranks
        (trainers_ldm_cond.py:1879-1914).  ``broadcast=True`` is COLLECTIVE (every rank must
        call it): rank 0's moments, step count and learning rates replace the other ranks' —
        for a state loaded on rank 0 only."""
        groups = self.reference_param_groups()
        exp_avg = torch.zeros_like(self.flat.data)          # whole-buffer moments, sharded below
        exp_avg_sq = torch.zeros_like(self.flat.data)
        if len(groups) != len(sd["param_groups"]):
            raise ValueError(f"optimizer has {len(groups)} parameter groups, checkpoint {len(sd['param_groups'])}")
        steps = set()
        for ((_, _), ps), g in zip(groups, sd["param_groups"]):
            if len(ps) != len(g["params"]):
                raise ValueError("parameter group sizes differ from the checkpoint's")
            for q, i in zip(ps, g["params"]):
                st = sd["state"].get(i, sd["state"].get(str(i)))
                seg = self.seg_hp[self.flat.index[id(q)]]
                seg[2], seg[3] = float(g["lr"]), float(g["weight_decay"])
                if st is None:
                    continue
                if tuple(st["exp_avg"].shape) != tuple(q.shape):
                    raise ValueError("optimizer state shape differs from the parameter's")
                self.flat.view_of(q, exp_avg).copy_(st["exp_avg"])
                self.flat.view_of(q, exp_avg_sq).copy_(st["exp_avg_sq"])
                steps.add(int(float(st["step"])))
        if len(steps) > 1:
            raise ValueError("per-parameter step counts differ; the fused AdamW keeps one count")
        self.step_count = steps.pop() if steps else 0
        if broadcast and self.world > 1:
            dev = self.flat.data.device
            cnt = torch.tensor([float(self.step_count)], dtype=torch.float64, device=dev)
            hp = torch.tensor([[s[2], s[3]] for s in self.seg_hp], dtype=torch.float32, device=dev)
            self._broadcast(exp_avg, exp_avg_sq, cnt, hp)
            self.step_count = int(cnt.item())
            for seg, (lr, wd) in zip(self.seg_hp, hp.tolist()):
                seg[2], seg[3] = lr, wd
        lo, hi = self.shard
        self.exp_avg.copy_(exp_avg[lo:hi])
        self.exp_avg_sq.copy_(exp_avg_sq[lo:hi])
        self._upload_segments()

    def broadcast_parameters(self):
        """Re-sync every rank's module state to rank 0's (collective), e.g. after a load on rank 0:
        the flat trainable buffer in one message, then the frozen parameters and buffers."""
        if self.world > 1:
            self._broadcast(self.flat.data)
            self._broadcast(*[q.data for q in self.unet.parameters() if id(q) not in self.flat.index],
                            *[b for b in self.unet.buffers()])
        self.unet.invalidate_packed()

    @contextlib.contextmanager
    def for_inference(self):
        """Inference with the module's own LayerNorm-fold setting (the fused QKV / feed-forward
        forms) between training iterations, e.g. validation sampling:

            with trainer.for_inference():
                latents = sample_latents(unet, ...)

        The packs are rebuilt for the folded plan on entry and for the training plan on exit
        (one prepare() each way).  The module is put in eval mode inside the context (the
        phase-form upsample conv runs only in eval mode) and its previous mode is restored on exit."""
        was_training = self.unet.training
        self.unet.set_ln_fold(self._inference_fold)
        self.unet.set_upsample_phases(self._inference_phases)
        self.unet.eval()
        try:
            yield self.unet
        finally:
            self.unet.train(was_training)
            self.unet.set_ln_fold(False)
            self.unet.set_upsample_phases(False)

    def _sink(self, p):
        return self.flat.view_of(p, self.flat.grad), False

    @torch.no_grad()
    def train_step(self, latents, rgb_latents, loss_mask=None, timesteps=None, noise=None):
        """One iteration; returns the (local) mean loss as a 0-d fp64 device tensor."""
        u, sch = self.unet, self.sched
        if u.ln_fold:                                       # re-enabled by the caller since construction
            u.set_ln_fold(False)
        if u.upsample_phases:
            u.set_upsample_phases(False)
        B = latents.shape[0]
        dev = latents.device
        if noise is None:
            noise = torch.randn(latents.shape, generator=self.gen, device=dev, dtype=latents.dtype)
        if timesteps is None:
            timesteps = torch.randint(self.min_noise_level, sch.num_train_timesteps, (B,), generator=self.gen,
                                      device=dev, dtype=torch.long)
        noisy = sch.add_noise(latents, noise, timesteps)
        sources = [noisy, rgb_latents]
        if self.self_condition:
            zeros = torch.zeros_like(noisy)
            pred0 = u.forward_sources([noisy, rgb_latents, zeros], timesteps)
            cond = sch.remove_noise(noisy, pred0.float(), timesteps)
            sources.append(cond)
        if sch.prediction_type == "epsilon":
            target = noise
        elif sch.prediction_type == "sample":
            target = latents
        else:
            raise ValueError(f"Unknown prediction type: {sch.prediction_type}")
        graph = UNetTrainGraph(u, self._sink, on_ready=self.bucketer.ready)
        pred = graph.forward(sources, timesteps)              # the conv_in gather casts each source
        weights = getattr(sch, "weights", None)
        loss_sum, dpred = K.mse_loss(pred, target, loss_mask, timesteps, weights,
                                     grad_scale=1.0 / (pred.numel() * self.world))
        graph.backward(dpred)
        self.bucketer.finish()
        self.optimizer_step()
        return loss_sum / pred.numel()

    def optimizer_step(self):
        """clip_grad_norm_ + AdamW step over the (reduced) flat gradient: this rank's shard under
        ZeRO, followed by the parameter all-gather."""
        self.step_count += 1
        self._consolidated = None                           # the consolidated moments are now stale
        K.sq_norm(self.flat.grad, out=self.sqsum)          # the whole reduced gradient (clip_grad_norm_)
        lo, hi = self.shard
        if self.nseg:
            K.adamw(self.flat.data[lo:hi], self.flat.grad[lo:hi], self.exp_avg, self.exp_avg_sq, self.segs, self.nseg,
                    self.step_count, self.betas[0], self.betas[1], self.eps, sqsum=self.sqsum,
                    max_norm=self.clip_grad if self.clip_grad > 0 else 0.0)
        if self.zero:
            self._gather_parameters()
        self.refresher.run()                               # packs rewritten in place (ldm_repack)
