"""AE training iteration on the HIP path (BASELINE config 1).

Follows TrainerAE.train_single_epoch for one batch, gradient_accumulate_every = 1, fp32 or bf16
compute, no inpainting / fuse_rgb / latent mask (trainers_ae.py:279-389):
  images = 2 * bits - 1; output = vae(images, sample_posterior=True)          :294, :324
  loss = w_ce * ce + w_mask * mask (+ w_kl * kl, weight 0 in base.yaml)     compute_point_loss :239-251
  loss.backward(); clip_grad_norm_(clip_grad); AdamW step                     :331-366
with SegmentationLosses.point_loss (losses.py:117-395):
  ce   : 3 * num_points random points, uncertainty top2[1] - top2[0] of the bilinear point logits,
         the 0.75 * num_points most uncertain + the rest random (detectron2_utils.py:20-72);
         labels by nearest sampling of the targets; CE / temperature with ignore_index, mean
  mask : one binary mask per (image, class present, != ignore) on the logit channel of that class
         (prepare_targets, :399-440); points by uncertainty -|x|; labels by bilinear sampling of the
         mask; BCE-with-logits mean over points + dice, both summed over masks / num_masks

Native pieces: the VAE forward keeps what its backward needs (conv pre-activations where a SiLU
follows, LayerNorm2d inputs, GroupNorm (mean, rstd)); the backward uses the data-gradient conv
(flipped weights; stride 2 by the zero-insert gather), ldm_conv2d_wgrad, ldm_colsum, the GN/LN
backward kernels, ldm_silu, ldm_space_to_depth2 (ConvTranspose k2s2) and ldm_posterior_bwd; the
losses are the point kernels of csrc/points.hip with an atomic scatter back to the logit planes;
clip + AdamW are the fused kernels over a flat fp32 parameter buffer.  Random numbers (point
coordinates, posterior noise) come from torch's generator; ``rand`` / ``randn`` can be injected
(the parity test feeds the reference's own draws).
"""
import torch
import torch.distributed as dist
import torch.nn as nn

from ..models.vae import LayerNorm2d
from ..ops import native as K
from .ddp import FlatParams


def _ceil8(c):
    return (c + 7) // 8 * 8


class VAETrainGraph:
    """Training forward (saved activations) + backward of GeneralVAESeg."""

    def __init__(self, vae, sink):
        self.v, self.sink = vae, sink
        self.dt = vae.dtype
        self.saved = []
        self._dg = {}

    # ------------------------------------------------------------------ helpers
    def _pc(self, m, **kw):
        return K.PackedConv(m.weight, m.bias, self.dt, **kw)

    def _dgrad_pc(self, m, cin_pad=None, out_pad=None):
        key = (id(m), cin_pad, out_pad)
        if key not in self._dg:
            from ..models.unet_train import packed_dgrad
            w = m.weight
            if out_pad is not None and out_pad != w.shape[1]:
                w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, out_pad - w.shape[1]))
            self._dg[key] = packed_dgrad(w, self.dt, cin_pad=cin_pad)
        return self._dg[key]

    def _param_grad(self, p, val):
        if p is None or not p.requires_grad:
            return
        dst, acc = self.sink(p)
        (dst.add_ if acc else dst.copy_)(val.view_as(dst))

    def _run_seq(self, seq, x, B, H, W, cin_pad, last_nchw, is_encoder):
        mods = list(seq)
        i = 0
        first = True
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            silu = isinstance(nxt, nn.SiLU)
            last = all(isinstance(q, (nn.Identity, nn.SiLU)) for q in mods[i + 1:])
            if isinstance(m, nn.Conv2d):
                stride = m.stride[0]
                pc = self._pc(m, cin_pad=cin_pad if first else None)
                if last and last_nchw:
                    y = K.conv2d(pc, x, B, H, W, stride=stride, out_layout=K.OUT_NCHW, out_dtype=torch.float32)
                    self.saved.append(("conv", m, dict(x=x, pc=pc, B=B, H=H, W=W, stride=stride, z=None,
                                                       first=first and is_encoder, nchw=True)))
                else:
                    z = K.conv2d(pc, x, B, H, W, stride=stride)
                    y = K.silu(z) if silu else z
                    self.saved.append(("conv", m, dict(x=x, pc=pc, B=B, H=H, W=W, stride=stride,
                                                       z=z if silu else None, first=first and is_encoder,
                                                       nchw=False)))
                if stride == 2:
                    H, W = H // 2, W // 2
                first = False
                x = y
            elif isinstance(m, nn.ConvTranspose2d):
                pc = self._pc(m, shuffle2=True)
                y = K.conv2d(pc, x, B, H, W, out_layout=K.OUT_SHUFFLE2)
                self.saved.append(("convT", m, dict(x=x, pc=pc, B=B, H=H, W=W)))
                H, W = 2 * H, 2 * W
                x = y
                silu = False
            elif isinstance(m, LayerNorm2d):
                g, b = m.weight.detach().float().contiguous(), m.bias.detach().float().contiguous()
                u = K.layer_norm(x, g, b, m.eps)
                y = K.silu(u) if silu else u
                self.saved.append(("ln", m, dict(x=x, u=u if silu else None, g=g)))
                x = y
            elif isinstance(m, nn.GroupNorm):
                g, b = m.weight.detach().float().contiguous(), m.bias.detach().float().contiguous()
                act = K.ACT_SILU if silu else K.ACT_NONE
                y, mr = K.group_norm_train(x, B, H * W, m.num_groups, g, b, m.eps, act)
                self.saved.append(("gn", m, dict(x=x, mr=mr, g=g, b=b, act=act, B=B, H=H, W=W)))
                x = y
            elif isinstance(m, (nn.Identity, nn.SiLU)):
                silu = False
            else:
                raise NotImplementedError(f"{type(m).__name__} in the VAE stack")
            i += 2 if silu else 1
        return x, H, W

    # ------------------------------------------------------------------ forward
    def forward(self, images, eps):
        """images [B, Cin, H, W] fp32 (already 2 * bits - 1) -> (logits fp32 NCHW, moments)."""
        v = self.v
        B, Cin, H, W = images.shape
        self.B = B
        self.enc_pad = _ceil8(Cin)
        x = K.nchw_to_nhwc([images], self.enc_pad, self.dt)
        self.saved.append(("enc_start", None, {}))
        moments, h, w = self._run_seq(v.encoder, x, B, H, W, self.enc_pad, last_nchw=True, is_encoder=True)
        if v.clamp_output or v.act_fn != "none":
            raise NotImplementedError("clamp_output / act_fn posteriors are not on the native AE training path")
        z = K.posterior_sample(moments, eps)
        self.post = dict(moments=moments, eps=eps, h=h, w=w)
        self.dec_pad = _ceil8(z.shape[1])
        zx = K.nchw_to_nhwc([z], self.dec_pad, self.dt)
        self.saved.append(("dec_start", None, {}))
        logits, _, _ = self._run_seq(v.decoder, zx, B, h, w, self.dec_pad, last_nchw=True, is_encoder=False)
        return logits, moments

    # ------------------------------------------------------------------ backward
    def backward(self, dlogits):
        """dlogits fp32 NCHW -> parameter gradients through the sink."""
        d = dlogits
        d_is_nchw = True
        for kind, m, s in reversed(self.saved):
            if kind == "dec_start":
                # d: NHWC [B, h, w, dec_pad] gradient of the decoder input -> posterior -> encoder
                p = self.post
                dm = K.posterior_bwd(p["moments"], p["eps"], d)
                d, d_is_nchw = dm, True
                continue
            if kind == "enc_start":
                break
            if kind == "conv":
                B, H, W, stride = s["B"], s["H"], s["W"], s["stride"]
                n = m.out_channels
                Ho, Wo = (H // 2, W // 2) if stride == 2 else (H, W)
                if d_is_nchw:
                    npad = _ceil8(n)
                    dy = K.nchw_to_nhwc([d], npad, self.dt)
                else:
                    npad = n
                    dy = d
                if s["z"] is not None:
                    dy = K.silu(s["z"], dy)
                # weight / bias gradients
                if m.weight.requires_grad:
                    pc = s["pc"]
                    if npad != n:
                        wpad = torch.nn.functional.pad(m.weight.detach(), (0, 0, 0, 0, 0, 0, 0, npad - n))
                        pc = K.PackedConv(wpad, None, self.dt, cin_pad=pc.cin if pc.cin != pc.cin_real else None)
                        tmp = K.conv2d_wgrad(pc, s["x"], B, H, W, dy, stride=stride)[:n]
                    else:
                        tmp = K.conv2d_wgrad(pc, s["x"], B, H, W, dy, stride=stride)
                    self._param_grad(m.weight, tmp)
                if m.bias is not None and m.bias.requires_grad:
                    self._param_grad(m.bias, K.colsum(dy, B * Ho * Wo, npad).view(-1)[:n])
                if s["first"]:
                    d = None
                    continue
                cin = m.in_channels
                dpc = self._dgrad_pc(m, cin_pad=npad if npad != n else None)
                if stride == 2:
                    d = K.conv2d(dpc, dy, B, Ho, Wo, upsample=2)
                else:
                    d = K.conv2d(dpc, dy, B, H, W)
                d_is_nchw = False
                assert d.shape[-1] == cin
            elif kind == "convT":
                B, H, W = s["B"], s["H"], s["W"]
                cout, cin = m.out_channels, m.in_channels
                ds = K.space_to_depth2(d, B, H, W)                          # [B, H, W, 4 cout]
                if m.weight.requires_grad:
                    lin = K.PackedConv(torch.empty(4 * cout, cin, device=d.device), None, self.dt)
                    tmp = K.conv2d_wgrad(lin, s["x"], B, H, W, ds)          # [(dy, dx, co), ci]
                    self._param_grad(m.weight, tmp.view(2, 2, cout, cin).permute(3, 2, 0, 1).contiguous())
                if m.bias is not None and m.bias.requires_grad:
                    self._param_grad(m.bias, K.colsum(ds, B * H * W, 4 * cout).view(4, cout).sum(0))
                key = ("convT", id(m))
                if key not in self._dg:
                    wp = m.weight.detach().permute(2, 3, 1, 0).reshape(4 * cout, cin)   # packed forward rows
                    self._dg[key] = K.PackedConv(wp.t().contiguous(), None, self.dt)     # [cin][4 cout]
                d = K.linear(self._dg[key], ds).view(B, H, W, cin)
            elif kind == "ln":
                dy = K.silu(s["u"], d) if s["u"] is not None else d
                dg = db = None
                acc = False
                if m.weight.requires_grad:
                    dg, acc = self.sink(m.weight)
                if m.bias.requires_grad:
                    db, acc = self.sink(m.bias)
                d = K.layer_norm_bwd(s["x"], dy.contiguous(), s["g"], m.eps, dgamma=dg, dbeta=db, acc_params=acc)
            elif kind == "gn":
                dg = db = None
                acc = False
                if m.weight.requires_grad:
                    dg, acc = self.sink(m.weight)
                if m.bias.requires_grad:
                    db, acc = self.sink(m.bias)
                d, _ = K.group_norm_bwd(s["x"], s["B"], s["H"] * s["W"], m.num_groups, s["mr"], s["g"], s["b"],
                                        s["act"], d.contiguous(), dgamma=dg, dbeta=db, acc_params=acc)
        self.saved.clear()


class PointLosses:
    """SegmentationLosses.point_loss on the point kernels (forward + gradient w.r.t. the logits)."""

    def __init__(self, num_points=12544, oversample_ratio=3, importance_sample_ratio=0.75, ignore_label=0,
                 temperature=1.0, rand=None, select=None):
        self.num_points = num_points
        self.oversample = oversample_ratio
        self.importance = importance_sample_ratio
        self.ignore_label = ignore_label
        self.temperature = temperature
        self.rand = rand or (lambda *shape, device: torch.rand(*shape, device=device))
        # select(u [boxes, n], k) -> int32 indices [boxes, k]; a test hook (default: ldm_topk_select)
        self.select = select or (lambda u, k: K.topk_select(u, k)[0])
        self.last_idx = []

    def _uncertain_coords(self, x, planes=None):
        """get_uncertain_point_coords_with_randomness (detectron2_utils.py:20-72)."""
        boxes = x.shape[0] if planes is None else planes.numel()
        n_s = int(self.num_points * self.oversample)
        coords = self.rand(boxes, n_s, 2, device=x.device).contiguous()
        pl = K.point_sample(x, coords, planes)
        u = K.point_uncertainty(pl)
        n_u = int(self.importance * self.num_points)
        n_r = self.num_points - n_u
        idx = self.select(u, n_u)
        self.last_idx.append(idx)
        sel = torch.gather(coords, 1, idx.long()[:, :, None].expand(-1, -1, 2))
        if n_r > 0:
            sel = torch.cat([sel, self.rand(boxes, n_r, 2, device=x.device)], dim=1)
        return sel.contiguous()

    def __call__(self, logits, targets):
        """logits fp32 NCHW [B, C, h, w], targets int64 [B, H, W] -> (ce, mask, dlogits fp32 NCHW)."""
        dlog = torch.zeros_like(logits)
        # (1) CE on uncertain points (loss_ce, losses.py:330-361)
        coords = self._uncertain_coords(logits)
        labels = K.point_labels_nearest(targets, coords)
        pl = K.point_sample(logits, coords)
        acc, g = K.point_ce(pl, labels, self.temperature, self.ignore_label)
        ce = acc[0] / acc[1]
        K.point_sample_bwd(g, coords, dlog, scale_t=(1.0 / acc[1]).float().reshape(1))
        # (2) BCE + dice per (image, class) mask (loss_masks, losses.py:117-185)
        B, C = logits.shape[:2]
        img, cls = [], []
        for b in range(B):
            u = torch.unique(targets[b])
            u = u[u != self.ignore_label]
            img += [b] * u.numel()
            cls += u.tolist()
        if not cls:
            return ce, logits.new_zeros(()), dlog
        if max(cls) >= C or min(cls) < 0:
            raise ValueError("target class ids must index the logit channels")
        img_t = torch.tensor(img, dtype=torch.int32, device=logits.device)
        cls_t = torch.tensor(cls, dtype=torch.int32, device=logits.device)
        planes = img_t * C + cls_t
        num_masks = float(len(cls))
        if dist.is_available() and dist.is_initialized():
            t = torch.tensor([num_masks], device=logits.device)
            dist.all_reduce(t)
            num_masks = float(t.item()) / dist.get_world_size()
        num_masks = max(num_masks, 1.0)
        mcoords = self._uncertain_coords(logits, planes)
        mlab = K.point_labels_mask(targets, img_t, cls_t, mcoords)
        mpl = K.point_sample(logits, mcoords, planes)
        macc, mg = K.point_bce_dice(mpl.view(len(cls), -1), mlab)
        mask = (macc[0] + macc[1]) / num_masks
        K.point_sample_bwd(mg.view(len(cls), 1, -1), mcoords, dlog, planes=planes, scale=1.0 / num_masks)
        return ce, mask, dlog


class AETrainStep:
    """One TrainerAE iteration: forward, point losses, backward, clip, AdamW (torch AdamW semantics)."""

    def __init__(self, vae, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, clip_grad=3.0,
                 loss_weights=None, loss_kwargs=None, ignore_label=0, rand=None, randn=None, select=None):
        import struct
        self.vae = vae
        self.w = dict(ce=1.0, mask=1.0, kl=0.0, **(loss_weights or {}))
        if self.w["kl"] != 0.0:
            raise NotImplementedError("a non-zero KL weight is not on the native AE path (base.yaml: kl 0.0)")
        kw = dict(loss_kwargs or {})
        kw.pop("cost_mask", None)
        kw.pop("cost_class", None)
        self.losses = PointLosses(ignore_label=ignore_label, rand=rand, select=select, **kw)
        self.randn = randn or (lambda shape, device: torch.randn(shape, device=device))
        self.betas, self.eps, self.clip = betas, eps, float(clip_grad)
        params = [p for p in vae.parameters() if p.requires_grad]
        self.flat = FlatParams(params)
        recs = struct.pack("<qqff", 0, self.flat.numel, float(lr), float(weight_decay))
        self.segs = torch.frombuffer(bytearray(recs), dtype=torch.uint8).to(self.flat.data.device)
        self.exp_avg = torch.zeros_like(self.flat.data)
        self.exp_avg_sq = torch.zeros_like(self.flat.data)
        self.sqsum = torch.zeros((), dtype=torch.float64, device=self.flat.data.device)
        self.step_count = 0
        # DDP (main_worker_ae.py:80-89): rank 0's weights at construction, averaged gradients
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if self.world > 1:
            dist.broadcast(self.flat.data, 0)
            for t in [q.data for q in vae.parameters() if id(q) not in self.flat.index] + list(vae.buffers()):
                dist.broadcast(t, 0)

    def _sink(self, p):
        return self.flat.view_of(p, self.flat.grad), False

    def _sink_acc(self, p):
        return self.flat.view_of(p, self.flat.grad), True

    @torch.no_grad()
    def train_step(self, bits, targets):
        """bits [B, Cin, H, W] in {0, 1} (data['image_semseg']), targets int64 [B, H, W].
        Returns (loss, ce, mask) as 0-d device tensors."""
        v = self.vae
        images = (2.0 * bits - 1.0).float()
        self.flat.grad.zero_()
        graph = VAETrainGraph(v, self._sink_acc)
        B = images.shape[0]
        f = v.downsample_factor
        eps = self.randn((B, v.latent_channels, images.shape[2] // f, images.shape[3] // f), device=images.device)
        logits, _ = graph.forward(images, eps.float().contiguous())
        ce, mask, dlog = self.losses(logits, targets)
        loss = self.w["ce"] * ce + self.w["mask"] * mask
        if self.w["ce"] != 1.0 or self.w["mask"] != 1.0:
            raise NotImplementedError("loss weights other than 1 (base.yaml) are not wired into the gradient")
        graph.backward(dlog)
        if self.world > 1:
            dist.all_reduce(self.flat.grad)
            self.flat.grad.mul_(1.0 / self.world)
        self.step_count += 1
        K.sq_norm(self.flat.grad, out=self.sqsum)
        K.adamw(self.flat.data, self.flat.grad, self.exp_avg, self.exp_avg_sq, self.segs, 1, self.step_count,
                self.betas[0], self.betas[1], self.eps, sqsum=self.sqsum,
                max_norm=self.clip if self.clip > 0 else 0.0)
        v._plan = None
        return loss, ce, mask
