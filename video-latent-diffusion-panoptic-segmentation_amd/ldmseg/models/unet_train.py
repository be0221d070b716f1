"""Training forward + hand-written backward of the drop-in UNet on the HIP kernels.

The reference trains the diffusers UNet with torch autograd (trainers_ldm_cond.py:592-604
prediction, :851-856 ``loss.backward()``).  Here the forward of ``UNet.forward`` is re-run in
a *training* flavour that keeps exactly the activations its backward needs, and the backward
walks the same graph in reverse calling the gfx950 backward kernels (include/ldmseg_hip.h,
"Training path"):

  conv / linear     dX = ldm_conv2d with the transposed, spatially flipped packed weight
                    (stride 2: the zero-insert gather; nearest-2x upsample: conv at 2H then a
                    2x2 sum pool); dW = ldm_conv2d_wgrad; db = ldm_colsum; the ResNet time
                    embedding term gives a per-batch colsum -> the batched time_emb_proj GEMM
  GroupNorm(+SiLU)  ldm_group_norm_bwd from the forward's saved (mean, rstd)
  LayerNorm         ldm_layer_norm_bwd (+ the residual stream's gradient in the same pass)
  attention         ldm_attention_bwd from the saved log-sum-exp (flash-attention backward)
  GEGLU             the ff.net.0 GEMM keeps its interleaved [h | g] output; ldm_geglu fwd/bwd

Gradients of activations use the compute dtype; parameter gradients are fp32 and are handed to
``grad_sink(param) -> (tensor, accumulate)`` so a trainer can place them in a flat buffer and
start bucketed all-reduces (``on_ready``) while the rest of the backward still runs.

Not supported natively (raises): a trainable time_embedding (the reference freezes it:
base.yaml ``freeze_layers: ['time_embedding']``), cross-attention (removed by
``image_descriptors: remove``, base.yaml:71).
"""
import torch

from ..ops import native as K


# --------------------------------------------------------------------------------------
# packed weights for the data gradient
# --------------------------------------------------------------------------------------
def packed_dgrad(weight, dtype, geglu=False, cin_pad=None):
    """PackedConv of the data-gradient conv: W'[ci][co][ky][kx] = W[co][ci][2-ky][2-kx]
    (a linear / 1x1: W^T).  geglu: rows of W follow the forward's GEGLU interleave so the
    incoming gradient (in the interleaved column order) contracts against the right rows."""
    w = weight.detach()
    if w.ndim == 2:
        w = w[:, :, None, None]
    if geglu:
        cout = w.shape[0]
        half = cout // 2
        wh, wg = w[:half].reshape(half // 16, 16, *w.shape[1:]), w[half:].reshape(half // 16, 16, *w.shape[1:])
        w = torch.stack([wh, wg], dim=1).reshape(cout, *w.shape[1:])
    wt = w.flip(-1, -2).transpose(0, 1).contiguous()
    pc = K.PackedConv(wt, None, dtype, cin_pad=cin_pad)
    pc.dg_src = (weight, geglu)            # models.repack.PackRefresher (ldm_repack mode 1)
    return pc


class _Grads:
    """Accumulating gradient buffers of activations (a tensor with several consumers —
    skip connections, residuals — gets one buffer every consumer adds into)."""

    def __init__(self):
        self.buf = {}

    def get(self, t):
        """(buffer, exists) for activation t (allocates an uninitialised buffer if new)."""
        k = id(t)
        if k in self.buf:
            return self.buf[k][1], True
        b = torch.empty_like(t)
        self.buf[k] = (t, b)       # keep t alive so its id stays unique
        return b, False

    def pop(self, t):
        return self.buf.pop(id(t))[1]


class UNetTrainGraph:
    """Forward with saved activations + backward for one call of the UNet."""

    def __init__(self, unet, grad_sink, on_ready=None):
        self.u = unet
        self.P = unet.prepare()
        self.Pd = unet.prepare_dgrad()
        self.sink = grad_sink
        self.on_ready = on_ready or (lambda params: None)
        self.saved = []
        self.G = _Grads()

    # ------------------------------------------------------------------ param grads
    def _wgrad(self, pc, conv_module_w, x0, B, H, W, dy, x1=None, stride=1, upsample=False):
        p = conv_module_w
        if not p.requires_grad:
            return
        dst, acc = self.sink(p)
        K.conv2d_wgrad(pc, x0, B, H, W, dy, x1=x1, stride=stride, upsample=upsample, dw=dst, accumulate=acc)

    def _bgrad(self, bias, dy, rows, n, geglu=False):
        if bias is None or not bias.requires_grad:
            return
        dst, acc = self.sink(bias)
        K.colsum(dy, rows, n, 1, geglu=geglu, out=dst, accumulate=acc)

    def _sink_pair(self, gamma, beta):
        dg = db = None
        acc = False
        if gamma.requires_grad:
            dg, acc = self.sink(gamma)
        if beta.requires_grad:
            db, acc_b = self.sink(beta)
            if dg is not None and acc_b != acc:
                raise RuntimeError("gamma/beta gradient accumulation state differs")
            acc = acc_b
        return dg, db, acc

    # ------------------------------------------------------------------ forward pieces
    def _resnet_fwd(self, r, x0, x1, B, H, W, temb_all):
        p = self.P[id(r)]
        h1, mr1 = K.group_norm_train(x0, B, H * W, r.groups, *p["n1"], r.eps, K.ACT_SILU, x1=x1)
        y1 = K.conv2d(p["c1"], h1, B, H, W, temb=temb_all[:, p["off"]:], temb_stride=temb_all.shape[1],
                      gn_stats=True)
        h2, mr2 = K.group_norm_train(y1, B, H * W, r.groups, *p["n2"], r.eps, K.ACT_SILU)
        res = K.conv2d(p["sc"], x0, B, H, W, x1=x1) if p["sc"] is not None else x0
        out = K.conv2d(p["c2"], h2, B, H, W, residual=res, gn_stats=True)
        self.saved.append(("resnet", r, dict(x0=x0, x1=x1, mr1=mr1, h1=h1, y1=y1, mr2=mr2, h2=h2, out=out, B=B, H=H,
                                             W=W)))
        return out

    def _transformer_fwd(self, t, x, B, H, W):
        p = self.P[id(t)]
        if p["attn2"] is not None:
            raise NotImplementedError("cross-attention training is off the reference path (attn2 removed)")
        C = x.shape[-1]
        N = H * W
        g, mr = K.group_norm_train(x, B, N, t.groups, *p["norm"], 1e-6)
        h0 = K.linear(p["proj_in"], g)
        n1 = K.layer_norm(h0, *p["ln1"], 1e-5)
        qkv = K.linear(p["qkv"], n1)
        heads, dh = p["heads"], p["dim_head"]
        a, lse = K.attention_fwd_lse(qkv, qkv[..., C:], qkv[..., 2 * C:], B, heads, dh, N, N, 3 * C, 3 * C, 3 * C)
        h1 = K.linear(p["out1"], a, residual=h0)
        n3 = K.layer_norm(h1, *p["ln3"], 1e-5)
        hg = K.linear(p["ff1"], n3)                         # raw [h | g] interleave
        f = K.geglu_fwd(hg)
        h2 = K.linear(p["ff2"], f, residual=h1)
        out = K.conv2d(p["proj_out"], h2, B, H, W, residual=x, gn_stats=True)
        self.saved.append(("transformer", t, dict(x=x, mr=mr, g=g, h0=h0, n1=n1, qkv=qkv, a=a, lse=lse, h1=h1, n3=n3,
                                                  hg=hg, f=f, h2=h2, out=out, B=B, H=H, W=W)))
        return out

    def forward(self, sources, timestep):
        s0 = sources[0]
        with K.gn_arena(("unet_train", id(self.u), tuple(s0.shape), self.u.compute_dtype), s0.device):
            return self._forward(sources, timestep)

    def _forward(self, sources, timestep):
        u, P = self.u, self.P
        if any(p.requires_grad for p in u.time_embedding.parameters()):
            raise NotImplementedError("a trainable time_embedding is not supported on the native training path "
                                      "(the reference freezes it: freeze_layers ['time_embedding'])")
        dt = u.compute_dtype
        sample = sources[0]
        dev = sample.device
        B, _, H, W = sample.shape
        Cin = sum(s.shape[1] for s in sources)
        if Cin != u.conv_in.in_channels:
            raise ValueError(f"UNet expects {u.conv_in.in_channels} input channels, got {Cin}")
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep], device=dev)
        t = timestep.reshape(-1).to(device=dev, dtype=torch.float32)
        emb = K.timestep_proj(t, B, P["freqs"], u.time_proj.num_channels, u.time_proj.flip_sin_to_cos, dt)
        emb = K.linear(P["lin1"], emb, act=K.ACT_SILU)
        semb = K.linear(P["lin2"], emb, act=K.ACT_SILU)
        temb_all = K.linear(P["temb_proj"], semb, out_dtype=torch.float32)
        self.semb, self.B = semb, B
        x_in = K.nchw_to_nhwc(sources, P["cin_pad"], dt)
        x = K.conv2d(P["conv_in"], x_in, B, H, W, gn_stats=True)
        self.saved.append(("conv_in", None, dict(x=x_in, out=x, B=B, H=H, W=W)))
        skips = [(x, H, W)]
        for blk in u.down_blocks:
            for j, r in enumerate(blk.resnets):
                x = self._resnet_fwd(r, x, None, B, H, W, temb_all)
                if blk.has_cross_attention:
                    x = self._transformer_fwd(blk.attentions[j], x, B, H, W)
                skips.append((x, H, W))
            if blk.downsamplers is not None:
                m = blk.downsamplers[0]
                xin = x
                x = K.conv2d(P[id(m)], xin, B, H, W, stride=2, gn_stats=True)
                self.saved.append(("down", m, dict(x=xin, out=x, B=B, H=H, W=W)))
                H, W = (H + 1) // 2, (W + 1) // 2
                skips.append((x, H, W))
        mb = u.mid_block
        x = self._resnet_fwd(mb.resnets[0], x, None, B, H, W, temb_all)
        x = self._transformer_fwd(mb.attentions[0], x, B, H, W)
        x = self._resnet_fwd(mb.resnets[1], x, None, B, H, W, temb_all)
        for blk in u.up_blocks:
            for j, r in enumerate(blk.resnets):
                s, sh, sw = skips.pop()
                x = self._resnet_fwd(r, x, s, B, H, W, temb_all)
                if blk.has_cross_attention:
                    x = self._transformer_fwd(blk.attentions[j], x, B, H, W)
            if blk.upsamplers is not None:
                m = blk.upsamplers[0]
                xin = x
                x = K.conv2d(P[id(m)], xin, B, H, W, upsample=True, gn_stats=True)
                self.saved.append(("up", m, dict(x=xin, out=x, B=B, H=H, W=W)))
                H, W = 2 * H, 2 * W
        hn, mr = K.group_norm_train(x, B, H * W, u.conv_norm_out.num_groups, *P["out_norm"], u.conv_norm_out.eps,
                                    K.ACT_SILU)
        out = K.conv2d(P["conv_out"], hn, B, H, W, out_layout=K.OUT_NCHW)
        self.saved.append(("out", None, dict(x=x, mr=mr, hn=hn, B=B, H=H, W=W)))
        return out

    # ------------------------------------------------------------------ backward pieces
    def _dgrad(self, key, dy, B, H, W, **kw):
        return K.conv2d(self.Pd[key], dy, B, H, W, **kw)

    def _resnet_bwd(self, r, s, dout):
        p = self.P[id(r)]
        B, H, W = s["B"], s["H"], s["W"]
        M = B * H * W
        x0, x1 = s["x0"], s["x1"]
        # conv2 (+ bias) ; residual branch
        self._wgrad(p["c2"], r.conv2.weight, s["h2"], B, H, W, dout)
        self._bgrad(r.conv2.bias, dout, M, r.out_channels)
        dh2 = self._dgrad(id(r.conv2), dout, B, H, W)
        add = dout
        if p["sc"] is not None:
            self._wgrad(p["sc"], r.conv_shortcut.weight, x0, B, H, W, dout, x1=x1)
            self._bgrad(r.conv_shortcut.bias, dout, M, r.out_channels)
            add = self._dgrad(id(r.conv_shortcut), dout, B, H, W)          # [M, c0 + c1]
        # norm2 + SiLU
        dg2, db2, acc2 = self._sink_pair(r.norm2.weight, r.norm2.bias)
        dy1, _ = K.group_norm_bwd(s["y1"], B, H * W, r.groups, s["mr2"], *p["n2"], K.ACT_SILU, dh2, dgamma=dg2,
                                  dbeta=db2, acc_params=acc2)
        # conv1 (+ bias + time embedding)
        self._wgrad(p["c1"], r.conv1.weight, s["h1"], B, H, W, dy1)
        self._bgrad(r.conv1.bias, dy1, M, r.out_channels)
        K.colsum(dy1, M, r.out_channels, B, out=self._dtemb_slice(p["off"], r.out_channels))   # d temb [B, Cout]
        dh1 = self._dgrad(id(r.conv1), dy1, B, H, W)
        # norm1 + SiLU, plus the residual / shortcut gradient, into the input buffers
        dg1, db1, acc1 = self._sink_pair(r.norm1.weight, r.norm1.bias)
        b0, e0 = self.G.get(x0)
        b1, e1 = (self.G.get(x1) if x1 is not None else (None, False))
        K.group_norm_bwd(x0, B, H * W, r.groups, s["mr1"], *p["n1"], K.ACT_SILU, dh1, x1=x1, add_src=add, dx0=b0,
                         dx1=b1, acc0=e0, acc1=e1, dgamma=dg1, dbeta=db1, acc_params=acc1)
        # time_emb_proj's gradient is written by _temb_bwd after the whole graph: report it there
        temb = {id(q) for q in r.time_emb_proj.parameters()}
        self.on_ready([q for q in r.parameters() if q.requires_grad and id(q) not in temb])

    def _dtemb_slice(self, off, n):
        return self.dtemb_parts.setdefault(off, torch.empty(self.B, n, dtype=torch.float32, device=self.dev))

    def _transformer_bwd(self, t, s, dout):
        p = self.P[id(t)]
        tb = t.transformer_blocks[0]
        a1 = tb.attn1
        B, H, W = s["B"], s["H"], s["W"]
        N = H * W
        M = B * N
        C = s["x"].shape[-1]
        heads, dh = p["heads"], p["dim_head"]
        # proj_out (+ residual x)
        self._wgrad(p["proj_out"], t.proj_out.weight, s["h2"], B, H, W, dout)
        self._bgrad(t.proj_out.bias, dout, M, C)
        dh2 = self._dgrad(id(t.proj_out), dout, M, 1, 1)
        # ff.net.2 (+ residual h1)
        self._wgrad(p["ff2"], tb.ff.net[2].weight, s["f"], M, 1, 1, dh2)
        self._bgrad(tb.ff.net[2].bias, dh2, M, C)
        df = self._dgrad(id(tb.ff.net[2]), dh2, M, 1, 1)
        # GEGLU + ff.net.0
        dhg = K.geglu_bwd(s["hg"], df)
        self._wgrad(p["ff1"], tb.ff.net[0].proj.weight, s["n3"], M, 1, 1, dhg)
        self._bgrad(tb.ff.net[0].proj.bias, dhg, M, dhg.shape[-1], geglu=True)
        dn3 = self._dgrad(id(tb.ff.net[0].proj), dhg, M, 1, 1)
        # norm3 (+ the residual-stream gradient dh2)
        dg, db, acc = self._sink_pair(tb.norm3.weight, tb.norm3.bias)
        dh1 = K.layer_norm_bwd(s["h1"], dn3, p["ln3"][0], 1e-5, add_src=dh2, dgamma=dg, dbeta=db, acc_params=acc)
        # to_out (+ residual h0)
        self._wgrad(p["out1"], a1.to_out[0].weight, s["a"], M, 1, 1, dh1)
        self._bgrad(a1.to_out[0].bias, dh1, M, C)
        da = self._dgrad(id(a1.to_out[0]), dh1, M, 1, 1)
        # attention
        qkv = s["qkv"]
        dqkv = torch.empty_like(qkv)
        K.attention_bwd(qkv, qkv[..., C:], qkv[..., 2 * C:], s["a"], da, s["lse"], B, heads, dh, N, N, 3 * C, 3 * C,
                        3 * C, dqkv, dqkv[..., C:], dqkv[..., 2 * C:], 3 * C, 3 * C)
        # fused QKV projection
        if a1.to_q.weight.requires_grad:
            sinks = [self.sink(lin.weight) for lin in (a1.to_q, a1.to_k, a1.to_v)]
            d0 = sinks[0][0]
            st0 = d0.untyped_storage().data_ptr()
            adjacent = all(d.untyped_storage().data_ptr() == st0 and d.data_ptr() == d0.data_ptr() + i * d0.numel() * 4
                           and d.is_contiguous() and a == sinks[0][1] for i, (d, a) in enumerate(sinks))
            if adjacent:
                # the trainer's flat buffer keeps to_q / to_k / to_v back to back: the fused [3C][C]
                # weight gradient lands in place (no temporary, no copies)
                dw = d0.as_strided((3 * C, C), (C, 1))
                K.conv2d_wgrad(p["qkv"], s["n1"], M, 1, 1, dqkv, dw=dw, accumulate=sinks[0][1])
            else:
                wq = torch.empty(3 * C, C, dtype=torch.float32, device=qkv.device)
                K.conv2d_wgrad(p["qkv"], s["n1"], M, 1, 1, dqkv, dw=wq)
                for i, (dst, accq) in enumerate(sinks):
                    if accq:
                        dst.add_(wq[i * C:(i + 1) * C].view_as(dst))
                    else:
                        dst.copy_(wq[i * C:(i + 1) * C].view_as(dst))
        dn1 = self._dgrad(id(a1), dqkv, M, 1, 1)
        # norm1 (+ residual dh1)
        dg, db, acc = self._sink_pair(tb.norm1.weight, tb.norm1.bias)
        dh0 = K.layer_norm_bwd(s["h0"], dn1, p["ln1"][0], 1e-5, add_src=dh1, dgamma=dg, dbeta=db, acc_params=acc)
        # proj_in
        self._wgrad(p["proj_in"], t.proj_in.weight, s["g"], B, H, W, dh0)
        self._bgrad(t.proj_in.bias, dh0, M, C)
        dgn = self._dgrad(id(t.proj_in), dh0, M, 1, 1)
        # GroupNorm (eps 1e-6, no act) + the outer residual gradient, into x's buffer
        dg, db, acc = self._sink_pair(t.norm.weight, t.norm.bias)
        bx, ex = self.G.get(s["x"])
        K.group_norm_bwd(s["x"], B, N, t.groups, s["mr"], *p["norm"], K.ACT_NONE, dgn, add_src=dout, dx0=bx, acc0=ex,
                         dgamma=dg, dbeta=db, acc_params=acc)
        self.on_ready([q for q in t.parameters() if q.requires_grad])

    def backward(self, d_out_nchw):
        u, P = self.u, self.P
        self.dev = d_out_nchw.device
        self.dtemb_parts = {}
        dt = u.compute_dtype
        for kind, m, s in reversed(self.saved):
            if kind == "out":
                B, H, W = s["B"], s["H"], s["W"]
                M = B * H * W
                dy = K.nchw_to_nhwc([d_out_nchw], 8, dt)                     # 4 channels padded to 8
                if u.conv_out.weight.requires_grad:
                    tmp = K.conv2d_wgrad(P["conv_out_t"], s["hn"], B, H, W, dy)
                    dst, acc = self.sink(u.conv_out.weight)
                    (dst.add_ if acc else dst.copy_)(tmp[:u.conv_out.out_channels])
                if u.conv_out.bias is not None and u.conv_out.bias.requires_grad:
                    tb = K.colsum(dy, M, 8)
                    dst, acc = self.sink(u.conv_out.bias)
                    (dst.add_ if acc else dst.copy_)(tb.view(-1)[:u.conv_out.out_channels])
                dhn = self._dgrad("conv_out", dy, B, H, W)
                dg, db, acc = self._sink_pair(u.conv_norm_out.weight, u.conv_norm_out.bias)
                bx, ex = self.G.get(s["x"])
                K.group_norm_bwd(s["x"], B, H * W, u.conv_norm_out.num_groups, s["mr"], *P["out_norm"], K.ACT_SILU,
                                 dhn, dx0=bx, acc0=ex, dgamma=dg, dbeta=db, acc_params=acc)
                self.on_ready([q for q in (u.conv_out.weight, u.conv_out.bias, u.conv_norm_out.weight,
                                           u.conv_norm_out.bias) if q is not None and q.requires_grad])
                continue
            dout = self.G.pop(s["out"])
            if kind == "resnet":
                self._resnet_bwd(m, s, dout)
            elif kind == "transformer":
                self._transformer_bwd(m, s, dout)
            elif kind == "up":
                B, H, W = s["B"], s["H"], s["W"]
                self._wgrad(P[id(m)], m.conv.weight, s["x"], B, H, W, dout, upsample=True)
                self._bgrad(m.conv.bias, dout, B * 4 * H * W, m.conv.out_channels)
                du = self._dgrad(id(m), dout, B, 2 * H, 2 * W)
                bx, ex = self.G.get(s["x"])
                K.sum_pool2(du, B, H, W, out=bx, accumulate=ex)
                self.on_ready([q for q in m.parameters() if q.requires_grad])
            elif kind == "down":
                B, H, W = s["B"], s["H"], s["W"]
                Ho, Wo = (H + 1) // 2, (W + 1) // 2
                self._wgrad(P[id(m)], m.conv.weight, s["x"], B, H, W, dout, stride=2)
                self._bgrad(m.conv.bias, dout, B * Ho * Wo, m.conv.out_channels)
                if H % 2 or W % 2:
                    raise NotImplementedError("stride-2 data gradient needs even spatial sizes")
                bx, ex = self.G.get(s["x"])
                self._dgrad(id(m), dout, B, Ho, Wo, upsample=2, out=bx, residual=bx if ex else None)
                self.on_ready([q for q in m.parameters() if q.requires_grad])
            elif kind == "conv_in":
                B, H, W = s["B"], s["H"], s["W"]
                self._wgrad(P["conv_in"], u.conv_in.weight, s["x"], B, H, W, dout)
                self._bgrad(u.conv_in.bias, dout, B * H * W, u.conv_in.out_channels)
                self.on_ready([q for q in u.conv_in.parameters() if q.requires_grad])
        # batched time_emb_proj: d temb_all [B, sum Cout] -> weight / bias of every ResNet's
        # time_emb_proj (the per-ResNet slices are adjacent in the packed GEMM)
        self._temb_bwd()
        self.saved.clear()

    def _temb_bwd(self):
        u, P = self.u, self.P
        resnets = P["resnets"]
        if not any(r.time_emb_proj.weight.requires_grad for r in resnets):
            return
        total = P["temb_total"]
        offs = sorted(self.dtemb_parts)
        if offs == [P[id(r), "temb_off"] for r in resnets]:       # every ResNet reported: one cat
            dtemb = torch.cat([self.dtemb_parts[o] for o in offs], dim=1)
        else:
            dtemb = torch.zeros(self.B, total, dtype=torch.float32, device=self.dev)
            for off, part in self.dtemb_parts.items():
                dtemb[:, off:off + part.shape[1]] = part
        dy = dtemb.to(u.compute_dtype).contiguous()
        wt = K.conv2d_wgrad(P["temb_proj"], self.semb, self.B, 1, 1, dy)        # [total, 1280] fp32
        bt = K.colsum(dtemb, self.B, total).view(-1)
        # scatter to the 22 ResNets' parameters with one multi-tensor launch per mode
        put, add = ([], []), ([], [])
        for r in resnets:
            off, n = P[id(r), "temb_off"], r.out_channels
            for prm, val in ((r.time_emb_proj.weight, wt[off:off + n]), (r.time_emb_proj.bias, bt[off:off + n])):
                if prm.requires_grad:
                    dst, acc = self.sink(prm)
                    tgt = add if acc else put
                    tgt[0].append(dst)
                    tgt[1].append(val.view_as(dst))
        if put[0]:
            torch._foreach_copy_(put[0], put[1])
        if add[0]:
            torch._foreach_add_(add[0], add[1])
        self.on_ready([q for r in resnets for q in r.time_emb_proj.parameters() if q.requires_grad])
