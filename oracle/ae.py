"""One AE training iteration (TrainerAE, row a16) — torch fp32 CPU restatement (test infrastructure
only, see oracle/__init__.py); autograd supplies the backward.

Follows:
  trainers_ae.py:293-331       images = 2 * bits - 1; vae(images, sample_posterior=True);
                               loss = ce + mask (+ 0 * kl)
  vae.py:371-413               posterior sample mean + std * randn
  losses.py:117-185, 330-395   loss_masks / loss_ce with uncertainty point sampling
  losses.py:187-247, 284-311   dice / sigmoid-CE, calculate_uncertainty(_seg)
  losses.py:399-440            prepare_targets (one mask per class present, != ignore)
  detectron2_utils.py:20-100   get_uncertain_point_coords_with_randomness, point_sample
Random draws come from the caller (``rand(*shape)``, ``randn(shape)``), selections optionally
forced (``select(u, k) -> idx``), so the reference's own draws can be replayed.
Pinned by tests/golden/ae.npz (the reference modules run with the same draws).
"""
import torch
import torch.nn.functional as F

from . import vae as ovae


def point_sample(x, coords, mode="bilinear"):
    return F.grid_sample(x, 2.0 * coords[:, :, None] - 1.0, mode=mode, align_corners=False)[..., 0]


def uncertain_coords(x, unc, rand, num_points, oversample, importance, select=None):
    n_s = int(num_points * oversample)
    coords = rand(x.shape[0], n_s, 2)
    u = unc(point_sample(x, coords))[:, 0]
    n_u = int(importance * num_points)
    idx = select(u, n_u).long() if select is not None else torch.topk(u, k=n_u, dim=1)[1]
    sel = torch.gather(coords, 1, idx[:, :, None].expand(-1, -1, 2))
    if num_points - n_u > 0:
        sel = torch.cat([sel, rand(x.shape[0], num_points - n_u, 2)], dim=1)
    return sel


def point_losses(logits, targets, rand, ignore_label=0, num_points=12544, oversample=3, importance=0.75,
                 temperature=1.0, select=None):
    def unc_seg(pl):
        t = torch.topk(pl, k=2, dim=1)[0]
        return (t[:, 1] - t[:, 0]).unsqueeze(1)

    with torch.no_grad():
        c = uncertain_coords(logits.detach(), unc_seg, rand, num_points, oversample, importance, select)
        lab = point_sample(targets[:, None].float(), c, mode="nearest")[:, 0].long()
    ce = F.cross_entropy(point_sample(logits, c) / temperature, lab, ignore_index=ignore_label)
    src, tgt = [], []
    for b in range(targets.shape[0]):
        for k in torch.unique(targets[b]):
            if int(k) == ignore_label:
                continue
            src.append(logits[b, int(k)])
            tgt.append((targets[b] == k).float())
    if not src:
        return ce, logits.sum() * 0.0
    sm = torch.stack(src)[:, None]
    tm = torch.stack(tgt)[:, None]
    nm = max(float(len(src)), 1.0)
    with torch.no_grad():
        mc = uncertain_coords(sm.detach(), lambda v: -torch.abs(v), rand, num_points, oversample, importance, select)
        ml = point_sample(tm, mc)[:, 0]
    mp = point_sample(sm, mc)[:, 0]
    bce = F.binary_cross_entropy_with_logits(mp, ml, reduction="none").mean(1).sum() / nm
    s = mp.sigmoid()
    dice = (1 - (2 * (s * ml).sum(-1) + 1) / (s.sum(-1) + ml.sum(-1) + 1)).sum() / nm
    return ce, bce + dice


def train_iteration(sd, cfg, bits, targets, rand, randn, select=None):
    """-> (loss, ce, mask, {param name: grad}) for weights ``sd`` (reference key names)."""
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    x = 2.0 * bits - 1.0
    moments = ovae.run_sequential(x, ovae.encoder_spec(cfg["in_channels"], cfg["block_out_channels"],
                                                       cfg["int_channels"], cfg["latent_channels"],
                                                       cfg.get("num_latents", 2)),
                                  params, "encoder", cfg["norm_num_groups"])
    mean, logvar = torch.chunk(moments, 2, dim=1)
    std = torch.exp(0.5 * logvar.clamp(-30.0, 20.0))
    z = mean + std * randn(mean.shape)
    logits = ovae.run_sequential(z, ovae.decoder_spec(cfg.get("num_upscalers", 1)), params, "decoder",
                                 cfg["norm_num_groups"])
    ce, mask = point_losses(logits, targets, rand, select=select)
    loss = ce + mask
    loss.backward()
    return loss.detach(), ce.detach(), mask.detach(), {k: p.grad for k, p in params.items()}
