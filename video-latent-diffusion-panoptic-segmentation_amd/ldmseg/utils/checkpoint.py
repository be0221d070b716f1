"""Checkpoint round-trip in the reference's on-disk layouts.

LDM ``model.pt`` (TrainerDiffusion.construct_save_dict / save / resume / load,
trainers_ldm_cond.py:1844-1944): a torch.save'd dict with keys
``step, epoch, vae_image, vae_semseg, unet, ema, opt, p, scaler`` — ``unet`` with diffusers key
names plus the ``new_conv.*`` alias of ``conv_in.*`` (unet.py:182,233), ``vae_semseg`` with the
nn.Sequential indices, ``opt`` a torch.optim.AdamW state_dict.  ``best_model.pt`` adds ``PQ``.
AE ``model.pt`` (TrainerAE, trainers_ae.py:534-587): ``step, epoch, vae (module.-prefixed),
opt, p, scaler``; GeneralVAESeg.load_pretrained (vae.py:117-122) strips ``module.``.

Loading uses ``torch.load(..., weights_only=True)`` by default: checkpoints written by this
package hold only tensors and plain containers.  A reference run stores its Hydra/EasyDict
config under ``p``, which the safe loader refuses; pass ``weights_only=False`` only for a file
you wrote yourself and trust.
"""
import torch
import torch.nn as nn

LDM_KEYS = ("step", "epoch", "vae_image", "vae_semseg", "unet", "ema", "opt", "p", "scaler")


def unwrap(model):
    """DistributedDataParallel -> its module (trainers_ldm_cond.py:1845-1848)."""
    return model.module if isinstance(model, nn.parallel.DistributedDataParallel) else model


def strip_module_prefix(sd):
    """``module.``-prefixed DDP keys -> plain keys (vae.py:119)."""
    return {k.replace("module.", ""): v for k, v in sd.items()}


def _plain(p):
    """Config -> plain dict/list/scalars (EasyDict / OmegaConf-like objects are dicts)."""
    if isinstance(p, dict):
        return {str(k): _plain(v) for k, v in p.items()}
    if isinstance(p, (list, tuple)):
        return [_plain(v) for v in p]
    return p


def construct_save_dict(unet, vae_semseg, vae_image=None, step=0, epoch=None, ema=None, opt=None, p=None,
                        scaler=None):
    """The reference's construct_save_dict (:1844-1867); ``opt`` is anything with state_dict()
    (torch optimizer or ldmseg.trainers.LDMTrainStep)."""
    return {
        "step": step,
        "epoch": epoch,
        "vae_image": vae_image.state_dict() if vae_image is not None else {},
        "vae_semseg": vae_semseg.state_dict(),
        "unet": unwrap(unet).state_dict(),
        "ema": ema.state_dict() if ema is not None else None,
        "opt": opt.state_dict() if opt is not None else None,
        "p": _plain(p) if p is not None else None,
        "scaler": scaler.state_dict() if scaler is not None else None,
    }


def save(path, **kw):
    """rank-0 ``torch.save(construct_save_dict(...), path)`` (:1869-1877).  Call it on EVERY
    rank: a sharded (ZeRO) optimizer is consolidated collectively first, then rank 0 alone
    builds and writes the dict."""
    import torch.distributed as dist
    opt = kw.get("opt")
    dist_on = dist.is_available() and dist.is_initialized()
    writer = 0                              # global rank that builds and writes the dict
    if hasattr(opt, "consolidate_state_dict"):
        # consolidate onto the writer: `to` is a rank of the optimizer's own process group, so map
        # global rank 0 into it; a group without global rank 0 consolidates to (and is written by)
        # its own first rank
        # (LDMTrainStep keeps its group in `group`, torch ZeroRedundancyOptimizer in `process_group`)
        to, group = 0, getattr(opt, "group", None) or getattr(opt, "process_group", None)
        if dist_on and group is not None:
            try:
                to = dist.get_group_rank(group, 0)
            except (ValueError, RuntimeError):
                writer = dist.get_global_rank(group, 0)
        opt.consolidate_state_dict(to=to)
    if dist_on and dist.get_rank() != writer:
        return
    torch.save(construct_save_dict(**kw), str(path))


def read(path, weights_only=True):
    return torch.load(str(path), map_location="cpu", weights_only=weights_only)


def load(path, unet, vae_semseg=None, ema=None, load_vae=True, weights_only=True):
    """TrainerDiffusion.load (:1916-1944): strict UNet (+ seg-VAE, + EMA) weights."""
    data = read(path, weights_only)
    unwrap(unet).load_state_dict(data["unet"])
    if load_vae and vae_semseg is not None:
        vae_semseg.load_state_dict(data["vae_semseg"])
    if ema is not None:
        ema.load_state_dict(data["ema"])
    if hasattr(unwrap(unet), "invalidate_packed"):
        unwrap(unet).invalidate_packed()
    return data


def resume(path, unet, vae_semseg=None, vae_image=None, opt=None, ema=None, scaler=None, load_vae=True,
           num_iters_per_epoch=1, weights_only=True):
    """TrainerDiffusion.resume (:1879-1914).  Returns (data, start_epoch, step) with
    start_epoch = epoch + 1 and step = (epoch + 1) * num_iters_per_epoch + 1 (:1901-1902)."""
    data = read(path, weights_only)
    unwrap(unet).load_state_dict(data["unet"])
    if load_vae:
        if vae_image is not None and data.get("vae_image"):
            vae_image.load_state_dict(data["vae_image"])
        if vae_semseg is not None:
            vae_semseg.load_state_dict(data["vae_semseg"])
    if opt is not None and data.get("opt") is not None:
        opt.load_state_dict(data["opt"])
    if ema is not None and data.get("ema") is not None:
        ema.load_state_dict(data["ema"])
    if scaler is not None and data.get("scaler") is not None:
        scaler.load_state_dict(data["scaler"])
    if hasattr(unwrap(unet), "invalidate_packed"):
        unwrap(unet).invalidate_packed()
    epoch = data["epoch"]
    return data, epoch + 1, (epoch + 1) * num_iters_per_epoch + 1


def save_ae(path, vae, step=0, epoch=None, opt=None, p=None, scaler=None, ddp_prefix=True):
    """TrainerAE's layout (trainers_ae.py:540-548): ``vae`` keys carry DDP's ``module.`` prefix."""
    sd = unwrap(vae).state_dict()
    if ddp_prefix:
        sd = {f"module.{k}": v for k, v in sd.items()}
    torch.save({"step": step, "epoch": epoch, "vae": sd, "opt": opt.state_dict() if opt is not None else None,
                "p": _plain(p) if p is not None else None,
                "scaler": scaler.state_dict() if scaler is not None else None}, str(path))
