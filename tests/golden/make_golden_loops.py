"""Golden vectors for the LOOP-level semantics of the reference trainer, made by running the
reference's own methods on stand-in objects (build container only; needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_loops.py

The UNet arithmetic of the reference lives in the un-vendored diffusers package, so every run
below that needs a UNet injects "oracle blocks": callables with the diffusers block signatures
(CrossAttnDownBlock2D / UNetMidBlock2DCrossAttn / CrossAttnUpBlock2D / ...) that compute with
oracle/unet.py on a state dict whose tensors are the parameters of this build's UNet module tree
(diffusers names and module types, loaded here under the alias ``ldmseg_amd`` so it does not
clash with the reference package).  What is pinned is the reference's own code around them:

  loops.npz
    modify__*     UNet.modify_encoder (unet.py:124-233) on a 4->320 conv_in shell, every
                  init-mode combination that does not raise; sha256 of the resulting conv_in
                  weight/bias + the full tensors of three combinations
    fwd__*        UNet.forward (unet.py:281-436) with oracle blocks: 0-d and per-frame [B]
                  timesteps, 12-channel input (self-conditioning layout)
    sample__*     TrainerDiffusion.sample (trainers_ldm_cond.py:1048-1173), self_condition
                  off / on, and return_all_latents
    enc__*        TrainerDiffusion.encode_inputs (:336-396) with the reference GeneralVAESeg
                  (vae.npz "kitti" weights): tuple resize, int resize, resize=None
    train__*      TrainerDiffusion.train_single_epoch (:792-900) for two iterations: self-cond
                  pre-pass, compute_loss (:530-619, l2, SNR weights, loss mask),
                  update_weights (:769-781: clip_grad_norm_ + AdamW of get_optim_unet); the
                  torch.randn_like / torch.randint draws are recorded; losses and the parameter
                  updates (full tensors for a named subset, L2 norms for all) are stored
    optim__*      get_optim_unet (optim.py:53-82) parameter groups: names, lr, weight_decay
    save__*       construct_save_dict (:1844-1867) keys, and resume (:1879-1914) of a file
                  written by this build's utils/checkpoint.save: start_epoch / step
    cmap          ldmseg/utils/utils.py color_map() (decode_latents' colour table)
"""
import functools
import hashlib
import importlib.util
import os
import sys
import tempfile
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (golden_utils)
sys.path.insert(0, ROOT)                            # oracle/
import _refstubs  # noqa: E402

_refstubs.install()

from golden_utils import LOOP_UNET, VAE_CONFIGS, build_loop_unet, load, state_hash, vae_state_dict  # noqa: E402
from oracle import unet as ounet  # noqa: E402

PKG = os.path.join(ROOT, "video-latent-diffusion-panoptic-segmentation_amd", "ldmseg")


def load_amd():
    """This build's package under the alias ``ldmseg_amd`` (its imports are all relative)."""
    if "ldmseg_amd" in sys.modules:
        return sys.modules["ldmseg_amd"]
    spec = importlib.util.spec_from_file_location("ldmseg_amd", os.path.join(PKG, "__init__.py"),
                                                  submodule_search_locations=[PKG])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ldmseg_amd"] = mod
    spec.loader.exec_module(mod)
    for sub in ("models", "utils", "utils.checkpoint"):
        importlib.import_module(f"ldmseg_amd.{sub}")
    return mod


# --------------------------------------------------------------------------------------
# oracle blocks with the diffusers call signatures
# --------------------------------------------------------------------------------------
class _Down:
    def __init__(self, sd, i, n, lpb, attn, G, eps, heads):
        self.sd, self.i, self.n, self.lpb, self.G, self.eps, self.heads = sd, i, n, lpb, G, eps, heads
        self.has_cross_attention = attn

    def __call__(self, hidden_states, temb, encoder_hidden_states=None, attention_mask=None,
                 cross_attention_kwargs=None):
        h, out = hidden_states, ()
        for j in range(self.lpb):
            h = ounet.resnet(self.sd, f"down_blocks.{self.i}.resnets.{j}", h, temb, self.G, self.eps)
            if self.has_cross_attention:
                h = ounet.transformer(self.sd, f"down_blocks.{self.i}.attentions.{j}", h, encoder_hidden_states,
                                      self.G, self.heads)
            out += (h,)
        if self.i < self.n - 1:
            h = ounet._conv(self.sd, f"down_blocks.{self.i}.downsamplers.0.conv", h, stride=2)
            out += (h,)
        return h, out


class _Mid:
    def __init__(self, sd, G, eps, heads):
        self.sd, self.G, self.eps, self.heads = sd, G, eps, heads

    def __call__(self, hidden_states, temb, encoder_hidden_states=None, attention_mask=None,
                 cross_attention_kwargs=None):
        h = ounet.resnet(self.sd, "mid_block.resnets.0", hidden_states, temb, self.G, self.eps)
        h = ounet.transformer(self.sd, "mid_block.attentions.0", h, encoder_hidden_states, self.G, self.heads)
        return ounet.resnet(self.sd, "mid_block.resnets.1", h, temb, self.G, self.eps)


class _Up:
    def __init__(self, sd, i, n, lpb, attn, G, eps, heads):
        self.sd, self.i, self.n, self.G, self.eps, self.heads = sd, i, n, G, eps, heads
        self.has_cross_attention = attn
        self.resnets = [None] * (lpb + 1)

    def __call__(self, hidden_states, temb, res_hidden_states_tuple, encoder_hidden_states=None,
                 cross_attention_kwargs=None, upsample_size=None, attention_mask=None):
        h, res = hidden_states, res_hidden_states_tuple
        for j in range(len(self.resnets)):
            h = torch.cat([h, res[-1]], dim=1)
            res = res[:-1]
            h = ounet.resnet(self.sd, f"up_blocks.{self.i}.resnets.{j}", h, temb, self.G, self.eps)
            if self.has_cross_attention:
                h = ounet.transformer(self.sd, f"up_blocks.{self.i}.attentions.{j}", h, encoder_hidden_states,
                                      self.G, self.heads)
        if self.i < self.n - 1:
            h = F.interpolate(h, scale_factor=2.0, mode="nearest") if upsample_size is None else \
                F.interpolate(h, size=upsample_size, mode="nearest")
            h = ounet._conv(self.sd, f"up_blocks.{self.i}.upsamplers.0.conv", h)
        return h


def oracle_unet_shell(module):
    """An object the reference UNet.forward (unet.py:281-436) can run on: its attributes are
    oracle blocks over ``module``'s parameters (autograd flows into them)."""
    cfg = dict(module.config)
    sd = dict(module.state_dict(keep_vars=True))
    G, eps, heads = cfg.get("norm_num_groups", 32), cfg.get("norm_eps", 1e-5), cfg.get("attention_head_dim", 8)
    boc, lpb = list(cfg["block_out_channels"]), cfg.get("layers_per_block", 2)
    downs, ups = cfg["down_block_types"], cfg["up_block_types"]
    ns = types.SimpleNamespace()
    ns.dtype = torch.float32
    ns.time_proj = lambda t: ounet.timestep_proj(t, boc[0], cfg.get("flip_sin_to_cos", True), cfg.get("freq_shift", 0))
    ns.time_embedding = lambda x, cond=None: ounet._lin(sd, "time_embedding.linear_2",
                                                        F.silu(ounet._lin(sd, "time_embedding.linear_1", x)))
    ns.encoder_hid_proj = None
    ns.conv_in = lambda x: ounet._conv(sd, "conv_in", x)
    ns.down_blocks = [_Down(sd, i, len(downs), lpb, "CrossAttn" in bt, G, eps, heads) for i, bt in enumerate(downs)]
    ns.mid_block = _Mid(sd, G, eps, heads)
    ns.up_blocks = [_Up(sd, i, len(ups), lpb, "CrossAttn" in bt, G, eps, heads) for i, bt in enumerate(ups)]
    ns.conv_norm_out = lambda x: F.group_norm(x, G, sd["conv_norm_out.weight"], sd["conv_norm_out.bias"], eps)
    ns.conv_act = F.silu
    ns.conv_out = lambda x: ounet._conv(sd, "conv_out", x)
    return ns


class RefUNetModel:
    """``self.unet_model`` of a stand-in trainer: reference UNet.forward over oracle blocks."""

    def __init__(self, module):
        from ldmseg.models.unet import UNet as RefUNet
        self.m, self.shell, self.fwd = module, oracle_unet_shell(module), RefUNet.forward

    def __call__(self, sample, timestep, encoder_hidden_states=None, timestep_img=None, **kw):
        out = self.fwd(self.shell, sample, timestep, encoder_hidden_states, timestep_img=timestep_img)
        # CPU conv2d may hand back a channels-last result; the GPU diffusers UNet's output is
        # contiguous, which compute_loss's ``loss.view(-1)`` (:601) relies on
        out.sample = out.sample.contiguous()
        return out

    def parameters(self):
        return self.m.parameters()


def _sha(*tensors):
    h = hashlib.sha256()
    for t in tensors:
        h.update(t.detach().contiguous().float().numpy().tobytes())
    return h.hexdigest()


# --------------------------------------------------------------------------------------
# modify_encoder
# --------------------------------------------------------------------------------------
MODES = ("copy", "div", "mean", "zero", "random")


def modify_cases():
    """(seg, image, cond_channels, cond_mode) combinations the reference accepts."""
    cases = [(s, i, 0, "zero") for s in MODES for i in MODES]
    for s in ("copy", "random"):
        for i in MODES:
            for c in ("zero", "random", "mean"):
                if c == "mean" and i != "mean":
                    continue                       # raises in the reference (:229-230)
                cases.append((s, i, 4, c))
    return cases


def gen_modify(out):
    from ldmseg.models.unet import UNet as RefUNet
    cases = modify_cases()
    full = {("copy", "zero", 0, "zero"), ("mean", "random", 4, "random"), ("div", "mean", 4, "mean")}
    for k, (s, i, c, cm) in enumerate(cases):
        torch.manual_seed(100 + k)
        shell = torch.nn.Module()
        shell.conv_in = torch.nn.Conv2d(4, 320, 3, padding=1)
        RefUNet.modify_encoder(shell, in_channels=8, init_mode_seg=s, init_mode_image=i, cond_channels=c,
                               init_mode_cond=cm)
        assert shell.conv_in is shell.new_conv
        out[f"modify__{k}__sha"] = np.array(_sha(shell.conv_in.weight, shell.conv_in.bias))
        if (s, i, c, cm) in full:
            out[f"modify__{k}__weight"] = shell.conv_in.weight.detach().numpy()
            out[f"modify__{k}__bias"] = shell.conv_in.bias.detach().numpy()
    out["modify__cases"] = np.array([f"{s},{i},{c},{cm}" for s, i, c, cm in cases])


# --------------------------------------------------------------------------------------
# forward / sample
# --------------------------------------------------------------------------------------
def _loop_unet():
    return build_loop_unet(load_amd().models.UNet)


def gen_forward(out):
    u = _loop_unet()
    out["unet__state_sha"] = np.array(state_hash(u))
    m = RefUNetModel(u)
    g = torch.Generator().manual_seed(31)
    x = torch.randn(2, 12, 16, 16, generator=g)
    with torch.no_grad():
        y0 = m(x, torch.tensor(731)).sample
        yb = m(x, torch.tensor([999, 19])).sample
    out["fwd__x"] = x.numpy()
    out["fwd__t0"] = np.int64(731)
    out["fwd__tb"] = np.array([999, 19], np.int64)
    out["fwd__out_t0"] = y0.numpy()
    out["fwd__out_tb"] = yb.numpy()


def _ref_scheduler(kind="base"):
    from golden_utils import DDIM_CONFIGS
    from ldmseg.schedulers.ddim_scheduler import DDIMNoiseScheduler
    return DDIMNoiseScheduler(**DDIM_CONFIGS[kind], device="cpu", verbose=False)


def gen_sample(out):
    from ldmseg.trainers.trainers_ldm_cond import TrainerDiffusion
    g = torch.Generator().manual_seed(41)
    B, L = 2, 16
    rgb = torch.randn(B, 4, L, L, generator=g)
    out["sample__rgb"] = rgb.numpy()
    for sc in (False, True):
        u8 = build_loop_unet(load_amd().models.UNet, cond=4 if sc else 0)
        fake = types.SimpleNamespace(
            noise_scheduler=_ref_scheduler(), args={"gpu": "cpu"}, image_descriptor_model=None, textencoder=None,
            self_condition=sc, unet_dtype=torch.float32, fp16_scaler=None, latent_size=L,
            unet_model=RefUNetModel(u8))
        lat = TrainerDiffusion.sample(fake, [""] * B, num_inference_steps=5, seed=0, rgb_latents=rgb,
                                      disable_progress_bar=True)
        out[f"sample__sc{int(sc)}__state_sha"] = np.array(state_hash(u8))
        out[f"sample__sc{int(sc)}__latents"] = lat.numpy()
        if sc:
            allv = TrainerDiffusion.sample(fake, [""] * B, num_inference_steps=3, seed=7, rgb_latents=rgb,
                                           disable_progress_bar=True, return_all_latents=True)
            out["sample__sc1__all3_seed7"] = allv.numpy()


# --------------------------------------------------------------------------------------
# encode_inputs
# --------------------------------------------------------------------------------------
def gen_encode(out):
    from ldmseg.models.vae import GeneralVAESeg
    from ldmseg.trainers.trainers_ldm_cond import TrainerDiffusion
    z = load("vae.npz")
    v = GeneralVAESeg(**VAE_CONFIGS["kitti"], encoder=None).eval()
    v.load_state_dict(vae_state_dict(z, "kitti"), strict=True)
    g = torch.Generator().manual_seed(51)
    fake = types.SimpleNamespace(latent_size=64, weight_dtype=torch.float32, vae_image=None)
    cases = {"tuple": ((100, 300), (192, 640)), "int": ((90, 130), 96), "none": ((96, 320), None)}
    for name, (hw, resize) in cases.items():
        x = (torch.rand(2, 10, *hw, generator=g) > 0.5).float()
        lat, lat_mean = TrainerDiffusion.encode_inputs(fake, x, encode_func=v.encode, scaling_factor=0.2,
                                                       resize=resize)
        assert torch.equal(lat, lat_mean)
        out[f"enc__{name}__x"] = x.numpy().astype(np.uint8)
        out[f"enc__{name}__resize"] = np.array([-1, -1] if resize is None else
                                               ([resize, resize] if isinstance(resize, int) else list(resize)))
        out[f"enc__{name}__is_int"] = np.bool_(isinstance(resize, int))
        out[f"enc__{name}__latents"] = lat.numpy()


# --------------------------------------------------------------------------------------
# train_single_epoch (two iterations)
# --------------------------------------------------------------------------------------
TRAIN_SUBSET = ("conv_in.weight", "conv_in.bias", "down_blocks.0.resnets.0.conv1.weight",
                "down_blocks.0.resnets.0.time_emb_proj.weight", "down_blocks.0.attentions.0.norm.weight",
                "down_blocks.1.attentions.0.transformer_blocks.0.attn1.to_q.weight",
                "mid_block.attentions.0.transformer_blocks.0.ff.net.0.proj.weight",
                "up_blocks.3.attentions.2.proj_out.bias", "up_blocks.1.upsamplers.0.conv.weight",
                "conv_norm_out.weight", "conv_out.weight", "conv_out.bias")
TRAIN_HP = dict(lr=1e-3, weight_decay=0.05, weight_decay_norm=0.0, clip_grad=1.0, lr_decay_rate=0.5)


class _Draws:
    """torch.randn_like / torch.randint replaced by seeded CPU draws, recorded in call order."""

    def __init__(self, seed):
        self.g = torch.Generator().manual_seed(seed)
        self.noise, self.t = [], []

    def __enter__(self):
        self.orig = (torch.randn_like, torch.randint)

        def randn_like(x, **kw):
            r = torch.randn(x.shape, generator=self.g, dtype=x.dtype)
            self.noise.append(r.clone())
            return r

        def randint(lo, hi, size, device=None, dtype=torch.long, **kw):
            r = self.orig[1](lo, hi, size, generator=self.g, dtype=dtype)
            self.t.append(r.clone())
            return r
        torch.randn_like, torch.randint = randn_like, randint
        return self

    def __exit__(self, *a):
        torch.randn_like, torch.randint = self.orig


def gen_train(out):
    import torch.distributed as dist
    import ldmseg.trainers.trainers_ldm_cond as T
    from ldmseg.models.unet import UNet as RefUNet
    from ldmseg.trainers.optim import get_optim_unet
    from ldmseg.utils import OutputDict
    u = build_loop_unet(load_amd().models.UNet, cond=4)
    u.train()
    out["train__state_sha"] = np.array(state_hash(u))
    before = {n: p.detach().clone() for n, p in u.named_parameters()}
    opt, _ = get_optim_unet(u, base_lr=TRAIN_HP["lr"], weight_decay=TRAIN_HP["weight_decay"],
                            weight_decay_norm=TRAIN_HP["weight_decay_norm"],
                            lr_factor_func=functools.partial(RefUNet.get_lr_func, u,
                                                             lr_decay_rate=TRAIN_HP["lr_decay_rate"]),
                            verbose=False)
    g = torch.Generator().manual_seed(61)
    B, L = 2, 16
    batches = []
    for _ in range(2):
        batches.append(dict(latents=torch.randn(B, 4, L, L, generator=g), rgb=torch.randn(B, 4, L, L, generator=g),
                            mask=(torch.rand(B, L, L, generator=g) > 0.1).float()))
    recorded = []

    class Meter:
        def update(self, val, n=1):
            recorded.append(val)
    fake = types.SimpleNamespace(
        dl=batches, noise_scheduler=_ref_scheduler("script"), min_noise_level=0, self_condition=True,
        fp16_scaler=None, unet_model=RefUNetModel(u), rgb_noise_level=0, cond_noise_level=0,
        training_loss_type="l2", ohem_ratio=1.0, gradient_accumulate_every=1, lr_scheduler=None,
        clip_grad=TRAIN_HP["clip_grad"], opt=opt, step=0, use_ema=False, print_freq=10 ** 6, batch_size_val=1)
    fake.process_inputs = lambda d: OutputDict(latents=d["latents"], rgb_latents=d["rgb"], loss_mask=d["mask"],
                                               encoder_hidden_states=None, original_latents=None,
                                               inpainting_masks=None, text=[""] * B)
    for meth in ("loss_fn", "compute_loss", "update_weights", "update_scheduler"):
        setattr(fake, meth, types.MethodType(getattr(T.TrainerDiffusion, meth), fake))
    fake.check_iter = lambda *a: False
    saved = (dist.barrier, torch.cuda.synchronize, T.gpu_gather)
    dist.barrier, torch.cuda.synchronize, T.gpu_gather = (lambda *a, **k: None), (lambda *a, **k: None), (lambda x: x)
    try:
        with _Draws(62) as dr:
            T.TrainerDiffusion.train_single_epoch(fake, 0, Meter(), {}, None)
    finally:
        dist.barrier, torch.cuda.synchronize, T.gpu_gather = saved
    assert len(dr.noise) == 2 and len(dr.t) == 2 and len(recorded) == 2
    for i, b in enumerate(batches):
        out[f"train__{i}__latents"] = b["latents"].numpy()
        out[f"train__{i}__rgb"] = b["rgb"].numpy()
        out[f"train__{i}__mask"] = b["mask"].numpy().astype(np.uint8)
        out[f"train__{i}__noise"] = dr.noise[i].numpy()
        out[f"train__{i}__t"] = dr.t[i].numpy()
    out["train__losses"] = np.array(recorded, np.float64)
    names = [n for n, p in u.named_parameters() if p.requires_grad]
    out["train__names"] = np.array(names)
    out["train__delta_norm"] = np.array([(p.detach() - before[n]).double().norm().item()
                                         for n, p in u.named_parameters() if p.requires_grad])
    for n in TRAIN_SUBSET:
        out[f"train__delta__{n}"] = (dict(u.named_parameters())[n].detach() - before[n]).numpy()
    out["train__hp"] = np.array([TRAIN_HP[k] for k in ("lr", "weight_decay", "weight_decay_norm", "clip_grad",
                                                        "lr_decay_rate")], np.float64)


# --------------------------------------------------------------------------------------
# get_optim_unet groups, construct_save_dict / resume
# --------------------------------------------------------------------------------------
def gen_optim(out):
    from ldmseg.models.unet import UNet as RefUNet
    from ldmseg.trainers.optim import get_optim_unet
    u = build_loop_unet(load_amd().models.UNet, cond=4)
    names = {id(p): n for n, p in u.named_parameters()}
    for tag, (wd, wdn, decay) in {"a": (0.05, 0.0, 0.5), "same_wd": (0.01, 0.01, 1.0)}.items():
        opt, save_optim = get_optim_unet(u, base_lr=1e-4, weight_decay=wd, weight_decay_norm=wdn,
                                         lr_factor_func=functools.partial(RefUNet.get_lr_func, u, lr_decay_rate=decay),
                                         verbose=False)
        assert save_optim
        groups = opt.param_groups
        out[f"optim__{tag}__hp"] = np.array([wd, wdn, decay], np.float64)
        out[f"optim__{tag}__lr"] = np.array([gr["lr"] for gr in groups], np.float64)
        out[f"optim__{tag}__wd"] = np.array([gr["weight_decay"] for gr in groups], np.float64)
        out[f"optim__{tag}__sizes"] = np.array([len(gr["params"]) for gr in groups], np.int64)
        out[f"optim__{tag}__names"] = np.array([names[id(p)] for gr in groups for p in gr["params"]])
        sd = opt.state_dict()
        out[f"optim__{tag}__group_keys"] = np.array(sorted(sd["param_groups"][0].keys()))


def gen_save(out):
    import torch.distributed.optim  # noqa: F401  (construct_save_dict reads dist.optim.ZeroRedundancyOptimizer)
    import ldmseg.trainers.trainers_ldm_cond as T
    from ldmseg.models.vae import GeneralVAESeg
    amd = load_amd()
    from ldmseg_amd.utils import checkpoint as ck
    u = build_loop_unet(amd.models.UNet, cond=4)
    vs = GeneralVAESeg(**VAE_CONFIGS["kitti"], encoder=None)
    opt = torch.optim.AdamW(u.parameters(), lr=1e-4)
    fake = types.SimpleNamespace(unet_model=u, save_optim=True, opt=opt, step=17, vae_image=torch.nn.Identity(),
                                 vae_semseg=vs, use_ema=False, p={"a": 1}, fp16_scaler=None)
    d = T.TrainerDiffusion.construct_save_dict(fake, epoch=3)
    out["save__keys"] = np.array(list(d))
    out["save__unet_keys"] = np.array(list(d["unet"]))
    out["save__vae_semseg_keys"] = np.array(list(d["vae_semseg"]))
    # the reference's resume() on a model.pt written by this build's checkpoint.save
    with tempfile.TemporaryDirectory() as tmp:
        ck.save(os.path.join(tmp, "model.pt"), unet=u, vae_semseg=vs, vae_image=torch.nn.Identity(), step=17, epoch=3,
                opt=opt, p={"a": 1})
        u2 = build_loop_unet(amd.models.UNet, cond=4, seed=9)
        vs2 = GeneralVAESeg(**VAE_CONFIGS["kitti"], encoder=None)
        fake2 = types.SimpleNamespace(results_folder=__import__("pathlib").Path(tmp), unet_model=u2,
                                      vae_image=torch.nn.Identity(), vae_semseg=vs2, num_iters_per_epoch=100,
                                      opt=torch.optim.AdamW(u2.parameters(), lr=1e-4), use_ema=False,
                                      fp16_scaler=None)
        T.TrainerDiffusion.resume(fake2)
        assert state_hash(u2) == state_hash(u)
        out["save__resume"] = np.array([fake2.start_epoch, fake2.step], np.int64)


def gen_cmap(out):
    from ldmseg.utils.utils import color_map
    out["cmap"] = color_map()
    out["cmap_norm"] = color_map(normalized=True).astype(np.float32)


def main():
    torch.set_num_threads(8)
    out = {}
    for fn in (gen_modify, gen_forward, gen_sample, gen_encode, gen_train, gen_optim, gen_save, gen_cmap):
        fn(out)
        print(fn.__name__, "done", flush=True)
    out["loop_unet_cfg"] = np.array(repr(LOOP_UNET))
    np.savez_compressed(os.path.join(HERE, "loops.npz"), **out)
    print("loops.npz:", len(out), "arrays")


if __name__ == "__main__":
    main()
