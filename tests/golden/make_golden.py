"""Generate the golden vectors under tests/golden/ from the REFERENCE implementation.

Run in the build container only (it needs /root/reference, which never travels to
the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is pinned (each array is data: inputs + the reference's outputs):
  codec.npz  bit-channel mask codec   ldmseg/data/cityscapes.py:256-270 (== kitti.py:292-306)
             + the reference's own known-answer PNGs sample_outputs/{semseg,bit_channel_*}.png
  ddim.npz   DDIMNoiseScheduler       ldmseg/schedulers/ddim_scheduler.py:32-269
  vae.npz    GeneralVAESeg            ldmseg/models/vae.py:42-323 (gaussian, no mid blocks)
  vpq.npz    eval_dvpq.vpq_eval       eval/eval_dvpq.py:25-101
  ae.npz     one AE training iteration's loss and parameter gradients: the reference
             GeneralVAESeg (train mode, sample_posterior=True) + SegmentationLosses.point_loss
             (trainers_ae.py:321-331, losses.py:117-395), torch.rand / torch.randn drawn from
             seeded CPU generators in call order (the GPU test replays the same draws)
  panoptic.npz  TrainerDiffusion.compute_pq's per-image panoptic head
             ldmseg/trainers/trainers_ldm_cond.py:1185-1330, run as the reference method on a
             stand-in trainer whose sample/decode_latents return seeded logits; the
             cleaned_pred each image hands to CityscapesPanopticEvaluator.add_image is recorded

The UNet has no golden vector: its arithmetic lives in the un-vendored `diffusers`
package — parity for it is pinned per op against torch.nn.functional.
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refstubs  # noqa: E402

_refstubs.install()
REF = _refstubs.REFERENCE_ROOT


# --------------------------------------------------------------------------------------
# bit codec
# --------------------------------------------------------------------------------------
def gen_codec():
    from PIL import Image
    from ldmseg.data.cityscapes import Cityscapes

    out = {}
    # (a) known-answer fixture committed in the reference (dataset_base.py:147-155,201-206:
    #     cityscapes bits, n=16, fill 0.5, ignore_label 0)
    sem = np.array(Image.open(os.path.join(REF, "sample_outputs", "semseg.png")))
    bits = np.stack([np.array(Image.open(os.path.join(REF, "sample_outputs", f"bit_channel_{i}.png")))
                     for i in range(16)])
    out["fixture_semseg"] = sem.astype(np.uint8)
    out["fixture_bits_u8"] = bits.astype(np.uint8)

    # (b) seeded cases through the reference functions
    g = torch.Generator().manual_seed(1234)
    cases = [
        # name, n, ignore_label, H, W, id_low, id_high
        ("cs16_ign127", 16, 127, 33, 47, 0, 130),
        ("cs16_ign0", 16, 0, 24, 80, 0, 40),
        ("kitti5_ign255", 5, 255, 64, 64, 0, 34),
        ("coco7_ign127", 7, 127, 17, 9, 0, 129),
        ("wide_ids", 5, 255, 8, 300, -3, 70000),
        ("single", 5, 255, 1, 1, 0, 32),
        ("empty", 5, 255, 0, 7, 0, 32),
    ]
    meta = []
    for name, n, ign, H, W, lo, hi in cases:
        obj = types.SimpleNamespace(ignore_label=ign)
        x = torch.randint(lo, hi, (H, W), generator=g, dtype=torch.int64)
        if H * W:
            m = torch.rand((H, W), generator=g) < 0.1
            x[m] = ign
        enc, ign_mask = Cityscapes.encode_bitmap(obj, x.clone(), n=n, fill_value=0.5)
        # decode: from 2*enc-1 (the trainer convention) and from noisy planes
        dec_clean = Cityscapes.decode_bitmap(obj, (2 * enc - 1).clone(), n=n)
        noisy = torch.randn((n, H, W), generator=g)
        if H * W:
            noisy.view(n, -1)[:, ::5] = 0.0          # exact zeros: (x > 0) must be False
            noisy[:, 0, 0] = 1.0 if H else 0.0        # an all-ones pixel -> value 2^n-1 (31 quirk at n=5)
        dec_noisy = Cityscapes.decode_bitmap(obj, noisy.clone(), n=n)
        out[f"{name}__ids"] = x.numpy()
        out[f"{name}__enc"] = enc.numpy()
        out[f"{name}__ignore_mask"] = ign_mask.numpy()
        out[f"{name}__dec_clean"] = dec_clean.numpy()
        out[f"{name}__noisy"] = noisy.numpy()
        out[f"{name}__dec_noisy"] = dec_noisy.numpy()
        meta.append((name, n, ign))
    out["cases"] = np.array([m[0] for m in meta])
    out["cases_n"] = np.array([m[1] for m in meta], dtype=np.int64)
    out["cases_ignore"] = np.array([m[2] for m in meta], dtype=np.int64)
    # reference check of the fixture itself: encode(semseg) * 255 == PNGs
    obj = types.SimpleNamespace(ignore_label=0)
    enc, _ = Cityscapes.encode_bitmap(obj, torch.from_numpy(sem.astype(np.int64)), n=16, fill_value=0.5)
    assert np.array_equal((enc.numpy() * 255).astype(np.uint8), bits)
    out["fixture_decode"] = Cityscapes.decode_bitmap(obj, 2 * enc - 1, n=16).numpy()
    np.savez_compressed(os.path.join(HERE, "codec.npz"), **out)
    print("codec.npz:", len(out), "arrays")


# --------------------------------------------------------------------------------------
# DDIM scheduler
# --------------------------------------------------------------------------------------
DDIM_CONFIGS = {
    # base.yaml:48-62
    "base": dict(prediction_type="epsilon", beta_schedule="scaled_linear", num_train_timesteps=1000,
                 beta_start=0.00085, beta_end=0.012, steps_offset=1, clip_sample=False,
                 set_alpha_to_one=False, thresholding=False, dynamic_thresholding_ratio=0.995,
                 clip_sample_range=1.0, sample_max_value=1.0, weight="none", max_snr=5.0),
    # tools/scripts/train_diffusion.sh:21-23 overrides
    "script": dict(prediction_type="epsilon", beta_schedule="scaled_linear", num_train_timesteps=1000,
                   beta_start=0.00085, beta_end=0.012, steps_offset=1, clip_sample=False,
                   set_alpha_to_one=False, weight="max_clamp_snr", max_snr=2.0),
    # NB: weight="inverse_log_snr" raises in the reference on torch>=2 (in-place
    # `weights /= weights[-1]` aliases its own element, ddim_scheduler.py:108); not pinnable.
    "linear_clip": dict(beta_schedule="linear", clip_sample=True, set_alpha_to_one=True,
                        weight="none", prediction_type="epsilon"),
    "cosine_v": dict(beta_schedule="squaredcos_cap_v2", prediction_type="v_prediction",
                     clip_sample=True, clip_sample_range=2.0, weight="linear"),
    "sigmoid_x0": dict(beta_schedule="sigmoid", beta_start=0.0001, beta_end=0.02,
                       prediction_type="sample", weight="fixed", clip_sample=False),
}


def gen_ddim():
    from ldmseg.schedulers.ddim_scheduler import DDIMNoiseScheduler

    out = {}
    g = torch.Generator().manual_seed(7)
    shape = (3, 4, 8, 8)
    for cname, kw in DDIM_CONFIGS.items():
        s = DDIMNoiseScheduler(**kw, device="cpu", verbose=False)
        out[f"{cname}__betas"] = s.betas.numpy()
        out[f"{cname}__alphas_cumprod"] = s.alphas_cumprod.numpy()
        out[f"{cname}__final_alpha_cumprod"] = np.float32(s.final_alpha_cumprod)
        out[f"{cname}__weights"] = s.weights.numpy()
        for nsteps in (50, 25, 7):
            s.set_timesteps_inference(nsteps)
            out[f"{cname}__timesteps_{nsteps}"] = s.timesteps.numpy()
        s.set_timesteps_inference(50, tmin=300)
        out[f"{cname}__timesteps_50_tmin300"] = s.timesteps.numpy()
        s.set_timesteps_inference(50)
        ts = [999, 979, 500, 39, 19]
        out[f"{cname}__step_t"] = np.array(ts, dtype=np.int64)
        mo = torch.randn(shape, generator=g)
        x = torch.randn(shape, generator=g)
        out[f"{cname}__step_model_output"] = mo.numpy()
        out[f"{cname}__step_sample"] = x.numpy()
        for t in ts:
            for clipped in (False, True):
                r = s.step(mo, t, x, use_clipped_model_output=clipped)
                out[f"{cname}__step_{t}_{int(clipped)}__prev"] = r.prev_sample.numpy()
                out[f"{cname}__step_{t}_{int(clipped)}__x0"] = r.pred_original_sample.numpy()
        # add_noise / remove_noise with per-sample timesteps
        tb = torch.tensor([0, 421, 999], dtype=torch.int64)
        x0 = torch.randn(shape, generator=g)
        eps = torch.randn(shape, generator=g)
        out[f"{cname}__an_t"] = tb.numpy()
        out[f"{cname}__an_x0"] = x0.numpy()
        out[f"{cname}__an_eps"] = eps.numpy()
        out[f"{cname}__an_out"] = s.add_noise(x0, eps.clone(), tb).numpy()
        out[f"{cname}__an_out_s2"] = s.add_noise(x0, eps.clone(), tb, scale=2.0).numpy()
        out[f"{cname}__rn_out"] = s.remove_noise(x, eps, tb).numpy()
        out[f"{cname}__rn_out_s2"] = s.remove_noise(x, eps, tb, scale=0.5).numpy()
    out["configs"] = np.array(list(DDIM_CONFIGS))
    np.savez_compressed(os.path.join(HERE, "ddim.npz"), **out)
    print("ddim.npz:", len(out), "arrays")


# --------------------------------------------------------------------------------------
# GeneralVAESeg
# --------------------------------------------------------------------------------------
VAE_CONFIGS = {
    # KITTI AE (screenlog: 10 bit planes in, 30-way out, 1.80 M params), num_upscalers 2 (base.yaml:29)
    "kitti": dict(in_channels=10, int_channels=256, out_channels=30, block_out_channels=(32, 64, 128, 256),
                  latent_channels=4, num_latents=2, num_upscalers=2, upscale_channels=256,
                  norm_num_groups=32, scaling_factor=0.18215, parametrization="gaussian",
                  num_mid_blocks=0, act_fn="none", clamp_output=False),
    # cityscapes-style input (16 planes), one upscaler, tanh bottleneck + clamp (branch coverage)
    "cs_tanh": dict(in_channels=16, int_channels=64, out_channels=19, block_out_channels=(16, 32, 64),
                    latent_channels=4, num_latents=2, num_upscalers=1, upscale_channels=64,
                    norm_num_groups=16, scaling_factor=0.2, parametrization="gaussian",
                    num_mid_blocks=0, act_fn="tanh", clamp_output=True),
}
VAE_INPUTS = {"kitti": (2, 48, 80), "cs_tanh": (1, 40, 56)}


def _quantized_init(model, gen):
    """Integer-grid weights (q * scale, q in [-7, 7]) so the fixture stores int8 + one scale per tensor."""
    q = {}
    with torch.no_grad():
        for name, p in model.named_parameters():
            if p.ndim > 1:
                fan_in = p[0].numel() if not isinstance(model.get_submodule(name.rsplit(".", 1)[0]),
                                                        torch.nn.ConvTranspose2d) else p.shape[0] * 4
                scale = 1.0 / (4.0 * np.sqrt(fan_in))
            elif name.endswith("weight"):
                scale = 1.0 / 32.0          # norm gammas: 1 + small
            else:
                scale = 1.0 / 64.0          # biases / betas
            qi = torch.randint(-7, 8, p.shape, generator=gen, dtype=torch.int64)
            val = qi.float() * scale
            if p.ndim == 1 and name.endswith("weight"):
                val = val + 1.0
            p.copy_(val)
            q[name] = (qi.to(torch.int8).numpy(), np.float32(scale), p.ndim == 1 and name.endswith("weight"))
    return q


def gen_vae():
    from ldmseg.models.vae import GeneralVAESeg

    out = {}
    for cname, kw in VAE_CONFIGS.items():
        torch.manual_seed(0)
        model = GeneralVAESeg(**kw, encoder=None).eval()
        gen = torch.Generator().manual_seed(11)
        q = _quantized_init(model, gen)
        for name, (qi, scale, plus_one) in q.items():
            out[f"{cname}__w__{name}__q"] = qi
            out[f"{cname}__w__{name}__scale"] = scale
            out[f"{cname}__w__{name}__plus1"] = np.bool_(plus_one)
        B, H, W = VAE_INPUTS[cname]
        bits = torch.randint(0, 2, (B, kw["in_channels"], H, W), generator=gen).float()
        bits[:, :, : H // 4, : W // 5] = 0.5                     # ignore region (fill 0.5)
        x = 2 * bits - 1                                          # trainers_ae.py:293-295 convention
        with torch.no_grad():
            post = model.encode(x).latent_dist
            z = post.mode()
            dec_i = model.decode(z, interpolate=True)
            dec_n = model.decode(z, interpolate=False)
            fwd = model(x, sample_posterior=False).sample
        out[f"{cname}__x"] = x.numpy()
        out[f"{cname}__moments"] = post.parameters.numpy()
        out[f"{cname}__mean"] = post.mean.numpy()
        out[f"{cname}__logvar"] = post.logvar.numpy()
        out[f"{cname}__std"] = post.std.numpy()
        out[f"{cname}__dec_interp"] = dec_i.numpy()
        out[f"{cname}__dec_nointerp"] = dec_n.numpy()
        out[f"{cname}__forward"] = fwd.numpy()
        out[f"{cname}__keys"] = np.array(list(model.state_dict().keys()))
        out[f"{cname}__interpolation_factor"] = np.int64(model.interpolation_factor)
    out["configs"] = np.array(list(VAE_CONFIGS))
    np.savez_compressed(os.path.join(HERE, "vae.npz"), **out)
    print("vae.npz:", len(out), "arrays")


# --------------------------------------------------------------------------------------
# vpq_eval (eval/eval_dvpq.py is a script: import it as a module with a neutral argv)
# --------------------------------------------------------------------------------------
def gen_vpq():
    argv = sys.argv
    sys.argv = ["eval_dvpq.py"]
    try:
        spec = importlib.util.spec_from_file_location("ref_eval_dvpq", os.path.join(REF, "eval", "eval_dvpq.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        sys.argv = argv
    max_ins = 2 ** 20
    rng = np.random.default_rng(5)
    out = {}
    n_cases = 6
    for c in range(n_cases):
        H, W = 32, 96 * (1 + c % 3)          # eval_frames 1..3 frames side by side
        gt_cat = rng.integers(0, 19, size=(H // 8, W // 8)).repeat(8, 0).repeat(8, 1)
        gt_ins = rng.integers(0, 3, size=(H // 8, W // 8)).repeat(8, 0).repeat(8, 1)
        gt_cat[rng.random((H, W)) < 0.05] = 255                # void pixels
        pred_cat = gt_cat.copy()
        pred_ins = gt_ins.copy()
        flip = rng.random((H, W)) < 0.1 * c                   # increasing disagreement
        pred_cat[flip] = rng.integers(0, 19, size=flip.sum())
        pred_ins[rng.random((H, W)) < 0.05 * c] = 7
        pred_cat[pred_cat == 255] = 0
        pred = pred_cat.astype(np.int32) * max_ins + pred_ins.astype(np.int32)
        gt = gt_cat.astype(np.int32) * max_ins + gt_ins.astype(np.int32)
        iou, tp, fn, fp = mod.vpq_eval([pred, gt])
        out[f"c{c}__pred"] = pred
        out[f"c{c}__gt"] = gt
        out[f"c{c}__iou"] = iou
        out[f"c{c}__tp"] = tp
        out[f"c{c}__fn"] = fn
        out[f"c{c}__fp"] = fp
    out["n_cases"] = np.int64(n_cases)
    np.savez_compressed(os.path.join(HERE, "vpq.npz"), **out)
    print("vpq.npz:", len(out), "arrays")


# --------------------------------------------------------------------------------------
# panoptic head: the reference compute_pq method itself, on a stand-in trainer
# --------------------------------------------------------------------------------------
class _HostTensor(torch.Tensor):
    """`.cuda()` stays on the host (the fixture container has no GPU)."""

    def cuda(self, *a, **k):
        return self.as_subclass(torch.Tensor)


class _Loader:
    def __init__(self, batches):
        self.batches = batches
        self.dataset = types.SimpleNamespace(meta_data={})

    def __iter__(self):
        return iter(self.batches)

    def __len__(self):
        return len(self.batches)


def _smooth_logits(gen, B, K, H, W, cell=12):
    """Segmentation-like logits: a blobby label map whose class gets a spatially varying boost
    over a negative background, a second class partly competing, and per-pixel noise — so the
    fixture exercises kept segments, the confidence threshold, small-count and low-overlap drops."""
    up = lambda t: torch.nn.functional.interpolate(t, size=(H, W), mode="bilinear", align_corners=False)
    field = up(torch.randn(B, K, max(2, H // cell), max(2, W // cell), generator=gen))
    lab = field.argmax(1)                                           # blobby label map
    second = field.topk(2, dim=1).indices[:, 1]
    boost = 1.0 + 6.0 * up(torch.rand(B, 1, max(2, H // 16), max(2, W // 16), generator=gen))[:, 0]
    x = torch.randn(B, K, H, W, generator=gen) - 4.0
    x.scatter_add_(1, lab[:, None], boost[:, None])
    x.scatter_add_(1, second[:, None], (0.6 * boost)[:, None] * (torch.rand(B, 1, H, W, generator=gen) < 0.5))
    # fp16-representable values, so the fixture stores them exactly as fp16
    return x.half().float()


def gen_panoptic():
    import ldmseg.evaluations.cityscapes_pap_eval as cpe
    from ldmseg.trainers.trainers_ldm_cond import TrainerDiffusion

    recorded = []
    cpe.CityscapesPanopticEvaluator.add_image = lambda self, pred, gt: recorded.append(np.array(pred))
    cpe.CityscapesPanopticEvaluator.evaluate = lambda self: {"pq": 0.0, "sq": 0.0, "rq": 0.0}
    gen = torch.Generator().manual_seed(77)
    cases = [
        # name, B, K, H, W, mask_th, count_th, overlap_th, ignore_label, threshold_output, mode, (Hi, Wi), (h, w)
        ("kitti_max", 2, 30, 48, 64, 0.5, 100, 0.5, 255, True, "max", None, None),
        ("kitti_ign0", 2, 30, 48, 64, 0.5, 60, 0.5, 0, True, "max", None, None),
        ("topk_diff", 1, 19, 40, 56, 0.3, 50, 0.7, 255, True, "topk_diff", None, None),
        ("no_threshold", 1, 16, 32, 32, 0.5, 0, 0.5, 255, False, "max", None, None),
        ("base_yaml", 1, 48, 80, 112, 0.5, 512, 0.5, 255, True, "max", None, None),
        ("resized", 1, 20, 32, 48, 0.5, 80, 0.5, 255, True, "max", (64, 96), (80, 120)),
    ]
    out = {}
    for (name, B, K, H, W, mth, cth, oth, ign, thr, mode, img_hw, orig_hw) in cases:
        logits = _smooth_logits(gen, B, K, H, W, cell=24 if cth >= 512 else 12)
        Hi, Wi = img_hw or (H, W)
        h, w = orig_hw or (Hi, Wi)
        pad = torch.zeros(B, Hi, Wi, dtype=torch.bool)
        pad[:, : Hi - (Hi // 8 if img_hw else 0), :] = True            # padded bottom rows when resized
        batch = {
            "meta": [{"image_file": f"f{i}", "image_id": i, "im_size": (h, w)} for i in range(B)],
            "image": torch.zeros(B, 3, Hi, Wi),
            "mask": pad.as_subclass(_HostTensor),
            "text": [""] * B,
            "semseg": torch.zeros(B, h, w, dtype=torch.int64).as_subclass(_HostTensor),
        }
        sched = types.SimpleNamespace(set_timesteps_inference=lambda num_inference_steps: None,
                                      move_timesteps_to=lambda dev: None, timesteps=torch.tensor([19]))
        fake = types.SimpleNamespace(
            noise_scheduler=sched, args={"gpu": "cpu"}, dl_val=None, rgb_size=64,
            vae_image=types.SimpleNamespace(encode=None, scaling_factor=1.0),
            ds=types.SimpleNamespace(ignore_label=ign), mask_th=mth, count_th=cth, overlap_th=oth,
            encode_inputs=lambda *a, **k: (torch.zeros(B, 4, 8, 8), None),
            sample=lambda *a, **k: torch.zeros(B, 4, 8, 8),
            decode_latents=lambda *a, **k: logits.clone(),
        )
        fake.crop_padding = types.MethodType(TrainerDiffusion.crop_padding, fake)
        recorded.clear()
        TrainerDiffusion.compute_pq(fake, num_inference_steps=1, threshold_output=thr, dataloader=_Loader([batch]),
                                    threshold_mode=mode)
        assert len(recorded) == B
        out[f"{name}__logits"] = logits.half().numpy()
        out[f"{name}__cleaned"] = np.stack(recorded).astype(np.int16)
        out[f"{name}__cfg"] = np.array([mth, cth, oth, ign, int(thr), {"max": 1, "topk_diff": 2}[mode],
                                        Hi, Wi, h, w, Hi - (Hi // 8 if img_hw else 0)], np.float64)
    out["names"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(HERE, "panoptic.npz"), **out)
    print("panoptic.npz:", len(out), "arrays")


# --------------------------------------------------------------------------------------
# AE training iteration (config 1): reference VAE forward + point losses + backward
# --------------------------------------------------------------------------------------
AE_CFG = dict(in_channels=10, int_channels=64, out_channels=30, block_out_channels=(16, 32, 32, 64),
              latent_channels=4, num_latents=2, num_upscalers=2, upscale_channels=64, norm_num_groups=16,
              scaling_factor=0.2, parametrization="gaussian", num_mid_blocks=0, act_fn="none", clamp_output=False)
AE_SEEDS = (123, 456)          # torch.rand / torch.randn replay generators


class _Replay:
    """torch.rand / torch.randn replaced by draws from seeded CPU generators (then moved)."""

    def __init__(self):
        self.g_rand = torch.Generator().manual_seed(AE_SEEDS[0])
        self.g_randn = torch.Generator().manual_seed(AE_SEEDS[1])
        self.orig = (torch.rand, torch.randn)

    def rand(self, *size, device=None, **kw):
        size = size[0] if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)) else size
        return self.orig[0](*size, generator=self.g_rand).to(device or "cpu")

    def randn(self, *size, generator=None, device=None, dtype=None, **kw):
        size = size[0] if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)) else size
        return self.orig[1](*size, generator=self.g_randn).to(device or "cpu", dtype or torch.float32)

    def topk(self, x, k, *a, **kw):
        r = self.orig_topk(x, k, *a, **kw)
        if k > 2:                                   # the point selection, not calculate_uncertainty_seg
            self.selected.append(r[1].clone())
        return r

    def __enter__(self):
        self.selected = []
        self.orig_topk = torch.topk
        torch.rand, torch.randn, torch.topk = self.rand, self.randn, self.topk
        return self

    def __exit__(self, *a):
        torch.rand, torch.randn = self.orig
        torch.topk = self.orig_topk


def _blob_labels(gen, B, H, W, n_cls, cell=16):
    lo = torch.randn(B, n_cls, max(2, H // cell), max(2, W // cell), generator=gen)
    return torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False).argmax(1)


def gen_ae():
    from ldmseg.models.vae import GeneralVAESeg
    from ldmseg.trainers.losses import SegmentationLosses

    torch.manual_seed(0)
    model = GeneralVAESeg(**AE_CFG, encoder=None).train()
    gen = torch.Generator().manual_seed(21)
    q = _quantized_init(model, gen)
    out = {}
    for name, (qi, scale, plus_one) in q.items():
        out[f"w__{name}__q"] = qi
        out[f"w__{name}__scale"] = scale
        out[f"w__{name}__plus1"] = np.bool_(plus_one)
    B, H, W = 2, 64, 160
    targets = _blob_labels(gen, B, H, W, 12)                       # classes 0..11, 0 = ignore_label
    ids = targets.clone()
    bits = torch.stack([(ids >> i) & 1 for i in range(5)] + [(ids >> i) & 1 for i in range(5)], 1).float()
    images = 2.0 * bits - 1.0                                       # trainers_ae.py:294-295
    losses = SegmentationLosses(num_points=12544, oversample_ratio=3, importance_sample_ratio=0.75,
                                ignore_label=0, temperature=1.0)
    with _Replay() as rp:
        output = model(images, sample_posterior=True)
        ls = losses.point_loss(output.sample, targets)
    # the reference's uncertain-point indices (CE boxes, then mask boxes), uint16 (< 37632)
    out["sel_ce"] = rp.selected[0].numpy().astype(np.uint16)
    out["sel_mask"] = rp.selected[1].numpy().astype(np.uint16)
    kl = torch.mean(output.posterior.kl())
    total = 1.0 * ls["ce"] + 1.0 * ls["mask"] + 0.0 * kl             # base.yaml loss_weights
    total.backward()
    out["bits"] = bits.numpy().astype(np.uint8)
    out["targets"] = targets.numpy().astype(np.int16)
    out["ce"] = np.float64(ls["ce"].item())
    out["mask"] = np.float64(ls["mask"].item())
    out["loss"] = np.float64(total.item())
    for name, p in model.named_parameters():
        out[f"g__{name}"] = p.grad.numpy().astype(np.float32)
    out["names"] = np.array([n for n, _ in model.named_parameters()])
    np.savez_compressed(os.path.join(HERE, "ae.npz"), **out)
    print("ae.npz:", len(out), "arrays", "ce", out["ce"], "mask", out["mask"])


# --------------------------------------------------------------------------------------
# PoseExpNet (config 5's pose network, posenet/posenet.py:21-96)
# --------------------------------------------------------------------------------------
POSE_CASES = {
    # name: (seed, B, H, W, nb_ref_imgs, output_exp, train_mode, init_weights)
    "kitti_256x512": (1, 2, 256, 512, 2, False, False, False),
    "exp_train_64x128": (2, 2, 64, 128, 2, True, True, True),
    "exp_eval_odd_72x100": (3, 1, 72, 100, 2, True, False, False),
    "one_ref_128x128": (4, 1, 128, 128, 1, False, False, True),
}


def _state_sha(m):
    import hashlib
    h = hashlib.sha256()
    for k, v in sorted(m.state_dict().items()):
        h.update(k.encode())
        h.update(v.detach().float().contiguous().numpy().tobytes())
    return h.hexdigest()


def gen_posenet():
    """The reference PoseExpNet, torch default init (or its init_weights: xavier_uniform) under
    torch.manual_seed(seed); inputs U(0,1) frames from a seeded generator.  The weights are not
    stored: the test rebuilds them with the drop-in module under the same seed and checks the
    state sha256 recorded here."""
    spec = importlib.util.spec_from_file_location("ref_posenet", os.path.join(REF, "posenet", "posenet.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}
    for name, (seed, B, H, W, nref, exp, train, xavier) in POSE_CASES.items():
        torch.manual_seed(seed)
        net = mod.PoseExpNet(nb_ref_imgs=nref, output_exp=exp)
        if xavier:
            net.init_weights()
        net.train(train)
        g = torch.Generator().manual_seed(100 + seed)
        tgt = torch.rand(B, 3, H, W, generator=g)
        refs = [torch.rand(B, 3, H, W, generator=g) for _ in range(nref)]
        with torch.no_grad():
            r = net(tgt, refs)
        masks, pose = r
        out[f"{name}__state_sha"] = np.array(_state_sha(net))
        out[f"{name}__pose"] = pose.numpy()
        if train:
            for i, m in enumerate(masks):
                if m is not None:
                    out[f"{name}__mask{i + 1}"] = m.numpy()
        elif masks is not None:
            out[f"{name}__mask1"] = masks.numpy()
        out[f"{name}__cfg"] = np.array([seed, B, H, W, nref, int(exp), int(train), int(xavier)], np.int64)
    out["names"] = np.array(list(POSE_CASES))
    np.savez_compressed(os.path.join(HERE, "posenet.npz"), **out)
    print("posenet.npz:", len(out), "arrays")


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["codec", "ddim", "vae", "vpq", "panoptic", "ae", "posenet"]
    for w in which:
        globals()[f"gen_{w}"]()
