"""Helpers to read tests/golden/*.npz (data only; np.load with allow_pickle=False)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def vae_state_dict(z, cname):
    """Rebuild the integer-grid VAE weights stored by make_golden._quantized_init."""
    sd = {}
    pref = f"{cname}__w__"
    for key in z.files:
        if key.startswith(pref) and key.endswith("__q"):
            name = key[len(pref):-3]
            q = z[key].astype(np.float32)
            val = q * z[f"{pref}{name}__scale"]
            if bool(z[f"{pref}{name}__plus1"]):
                val = val + np.float32(1.0)
            sd[name] = torch.from_numpy(val.astype(np.float32))
    return sd


VAE_CONFIGS = {
    "kitti": dict(in_channels=10, int_channels=256, out_channels=30, block_out_channels=(32, 64, 128, 256),
                  latent_channels=4, num_latents=2, num_upscalers=2, upscale_channels=256,
                  norm_num_groups=32, scaling_factor=0.18215, parametrization="gaussian",
                  num_mid_blocks=0, act_fn="none", clamp_output=False),
    "cs_tanh": dict(in_channels=16, int_channels=64, out_channels=19, block_out_channels=(16, 32, 64),
                    latent_channels=4, num_latents=2, num_upscalers=1, upscale_channels=64,
                    norm_num_groups=16, scaling_factor=0.2, parametrization="gaussian",
                    num_mid_blocks=0, act_fn="tanh", clamp_output=True),
}

DDIM_CONFIGS = {
    "base": dict(prediction_type="epsilon", beta_schedule="scaled_linear", num_train_timesteps=1000,
                 beta_start=0.00085, beta_end=0.012, steps_offset=1, clip_sample=False,
                 set_alpha_to_one=False, thresholding=False, dynamic_thresholding_ratio=0.995,
                 clip_sample_range=1.0, sample_max_value=1.0, weight="none", max_snr=5.0),
    "script": dict(prediction_type="epsilon", beta_schedule="scaled_linear", num_train_timesteps=1000,
                   beta_start=0.00085, beta_end=0.012, steps_offset=1, clip_sample=False,
                   set_alpha_to_one=False, weight="max_clamp_snr", max_snr=2.0),
    "linear_clip": dict(beta_schedule="linear", clip_sample=True, set_alpha_to_one=True,
                        weight="none", prediction_type="epsilon"),
    "cosine_v": dict(beta_schedule="squaredcos_cap_v2", prediction_type="v_prediction",
                     clip_sample=True, clip_sample_range=2.0, weight="linear"),
    "sigmoid_x0": dict(beta_schedule="sigmoid", beta_start=0.0001, beta_end=0.02,
                       prediction_type="sample", weight="fixed", clip_sample=False),
}


# ------------------------------------------------------------------ loop-level fixtures
# (tests/golden/make_golden_loops.py): a reduced-width UNet built by this package's module tree
# with seeded torch default init, non-trivial norm affines / biases, and this package's
# modify_encoder (pinned separately against the reference's at 320 channels).  The fixture
# stores state_hash() of the weights it ran with, so a drift in construction order fails loudly.
LOOP_UNET = dict(block_out_channels=(64, 128, 128, 128), cross_attention_dim=None)


def build_loop_unet(UNet, cond=4, seed=0):
    torch.manual_seed(seed)
    u = UNet(**LOOP_UNET)
    with torch.no_grad():
        for _, p in u.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="random", cond_channels=cond,
                     init_mode_cond="random")
    u.freeze_layers(["time_embedding"])
    return u


def state_hash(module):
    import hashlib
    h = hashlib.sha256()
    for k, v in sorted(module.state_dict().items()):
        h.update(k.encode())
        h.update(v.detach().float().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()
