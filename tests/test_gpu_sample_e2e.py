"""BASELINE config 4 end to end on the HIP path (TrainerDiffusion.compute_pq's per-batch body,
trainers_ldm_cond.py:1222-1330): RGB encode -> DDIM denoise -> seg-VAE decode -> panoptic head,
against the oracle chain on the CPU (oracle/autoencoder_kl -> oracle/unet + oracle/ddim ->
oracle/vae -> oracle/panoptic; the DDIM, VAE and panoptic oracles are pinned to reference
goldens, the UNet and RGB encoder restate diffusers).  Then both outputs are written as the
DVPQ PNGs eval/eval_dvpq.py reads and scored with the pinned vpq_eval oracle.

The seg-VAE is the golden "kitti" model with its last conv scaled x20 and shifted by -1 (per
unit), so the decoder's logits are peaked and segments survive mask_th / count_th / overlap_th
(random-init weights otherwise give near-uniform softmax and nothing survives — the bench's
``segments_frame0: 0``).  Bars (fp32): label maps equal on >= 99.5 % of pixels, the same surviving
segments, DVPQ within 0.1 (percent points) of the oracle chain's DVPQ against the same ground truth.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_utils import VAE_CONFIGS, build_loop_unet, load, vae_state_dict
from ldmseg.evaluations.dvpq import dvpq_summary, panoptic_to_dvpq, write_dvpq_frame
from ldmseg.models import GeneralVAESeg, UNet
from ldmseg.models.autoencoder_kl import GeneralVAEImage
from ldmseg.pipelines.sample import sample_panoptic
from ldmseg.schedulers import DDIMNoiseScheduler
from oracle import autoencoder_kl as oae
from oracle import ddim as oddim
from oracle import dvpq as odvpq
from oracle import panoptic as opan
from oracle import unet as ounet
from oracle import vae as ovae

pytestmark = pytest.mark.gpu
DEV = "cuda"
B, H, W, L, STEPS, RGB = 2, 64, 192, 16, 5, 64
HEAD = dict(mask_th=0.5, count_th=400, overlap_th=0.5, ignore_label=255)
MAX_INS = 2 ** 20


def _models():
    torch.manual_seed(3)
    ae = GeneralVAEImage(block_out_channels=(32, 64, 64, 64), norm_num_groups=16).eval()
    u = build_loop_unet(UNet, cond=0).eval()
    sd_v = vae_state_dict(load("vae.npz"), "kitti")
    sd_v["decoder.10.weight"] = sd_v["decoder.10.weight"] * 20.0
    sd_v["decoder.10.bias"] = (sd_v["decoder.10.bias"] - 1.0) * 20.0
    vs = GeneralVAESeg(**VAE_CONFIGS["kitti"]).eval()
    vs.load_state_dict(sd_v, strict=True)
    return ae, u, vs


def _oracle_chain(ae, u, vs, rgb):
    sd_ae = {k: t.detach().clone() for k, t in ae.state_dict().items()}
    sd_u = {k: t.detach().clone() for k, t in u.state_dict().items()}
    sd_v = {k: t.detach().clone() for k, t in vs.state_dict().items()}
    torch.set_num_threads(16)
    with torch.no_grad():
        x = 2 * F.interpolate(rgb, size=(RGB, RGB), mode="bilinear", align_corners=False) - 1   # :1230-1236
        mean = oae.encode_moments(sd_ae, x, groups=16)[:, :4]
        rl = F.interpolate(mean, size=(L, L), mode="bilinear", align_corners=False) * ae.scaling_factor
        _, ac, final = oddim.tables("scaled_linear", 1000, 0.00085, 0.012, False)
        lat = torch.randn((B, 4, L, L), generator=torch.Generator().manual_seed(0))             # :1091-1095
        ts = oddim.inference_timesteps(1000, STEPS)
        for i, t in enumerate(ts):
            eps = ounet.forward(sd_u, dict(u.config), torch.cat([lat, rl], 1), torch.tensor(int(t)))
            prev, x0 = oddim.step(ac, final, 1000, STEPS, eps, int(t), lat)
            lat = x0 if i == len(ts) - 1 else prev
        logits = ovae.decode(sd_v, lat / vs.scaling_factor, VAE_CONFIGS["kitti"])              # :1253-1259
        return opan.postprocess(logits, (H, W), torch.ones(B, H, W, dtype=torch.bool), [(H, W)] * B, **HEAD)


def _panoptic_pngs(d, cleaned_frames, tag, gt=False):
    """Predictions through panoptic_to_dvpq (segments -> category 0, dropped -> 19); the ground
    truth's dropped pixels are void (255)."""
    for f, c in enumerate(cleaned_frames):
        cat, ins = panoptic_to_dvpq(c, dropped_category=255 if gt else 19)
        write_dvpq_frame(os.path.join(d, tag), f"000000_{f:06d}_", cat, ins)


def _read_clip(d, tag):
    """eval_dvpq.py:105-122: ids = cat * 2**20 + ins, the window's frames side by side."""
    from PIL import Image
    files = sorted(os.listdir(os.path.join(d, tag)))
    cats = [f for f in files if f.endswith("cat.png")]
    inss = [f for f in files if f.endswith("ins.png")]
    ids = [np.array(Image.open(os.path.join(d, tag, c))).astype(np.int32) * MAX_INS +
           np.array(Image.open(os.path.join(d, tag, i))).astype(np.int32) for c, i in zip(cats, inss)]
    return np.concatenate(ids, axis=1)


def _ground_truth(r, seed):
    g2 = r.copy()
    g2[np.random.default_rng(seed).random(r.shape) < 0.1] = -1
    vals, cnt = np.unique(r[r >= 0], return_counts=True)
    order = vals[np.argsort(cnt)]
    g2[r == order[-1]] = -1
    g2[r == order[1]] = order[0]
    return g2


@pytest.mark.parametrize("graph", [False, True])
def test_sample_panoptic_matches_oracle_chain_and_dvpq(graph, tmp_path):
    ae, u, vs = _models()
    g = torch.Generator().manual_seed(5)
    rgb = torch.rand(B, 3, H, W, generator=g)
    ref = _oracle_chain(ae, u, vs, rgb)
    assert all(len(np.unique(r[r >= 0])) >= 3 for r in ref), "fixture must leave surviving segments"
    sched = DDIMNoiseScheduler(prediction_type="epsilon", beta_schedule="scaled_linear", beta_start=0.00085,
                               beta_end=0.012, steps_offset=1, clip_sample=False, set_alpha_to_one=False,
                               device=DEV, verbose=False)
    res = sample_panoptic(rgb.to(DEV), ae.to(DEV), vs.to(DEV), u.to(DEV), sched, rgb_size=RGB, latent_size=L,
                          num_inference_steps=STEPS, seed=0, use_graph=graph, **HEAD)
    mine = [r["cleaned_pred"].cpu().numpy() for r in res]
    for f in range(B):
        assert (mine[f] == ref[f]).mean() >= 0.995, f
        ids, info = res[f]["panoptic_seg"]
        assert sorted(s["id"] for s in info) == sorted((np.unique(ref[f][ref[f] >= 0]) + 1).tolist())
        assert torch.equal(ids.cpu(), torch.from_numpy(mine[f]) + 1)
    # DVPQ: both outputs as eval_dvpq PNGs, scored against one ground truth: the oracle's own map
    # with 10 % of its pixels void, its largest segment void and its two smallest merged
    gt = [_ground_truth(r, seed=f) for f, r in enumerate(ref)]
    _panoptic_pngs(tmp_path, mine, "pred")
    _panoptic_pngs(tmp_path, ref, "oracle")
    _panoptic_pngs(tmp_path, gt, "gt", gt=True)
    pq = {}
    for tag in ("pred", "oracle"):
        acc = odvpq.vpq_eval(_read_clip(tmp_path, tag), _read_clip(tmp_path, "gt"))
        pq[tag] = dvpq_summary(*acc, num_things=1, num_classes=1)[0]
    assert 0.0 < pq["oracle"] < 100.0
    assert abs(pq["pred"] - pq["oracle"]) <= 0.1, pq
