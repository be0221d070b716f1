"""BASELINE configs 4 and 1 at their full sizes on the HIP path, through size-independent
properties (the oracle chain cannot run these sizes in test time; the reduced-size parity tests
pin the arithmetic: test_gpu_sample_e2e.py, test_gpu_train_ae.py).

Config 4 (TrainerDiffusion.compute_pq's per-batch body, trainers_ldm_cond.py:1222-1330, with the
sampler :1048-1173): a T=8 clip of 192x640 RGB frames -> SD-1.x VAE encoder (192x192) -> 50 DDIM
steps of the full SD-1.4 UNet (bf16, 8x64x64) -> seg-VAE decode to K=128 logits -> panoptic head.
The seg-VAE's last conv is scaled x20 and shifted (as in the reduced test) so random-init logits
are peaked and segments survive the mask / count / overlap thresholds.  Properties: graph replay
== eager bit for bit, finite outputs, surviving segments, the head's histogram / relabel
consistency (every kept id is present in the map and nothing else is), and the DVPQ PNGs of the
prediction scored by the pinned vpq_eval oracle (prediction vs itself 100, vs a perturbed ground
truth strictly between 0 and 100).

Config 1 (TrainerAE, trainers_ae.py:279-389, main_worker_ae.py): one iteration of the 1.80 M
GeneralVAESeg on B=4 10x192x640 bit planes with the point losses, clip 3.0 and AdamW: finite
losses, finite gradients with every parameter tensor receiving a non-zero gradient, and the
parameter update equal to torch.optim.AdamW applied to the same (clipped) gradient.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ldmseg.evaluations.dvpq import dvpq_summary, panoptic_to_dvpq, write_dvpq_frame
from ldmseg.models import GeneralVAESeg, UNet
from ldmseg.models.autoencoder_kl import GeneralVAEImage
from ldmseg.pipelines.sample import sample_panoptic
from ldmseg.schedulers import DDIMNoiseScheduler
from ldmseg.trainers.ae import AETrainStep
from oracle import dvpq as odvpq

pytestmark = pytest.mark.gpu
DEV = "cuda"
T, H, W, K = 8, 192, 640, 128
HEAD = dict(mask_th=0.5, count_th=512, overlap_th=0.5, ignore_label=255)      # base.yaml eval thresholds
MAX_INS = 2 ** 20


def _config4_models():
    torch.manual_seed(0)
    with torch.device(DEV):
        u = UNet()
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero")
    u = u.to(torch.bfloat16).eval()
    ae = GeneralVAEImage().to(DEV, torch.bfloat16).eval()
    vs = GeneralVAESeg(in_channels=16, int_channels=256, out_channels=K, block_out_channels=(32, 64, 128, 256),
                       num_upscalers=2, scaling_factor=0.2)
    with torch.no_grad():
        vs.decoder[10].weight.mul_(20.0)
        vs.decoder[10].bias.sub_(1.0).mul_(20.0)
    return u, ae, vs.to(DEV, torch.bfloat16).eval()


def _sched():
    s = DDIMNoiseScheduler(prediction_type="epsilon", beta_schedule="scaled_linear", beta_start=0.00085,
                           beta_end=0.012, steps_offset=1, clip_sample=False, set_alpha_to_one=False, device=DEV,
                           verbose=False)
    return s


def _write(d, tag, maps, gt=False):
    for f, c in enumerate(maps):
        cat, ins = panoptic_to_dvpq(c, dropped_category=255 if gt else 19)
        write_dvpq_frame(os.path.join(d, tag), f"000000_{f:06d}_", cat, ins)


def _read(d, tag):
    from PIL import Image
    files = sorted(os.listdir(os.path.join(d, tag)))
    cats = [f for f in files if f.endswith("cat.png")]
    inss = [f for f in files if f.endswith("ins.png")]
    ids = [np.array(Image.open(os.path.join(d, tag, c))).astype(np.int32) * MAX_INS +
           np.array(Image.open(os.path.join(d, tag, i))).astype(np.int32) for c, i in zip(cats, inss)]
    return np.concatenate(ids, axis=1)


def test_config4_full_clip_sampling(tmp_path):
    u, ae, vs = _config4_models()
    g = torch.Generator().manual_seed(7)
    # blobby frames: low-resolution noise upsampled, so the encoder sees structure
    rgb = F.interpolate(torch.rand(T, 3, 12, 40, generator=g), size=(H, W), mode="bilinear").to(DEV)
    kw = dict(rgb_size=192, latent_size=64, num_inference_steps=50, seed=0, **HEAD)
    res_g = sample_panoptic(rgb, ae, vs, u, _sched(), use_graph=True, **kw)
    res_e = sample_panoptic(rgb, ae, vs, u, _sched(), use_graph=False, **kw)
    torch.cuda.synchronize()
    maps = []
    nseg = []
    for f in range(T):
        cg, ce = res_g[f]["cleaned_pred"], res_e[f]["cleaned_pred"]
        assert torch.equal(cg, ce), f                              # graph replay == eager
        ids, info = res_g[f]["panoptic_seg"]
        assert ids.shape == (H, W) and torch.equal(ids, cg + 1)
        c = cg.cpu().numpy()
        assert c.min() >= -1 and c.max() < K
        present = set(np.unique(c[c >= 0]).tolist())
        kept = {s["id"] - 1 for s in info}
        assert present == kept, (f, sorted(present), sorted(kept))  # relabel == histogram filter
        assert all(s["category_id"] == 1 and s["isthing"] for s in info)
        nseg.append(len(kept))
        maps.append(c)
    assert sum(nseg) >= T and max(nseg) >= 2, nseg                 # segments survive the thresholds
    # DVPQ PNGs (eval_dvpq.py's input) scored by the pinned vpq_eval
    rng = np.random.default_rng(0)
    gt = []
    for c in maps:
        g2 = c.copy()
        g2[rng.random(c.shape) < 0.1] = -1
        vals = np.unique(c[c >= 0])
        if len(vals) >= 2:
            g2[c == vals[0]] = vals[1]                              # merge two segments
        gt.append(g2)
    _write(tmp_path, "pred", maps)
    _write(tmp_path, "gt", gt, gt=True)
    _write(tmp_path, "self", maps, gt=True)
    pred, gtc, selfc = _read(tmp_path, "pred"), _read(tmp_path, "gt"), _read(tmp_path, "self")
    pq_self = dvpq_summary(*odvpq.vpq_eval(pred, selfc), num_things=1, num_classes=1)[0]
    pq_gt = dvpq_summary(*odvpq.vpq_eval(pred, gtc), num_things=1, num_classes=1)[0]
    assert abs(pq_self - 100.0) < 1e-6, pq_self
    assert 0.0 < pq_gt < 100.0, pq_gt


def test_config1_full_ae_iteration():
    torch.manual_seed(0)
    vae = GeneralVAESeg(in_channels=10, int_channels=256, out_channels=30, block_out_channels=(32, 64, 128, 256),
                        num_upscalers=2, scaling_factor=0.2).to(DEV).train()
    assert 1.7e6 < sum(p.numel() for p in vae.parameters()) < 2.1e6
    g = torch.Generator().manual_seed(1)
    lo = torch.randn(4, 20, 12, 40, generator=g)
    targets = F.interpolate(lo, size=(192, 640), mode="bilinear").argmax(1).to(DEV)
    bits = torch.stack([(targets >> i) & 1 for i in range(5)] * 2, 1).float()
    lr, clip = 1e-4, 3.0
    st = AETrainStep(vae, lr=lr, clip_grad=clip, ignore_label=0)
    before = st.flat.data.clone()
    loss, ce, mask = st.train_step(bits, targets)
    torch.cuda.synchronize()
    for v in (loss, ce, mask):
        assert torch.isfinite(v).item()
    assert loss.item() > 0
    grad = st.flat.grad.clone()
    assert torch.isfinite(grad).all()
    zero = [n for n, p in vae.named_parameters() if p.requires_grad and st.flat.view_of(p, grad).abs().max() == 0]
    assert not zero, zero
    # the same step by torch: clip_grad_norm_ (max_norm / (norm + 1e-6), capped at 1) + AdamW
    norm = grad.double().norm().item()
    coef = min(1.0, clip / (norm + 1e-6))
    p = torch.nn.Parameter(before.clone())
    p.grad = grad * coef
    opt = torch.optim.AdamW([p], lr=lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0)
    opt.step()
    assert torch.allclose(st.flat.data, p.detach(), rtol=1e-6, atol=1e-9)
    assert not torch.equal(st.flat.data, before)
