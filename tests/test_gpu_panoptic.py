"""Panoptic head on the HIP path (ldm_panoptic_pixels / ldm_panoptic_finalize) against the
reference's own compute_pq outputs (tests/golden/panoptic.npz) and the golden-pinned oracle.

Integer outputs: the bar is bit-exact.  The one documented exception is the ``resized`` case,
whose logits first pass two bilinear resamples (ldm_resize_bilinear vs torch F.interpolate,
≤1 ulp apart): an argmax can flip where two channels tie to that precision, so that case
allows 0.2 % of pixels to differ; the head itself (identity-size cases) must match exactly."""
import numpy as np
import pytest
import torch

from golden_utils import load
from ldmseg.ops import native as K
from ldmseg.pipelines.panoptic import panoptic_head, postprocess_panoptic, segments_info, threshold_predictions
from oracle import panoptic as opan

pytestmark = pytest.mark.gpu
DEV = "cuda"
MODES = {1: "max", 2: "topk_diff"}


def _case(name):
    z = load("panoptic.npz")
    logits = torch.from_numpy(z[f"{name}__logits"].astype(np.float32))
    mth, cth, oth, ign, thr, mode, Hi, Wi, h, w, rows = z[f"{name}__cfg"].tolist()
    kw = dict(mask_th=mth, count_th=int(cth), overlap_th=oth, ignore_label=int(ign), threshold_output=bool(thr),
              threshold_mode=MODES[int(mode)])
    return logits, kw, (int(Hi), int(Wi)), (int(h), int(w)), int(rows), z[f"{name}__cleaned"].astype(np.int64)


@pytest.mark.parametrize("name", ["kitti_max", "kitti_ign0", "topk_diff", "no_threshold", "base_yaml"])
def test_head_matches_reference_golden(name):
    logits, kw, _, _, _, exp = _case(name)
    cleaned, keep = panoptic_head(logits.to(DEV), **kw)
    np.testing.assert_array_equal(cleaned.cpu().numpy(), exp)
    for i in range(exp.shape[0]):
        labels = sorted(set(np.unique(exp[i]).tolist()) - {-1})
        assert [s["id"] for s in segments_info(keep[i])] == [l + 1 for l in labels]


def test_postprocess_with_crop_and_resizes_matches_reference_golden():
    logits, kw, img_hw, orig_hw, rows, exp = _case("resized")
    pad = torch.zeros(logits.shape[0], *img_hw, dtype=torch.bool)
    pad[:, :rows, :] = True
    res = postprocess_panoptic(logits.to(DEV), img_hw, pad.to(DEV), [orig_hw] * logits.shape[0], **kw)
    for i, r in enumerate(res):
        got = r["cleaned_pred"].cpu().numpy()
        assert got.shape == exp[i].shape
        assert (got != exp[i]).mean() <= 2e-3
        np.testing.assert_array_equal(r["panoptic_seg"][0].cpu().numpy(), got + 1)


@pytest.mark.parametrize("K_,H,W,ign,cth,oth,mode", [
    (1, 7, 9, 255, 0, 0.5, "max"),            # single channel, ragged pixel count
    (30, 37, 53, 0, 20, 0.5, "max"),          # ignore label inside [0, K)
    (30, 37, 53, 3, 0, 0.0, "none"),          # no threshold, keep everything but the ignore label
    (128, 64, 96, 255, 512, 0.5, "topk_diff"),
    (19, 1, 300, 255, 5, 0.9, "max"),
])
def test_head_matches_oracle_edge_cases(K_, H, W, ign, cth, oth, mode):
    g = torch.Generator().manual_seed(K_ * 1000 + H)
    lo = torch.randn(2, K_, max(2, H // 8), max(2, W // 8), generator=g) * 4
    logits = torch.nn.functional.interpolate(lo, size=(H, W), mode="bilinear", align_corners=False)
    logits = logits + 0.5 * torch.randn(2, K_, H, W, generator=g) - 2.0
    kw = dict(mask_th=0.5, count_th=cth, overlap_th=oth, ignore_label=ign, threshold_output=mode != "none",
              threshold_mode="max" if mode == "none" else mode)
    cleaned, _ = panoptic_head(logits.to(DEV), **kw)
    for i in range(2):
        np.testing.assert_array_equal(cleaned[i].cpu().numpy(), opan.head(logits[i].clone(), **kw))


def test_full_size_properties():
    """B=8 frames of K=128 logits at 512x512 (decode_latents' output size, base.yaml K): the
    relabel is consistent with the histograms (kept labels are exactly those whose pixel count
    and overlap pass), and every kept pixel carries its argmax label."""
    torch.manual_seed(0)
    B, Kc, H, W = 8, 128, 512, 512
    lo = torch.randn(B, Kc, 16, 16, device=DEV) * 5
    logits = K.resize_bilinear(lo, size=(H, W)) - 3.0
    pred, counts, mcounts = K.panoptic_pixels(logits, 0.5, 255, "max")
    assert int(counts.sum()) + int((pred == 255).sum()) == B * H * W
    cleaned, keep = panoptic_head(logits, 0.5, 512, 0.5, 255)
    am = logits.argmax(1)
    kept_px = cleaned >= 0
    assert torch.equal(cleaned[kept_px], am[kept_px])
    ratio = counts.double() / mcounts.double().clamp_min(1)
    want = (counts >= 512) & ((mcounts == 0) | (ratio >= 0.5))
    assert torch.equal(keep, want)
    lab_ok = torch.gather(keep, 1, pred.long().clamp(0, Kc - 1).flatten(1)).view_as(pred) & (pred < Kc)
    assert torch.equal(kept_px, lab_ok)


def test_threshold_predictions_matches_decode_latents_branch():
    torch.manual_seed(3)
    x = torch.randn(2, 30, 40, 52) * 2
    got = threshold_predictions(x.to(DEV), 0.5, 255).cpu()
    ref = torch.argmax(x, dim=1)
    ref[torch.softmax(x, dim=1).max(dim=1)[0] < 0.5] = 255
    assert torch.equal(got, ref)
    assert torch.equal(threshold_predictions(x.to(DEV), 0.5, 255, threshold_output=False).cpu(), x.argmax(1))


def test_rejects_bad_arguments():
    with pytest.raises(TypeError):
        K.panoptic_pixels(torch.zeros(1, 3, 4, 4, device=DEV, dtype=torch.float16), 0.5, 255)
    with pytest.raises(RuntimeError):
        K.panoptic_pixels(torch.zeros(1, 2000, 4, 4, device=DEV), 0.5, 255)     # K > 1024
