"""encode_inputs / decode_latents (trainers_ldm_cond.py:336-444) on the HIP path against the
same composition of torch F.interpolate and the golden-pinned seg-VAE oracle (oracle/vae.py),
and the RGB path through GeneralVAEImage against oracle/autoencoder_kl.py (unpinned)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_utils import VAE_CONFIGS
from ldmseg.models import GeneralVAESeg
from ldmseg.models.autoencoder_kl import GeneralVAEImage
from ldmseg.pipelines.latents import color_map, decode_latents, encode_inputs
from oracle import autoencoder_kl as oae
from oracle import vae as ovae

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    return ((a.float().cpu() - b.float()).norm() / b.float().norm()).item()


def _seg_vae():
    torch.manual_seed(0)
    v = GeneralVAESeg(**VAE_CONFIGS["kitti"]).eval()
    return v, {k: t.detach().clone() for k, t in v.state_dict().items()}


def test_encode_inputs_seg_matches_reference_composition():
    v, sd = _seg_vae()
    torch.manual_seed(1)
    bits = (torch.rand(2, 10, 160, 512) > 0.5).float()          # bit planes in {0, 1}
    lat, lat_mean = encode_inputs(bits.to(DEV), v.to(DEV).encode, 0.2, 64, resize=(192, 640))
    x = 2.0 * F.interpolate(bits, size=(192, 640), mode="bilinear", align_corners=False) - 1.0
    _, mean, _, _ = ovae.encode(sd, x, VAE_CONFIGS["kitti"])
    ref = F.interpolate(mean, size=(64, 64), mode="bilinear", align_corners=False) * 0.2
    assert lat.shape == (2, 4, 64, 64)
    assert rel(lat, ref) < 1e-4
    assert torch.equal(lat, lat_mean)


def test_decode_latents_logits_and_predictions():
    v, sd = _seg_vae()
    torch.manual_seed(2)
    z = torch.randn(2, 4, 24, 80)
    logits = decode_latents(v.to(DEV), z.to(DEV), return_logits=True)
    ref = ovae.decode(sd, z * (1.0 / v.scaling_factor), VAE_CONFIGS["kitti"])
    assert rel(logits, ref) < 1e-4
    pred = decode_latents(v, z.to(DEV), threshold_output=True, mask_th=0.5, ignore_label=255,
                          return_predictions=True).cpu()
    exp = logits.cpu().argmax(1)
    exp[torch.softmax(logits.cpu(), 1).max(1)[0] < 0.5] = 255
    assert torch.equal(pred, exp)
    # the reference's return value (:437-438): encode_seg colour map of the predictions, uint8 NHWC
    img = decode_latents(v, z.to(DEV), threshold_output=True, mask_th=0.5, ignore_label=255)
    assert isinstance(img, np.ndarray) and img.dtype == np.uint8 and img.shape == (*exp.shape, 3)
    assert np.array_equal(img, color_map()[exp.numpy().astype(np.uint8)])


def test_encode_inputs_rgb_path():
    """RGB frames squashed to rgb_size x rgb_size (:705) -> SD latents -> L x L (x 0.18215)."""
    torch.manual_seed(3)
    m = GeneralVAEImage(block_out_channels=(32, 64, 64, 64), norm_num_groups=16).eval()
    sd = {k: t.detach().clone() for k, t in m.state_dict().items()}
    rgb = torch.rand(2, 3, 200, 600)
    lat, _ = encode_inputs(rgb.to(DEV), m.to(DEV).encode, 0.18215, 64, resize=192)
    x = 2.0 * F.interpolate(rgb, size=(192, 192), mode="bilinear", align_corners=False) - 1.0
    mean = oae.encode_moments(sd, x, groups=16)[:, :4]
    ref = F.interpolate(mean, size=(64, 64), mode="bilinear", align_corners=False) * 0.18215
    assert rel(lat, ref) < 1e-3
