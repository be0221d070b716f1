"""RGB image encoder (GeneralVAEImage = diffusers AutoencoderKL encoder + quant_conv, row f3) on
the HIP path vs oracle/autoencoder_kl.py (torch fp32 restatement).

PARITY UNPINNED: diffusers is absent and no reference file holds an encoder output (SURVEY.md
§8c); the oracle restates the published SD-1.x encoder and each op it uses is stock torch.
Bars: fp32 1e-3 rel (north star), bf16 5e-2."""
import pytest
import torch
import torch.nn.functional as F

from ldmseg.models.autoencoder_kl import GeneralVAEImage
from ldmseg.ops import native as K
from oracle import autoencoder_kl as oae

pytestmark = pytest.mark.gpu
DEV = "cuda"
SMALL = dict(block_out_channels=(32, 64, 64), layers_per_block=1, norm_num_groups=16)


def rel(a, b):
    return ((a.float().cpu() - b.float()).norm() / b.float().norm()).item()


def _model(cfg, seed=0):
    torch.manual_seed(seed)
    m = GeneralVAEImage(**cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn_like(p) * 0.1)
    return m.eval()


@pytest.mark.parametrize("H,W", [(64, 64), (72, 40)])       # 72x40 -> 4x... tokens not a multiple of 64
def test_small_encoder_fp32_matches_oracle(H, W):
    m = _model(SMALL)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    torch.manual_seed(1)
    x = torch.rand(2, 3, H, W) * 2 - 1
    with torch.no_grad():
        ref = oae.encode_moments(sd, x, n_blocks=3, layers_per_block=1, groups=16)
    got = m.to(DEV).encode_moments(x.to(DEV))
    assert got.shape == ref.shape
    assert rel(got, ref) < 1e-3
    mode = m.encode(x.to(DEV)).latent_dist.mode()
    assert rel(mode, ref[:, :4]) < 1e-3


def test_small_encoder_bf16_close_to_oracle():
    m = _model(SMALL, seed=3)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    x = torch.rand(2, 3, 64, 96) * 2 - 1
    with torch.no_grad():
        ref = oae.encode_moments(sd, x, n_blocks=3, layers_per_block=1, groups=16)
    got = m.to(DEV, torch.bfloat16).encode_moments(x.to(DEV, torch.bfloat16))
    assert rel(got, ref) < 5e-2


def test_sd14_encoder_fullsize_fp32_matches_oracle():
    """SD-1.4 VAE encoder (34.2 M params) on the reference's squashed RGB frames, 192x192
    (encode_inputs resize=self.rgb_size, trainers_ldm_cond.py:705): 576 mid-block tokens."""
    m = _model({}, seed=5)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    x = torch.rand(2, 3, 192, 192) * 2 - 1
    torch.set_num_threads(16)
    with torch.no_grad():
        ref = oae.encode_moments(sd, x)
    got = m.to(DEV).encode_moments(x.to(DEV))
    assert got.shape == (2, 8, 24, 24)
    assert rel(got, ref) < 1e-3


def test_downsample_pad_mode_matches_fpad_conv():
    torch.manual_seed(7)
    for dt, tol in ((torch.float32, 1e-5), (torch.bfloat16, 2e-2)):
        x = torch.randn(2, 64, 18, 26)
        w = torch.randn(64, 64, 3, 3) * 0.05
        b = torch.randn(64)
        ref = F.conv2d(F.pad(x, (0, 1, 0, 1)), w, b, stride=2)
        pc = K.PackedConv(w.to(DEV), b.to(DEV), dt)
        xh = x.permute(0, 2, 3, 1).contiguous().to(DEV, dt)
        y = K.conv2d(pc, xh, 2, 18, 26, stride=2, pad_mode=1)
        assert y.shape == (2, 9, 13, 64)
        assert rel(y.permute(0, 3, 1, 2), ref) < tol


@pytest.mark.parametrize("n,stride", [(576, 576), (425, 448), (4096, 4096), (1, 64)])
def test_softmax_rows(n, stride):
    torch.manual_seed(n)
    s = torch.randn(37, stride, device=DEV) * 4
    p = K.softmax_rows(s, n, 0.3, torch.float32)
    ref = torch.softmax(s[:, :n].cpu() * 0.3, dim=-1)
    assert torch.allclose(p[:, :n].cpu(), ref, rtol=1e-5, atol=1e-7)
    assert bool((p[:, n:] == 0).all())
    pb = K.softmax_rows(s, n, 0.3, torch.bfloat16)
    assert torch.allclose(pb[:, :n].float().cpu(), ref, rtol=1e-2, atol=1e-3)
