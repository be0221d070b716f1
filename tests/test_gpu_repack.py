"""In-place pack refresh after an optimizer update (ldm_repack, ldmseg/models/repack.py).

LDMTrainStep no longer rebuilds the UNet's packed weights with torch ops after each AdamW step
(trainers_ldm_cond.py:769-781 updates the parameters in place; the HIP path then needs fresh
packs): one ldm_repack launch rewrites every forward pack, data-gradient pack and concatenated /
interleaved bias vector from the fp32 master weights.  The refreshed packs must equal, bit for
bit, what UNet.prepare() / prepare_dgrad() build from scratch from the same weights — including
the GEGLU interleave, the fused QKV (three sources), the 22 concatenated time_emb_proj weights
and biases, conv_in's channel padding and conv_out's row-padded weight-gradient pack.
"""
import pytest
import torch

from golden_utils import DDIM_CONFIGS, build_loop_unet
from ldmseg.models import UNet
from ldmseg.models.repack import _iter_packs
from ldmseg.schedulers import DDIMNoiseScheduler
from ldmseg.trainers import LDMTrainStep

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _packs(unet):
    P, D = unet.prepare(), unet.prepare_dgrad()
    out = []
    for pc in list(_iter_packs(P)) + list(_iter_packs(D)):
        out.append((pc.w.clone(), None if pc.bias is None else pc.bias.clone()))
    return out


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_refreshed_packs_equal_fresh_packs(dtype):
    torch.manual_seed(3)
    u = build_loop_unet(UNet, cond=4, seed=21).to(DEV)
    sched = DDIMNoiseScheduler(**DDIM_CONFIGS["script"], device=DEV, verbose=False)
    st = LDMTrainStep(u, sched, lr=1e-2, weight_decay=0.05, clip_grad=1.0, self_condition=True, compute_dtype=dtype)
    g = torch.Generator().manual_seed(2)
    B, L = 2, 16
    lat, rgb = torch.randn(B, 4, L, L, generator=g).to(DEV), torch.randn(B, 4, L, L, generator=g).to(DEV)
    mask = torch.ones(B, L, L, device=DEV)
    before = _packs(u)
    for _ in range(2):
        st.train_step(lat, rgb, mask)
    torch.cuda.synchronize()
    assert st.refresher.ndesc > 50 and not st.refresher.fallback
    refreshed = _packs(u)                                   # the plan kept by the refresher
    assert any(not torch.equal(a[0], b[0]) for a, b in zip(before, refreshed))   # weights moved
    u.invalidate_packed()
    fresh = _packs(u)                                       # rebuilt from scratch, same weights
    assert len(fresh) == len(refreshed)
    for i, ((w1, b1), (w2, b2)) in enumerate(zip(refreshed, fresh)):
        assert torch.equal(w1, w2), i
        assert (b1 is None) == (b2 is None) and (b1 is None or torch.equal(b1, b2)), i
