"""AE training iteration (row a16, config 1) on the HIP path against the reference's own
forward + point losses + backward (tests/golden/ae.npz: GeneralVAESeg train mode with
sample_posterior=True, SegmentationLosses.point_loss, loss.backward()).  The reference's
torch.rand / torch.randn draws are replayed from the same seeded CPU generators, so both sides
sample the same points and posterior noise.  Bars (fp32): losses 1e-4 rel; every parameter
gradient 1e-3 rel (L2) — the top-k of 37632 uncertainty values could swap one point at the
threshold under rounding, which moves a gradient by far less than that."""
import numpy as np
import pytest
import torch

from golden_utils import load
from ldmseg.models import GeneralVAESeg
from ldmseg.ops import native as K
from ldmseg.trainers.ae import AETrainStep, PointLosses, VAETrainGraph

pytestmark = pytest.mark.gpu
DEV = "cuda"
AE_CFG = dict(in_channels=10, int_channels=64, out_channels=30, block_out_channels=(16, 32, 32, 64),
              latent_channels=4, num_latents=2, num_upscalers=2, upscale_channels=64, norm_num_groups=16,
              scaling_factor=0.2, parametrization="gaussian", num_mid_blocks=0, act_fn="none", clamp_output=False)


class Replay:
    def __init__(self):
        self.g_rand = torch.Generator().manual_seed(123)
        self.g_randn = torch.Generator().manual_seed(456)

    def rand(self, *shape, device):
        return torch.rand(*shape, generator=self.g_rand).to(device)

    def randn(self, shape, device):
        return torch.randn(*shape, generator=self.g_randn).to(device)


def _model(z, dtype=torch.float32):
    torch.manual_seed(0)
    m = GeneralVAESeg(**AE_CFG)
    sd = {}
    for name in z["names"]:
        name = str(name)
        val = z[f"w__{name}__q"].astype(np.float32) * z[f"w__{name}__scale"]
        if bool(z[f"w__{name}__plus1"]):
            val = val + np.float32(1.0)
        sd[name] = torch.from_numpy(val.astype(np.float32))
    m.load_state_dict(sd)
    return m.to(DEV, dtype).train()


def _inputs(z):
    bits = torch.from_numpy(z["bits"].astype(np.float32)).to(DEV)
    targets = torch.from_numpy(z["targets"].astype(np.int64)).to(DEV)
    return bits, targets


def _grads(m, bits, targets, rp, select=None, losses_out=None):
    grads = {}

    def sink(p):
        g = grads.get(p)
        if g is None:
            g = grads[p] = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
        return g, True
    graph = VAETrainGraph(m, sink)
    B = bits.shape[0]
    eps = rp.randn((B, 4, bits.shape[2] // 8, bits.shape[3] // 8), device=DEV)
    logits, _ = graph.forward((2.0 * bits - 1.0).contiguous(), eps)
    pl = PointLosses(ignore_label=0, rand=rp.rand, select=select)
    ce, mask, dlog = pl(logits, targets)
    if losses_out is not None:
        losses_out.append(pl)
    graph.backward(dlog)
    return ce, mask, grads


def _forced(z):
    """select hook returning the reference's own uncertain-point indices (CE call, then masks)."""
    sels = [torch.from_numpy(z["sel_ce"].astype(np.int32)), torch.from_numpy(z["sel_mask"].astype(np.int32))]
    return lambda u, k: sels.pop(0).to(u.device)


def test_ae_point_selection_matches_reference():
    """ldm_topk_select picks the reference's uncertain points up to rounding at the threshold."""
    z = load("ae.npz")
    m = _model(z)
    bits, targets = _inputs(z)
    out = []
    _grads(m, bits, targets, Replay(), losses_out=out)
    mine = out[0].last_idx
    for got, key in zip(mine, ("sel_ce", "sel_mask")):
        ref = z[key].astype(np.int64)
        got = got.cpu().numpy()
        assert got.shape == ref.shape
        diff = sum(len(set(a.tolist()) - set(b.tolist())) for a, b in zip(got, ref))
        assert diff <= 1e-3 * ref.size, (key, diff)


def test_ae_losses_and_gradients_match_reference():
    """With the reference's point selection, the whole forward + losses + backward chain."""
    z = load("ae.npz")
    m = _model(z)
    bits, targets = _inputs(z)
    ce, mask, grads = _grads(m, bits, targets, Replay(), select=_forced(z))
    assert abs(ce.item() - float(z["ce"])) <= 1e-4 * abs(float(z["ce"]))
    assert abs(mask.item() - float(z["mask"])) <= 1e-4 * abs(float(z["mask"]))
    named = dict(m.named_parameters())
    worst = []
    for name in z["names"]:
        name = str(name)
        ref = torch.from_numpy(z[f"g__{name}"])
        got = grads[named[name]].cpu()
        worst.append((((got - ref).norm() / ref.norm().clamp_min(1e-20)).item(), name))
    worst.sort(reverse=True)
    assert worst[0][0] < 1e-3, worst[:5]


def test_ae_bf16_gradients_close():
    z = load("ae.npz")
    m = _model(z, torch.bfloat16)
    bits, targets = _inputs(z)
    ce, mask, grads = _grads(m, bits, targets, Replay())
    assert abs(ce.item() - float(z["ce"])) <= 3e-2 * abs(float(z["ce"]))
    named = dict(m.named_parameters())
    errs = [((grads[named[str(n)]].cpu() - torch.from_numpy(z[f"g__{n}"])).norm() /
             torch.from_numpy(z[f"g__{n}"]).norm()).item() for n in z["names"]]
    assert max(errs) < 1.5e-1, sorted(errs)[-3:]


def test_ae_train_step_is_one_torch_adamw_step():
    """AETrainStep: its gradients match the reference's (with the reference's point selection), and
    its update is clip_grad_norm_(3.0) + torch AdamW (lr 1e-4) applied to those gradients."""
    z = load("ae.npz")
    m = _model(z)
    before = {n: p.detach().clone().cpu() for n, p in m.named_parameters()}
    bits, targets = _inputs(z)
    rp = Replay()
    st = AETrainStep(m, lr=1e-4, clip_grad=3.0, ignore_label=0, rand=rp.rand, randn=rp.randn, select=_forced(z))
    loss, ce, mask = st.train_step(bits, targets)
    assert abs(loss.item() - float(z["loss"])) <= 1e-4 * abs(float(z["loss"]))
    named = dict(m.named_parameters())
    ref = {}
    for n in before:
        g = st.flat.view_of(named[n], st.flat.grad).detach().cpu().clone()
        gr = torch.from_numpy(z[f"g__{n}"])
        assert (g - gr).norm() <= 1e-3 * gr.norm(), n
        ref[n] = torch.nn.Parameter(before[n].clone())
        ref[n].grad = g
    torch.nn.utils.clip_grad_norm_(list(ref.values()), 3.0)
    opt = torch.optim.AdamW(list(ref.values()), lr=1e-4, betas=(0.9, 0.999), weight_decay=0.0)
    opt.step()
    for n, p in m.named_parameters():
        assert torch.allclose(p.detach().cpu(), ref[n].detach(), rtol=0, atol=1e-6), n


@pytest.mark.parametrize("n,k", [(37632, 9408), (1000, 1), (64, 64), (5000, 2500)])
def test_topk_select_set(n, k):
    torch.manual_seed(n)
    u = torch.randn(3, n, device=DEV)
    u[1, :n // 2] = 0.25                                   # ties across the threshold
    idx, _ = K.topk_select(u, k)
    for r in range(3):
        got = set(idx[r].cpu().tolist())
        assert len(got) == k
        thr = torch.topk(u[r].cpu(), k).values[-1]
        vals = u[r].cpu()
        assert all(vals[i] >= thr for i in got)
        assert (vals > thr).sum().item() <= k


def test_point_sample_matches_grid_sample_and_its_adjoint():
    torch.manual_seed(5)
    x = torch.randn(2, 7, 13, 29, device=DEV)
    c = torch.rand(2, 300, 2, device=DEV)
    c[:, :4] = torch.tensor([[0.0, 0.0], [1.0, 1.0], [0.999, 0.0], [0.5, 0.5]], device=DEV)
    ref = torch.nn.functional.grid_sample(x, 2 * c[:, :, None] - 1, align_corners=False)[..., 0]
    assert torch.allclose(K.point_sample(x, c), ref, atol=1e-5, rtol=1e-5)
    g = torch.randn(2, 7, 300, device=DEV)
    xr = x.clone().requires_grad_(True)
    torch.nn.functional.grid_sample(xr, 2 * c[:, :, None] - 1, align_corners=False)[..., 0].mul(g).sum().backward()
    din = torch.zeros_like(x)
    K.point_sample_bwd(g, c, din)
    assert torch.allclose(din, xr.grad, atol=1e-4, rtol=1e-4)
