"""PoseExpNet (posenet/posenet.py:21-96, BASELINE config 5) on the HIP path against the
REFERENCE module's own outputs (tests/golden/posenet.npz: seeded weights — the state sha256 is
checked so both ran with identical parameters — and seeded frames).  fp32 (exact-fp32 MFMA)
1e-3 relative to the tensor's max-abs; bf16 5e-2.  Cases: the config-5 KITTI frame 256x512,
the explainability branch in train mode (all four masks) and in eval mode at an odd size
(72x100: every ConvTranspose output is cropped), one reference image."""
import hashlib

import numpy as np
import pytest
import torch

from golden_utils import load
from posenet.posenet import PoseExpNet

pytestmark = pytest.mark.gpu
DEV = "cuda"
Z = load("posenet.npz")


def _sha(m):
    h = hashlib.sha256()
    for k, v in sorted(m.state_dict().items()):
        h.update(k.encode())
        h.update(v.detach().float().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def rel(a, b):
    a, b = a.detach().float().cpu(), torch.as_tensor(b).float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _case(name):
    seed, B, H, W, nref, exp, train, xavier = Z[f"{name}__cfg"].tolist()
    torch.manual_seed(seed)
    net = PoseExpNet(nb_ref_imgs=nref, output_exp=bool(exp))
    if xavier:
        net.init_weights()
    assert _sha(net) == str(Z[f"{name}__state_sha"]), "weights differ from the reference run's"
    net.train(bool(train))
    g = torch.Generator().manual_seed(100 + seed)
    tgt = torch.rand(B, 3, H, W, generator=g)
    refs = [torch.rand(B, 3, H, W, generator=g) for _ in range(nref)]
    return net, tgt, refs, bool(exp), bool(train)


@pytest.mark.parametrize("name", [str(n) for n in Z["names"]])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_posenet_matches_reference(name, dtype):
    net, tgt, refs, exp, train = _case(name)
    net = net.to(DEV, dtype)
    masks, pose = net(tgt.to(DEV, dtype), [r.to(DEV, dtype) for r in refs])
    tol = 1e-3 if dtype == torch.float32 else 5e-2
    assert pose.shape == Z[f"{name}__pose"].shape
    assert rel(pose, Z[f"{name}__pose"]) < tol
    if not exp:
        assert masks == ([None] * 4 if train else None)
        return
    got = masks if train else [masks]
    for i, m in enumerate(got):
        ref = Z[f"{name}__mask{i + 1}"]
        assert tuple(m.shape) == ref.shape
        assert rel(m, ref) < tol, i


def test_posenet_reference_checkpoint_keys_load():
    net, *_ = _case("exp_train_64x128")
    sd = net.state_dict()
    assert "conv1.0.weight" in sd and "upconv5.0.weight" in sd and "predict_mask1.weight" in sd
    PoseExpNet(nb_ref_imgs=2, output_exp=True).load_state_dict(sd, strict=True)
