"""Checkpoint round-trip in the reference's layouts (CPU, host logic only).

LDM model.pt: trainers_ldm_cond.py:1844-1944; AE model.pt: trainers_ae.py:534-587;
GeneralVAESeg.load_pretrained: vae.py:117-122.  Files are read back with the safe loader
(weights_only=True).  The optimizer entry is torch.optim.AdamW's state_dict of the reference's
parameter grouping (trainers/optim.py:196-217): checked against a real torch AdamW."""
import torch
import torch.nn as nn

from golden_utils import VAE_CONFIGS
from ldmseg.models import GeneralVAESeg, UNet
from ldmseg.schedulers import DDIMNoiseScheduler
from ldmseg.trainers.ldm import LDMTrainStep
from ldmseg.utils import checkpoint as ck

SMALL = dict(block_out_channels=(32, 64, 64, 64), cross_attention_dim=None, norm_num_groups=32)


def _unet(seed):
    torch.manual_seed(seed)
    u = UNet(**SMALL)
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero")
    u.freeze_layers(["time_embedding"])
    return u


def _vae(seed):
    torch.manual_seed(seed)
    return GeneralVAESeg(**VAE_CONFIGS["kitti"])


def _same(a, b):
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_ldm_model_pt_round_trip(tmp_path):
    u, v = _unet(0), _vae(1)
    path = tmp_path / "model.pt"
    ck.save(path, unet=u, vae_semseg=v, step=11, epoch=2, p={"train_kwargs": {"lr": 1e-4}, "sizes": (1, 2)})
    data = ck.read(path)                                  # weights_only=True
    assert tuple(data) == ck.LDM_KEYS
    assert "new_conv.weight" in data["unet"] and "conv_in.weight" in data["unet"]
    assert not any(".attn2." in k or ".norm2." in k and "transformer_blocks" in k for k in data["unet"])
    u2, v2 = _unet(5), _vae(6)
    got, start_epoch, step = ck.resume(path, u2, vae_semseg=v2, num_iters_per_epoch=100)
    assert (start_epoch, step) == (3, 301)                # trainers_ldm_cond.py:1901-1902
    _same(u.state_dict(), u2.state_dict())
    _same(v.state_dict(), v2.state_dict())
    u3 = _unet(7)
    ck.load(path, u3, load_vae=False)
    _same(u.state_dict(), u3.state_dict())


def test_ddp_wrapped_unet_saves_plain_keys(tmp_path):
    u = _unet(0)

    class FakeDDP(nn.parallel.DistributedDataParallel):     # unwrap() only looks at the type
        def __init__(self, m):
            nn.Module.__init__(self)
            self.module = m
    d = ck.construct_save_dict(FakeDDP(u), _vae(1))
    assert not any(k.startswith("module.") for k in d["unet"])


def test_ae_checkpoint_and_load_pretrained(tmp_path):
    v = _vae(3)
    path = tmp_path / "ae.pt"
    ck.save_ae(path, v, step=5, epoch=0)
    data = ck.read(path)
    assert set(data) == {"step", "epoch", "vae", "opt", "p", "scaler"}
    assert all(k.startswith("module.") for k in data["vae"])
    v2 = _vae(4)
    v2.load_pretrained(str(path))
    _same(v.state_dict(), v2.state_dict())


def _reference_adamw(unet, lr, wd, wd_norm, lr_func):
    """get_optim_unet (optim.py:196-217 + reduce_param_groups) restated with torch AdamW."""
    norm = (nn.GroupNorm, nn.LayerNorm, nn.BatchNorm2d)
    memo, groups = set(), {}
    for mname, m in unet.named_modules():
        for pname, q in m.named_parameters(recurse=False):
            if not q.requires_grad or q in memo:
                continue
            memo.add(q)
            hp = (lr * lr_func(f"{mname}.{pname}"), wd_norm if isinstance(m, norm) else wd)
            groups.setdefault(hp, []).append(q)
    return torch.optim.AdamW([{"params": ps, "lr": a, "weight_decay": b} for (a, b), ps in groups.items()],
                             lr=lr, betas=(0.9, 0.999), eps=1e-8)


def test_optimizer_state_is_torch_adamw_format():
    lr_func = lambda name: 0.1 if "conv_in" in name else 1.0      # noqa: E731
    u_ref = _unet(2)
    u = _unet(2)
    ref = _reference_adamw(u_ref, 1e-4, 0.01, 0.0, lr_func)
    for q in u_ref.parameters():
        if q.requires_grad:
            q.grad = torch.randn_like(q)
    ref.step()
    ts = LDMTrainStep(u, DDIMNoiseScheduler(), lr=1e-4, weight_decay=0.01, weight_decay_norm=0.0,
                      lr_factor_func=lr_func)
    ts.load_state_dict(ref.state_dict())                   # a reference run's optimizer -> native
    assert ts.step_count == 1
    mine = ts.state_dict()
    theirs = ref.state_dict()
    assert [sorted(g) for g in mine["param_groups"]] == [sorted(g) for g in theirs["param_groups"]]
    for gm, gt in zip(mine["param_groups"], theirs["param_groups"]):
        assert gm["params"] == gt["params"]
        assert gm["lr"] == gt["lr"] and gm["weight_decay"] == gt["weight_decay"]
    assert mine["state"].keys() == theirs["state"].keys()
    for i in theirs["state"]:
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(mine["state"][i][k], theirs["state"][i][k]), (i, k)
        assert float(mine["state"][i]["step"]) == float(theirs["state"][i]["step"])
    ref2 = _reference_adamw(_unet(2), 1e-4, 0.01, 0.0, lr_func)
    ref2.load_state_dict(mine)                             # native -> torch AdamW loads it


def test_train_step_keeps_inference_ln_fold():
    """LDMTrainStep turns the LayerNorm fold off for its own forward/backward; for_inference()
    gives validation sampling the module's original (folded) setting back, and the next
    train_step turns it off again (the fold was silently lost for inference)."""
    from ldmseg.schedulers import DDIMNoiseScheduler
    from ldmseg.trainers.ldm import LDMTrainStep
    u = _unet(0)
    assert u.ln_fold
    ts = LDMTrainStep(u, DDIMNoiseScheduler())
    assert not u.ln_fold
    u.train()
    with ts.for_inference() as m:
        assert m is u and u.ln_fold
        assert not u.training and u.upsample_phases        # eval mode inside: the phase form runs
    assert not u.ln_fold and u.training
