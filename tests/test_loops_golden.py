"""Host-side loop semantics against the REFERENCE's own runs (tests/golden/loops.npz, made by
tests/golden/make_golden_loops.py with the reference methods on stand-in objects).  CPU only:

  UNet.modify_encoder   unet.py:124-233 at 320 channels, every accepted init-mode combination
  get_optim_unet        optim.py:53-82 parameter groups (order, members, lr, weight_decay)
  construct_save_dict   trainers_ldm_cond.py:1844-1867 top-level / VAE keys; resume :1879-1914
  color_map             utils.py:240-258 (decode_latents' colour table)
"""
import functools
import hashlib

import numpy as np
import pytest
import torch

from golden_utils import VAE_CONFIGS, build_loop_unet, load, state_hash
from ldmseg.models import GeneralVAESeg, UNet
from ldmseg.pipelines.latents import color_map
from ldmseg.schedulers import DDIMNoiseScheduler
from ldmseg.trainers.ldm import LDMTrainStep
from ldmseg.utils import checkpoint as ck

Z = load("loops.npz")


def _sha(*tensors):
    h = hashlib.sha256()
    for t in tensors:
        h.update(t.detach().contiguous().float().numpy().tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("k", range(len(Z["modify__cases"])))
def test_modify_encoder_matches_reference(k):
    s, i, c, cm = str(Z["modify__cases"][k]).split(",")
    torch.manual_seed(100 + k)
    shell = torch.nn.Module()
    shell.conv_in = torch.nn.Conv2d(4, 320, 3, padding=1)
    UNet.modify_encoder(shell, in_channels=8, init_mode_seg=s, init_mode_image=i, cond_channels=int(c),
                        init_mode_cond=cm)
    assert shell.conv_in is shell.new_conv                      # the aliased registration (:182,233)
    if f"modify__{k}__weight" in Z.files:
        assert np.array_equal(shell.conv_in.weight.detach().numpy(), Z[f"modify__{k}__weight"])
        assert np.array_equal(shell.conv_in.bias.detach().numpy(), Z[f"modify__{k}__bias"])
    assert _sha(shell.conv_in.weight, shell.conv_in.bias) == str(Z[f"modify__{k}__sha"]), (s, i, c, cm)


def test_modify_encoder_rejects_what_the_reference_rejects():
    torch.manual_seed(0)
    shell = torch.nn.Module()
    shell.conv_in = torch.nn.Conv2d(4, 320, 3, padding=1)
    with pytest.raises(NotImplementedError):                     # cond 'mean' needs image 'mean' (:225-230)
        UNet.modify_encoder(shell, in_channels=8, init_mode_image="copy", cond_channels=4, init_mode_cond="mean")


@pytest.mark.parametrize("tag", ["a", "same_wd"])
def test_param_groups_match_get_optim_unet(tag):
    wd, wdn, decay = Z[f"optim__{tag}__hp"].tolist()
    u = build_loop_unet(UNet, cond=4)
    names = {id(p): n for n, p in u.named_parameters()}
    st = LDMTrainStep(u, DDIMNoiseScheduler(verbose=False), lr=1e-4, weight_decay=wd, weight_decay_norm=wdn,
                      lr_factor_func=functools.partial(u.get_lr_func, lr_decay_rate=decay))
    groups = st.reference_param_groups()
    assert [len(ps) for _, ps in groups] == Z[f"optim__{tag}__sizes"].tolist()
    assert [names[id(p)] for _, ps in groups for p in ps] == Z[f"optim__{tag}__names"].tolist()
    sd = st.state_dict()
    np.testing.assert_allclose([g["lr"] for g in sd["param_groups"]], Z[f"optim__{tag}__lr"], rtol=1e-6)
    np.testing.assert_allclose([g["weight_decay"] for g in sd["param_groups"]], Z[f"optim__{tag}__wd"], rtol=1e-6)
    assert sorted(sd["param_groups"][0].keys()) == Z[f"optim__{tag}__group_keys"].tolist()


def test_param_groups_survive_set_lr_round_trip():
    """A scheduled lr (update_scheduler, trainers_ldm_cond.py:783-790) sets every group's lr; the
    groups themselves — and so a resume — must not change (lr_decay_rate != 1)."""
    wd, wdn, decay = Z["optim__a__hp"].tolist()
    u = build_loop_unet(UNet, cond=4)
    st = LDMTrainStep(u, DDIMNoiseScheduler(verbose=False), lr=1e-4, weight_decay=wd, weight_decay_norm=wdn,
                      lr_factor_func=functools.partial(u.get_lr_func, lr_decay_rate=decay))
    n_groups = len(st.state_dict()["param_groups"])
    st.set_lr(3e-5)
    sd = st.state_dict()
    assert len(sd["param_groups"]) == n_groups == len(Z["optim__a__sizes"])
    assert all(abs(g["lr"] - 3e-5) < 1e-12 for g in sd["param_groups"])
    u2 = build_loop_unet(UNet, cond=4)
    st2 = LDMTrainStep(u2, DDIMNoiseScheduler(verbose=False), lr=1e-4, weight_decay=wd, weight_decay_norm=wdn,
                       lr_factor_func=functools.partial(u2.get_lr_func, lr_decay_rate=decay))
    st2.load_state_dict(sd)
    assert all(abs(s[2] - 3e-5) < 1e-12 for s in st2.seg_hp)


def test_save_dict_layout_and_resume_match_reference(tmp_path):
    u = build_loop_unet(UNet, cond=4)
    vs = GeneralVAESeg(**VAE_CONFIGS["kitti"])
    d = ck.construct_save_dict(u, vs, vae_image=torch.nn.Identity(), step=17, epoch=3,
                               opt=torch.optim.AdamW(u.parameters(), lr=1e-4), p={"a": 1})
    assert list(d) == Z["save__keys"].tolist()
    assert list(d["vae_semseg"]) == Z["save__vae_semseg_keys"].tolist()   # the REFERENCE GeneralVAESeg's keys
    assert list(d["unet"]) == Z["save__unet_keys"].tolist()
    path = tmp_path / "model.pt"
    ck.save(path, unet=u, vae_semseg=vs, vae_image=torch.nn.Identity(), step=17, epoch=3, p={"a": 1})
    u2 = build_loop_unet(UNet, cond=4, seed=9)
    _, start_epoch, step = ck.resume(path, u2, vae_semseg=GeneralVAESeg(**VAE_CONFIGS["kitti"]),
                                     num_iters_per_epoch=100)
    assert [start_epoch, step] == Z["save__resume"].tolist()      # what the reference's resume() computed
    assert state_hash(u2) == state_hash(u)


def test_color_map_matches_reference():
    assert np.array_equal(color_map(), Z["cmap"])
    np.testing.assert_allclose(color_map(normalized=True), Z["cmap_norm"], rtol=0, atol=1e-7)


def test_loop_unet_weights_are_the_fixtures():
    assert state_hash(build_loop_unet(UNet, cond=4)) == str(Z["unet__state_sha"])
    assert state_hash(build_loop_unet(UNet, cond=0)) == str(Z["sample__sc0__state_sha"])
