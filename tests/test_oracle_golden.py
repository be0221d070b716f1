"""Pin the CPU oracle (oracle/) against the reference's golden vectors (tests/golden/)."""
import numpy as np
import pytest
import torch

from golden_utils import DDIM_CONFIGS, VAE_CONFIGS, load, vae_state_dict
from oracle import codec, ddim, dvpq, vae


# ----------------------------------------------------------------------------- codec
def test_codec_known_answer_pngs():
    z = load("codec.npz")
    planes, _ = codec.encode_bitmap(z["fixture_semseg"].astype(np.int64), n=16, ignore_label=0)
    assert np.array_equal((planes * 255).astype(np.uint8), z["fixture_bits_u8"])
    dec = codec.decode_bitmap(2 * planes - 1)
    assert np.array_equal(dec, z["fixture_decode"])


@pytest.mark.parametrize("case", list(load("codec.npz")["cases"]))
def test_codec_cases(case):
    z = load("codec.npz")
    i = list(z["cases"]).index(case)
    n, ign = int(z["cases_n"][i]), int(z["cases_ignore"][i])
    planes, mask = codec.encode_bitmap(z[f"{case}__ids"], n=n, ignore_label=ign)
    assert planes.dtype == np.float32
    assert np.array_equal(planes, z[f"{case}__enc"])
    assert np.array_equal(mask, z[f"{case}__ignore_mask"])
    assert np.array_equal(codec.decode_bitmap(2 * planes - 1), z[f"{case}__dec_clean"])
    assert np.array_equal(codec.decode_bitmap(z[f"{case}__noisy"]), z[f"{case}__dec_noisy"])


# ----------------------------------------------------------------------------- ddim
@pytest.mark.parametrize("cname", list(DDIM_CONFIGS))
def test_ddim_tables_and_steps(cname):
    z = load("ddim.npz")
    kw = DDIM_CONFIGS[cname]
    betas, ac, final = ddim.tables(kw.get("beta_schedule", "linear"), kw.get("num_train_timesteps", 1000),
                                   kw.get("beta_start", 0.0001), kw.get("beta_end", 0.02),
                                   kw.get("set_alpha_to_one", True))
    np.testing.assert_array_equal(betas.numpy(), z[f"{cname}__betas"])
    np.testing.assert_array_equal(ac.numpy(), z[f"{cname}__alphas_cumprod"])
    assert float(final) == float(z[f"{cname}__final_alpha_cumprod"])
    w = ddim.loss_weights(ac, kw.get("weight", "none"), kw.get("max_snr", 5.0))
    np.testing.assert_array_equal(w.numpy(), z[f"{cname}__weights"])
    for n in (50, 25, 7):
        np.testing.assert_array_equal(ddim.inference_timesteps(1000, n), z[f"{cname}__timesteps_{n}"])
    np.testing.assert_array_equal(ddim.inference_timesteps(1000, 50, 300), z[f"{cname}__timesteps_50_tmin300"])
    mo = torch.from_numpy(z[f"{cname}__step_model_output"])
    x = torch.from_numpy(z[f"{cname}__step_sample"])
    for t in z[f"{cname}__step_t"]:
        for clipped in (0, 1):
            prev, x0 = ddim.step(ac, final, 1000, 50, mo, int(t), x, kw.get("prediction_type", "epsilon"),
                                 kw.get("clip_sample", True), kw.get("clip_sample_range", 1.0), bool(clipped))
            np.testing.assert_allclose(prev.numpy(), z[f"{cname}__step_{t}_{clipped}__prev"], rtol=1e-6, atol=1e-6)
            np.testing.assert_allclose(x0.numpy(), z[f"{cname}__step_{t}_{clipped}__x0"], rtol=1e-6, atol=1e-6)
    tb = torch.from_numpy(z[f"{cname}__an_t"])
    x0 = torch.from_numpy(z[f"{cname}__an_x0"])
    eps = torch.from_numpy(z[f"{cname}__an_eps"])
    np.testing.assert_allclose(ddim.add_noise(ac, x0, eps, tb).numpy(), z[f"{cname}__an_out"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(ddim.add_noise(ac, x0, eps, tb, 2.0).numpy(), z[f"{cname}__an_out_s2"],
                               rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(ddim.remove_noise(ac, x, eps, tb).numpy(), z[f"{cname}__rn_out"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(ddim.remove_noise(ac, x, eps, tb, 0.5).numpy(), z[f"{cname}__rn_out_s2"],
                               rtol=1e-6, atol=1e-6)


# ----------------------------------------------------------------------------- vae
@pytest.mark.parametrize("cname", list(VAE_CONFIGS))
def test_vae_encode_decode(cname):
    torch.set_num_threads(8)
    z = load("vae.npz")
    cfg = VAE_CONFIGS[cname]
    sd = vae_state_dict(z, cname)
    assert sorted(sd) == sorted(z[f"{cname}__keys"])
    x = torch.from_numpy(z[f"{cname}__x"])
    with torch.no_grad():
        moments, mean, logvar, std = vae.encode(sd, x, cfg)
        np.testing.assert_allclose(moments.numpy(), z[f"{cname}__moments"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(mean.numpy(), z[f"{cname}__mean"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(logvar.numpy(), z[f"{cname}__logvar"], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(std.numpy(), z[f"{cname}__std"], rtol=1e-5, atol=1e-5)
        dec_n = vae.decode(sd, mean, cfg, interpolate=False)
        dec_i = vae.decode(sd, mean, cfg, interpolate=True)
    np.testing.assert_allclose(dec_n.numpy(), z[f"{cname}__dec_nointerp"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(dec_i.numpy(), z[f"{cname}__dec_interp"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(dec_n.numpy(), z[f"{cname}__forward"], rtol=1e-5, atol=1e-5)


# ----------------------------------------------------------------------------- dvpq
def test_vpq_eval():
    z = load("vpq.npz")
    for c in range(int(z["n_cases"])):
        iou, tp, fn, fp = dvpq.vpq_eval(z[f"c{c}__pred"], z[f"c{c}__gt"])
        np.testing.assert_allclose(iou, z[f"c{c}__iou"], rtol=1e-12)
        np.testing.assert_array_equal(tp, z[f"c{c}__tp"])
        np.testing.assert_array_equal(fn, z[f"c{c}__fn"])
        np.testing.assert_array_equal(fp, z[f"c{c}__fp"])


def _panoptic_cases():
    z = load("panoptic.npz")
    return z, [str(n) for n in z["names"]]


@pytest.mark.parametrize("name", ["kitti_max", "kitti_ign0", "topk_diff", "no_threshold", "base_yaml", "resized"])
def test_panoptic_head_oracle(name):
    """oracle/panoptic.py == the reference compute_pq method's cleaned_pred (panoptic.npz)."""
    from oracle import panoptic as opan
    z, _ = _panoptic_cases()
    logits = torch.from_numpy(z[f"{name}__logits"].astype(np.float32))
    mth, cth, oth, ign, thr, mode, Hi, Wi, h, w, rows = z[f"{name}__cfg"].tolist()
    kw = dict(mask_th=mth, count_th=int(cth), overlap_th=oth, ignore_label=int(ign), threshold_output=bool(thr),
              threshold_mode={1: "max", 2: "topk_diff"}[int(mode)])
    B = logits.shape[0]
    pad = torch.zeros(B, int(Hi), int(Wi), dtype=torch.bool)
    pad[:, :int(rows), :] = True
    got = opan.postprocess(logits, (int(Hi), int(Wi)), pad, [(int(h), int(w))] * B, **kw)
    exp = z[f"{name}__cleaned"].astype(np.int64)
    for i in range(B):
        np.testing.assert_array_equal(got[i], exp[i])


def test_ae_iteration_oracle():
    """oracle/ae.py (autograd over the restated VAE + point losses) == the reference's AE iteration
    (ae.npz) with the reference's draws replayed and its point selection forced."""
    from oracle import ae as oae
    z = load("ae.npz")
    cfg = dict(in_channels=10, int_channels=64, out_channels=30, block_out_channels=(16, 32, 32, 64),
               latent_channels=4, num_latents=2, num_upscalers=2, norm_num_groups=16)
    sd = {}
    for name in z["names"]:
        name = str(name)
        v = z[f"w__{name}__q"].astype(np.float32) * z[f"w__{name}__scale"]
        if bool(z[f"w__{name}__plus1"]):
            v = v + np.float32(1.0)
        sd[name] = torch.from_numpy(v.astype(np.float32))
    g_rand = torch.Generator().manual_seed(123)
    g_randn = torch.Generator().manual_seed(456)
    sels = [torch.from_numpy(z["sel_ce"].astype(np.int64)), torch.from_numpy(z["sel_mask"].astype(np.int64))]
    torch.set_num_threads(8)
    loss, ce, mask, grads = oae.train_iteration(
        sd, cfg, torch.from_numpy(z["bits"].astype(np.float32)), torch.from_numpy(z["targets"].astype(np.int64)),
        rand=lambda *s: torch.rand(*s, generator=g_rand), randn=lambda s: torch.randn(*s, generator=g_randn),
        select=lambda u, k: sels.pop(0))
    assert abs(ce.item() - float(z["ce"])) <= 1e-5 * float(z["ce"])
    assert abs(mask.item() - float(z["mask"])) <= 1e-5 * float(z["mask"])
    for name in z["names"]:
        ref = torch.from_numpy(z[f"g__{name}"])
        assert (grads[str(name)] - ref).norm() <= 1e-4 * ref.norm(), name


def test_posenet_oracle_matches_reference_golden():
    """oracle/posenet.py against the reference PoseExpNet's outputs (posenet.npz), weights rebuilt
    by the drop-in module under the same seed (state sha256 checked)."""
    import hashlib
    from oracle import posenet as opose
    from posenet.posenet import PoseExpNet
    z = load("posenet.npz")
    for name in [str(n) for n in z["names"]]:
        seed, B, H, W, nref, exp, train, xavier = z[f"{name}__cfg"].tolist()
        torch.manual_seed(seed)
        net = PoseExpNet(nb_ref_imgs=nref, output_exp=bool(exp))
        if xavier:
            net.init_weights()
        h = hashlib.sha256()
        for k, v in sorted(net.state_dict().items()):
            h.update(k.encode())
            h.update(v.detach().float().contiguous().numpy().tobytes())
        assert h.hexdigest() == str(z[f"{name}__state_sha"])
        g = torch.Generator().manual_seed(100 + seed)
        tgt = torch.rand(B, 3, H, W, generator=g)
        refs = [torch.rand(B, 3, H, W, generator=g) for _ in range(nref)]
        with torch.no_grad():
            pose, masks = opose.forward(net.state_dict(), tgt, refs, output_exp=bool(exp))
        np.testing.assert_allclose(pose.numpy(), z[f"{name}__pose"], rtol=1e-5, atol=1e-7)
        if exp:
            for i in range(4 if train else 1):
                np.testing.assert_allclose(masks[i].numpy(), z[f"{name}__mask{i + 1}"], rtol=1e-5, atol=1e-6)
