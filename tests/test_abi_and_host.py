"""CPU-only checks: the C-ABI library loads and exports every declared symbol; host-side
logic of the drop-in modules (structure, checkpoint keys, schedule tables, weight packing)."""
import os
import re

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_utils import DDIM_CONFIGS, VAE_CONFIGS, load
from ldmseg.models import GeneralVAESeg, UNet
from ldmseg.ops import native as K
from ldmseg.schedulers import DDIMNoiseScheduler

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "ldmseg_hip.h")).read()
    return sorted(set(re.findall(r"^(?:int|void|size_t|const char\*)\s+(ldm_\w+)\(", src, re.M)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = K.load_library()
    syms = _declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(K.EXPORTS), "python binding and header disagree"
    assert lib.ldm_abi_version() == 1
    assert lib.ldm_status_string(2).decode().startswith("pointer")


def test_workspace_size_is_host_only():
    lib = K.load_library()
    assert lib.ldm_group_norm_workspace_bytes(8, 4096, 320) >= 8 * 320 * 2 * 8   # fp64 (sum, sumsq)


def test_ops_refuse_cpu_tensors():
    pc = K.PackedConv(torch.randn(8, 8, 3, 3), torch.randn(8), torch.float32)
    with pytest.raises(RuntimeError, match="GPU tensors only"):
        K.conv2d(pc, torch.randn(1, 4, 4, 8), 1, 4, 4)
    with pytest.raises(RuntimeError, match="GPU tensors only"):
        K.bit_encode(torch.zeros(4, 4, dtype=torch.int64), 5, 255, 0.5)


def test_group_norm_refuses_out_of_range_shapes_before_launch():
    """ldm_group_norm stages <= 64 groups and <= 2560 channels in LDS; wider calls get a clear
    error on the host (no launch, no GPU needed)."""
    x = torch.zeros(1, 4, 128)
    g, b = torch.ones(128), torch.zeros(128)
    with pytest.raises(ValueError, match="outside the HIP kernel's range"):
        K.group_norm(x, 1, 4, 128, g, b, 1e-5)            # 128 groups
    x = torch.zeros(1, 4, 2600)
    with pytest.raises(ValueError, match="outside the HIP kernel's range"):
        K.group_norm(x, 1, 4, 26, torch.ones(2600), torch.zeros(2600), 1e-5)
    with pytest.raises(RuntimeError, match="GPU tensors only"):   # in range: reaches the device check
        K.group_norm(torch.zeros(1, 4, 2560), 1, 4, 32, torch.ones(2560), torch.zeros(2560), 1e-5)


# --------------------------------------------------------------------------- UNet structure
def test_unet_structure_and_param_counts():
    u = UNet()
    n = sum(p.numel() for p in u.parameters())
    assert n == 859_520_964                    # SD-1.4 UNet2DConditionModel
    u.remove_cross_attention()
    u.modify_encoder(in_channels=8, init_mode_seg="copy", init_mode_image="zero")
    assert sum(p.numel() for p in u.parameters()) == 815_544_964   # SURVEY §2.3 (815.5 M)
    sd = u.state_dict()
    keys = list(sd)
    # diffusers names + the new_conv alias registered last (unet.py:182,233)
    assert keys[:2] == ["conv_in.weight", "conv_in.bias"] and keys[-2:] == ["new_conv.weight", "new_conv.bias"]
    assert sd["conv_in.weight"].shape == (320, 8, 3, 3)
    assert "down_blocks.0.attentions.0.transformer_blocks.0.attn1.to_q.weight" in sd
    assert not any(".attn2." in k or ".norm2." in k and "transformer_blocks" in k for k in keys)
    assert "up_blocks.1.upsamplers.0.conv.weight" in sd and "down_blocks.2.downsamplers.0.conv.weight" in sd
    assert sd["up_blocks.3.resnets.0.conv1.weight"].shape == (320, 960, 3, 3)
    assert sd["mid_block.attentions.0.transformer_blocks.0.ff.net.0.proj.weight"].shape == (10240, 1280)


def test_modify_encoder_quirks():
    u = UNet(block_out_channels=(32, 64, 64, 64), cross_attention_dim=None)
    w0 = u.conv_in.weight.detach().clone()
    u.modify_encoder(in_channels=8, init_mode_seg="div", init_mode_image="div", cond_channels=4,
                     init_mode_cond="zero")
    w = u.conv_in.weight.detach()
    assert torch.equal(w[:, :4], w0) and torch.equal(w[:, 4:8], w0)    # 'div' is a no-op (unet.py:188,202)
    assert torch.all(w[:, 8:] == 0)
    assert u.get_lr_func("module.down_blocks.0.x", 0.1) == 0.1 and u.get_lr_func("up_blocks.x", 0.1) == 1.0


# --------------------------------------------------------------------------- scheduler host side
@pytest.mark.parametrize("cname", list(DDIM_CONFIGS))
def test_scheduler_tables_match_reference(cname):
    z = load("ddim.npz")
    s = DDIMNoiseScheduler(**DDIM_CONFIGS[cname], device="cpu", verbose=False)
    np.testing.assert_array_equal(s.betas.numpy(), z[f"{cname}__betas"])
    np.testing.assert_array_equal(s.alphas_cumprod.numpy(), z[f"{cname}__alphas_cumprod"])
    np.testing.assert_array_equal(s.weights.numpy(), z[f"{cname}__weights"])
    assert float(s.final_alpha_cumprod) == float(z[f"{cname}__final_alpha_cumprod"])
    for n in (50, 25, 7):
        s.set_timesteps_inference(n)
        np.testing.assert_array_equal(s.timesteps.numpy(), z[f"{cname}__timesteps_{n}"])
    s.set_timesteps_inference(50, tmin=300)
    np.testing.assert_array_equal(s.timesteps.numpy(), z[f"{cname}__timesteps_50_tmin300"])
    assert len(s) == 1000 and "DDIMScheduler(" in str(s)


def test_scheduler_known_answers():
    s = DDIMNoiseScheduler(**DDIM_CONFIGS["script"], device="cpu", verbose=False)
    assert abs(float(s.alphas_cumprod[999]) - 0.0046601) < 1e-6
    assert abs(float(s.alphas_cumprod[19]) - 0.9822440) < 1e-6
    assert abs(float(s.final_alpha_cumprod) - 0.9991500) < 1e-6
    assert abs(float(s.weights[0]) - 0.0017015) < 1e-6 and float(s.weights[999]) == 1.0


# --------------------------------------------------------------------------- weight packing
def _emulate_packed_gemm(pc, x_nhwc, h, w, upsample=False, stride=1):
    """CPU emulation of ldm_conv2d's contraction order from the PACKED weights (im2col)."""
    B, _, _, C = x_nhwc.shape
    x = x_nhwc.permute(0, 3, 1, 2)
    if upsample:
        x = F.interpolate(x, scale_factor=2.0, mode="nearest")
    k = pc.ksize
    cols = F.unfold(x, k, padding=k // 2, stride=stride)                       # [B, C*k*k, L] (c-major)
    cols = cols.view(B, C, k * k, -1).permute(0, 3, 2, 1).reshape(B, -1, k * k * C)   # tap-major
    Wp = pc.w[:, : k * k * C].float()
    y = cols @ Wp.t()
    if pc.bias is not None:
        y = y + pc.bias
    return y


def test_packing_conv3x3_tap_major():
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(12, 24, 3, padding=1)
    pc = K.PackedConv(conv.weight, conv.bias, torch.float32, cin_pad=16)
    assert pc.kpad % 64 == 0 and pc.cin == 16
    x = torch.randn(2, 12, 9, 7)
    xp = F.pad(x, (0, 0, 0, 0, 0, 4)).permute(0, 2, 3, 1)
    y = _emulate_packed_gemm(pc, xp, 9, 7)
    ref = conv(x).permute(0, 2, 3, 1).reshape(2, -1, 24)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)


def test_packing_geglu_interleave():
    torch.manual_seed(0)
    lin = torch.nn.Linear(32, 128)
    pc = K.PackedConv(lin.weight, lin.bias, torch.float32, geglu=True)
    x = torch.randn(5, 32)
    y = x @ pc.w[:, :32].t() + pc.bias                                         # packed columns
    y = y.view(5, -1, 2, 16)                                                   # (block, h|g, 16)
    out = (y[:, :, 0] * F.gelu(y[:, :, 1])).reshape(5, 64)
    h, g = lin(x).chunk(2, dim=-1)
    torch.testing.assert_close(out, h * F.gelu(g), rtol=1e-5, atol=1e-5)


def test_packing_convT_shuffle():
    torch.manual_seed(0)
    ct = torch.nn.ConvTranspose2d(16, 8, 2, stride=2)
    pc = K.PackedConv(ct.weight, ct.bias, torch.float32, shuffle2=True)
    x = torch.randn(2, 16, 3, 5)
    y = x.permute(0, 2, 3, 1).reshape(-1, 16) @ pc.w[:, :16].t() + pc.bias     # [B*H*W, 4*Cout]
    y = y.view(2, 3, 5, 2, 2, 8).permute(0, 5, 1, 3, 2, 4).reshape(2, 8, 6, 10)  # (b,co,y,dy,x,dx)
    torch.testing.assert_close(y, ct(x), rtol=1e-5, atol=1e-5)


# --------------------------------------------------------------------------- VAE structure
@pytest.mark.parametrize("cname", list(VAE_CONFIGS))
def test_vae_state_dict_keys_match_reference(cname):
    z = load("vae.npz")
    v = GeneralVAESeg(**VAE_CONFIGS[cname])
    assert list(v.state_dict().keys()) == list(z[f"{cname}__keys"])
    assert v.interpolation_factor == int(z[f"{cname}__interpolation_factor"])


def test_alias_package_imports_next_to_reference_name():
    """the drop-in modules load as ``ldmseg_mi355x`` (no GPU needed)."""
    import importlib
    m = importlib.import_module("ldmseg_mi355x")
    from ldmseg_mi355x.models import GeneralVAESeg, UNet  # noqa: F401
    from ldmseg_mi355x.schedulers import DDIMNoiseScheduler  # noqa: F401
    assert m.__name__ == "ldmseg_mi355x" and UNet.__module__ == "ldmseg_mi355x.models.unet"


def test_autoencoder_kl_structure_and_legacy_keys():
    """GeneralVAEImage keeps diffusers' AutoencoderKL names (encoder.*, quant_conv, post_quant_conv;
    no decoder keys, tools/main_ldm.py:139) and accepts the pre-0.14 attention names."""
    from ldmseg.models.autoencoder_kl import GeneralVAEImage
    m = GeneralVAEImage()
    sd = m.state_dict()
    n_enc = sum(v.numel() for k, v in sd.items() if k.startswith("encoder."))
    assert n_enc == 34_163_592                      # SD-1.x VAE encoder
    assert "encoder.mid_block.attentions.0.to_out.0.weight" in sd
    assert "encoder.down_blocks.0.downsamplers.0.conv.weight" in sd
    assert "encoder.down_blocks.3.downsamplers.0.conv.weight" not in sd
    assert not any(k.startswith("decoder.") for k in sd)
    legacy = {k.replace(".to_q.", ".query.").replace(".to_out.0.", ".proj_attn."): v.clone() for k, v in sd.items()}
    legacy["decoder.conv_in.weight"] = torch.zeros(1)          # decoder weights of a full checkpoint are skipped
    m2 = GeneralVAEImage()
    m2.load_state_dict(legacy)
    assert torch.equal(m2.encoder.mid_block.attentions[0].to_q.weight, m.encoder.mid_block.attentions[0].to_q.weight)
    m2.set_scaling_factor(0.2)
    assert m2.scaling_factor == 0.2
