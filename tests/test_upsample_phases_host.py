"""The phase form of the Upsample2D conv on the host (no GPU): nearest-2x upsample + 3x3 conv
(diffusers Upsample2D, reached via /root/reference/ldmseg/models/unet.py:281-436) equals four 2x2
convs over the low-res input, one per output phase, whose weights sum the 3x3 taps that read the
same source pixel (PackedConv(upsample_phases=True), csrc/igemm.hip phase mode).  Checked here
in fp64 on the packed layout itself — rows (dy, dx, co), K (ty, tx, ci) — so the GPU kernel's
addressing is the only thing left to the GPU test (tests/test_gpu_ops.py)."""
import torch
import torch.nn.functional as F

from ldmseg.ops import native as K


def test_phase_pack_reproduces_upsample_conv():
    torch.manual_seed(0)
    B, cin, cout, H, W = 2, 24, 16, 5, 7
    x = torch.randn(B, cin, H, W, dtype=torch.float64)
    w = torch.randn(cout, cin, 3, 3, dtype=torch.float64)
    b = torch.randn(cout, dtype=torch.float64)
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), w, b, padding=1)
    pc = K.PackedConv(w.float(), b.float(), torch.float32, upsample_phases=True)
    assert pc.ksize == 2 and pc.n == cout and pc.phases and pc.w.shape == (4 * cout, pc.kpad)
    wp = pc.w[:, :4 * cin].double().reshape(2, 2, cout, 2, 2, cin)          # (dy, dx, co, ty, tx, ci)
    xp = F.pad(x, (1, 1, 1, 1))                                             # source rows y - 1 .. y + 1
    out = torch.zeros(B, cout, 2 * H, 2 * W, dtype=torch.float64)
    for dy in range(2):
        for dx in range(2):
            k = wp[dy, dx].permute(0, 3, 1, 2)                             # [co, ci, ty, tx]
            # taps ty at source row y - 1 + dy + ty: a 2x2 conv over xp starting at row dy
            o = F.conv2d(xp[:, :, dy:dy + H + 1, dx:dx + W + 1], k, pc.bias.double())
            out[:, :, dy::2, dx::2] = o
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-4)


def test_phase_pack_needs_upsample_flag():
    """The upsample check comes before any device check: a phase pack called without
    upsample=True is rejected with ValueError on any tensor (a CPU tensor used to
    satisfy the test through the device check alone)."""
    pc = K.PackedConv(torch.randn(8, 8, 3, 3), None, torch.float32, upsample_phases=True)
    import pytest
    with pytest.raises(ValueError, match="upsample_phases"):
        K.conv2d(pc, torch.empty(1, 4, 4, 8), 1, 4, 4)
