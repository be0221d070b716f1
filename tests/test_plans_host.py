"""ldm_conv2d's planner on the host (ldm_conv2d_describe_plan; no GPU, nothing launches).

The plans of the headline workload (BASELINE config: B = 8 frames at 64x64 latents) are pinned —
they are the ones the bench and its rocprof profiles measure — and config 2's single frame must
fill the chip: at B = 1 every 3x3 conv and deep-K GEMM is split into >= 128 blocks instead of the
32 halo tiles / 64-160 blocks the B = 8 rules gave (profiles/r03g_b1_plans.txt).
"""
import pytest

from ldmseg.ops import native as K


def _p(**kw):
    return K.describe_plan(**kw)


def test_headline_plans_pinned():
    # 3x3 at the 64x64 and 32x32 levels: halo-tiled, one block per CU
    for hw, c in ((64, 320), (32, 640)):
        pl = _p(batch=8, h=hw, w=hw, c0=c, n=c, temb=True, gn_stats=True)
        assert pl["kind"] == "halo" and pl["blocks"] == 256, pl
    # the [640 || 320] -> 320 up-block conv reads the concat in place on the halo kernel
    assert _p(batch=8, h=64, w=64, c0=640, c1=320, n=320, residual=True, gn_stats=True)["kind"] == "halo"
    # GEGLU: A-register-stationary at K = 320, the wide persistent tile at K = 640 / 1280
    assert _p(batch=8 * 4096, h=1, w=1, c0=320, n=2560, ksize=1, ln=True, out_layout=K.OUT_GEGLU)["kind"] == "ars"
    for hw, c in ((32, 640), (16, 1280)):
        pl = _p(batch=8 * hw * hw, h=1, w=1, c0=c, n=8 * c, ksize=1, ln=True, out_layout=K.OUT_GEGLU)
        assert pl["kind"] == "wide", pl
    # QKV at K = 320 stays on the two-blocks-per-CU tiles (the wide tile lost there, r03a)
    pl = _p(batch=8 * 4096, h=1, w=1, c0=320, n=960, ksize=1, ln=True, geglu_bias=False)
    assert (pl["kind"], pl["bm"], pl["bn"]) == ("tile", 128, 160), pl
    # the 16x16 level: whole-image halo tiles (256 rows) split over channel blocks to 256+ blocks
    for c0, c1, ks in ((1280, 0, 4), (1280, 1280, 4), (1280, 640, 5)):
        pl = _p(batch=8, h=16, w=16, c0=c0, c1=c1, n=1280, temb=True, gn_stats=True)
        assert (pl["kind"], pl["bm"], pl["bn"], pl["ksplit"]) == ("halo", 256, 160, ks), pl
        assert pl["blocks"] >= 256 and (c0 + c1) // 64 // ks >= 4, pl
    # the 32x32 level's wide up-block concats: 256-row halo tiles split over channel blocks (the
    # [640 || 320] -> 640 concat and the single-source convs keep 4-row tiles)
    for c0, c1, ks in ((1280, 640, 2), (640, 640, 2)):
        pl = _p(batch=8, h=32, w=32, c0=c0, c1=c1, n=640, temb=True, gn_stats=True)
        assert (pl["kind"], pl["bm"], pl["bn"], pl["ksplit"], pl["blocks"]) == ("halo", 256, 160, ks, 256), pl
    pl = _p(batch=8, h=32, w=32, c0=640, c1=320, n=640, temb=True, gn_stats=True)
    assert (pl["kind"], pl["bm"], pl["ksplit"]) == ("halo", 128, 1), pl
    # 640 -> 1280 would need 2-channel-block splits: the split 128x160 tiles stay faster
    pl = _p(batch=8, h=16, w=16, c0=640, n=1280, temb=True, gn_stats=True)
    assert (pl["kind"], pl["bm"], pl["bn"], pl["ksplit"]) == ("tile", 128, 160, 4), pl
    pl = _p(batch=8, h=8, w=8, c0=1280, n=1280, temb=True, gn_stats=True)
    assert (pl["bm"], pl["bn"], pl["ksplit"], pl["blocks"]) == (64, 160, 8, 512), pl
    pl = _p(batch=8, h=8, w=8, c0=1280, c1=1280, n=1280, residual=True, gn_stats=True)
    assert (pl["bm"], pl["bn"], pl["ksplit"]) == (128, 160, 16), pl


@pytest.mark.parametrize("hw,c0,c1,n", [(64, 320, 0, 320), (64, 640, 320, 320), (32, 320, 0, 640), (32, 640, 0, 640),
                                        (32, 1280, 640, 640), (16, 640, 0, 1280), (16, 1280, 0, 1280),
                                        (16, 2560, 0, 1280), (8, 1280, 0, 1280), (8, 1280, 1280, 1280)])
def test_single_frame_convs_fill_the_chip(hw, c0, c1, n):
    pl = _p(batch=1, h=hw, w=hw, c0=c0, c1=c1, n=n, residual=True, gn_stats=True)
    assert pl["kind"] == "tile" and pl["blocks"] >= 128, pl
    if hw >= 16:
        assert pl["blocks"] >= 256, pl


@pytest.mark.parametrize("M,kin,n", [(1024, 2560, 640), (256, 5120, 1280), (64, 5120, 1280)])
def test_single_frame_deep_gemms_split(M, kin, n):
    """Few rows, deep K: split K over >= 128 blocks, or one deep-ring tile per CU (no split)."""
    pl = _p(batch=M, h=1, w=1, c0=kin, n=n, ksize=1, residual=True)
    assert (pl["ksplit"] > 1 or pl["kind"] == "ring") and pl["blocks"] >= 128, pl


def test_deep_level_gemms_on_the_ring():
    """The 16x16 / 8x8 levels' 1x1 GEMMs at B = 8 (proj_in / to_out / proj_out, the
    16x16 up-block shortcuts) run on the deep-ring kernel, one tile per CU."""
    for M, c0, c1, n, kw in ((2048, 1280, 0, 1280, dict(residual=True, gn_stats=True)),
                             (2048, 1280, 0, 1280, dict(row_stats=True)),
                             (2048, 1280, 1280, 1280, {}), (2048, 1280, 640, 1280, {}),
                             (512, 1280, 0, 1280, dict(residual=True, gn_stats=True))):
        pl = _p(batch=M // 64 if kw.get("gn_stats") else M, h=8 if kw.get("gn_stats") else 1,
                w=8 if kw.get("gn_stats") else 1, c0=c0, c1=c1, n=n, ksize=1, **kw)
        assert pl["kind"] == "ring" and pl["blocks"] == 256, (M, c0, c1, n, kw, pl)
    # ff.net.2 (K = 5120) and the 8x8 concat shortcut keep their split-K tiles
    for M, c0, c1 in ((2048, 5120, 0), (512, 5120, 0), (512, 1280, 1280)):
        assert _p(batch=M, h=1, w=1, c0=c0, c1=c1, n=1280, ksize=1, residual=True)["kind"] == "tile"


def test_describe_plan_rejects_what_conv2d_rejects():
    assert _p(batch=1, h=8, w=8, c0=12, n=64)["kind"] == "tile"     # c0 padded to 16: legal
    with pytest.raises(RuntimeError):
        _p(batch=1, h=8, w=8, c0=16, n=64, ksize=3, stride=2, upsample=True)   # upsample + stride 2


def test_feedforward_fused_only_where_it_fills_the_chip():
    """ldm_feedforward (one 128-row tile per CU) takes the 64x64 level's FeedForward at B >= 8
    frames; a single frame (32 tiles) keeps the two-launch form."""
    import torch
    bf = torch.bfloat16
    w1, w2 = torch.randn(2560, 320) * 0.05, torch.randn(320, 1280) * 0.03
    pc1 = K.PackedConv(w1, torch.zeros(2560), bf, geglu=True)
    pc2 = K.PackedConv(w2, torch.zeros(320), bf)
    assert K.feedforward_ok(pc1, pc2, torch.empty(8, 4096, 320, dtype=bf))
    assert not K.feedforward_ok(pc1, pc2, torch.empty(1, 4096, 320, dtype=bf))
    assert not K.feedforward_ok(K.PackedConv(w1, None, bf), pc2, torch.empty(8, 4096, 320, dtype=bf))
    with pytest.raises(RuntimeError):           # CPU tensors: no fallback path
        K.feedforward(pc1, pc2, torch.empty(8, 4096, 320, dtype=bf))
