"""ctypes binding of lib/libldmseg_hip.so (C ABI: include/ldmseg_hip.h) + tensor-level wrappers.

Every op here launches a hand-written gfx950 kernel on the current torch stream.  There is
no fallback: if the library is missing, or a tensor is not on the GPU, the call raises.
Host-side checks (device, dtype, contiguity, shapes) run before any launch so that a bad
call can never reach the GPU as an out-of-bounds kernel.
"""
import contextlib
import ctypes
import math
import os
import threading

import torch

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libldmseg_hip.so")

F32, BF16 = 0, 1
OUT_NHWC, OUT_NCHW, OUT_GEGLU, OUT_SHUFFLE2 = 0, 1, 2, 3
ACT_NONE, ACT_SILU, ACT_RELU, ACT_SIGMOID = 0, 1, 2, 3
PRED = {"epsilon": 0, "sample": 1, "v_prediction": 2}
POST_ACT = {"none": 0, "tanh": 1, "sigmoid": 2, "clip": 3}

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_i64 = ctypes.c_int64
_d = ctypes.c_double


class ConvParams(ctypes.Structure):
    _fields_ = [("a0", _vp), ("a1", _vp), ("c0", _i), ("c1", _i), ("batch", _i), ("h_in", _i), ("w_in", _i),
                ("h_out", _i), ("w_out", _i), ("ksize", _i), ("stride", _i), ("upsample", _i), ("w", _vp),
                ("n", _i), ("kpad", _i), ("bias", _vp), ("temb", _vp), ("temb_stride", _i), ("residual", _vp),
                ("out", _vp), ("out_layout", _i), ("act", _i), ("dtype", _i), ("out_f32", _i),
                ("workspace", _vp), ("workspace_bytes", _i64), ("gn_partial", _vp), ("pad_mode", _i), ("gn_unit", _i), ("gn_slots", _i),
                ("row_stats", _vp), ("ln_rows", _vp), ("ln_c1", _vp), ("ln_inv_k", _f), ("ln_eps", _f),
                ("gn_out", _vp), ("gn_gamma", _vp), ("gn_beta", _vp), ("gn_groups", _i), ("gn_act", _i),
                ("gn_eps", _f), ("gn_skip_out", _i)]


class ConvInParams(ctypes.Structure):
    _fields_ = [("src", _vp * 3), ("c", _i * 3), ("src_dtype", _i * 3), ("batch", _i), ("height", _i), ("width", _i),
                ("dtype", _i), ("w", _vp), ("n", _i), ("kpad", _i), ("bias", _vp), ("out", _vp), ("gn_partial", _vp),
                ("gn_unit", _i), ("gn_slots", _i)]


class GnFold(ctypes.Structure):
    _fields_ = [("acc", _vp), ("unit", _i), ("slots", _i), ("groups", _i), ("eps", _f), ("gamma", _vp),
                ("beta", _vp)]


class AttnParams(ctypes.Structure):
    _fields_ = [("q", _vp), ("k", _vp), ("v", _vp), ("o", _vp), ("q_stride", _i), ("k_stride", _i),
                ("v_stride", _i), ("o_stride", _i), ("batch", _i), ("heads", _i), ("head_dim", _i),
                ("n_q", _i), ("n_kv", _i), ("scale", _f), ("dtype", _i)]


class UnetTailParams(ctypes.Structure):
    _fields_ = [("h", _vp), ("batch", _i), ("height", _i), ("width", _i), ("c", _i), ("gn_acc", _vp),
                ("gn_unit", _i), ("gn_slots", _i), ("groups", _i), ("eps", _f), ("gamma", _vp), ("beta", _vp),
                ("w", _vp), ("kpad", _i), ("cout", _i), ("bias", _vp), ("eps_out", _vp), ("eps_dtype", _i),
                ("sample", _vp), ("sample_dtype", _i), ("t", _vp), ("alphas_cumprod", _vp),
                ("final_alpha_cumprod", _f), ("step_ratio", _i), ("prediction_type", _i), ("clip_sample", _i),
                ("clip_range", _f), ("use_clipped_model_output", _i), ("num_train_timesteps", _i), ("prev", _vp),
                ("x0", _vp), ("out_dtype", _i)]


class WgradParams(ctypes.Structure):
    _fields_ = [("a0", _vp), ("a1", _vp), ("c0", _i), ("c1", _i), ("batch", _i), ("h_in", _i), ("w_in", _i),
                ("h_out", _i), ("w_out", _i), ("ksize", _i), ("stride", _i), ("upsample", _i), ("dy", _vp),
                ("n", _i), ("kpad", _i), ("cin_real", _i), ("geglu", _i), ("dw", _vp), ("accumulate", _i),
                ("dtype", _i), ("workspace", _vp), ("workspace_bytes", _i64)]


class DdimParams(ctypes.Structure):
    _fields_ = [("model_output", _vp), ("mo_dtype", _i), ("sample", _vp), ("x_dtype", _i), ("prev", _vp),
                ("x0", _vp), ("out_dtype", _i), ("n", _i64), ("t", _vp), ("alphas_cumprod", _vp),
                ("final_alpha_cumprod", _f), ("step_ratio", _i), ("prediction_type", _i), ("clip_sample", _i),
                ("clip_range", _f), ("use_clipped_model_output", _i), ("num_train_timesteps", _i)]


EXPORTS = {
    "ldm_conv2d": (_i, [ctypes.POINTER(ConvParams), _vp]),
    "ldm_conv2d_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(ConvParams)]),
    "ldm_conv2d_force_plan": (None, [_i, _i, _i]),
    "ldm_conv2d_describe_plan": (_i, [ctypes.POINTER(ConvParams), ctypes.POINTER(ctypes.c_int)]),
    "ldm_conv2d_gn_fusable": (_i, [ctypes.POINTER(ConvParams)]),
    "ldm_conv_in": (_i, [ctypes.POINTER(ConvInParams), _vp]),
    "ldm_conv2d_set_gn_fuse_min_blocks": (None, [_i]),
    "ldm_conv2d_force_stages": (None, [_i]),
    "ldm_conv2d_set_raster_group": (None, [_i]),
    "ldm_conv2d_set_halo": (None, [_i]),
    "ldm_conv2d_set_halo_split": (None, [_i]),
    "ldm_conv2d_set_halo_rows32": (None, [_i]),
    "ldm_conv2d_set_ars": (None, [_i]),
    "ldm_conv2d_set_wide": (None, [_i]),
    "ldm_conv2d_set_ring": (None, [_i]),
    "ldm_conv2d_set_ring_split": (None, [_i]),
    "ldm_conv2d_set_splitk_cols": (None, [_i]),
    "ldm_conv2d_set_splitk_rows": (None, [_i]),
    "ldm_conv2d_set_fast_addressing": (None, [_i]),
    "ldm_conv2d_set_fewblock_ring": (None, [_i]),
    "ldm_conv2d_set_epilogue": (None, [_i]),
    "ldm_feedforward": (_i, [ctypes.POINTER(ConvParams), ctypes.POINTER(ConvParams), ctypes.POINTER(ConvParams), _vp]),
    "ldm_transformer_in": (_i, [ctypes.POINTER(GnFold), ctypes.POINTER(ConvParams), ctypes.POINTER(ConvParams), _vp]),
    "ldm_transformer_in_set_mode": (None, [_i]),
    "ldm_attention": (_i, [ctypes.POINTER(AttnParams), _vp]),
    "ldm_attention_fp8": (_i, [ctypes.POINTER(AttnParams), _vp, _i64, _vp]),
    "ldm_attention_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(AttnParams)]),
    "ldm_attention_ws": (_i, [ctypes.POINTER(AttnParams), _vp, _i64, _vp]),
    "ldm_attention_set_kvsplit": (None, [_i]),
    "ldm_attention_set_pair": (None, [_i]),
    "ldm_attention_fp8_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(AttnParams)]),
    "ldm_attention_set_fp8_scaled": (None, [_i]),
    "ldm_attention_set_maxcol": (None, [_i]),
    "ldm_group_norm_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i]),
    "ldm_group_norm": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _f, _i, _vp, _vp, _vp, _i, _i, _vp, _i, _vp]),
    "ldm_layer_norm": (_i, [_vp, _i, _i, _vp, _vp, _f, _i, _vp, _i, _vp]),
    "ldm_timestep_proj": (_i, [_vp, _i, _i, _vp, _i, _i, _vp, _i, _vp]),
    "ldm_unet_tail": (_i, [ctypes.POINTER(UnetTailParams), _vp]),
    "ldm_linear_rows": (_i, [_vp, _vp, _i, _vp, _i, _vp, _i, _i, _i, _vp, _i, _i, _vp, _i, _vp]),
    "ldm_ddim_step": (_i, [ctypes.POINTER(DdimParams), _vp]),
    "ldm_ddim_add_noise": (_i, [_vp, _vp, _vp, _vp, _i, _f, _i, _i64, _vp, _i, _vp]),
    "ldm_ddim_remove_noise": (_i, [_vp, _vp, _vp, _vp, _i, _f, _i, _i64, _vp, _i, _vp]),
    "ldm_bit_encode": (_i, [_vp, _i, _i64, _i, _i64, _f, _vp, _vp, _vp]),
    "ldm_bit_decode": (_i, [_vp, _i, _i, _i64, _i, _vp, _i, _vp]),
    "ldm_nchw_to_nhwc": (_i, [_vp, _i, _i, _vp, _i, _i, _vp, _i, _i, _i, _i, _i, _vp, _i, _vp]),
    "ldm_resize_bilinear": (_i, [_vp, _i, _i, _i, _i, _i, _f, _f, _f, _f, _vp, _i, _i, _vp]),
    "ldm_gaussian_posterior": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _vp]),
    "ldm_attention_fwd_lse": (_i, [ctypes.POINTER(AttnParams), _vp, _vp]),
    "ldm_attention_force_legacy": (None, [_i]),
    "ldm_attention_set_d80": (None, [_i]),
    "ldm_attention_set_qs2": (None, [_i]),
    "ldm_attention_set_il": (None, [_i]),
    "ldm_attention_set_skew": (None, [_i]),
    "ldm_attention_set_d160": (None, [_i]),
    "ldm_attention_set_bwd32": (None, [_i]),
    "ldm_conv2d_wgrad_set_ring": (None, [_i]),
    "ldm_conv2d_wgrad_set_fast_loader": (None, [_i]),
    "ldm_conv2d_wgrad_set_reduce3": (None, [_i]),
    "ldm_attention_set_waves": (None, [_i]),
    "ldm_attention_bwd_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(AttnParams)]),
    "ldm_attention_bwd": (_i, [ctypes.POINTER(AttnParams), _vp, _vp, _i, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp]),
    "ldm_group_norm_ex": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _f, _i, _vp, _vp, _vp, _i, _i, _vp, _vp,
                               _i, _vp]),
    "ldm_conv2d_wgrad_workspace_bytes": (ctypes.c_size_t, [ctypes.POINTER(WgradParams)]),
    "ldm_conv2d_wgrad": (_i, [ctypes.POINTER(WgradParams), _vp]),
    "ldm_colsum_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i]),
    "ldm_colsum": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp, _i, _vp]),
    "ldm_group_norm_bwd_workspace_bytes": (ctypes.c_size_t, [_i, _i, _i, _i]),
    "ldm_group_norm_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _i, _i, _vp,
                                _vp, _i, _vp, _i, _vp]),
    "ldm_layer_norm_bwd_workspace_bytes": (ctypes.c_size_t, [_i, _i]),
    "ldm_layer_norm_bwd": (_i, [_vp, _vp, _i, _i, _vp, _f, _vp, _vp, _vp, _vp, _i, _vp, _i, _vp]),
    "ldm_geglu": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _vp]),
    "ldm_sum_pool2": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _vp]),
    "ldm_mse_loss": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _f, _vp, _vp, _vp, _i, _vp]),
    "ldm_sq_norm": (_i, [_vp, _i64, _vp, _i, _vp, _vp]),
    "ldm_reduce_workspace_bytes": (ctypes.c_size_t, []),
    "ldm_repack": (_i, [_vp, _i, _i64, _vp]),
    "ldm_adamw": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i64, _f, _f, _f, _i, _vp, _f, _vp]),
    "ldm_panoptic_pixels": (_i, [_vp, _i, _i, _i, _i, _f, _i, _vp, _vp, _vp, _vp]),
    "ldm_panoptic_finalize": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _d, _i, _vp, _vp, _vp]),
    "ldm_softmax_rows": (_i, [_vp, _i, _i, _i, _f, _vp, _i, _vp]),
    "ldm_point_sample": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp]),
    "ldm_point_sample_bwd": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _f, _vp, _vp]),
    "ldm_point_labels": (_i, [_vp, _i, _i, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "ldm_point_uncertainty": (_i, [_vp, _i, _i, _i, _vp, _vp]),
    "ldm_topk_select": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "ldm_point_ce": (_i, [_vp, _vp, _i, _i, _i, _f, _i64, _vp, _vp, _vp]),
    "ldm_point_bce_dice": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp]),
    "ldm_silu": (_i, [_vp, _vp, _i64, _vp, _i, _vp]),
    "ldm_space_to_depth2": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp]),
    "ldm_posterior_sample": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp]),
    "ldm_posterior_bwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _i, _vp]),
    "ldm_status_string": (ctypes.c_char_p, [_i]),
    "ldm_abi_version": (_i, []),
}

_lib = None
_lock = threading.Lock()


def load_library(path=None):
    """Load the HIP library (no GPU needed to load it; kernels need one to run).  The env variable
    LDMSEG_HIP_LIB selects another build of it (A/B runs of an ablation or older build, whose
    tuning hooks may be missing: only those are then skipped)."""
    global _lib
    override = path is not None or bool(os.environ.get("LDMSEG_HIP_LIB"))
    path = path or os.environ.get("LDMSEG_HIP_LIB") or LIB_PATH
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise RuntimeError(f"ldmseg HIP library not found at {path}: run "
                                   f"`python video-latent-diffusion-panoptic-segmentation_amd/build.py` "
                                   f"(or __graft_entry__.build()) first")
            lib = ctypes.CDLL(path)
            for name, (res, args) in EXPORTS.items():
                if override and not hasattr(lib, name) and ("_set_" in name or "describe" in name):
                    continue
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def _check(status, what):
    if status != 0:
        msg = load_library().ldm_status_string(status).decode()
        raise RuntimeError(f"{what} failed: {msg} (status {status})")


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise TypeError(f"unsupported dtype {dt}: the HIP path computes in float32 or bfloat16")


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("ldmseg HIP ops take GPU tensors only (no CPU fallback); got a tensor on "
                               f"{t.device}")


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _contig(t, name):
    if t is not None and not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


# ======================================================================================
# launch profiler (bench.py roofline): HIP events around each launch on its stream
# ======================================================================================
class LaunchProfiler:
    """Records (family, algorithmic flops, algorithmic bytes, start/end events) per launch."""

    def __init__(self):
        self.records = []

    def start(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def stop(self, family, flops, nbytes, ev0, detail=""):
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self.records.append((family, flops, nbytes, ev0, ev1, detail))

    def summary(self, by_detail=False):
        torch.cuda.synchronize()
        fam = {}
        for f, fl, by, e0, e1, det in self.records:
            d = fam.setdefault((f, det) if by_detail else f, dict(launches=0, ms=0.0, flops=0.0, bytes=0.0))
            d["launches"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["flops"] += fl
            d["bytes"] += by
        return fam


_PROFILER = None


def set_profiler(p):
    global _PROFILER
    _PROFILER = p


def _prof_start():
    return _PROFILER.start() if _PROFILER is not None else None


def _prof_stop(ev0, family, flops, nbytes, detail=""):
    if ev0 is not None:
        _PROFILER.stop(family, flops, nbytes, ev0, detail)


# ======================================================================================
# packed weights
# ======================================================================================
def _kpad(k):
    return (k + 63) // 64 * 64


class PackedConv:
    """A conv/linear weight packed for ldm_conv2d: [n][kpad], k = (ky, kx, c) tap-major.

    ``cin_pad`` zero-pads the input channels (e.g. conv_in's 8/12 -> 16 so every 16-byte
    chunk of the NHWC input is one tap).  ``geglu`` interleaves the hidden/gate halves of a
    GEGLU projection in 16-column blocks; ``shuffle2`` packs a ConvTranspose2d(k=2, s=2).
    """

    def __init__(self, weight, bias, dtype, cin_pad=None, geglu=False, shuffle2=False, convt4=False,
                 upsample_phases=False):
        w = weight.detach()
        self.phases = bool(upsample_phases)
        if upsample_phases:
            # conv3x3(nearest_upsample_2x(x)) as four 2x2 convs over x, one per output phase (dy, dx):
            # out[2y+dy, 2x+dx] = sum_{ty,tx in 0..1} x[y-1+dy+ty, x-1+dx+tx] . Wp[dy,dx][:, :, ty, tx]
            # with the taps that read the same source pixel summed (in fp32, then rounded once):
            # rows dy = 0: ty 0 <- ky 0, ty 1 <- ky 1 + 2;  dy = 1: ty 0 <- ky 0 + 1, ty 1 <- ky 2
            cout, cin, kh, kw = w.shape
            assert kh == kw == 3, "upsample phases take a 3x3 kernel"
            wf = w.float()
            R = torch.tensor([[[1., 0., 0.], [0., 1., 1.]], [[1., 1., 0.], [0., 0., 1.]]], device=w.device)
            wph = torch.einsum("ayk,bxl,oikl->abyxoi", R, R, wf)      # [dy, dx, ty, tx, cout, cin]
            wp = wph.permute(0, 1, 4, 2, 3, 5).reshape(4 * cout, 4 * cin)  # rows (dy, dx, co), k (ty, tx, ci)
            b = None if bias is None else bias.detach().float()
            self.ksize, self.cin, self.n = 2, cin, cout
            self.cin_real = cin
            # the gather form for images the phase kernel cannot tile (a tile's rows must lie in one
            # phase: h * w % 32 == 0); packed now, so a captured graph never packs
            self.gather = PackedConv(weight, bias, dtype)
        elif convt4:
            # ConvTranspose2d(k=4, s=2, p=1) weight [cin, cout, 4, 4] as a 3x3 conv (pad 1) with
            # 4 * cout outputs, one per output phase (dy, dx), + the pixel-shuffle epilogue:
            # out[2y+dy, 2x+dx] = sum over taps (ty, tx) of in[y-1+ty, x-1+tx] . W[:, :, ky, kx]
            # with ky = 3 + dy - 2 ty (valid 0..3), kx likewise
            cin, cout = w.shape[0], w.shape[1]
            cp = cin_pad or cin
            w3 = torch.zeros(2, 2, cout, 3, 3, cp, dtype=w.dtype, device=w.device)
            for dy in range(2):
                for dx in range(2):
                    for ty in range(3):
                        for tx in range(3):
                            ky, kx = 3 + dy - 2 * ty, 3 + dx - 2 * tx
                            if 0 <= ky <= 3 and 0 <= kx <= 3:
                                w3[dy, dx, :, ty, tx, :cin] = w[:, :, ky, kx].t()
            wp = w3.reshape(4 * cout, 9 * cp)
            b = None if bias is None else bias.detach().float().repeat(4)
            self.ksize, self.cin, self.n = 3, cp, 4 * cout
            self.cin_real = cin
        elif shuffle2:                     # ConvTranspose2d weight [cin, cout, 2, 2]
            cin, cout = w.shape[0], w.shape[1]
            wp = w.permute(2, 3, 1, 0).reshape(4 * cout, cin)          # n = (dy*2+dx)*cout + co
            b = None if bias is None else bias.detach().float().repeat(4)
            self.ksize, self.cin, self.n = 1, cin, 4 * cout
            self.cin_real = cin
        else:
            if w.ndim == 2:
                w = w[:, :, None, None]
            cout, cin, kh, kw = w.shape
            assert kh == kw and kh in (1, 3, 5, 7), "1x1 / 3x3 / 5x5 / 7x7 kernels"
            cp = cin_pad or cin
            self.cin_real = cin
            if cp != cin:
                w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, cp - cin))
            wp = w.permute(0, 2, 3, 1).reshape(cout, kh * kw * cp)
            b = None if bias is None else bias.detach().float()
            if geglu:
                half = cout // 2
                assert half % 16 == 0, "GEGLU packing needs 16-aligned halves"
                wh, wg = wp[:half].reshape(half // 16, 16, -1), wp[half:].reshape(half // 16, 16, -1)
                wp = torch.stack([wh, wg], dim=1).reshape(cout, -1)
                if b is not None:
                    bh, bg = b[:half].reshape(-1, 16), b[half:].reshape(-1, 16)
                    b = torch.stack([bh, bg], dim=1).reshape(-1)
            self.ksize, self.cin, self.n = kh, cp, cout
        K = wp.shape[1]
        self.kpad = _kpad(K)
        packed = torch.zeros(wp.shape[0], self.kpad, dtype=dtype, device=wp.device)
        packed[:, :K] = wp.to(dtype)
        self.w = packed.contiguous()
        self.bias = None if b is None else b.contiguous()
        self.dtype = dtype
        self.geglu = geglu
        self.shuffle2 = shuffle2 or convt4


def packed_ln_fold(weight, bias, gamma, beta, dtype, geglu=False):
    """Linear(LayerNorm(x)) as one GEMM on the raw rows x (ldm_conv_params ln_rows): the packed
    weight is W' = W diag(gamma), the bias W beta + b, and ``ln_c1`` the column sums of the
    packed (rounded) W', so that rstd (x W'^T - mean c1) cancels the mean exactly as packed."""
    w = weight.detach().float()
    wf = w * gamma.detach().float()[None, :]
    b = w @ beta.detach().float()
    if bias is not None:
        b = b + bias.detach().float()
    pc = PackedConv(wf, b, dtype, geglu=geglu)
    pc.ln_c1 = pc.w.float().sum(1).contiguous()
    return pc


def packed_rows(t, bias=None):
    """Wrap a contiguous [n][k] activation tensor (k % 64 == 0) as the B operand of a 1x1
    ldm_conv2d without copying: out[m, j] = sum_k A[m, k] * t[j, k] (+ bias[j])."""
    if t.ndim != 2 or not t.is_contiguous() or t.shape[1] % 64:
        raise ValueError("packed_rows: need a contiguous [n, k] tensor with k % 64 == 0")
    pc = PackedConv.__new__(PackedConv)
    pc.ksize, pc.cin, pc.cin_real, pc.n, pc.kpad = 1, t.shape[1], t.shape[1], t.shape[0], t.shape[1]
    pc.w, pc.dtype, pc.geglu, pc.shuffle2 = t, t.dtype, False, False
    pc.bias = None if bias is None else bias.detach().float().contiguous()
    return pc


GN_PART_ATTR = "_ldm_gn_part"
GN_DONE_ATTR = "_ldm_gn_done"     # (key, normalised tensor) a split-K conv's reduction already produced


def gn_key(groups, gamma, beta, eps, act):
    """Identity of one GroupNorm application (ldm_conv2d gn_out <-> group_norm)."""
    return (int(groups), gamma.data_ptr(), beta.data_ptr(), float(eps), int(act))


def gn_stats_of(t):
    """The fp64 [batch, slots, c / unit, 2] (sum, sumsq) accumulators a conv epilogue attached to
    ``t`` (or None); unit = channels per accumulator, slots = copies the row tiles spread over."""
    return getattr(t, GN_PART_ATTR, None) if t is not None else None


GN_UNIT_MAX = 10          # tuning hook (A/B only): 1 = one accumulator per channel


def gn_unit_for(n):
    """Channels per GroupNorm accumulator of an n-channel conv output: 10 for the SD UNet widths
    (it divides every group size, 10..80, and every concat offset), else gcd(n, 10)."""
    return math.gcd(n, GN_UNIT_MAX)


def gn_slots_for(hw):
    """Accumulator copies for an output of hw pixels per image: same-address fp64 atomics
    serialise, so the ~hw/128 row tiles of one image are spread over up to 8 copies."""
    return max(1, min(8, hw // 256))


_gn_arena_tls = threading.local()
_gn_arena_sizes = {}


@contextlib.contextmanager
def gn_arena(key, device):
    """Scope (one forward) in which conv2d(gn_stats=True) takes its zeroed GroupNorm accumulators
    as slices of ONE zero-filled fp64 buffer — one memset per forward instead of one per conv.
    The buffer is sized from the previous forward with the same ``key`` (the first one falls back
    to a torch.zeros per conv and records how much it needed)."""
    need = _gn_arena_sizes.get(key, 0)
    st = {"buf": torch.zeros(need, dtype=torch.float64, device=device) if need else None, "off": 0, "used": 0}
    stack = getattr(_gn_arena_tls, "stack", None)
    if stack is None:
        stack = _gn_arena_tls.stack = []
    stack.append(st)
    try:
        yield
    finally:
        stack.pop()
        _gn_arena_sizes[key] = max(need, st["used"])


def zeroed_f64(count, device):
    """A zeroed fp64 tensor of ``count`` (even) elements, from the enclosing gn_arena if any
    (LayerNorm row statistics share the GroupNorm accumulators' one memset)."""
    return _gn_accumulators(1, 1, (count + 1) // 2, device).view(-1)[:count]


def _gn_accumulators(batch, slots, n, device):
    """Zeroed fp64 [batch, slots, n, 2] accumulators (n = units), from the enclosing gn_arena if any."""
    cnt = batch * slots * n * 2                   # even -> every slice stays 16-B aligned
    stack = getattr(_gn_arena_tls, "stack", None)
    if stack:
        st = stack[-1]
        st["used"] += cnt
        buf = st["buf"]
        if buf is not None and buf.device == device and st["off"] + cnt <= buf.numel():
            v = buf[st["off"]:st["off"] + cnt].view(batch, slots, n, 2)
            st["off"] += cnt
            return v
    return torch.zeros(batch, slots, n, 2, dtype=torch.float64, device=device)


GN_FUSE = True            # A/B hook (set_gn_fuse): GroupNorm in the split-K reduction's launch


def set_gn_fuse(enabled=True):
    """A/B hook: let conv2d(gn_next=...) run the consumer GroupNorm inside the split-K reduction
    (default on); off runs the reduction and ldm_group_norm as two launches."""
    global GN_FUSE
    GN_FUSE = bool(enabled)


def set_gn_fuse_min_blocks(n=16):
    """Tuning hook: the fewest reduction blocks (images x 40-channel segments) the fused split-K
    GroupNorm takes (ldm_conv2d_set_gn_fuse_min_blocks; smaller grids keep the two launches)."""
    load_library().ldm_conv2d_set_gn_fuse_min_blocks(int(n))


def conv2d(pc: PackedConv, x0, batch, h, w, *, x1=None, stride=1, upsample=False, temb=None, temb_stride=0,
           residual=None, out=None, out_layout=OUT_NHWC, act=ACT_NONE, out_dtype=None, gn_stats=False, pad_mode=0,
           row_stats=None, ln=None, gn_next=None):
    """Run ldm_conv2d.  x0/x1: NHWC [batch, h, w, c] (any contiguous view with that numel).

    gn_stats=True also has the epilogue sum the per-(batch, channel) (sum, sumsq) of the output
    into fp64 accumulators (from the enclosing gn_arena when there is one); they are attached to
    the returned tensor and consumed by group_norm().

    gn_next = (groups, gamma, beta, eps, act, keep_out): the GroupNorm that will consume the output.
    When the plan splits K and the shape is in scope (ldm_conv2d_gn_fusable: the deep levels), the
    reduction applies it in the same launch and the normalised tensor is attached to the output, so
    the following group_norm() with the same arguments returns it without a launch.  keep_out=False:
    the pre-norm output is dead — it is not written and the normalised tensor is returned instead.

    row_stats: a zeroed fp64 [M, 2] tensor the epilogue adds each output row's (sum, sumsq) to.
    ln = (rows, eps): x0's rows are LayerNorm'd inside the GEMM (pc from packed_ln_fold, rows =
    the producer's row_stats)."""
    if getattr(pc, "phases", False) and not upsample:
        raise ValueError("an upsample_phases pack is the nearest-2x upsample conv: pass upsample=True")
    lib = load_library()
    _gpu(x0, x1, pc.w, temb, residual, out)
    c0 = x0.numel() // (batch * h * w)
    c1 = 0 if x1 is None else x1.numel() // (batch * h * w)
    if c0 * batch * h * w != x0.numel() or (x1 is not None and c1 * batch * h * w != x1.numel()):
        raise ValueError("input numel does not match batch*h*w*c")
    if c0 + c1 != pc.cin:
        raise ValueError(f"conv expects {pc.cin} input channels, got {c0}+{c1}")
    for t, nm in ((x0, "x0"), (x1, "x1"), (residual, "residual")):
        _contig(t, nm)
    if x0.dtype != pc.dtype or (x1 is not None and x1.dtype != pc.dtype):
        raise TypeError(f"conv input dtype {x0.dtype} != packed weight dtype {pc.dtype}")
    if getattr(pc, "phases", False):
        if (h * w) % 32 or x1 is not None or stride != 1 or pad_mode or out_layout != OUT_NHWC or \
                row_stats is not None or ln is not None:
            pc = pc.gather                 # shapes the phase form does not take: the 3x3 gather form
    k = pc.ksize
    if k == 1:
        ho, wo = h, w
    elif upsample:
        ho, wo = 2 * h, 2 * w
    elif pad_mode == 1:                    # diffusers Downsample2D(padding=0): F.pad (0, 1, 0, 1)
        ho, wo = (h + 1 - 3) // stride + 1, (w + 1 - 3) // stride + 1
    else:                                  # padding (k - 1) // 2
        ho, wo = (h + k - 1 - k) // stride + 1, (w + k - 1 - k) // stride + 1
    n = pc.n
    if out_layout == OUT_GEGLU:
        shape = (batch, ho, wo, n // 2)
    elif out_layout == OUT_NCHW:
        shape = (batch, n, ho, wo)
    elif out_layout == OUT_SHUFFLE2:
        shape = (batch, 2 * ho, 2 * wo, n // 4)
    else:
        shape = (batch, ho, wo, n)
    odt = out_dtype or pc.dtype
    if out is None:
        out = torch.empty(shape, dtype=odt, device=x0.device)
    elif out.numel() != math.prod(shape) or out.dtype != odt:
        raise ValueError("preallocated out has the wrong size / dtype")
    if residual is not None and (residual.numel() != out.numel() or residual.dtype != pc.dtype):
        raise ValueError("residual must match the output size and the compute dtype")
    if temb is not None:
        # temb may be a column slice [B, n:] of the batched time_emb_proj output: element
        # (b, j) lives at temb.data_ptr() + (b * temb_stride + j) * 4
        if temb.dtype != torch.float32 or temb.ndim != 2 or temb.stride(-1) != 1 or temb.shape[0] != batch:
            raise ValueError("temb must be an fp32 [batch, >=n] row-major view")
        if temb.shape[1] < n or temb.stride(0) != temb_stride:
            raise ValueError("temb view narrower than n or stride mismatch")
    M = batch * ho * wo
    part, unit, slots = None, 0, 0
    if gn_stats and out_layout == OUT_NHWC and M % 64 == 0 and (ho * wo) % 64 == 0:
        unit, slots = gn_unit_for(n), gn_slots_for(ho * wo)
        part = _gn_accumulators(batch, slots, n // unit, x0.device)
    ln_rows, ln_c1, ln_inv_k, ln_eps = None, None, 0.0, 0.0
    if row_stats is not None and (row_stats.dtype != torch.float64 or row_stats.numel() != 2 * M
                                  or not row_stats.is_contiguous()):
        raise ValueError("row_stats must be a contiguous fp64 [M, 2] tensor")
    if ln is not None:
        ln_rows, eps = ln
        if getattr(pc, "ln_c1", None) is None:
            raise ValueError("ln needs a packed_ln_fold weight")
        if ln_rows.dtype != torch.float64 or ln_rows.numel() != 2 * M or not ln_rows.is_contiguous():
            raise ValueError("ln rows must be a contiguous fp64 [M, 2] tensor")
        ln_c1, ln_inv_k, ln_eps = pc.ln_c1, 1.0 / (c0 + c1), float(eps)
    up_mode = 3 if getattr(pc, "phases", False) else int(upsample)
    p = ConvParams(_ptr(x0), _ptr(x1), c0, c1, batch, h, w, ho, wo, pc.ksize, stride, up_mode, _ptr(pc.w),
                   n, pc.kpad, _ptr(pc.bias), _ptr(temb), temb_stride, _ptr(residual), _ptr(out), out_layout, act,
                   dtype_code(pc.dtype), int(odt == torch.float32 and pc.dtype != torch.float32), None, 0,
                   _ptr(part), int(pad_mode), unit, slots, _ptr(row_stats), _ptr(ln_rows), _ptr(ln_c1),
                   float(ln_inv_k), float(ln_eps))
    ws_bytes = int(lib.ldm_conv2d_workspace_bytes(ctypes.byref(p)))
    if ws_bytes:
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x0.device)
        p.workspace, p.workspace_bytes = _ptr(ws), ws_bytes
    gn_done = None
    if gn_next is not None and ws_bytes and GN_FUSE and odt == torch.bfloat16 and out_layout == OUT_NHWC:
        groups, gamma, beta, eps, gact, keep = gn_next
        _gpu(gamma, beta)
        if gamma.dtype != torch.float32 or beta.dtype != torch.float32 or gamma.numel() != n or beta.numel() != n:
            raise ValueError("gn_next gamma / beta must be fp32 [n]")
        p.gn_out, p.gn_gamma, p.gn_beta = p.out, _ptr(gamma), _ptr(beta)
        p.gn_groups, p.gn_act, p.gn_eps = int(groups), int(gact), float(eps)
        if not p.gn_unit:
            p.gn_unit = gn_unit_for(n)
        if lib.ldm_conv2d_gn_fusable(ctypes.byref(p)):
            if keep:
                gout = torch.empty_like(out)
                p.gn_out = _ptr(gout)
            else:                          # the pre-norm tensor is dead: normalise into out itself
                gout, part = out, None
                p.gn_skip_out, p.gn_partial = 1, None
            gn_done = (gn_key(groups, gamma, beta, eps, gact), gout)
        else:
            p.gn_out = p.gn_gamma = p.gn_beta = None
            p.gn_groups = p.gn_act = 0
    ev = _prof_start()
    _check(lib.ldm_conv2d(ctypes.byref(p), _stream(x0)), "ldm_conv2d")
    setattr(out, GN_PART_ATTR, part)     # never leave a stale slab on a rewritten tensor
    setattr(out, GN_DONE_ATTR, gn_done)
    if ev is not None:
        flops = 2.0 * M * n * pc.ksize * pc.ksize * pc.cin_real
        nbytes = (x0.numel() + (0 if x1 is None else x1.numel()) + pc.w.numel()) * x0.element_size() + \
            out.numel() * out.element_size() + (0 if residual is None else residual.numel() * residual.element_size())
        det = f"k{pc.ksize}{'s2' if stride == 2 else ''}{'up' if upsample else ''} M={M} N={n} " \
              f"Cin={c0}+{c1} L{out_layout}"
        _prof_stop(ev, "igemm", flops, nbytes, det)
    return out


PLAN_KINDS = {0: "tile", 1: "halo", 2: "wide", 3: "ars", 4: "big", 5: "ring"}


def describe_plan(batch, h, w, c0, n, *, c1=0, ksize=3, stride=1, upsample=False, out_layout=OUT_NHWC,
                  dtype=torch.bfloat16, residual=False, temb=False, gn_stats=False, row_stats=False, ln=False,
                  act=ACT_NONE, geglu_bias=True):
    """The kernel / tile plan ldm_conv2d picks for a call of this shape (host only: the library's
    planner on a parameter block with placeholder 16-byte-aligned addresses; nothing launches).
    Returns {"kind", "bm", "bn", "ksplit", "stages", "blocks"}."""
    lib = load_library()
    fake = ctypes.c_void_p(1 << 20)
    ce = 16 // (4 if dtype == torch.float32 else 2)
    c0p = (c0 + ce - 1) // ce * ce
    k = ksize
    if k == 1:
        ho, wo = h, w
    elif upsample:
        ho, wo = 2 * h, 2 * w
    else:
        ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1
    M = batch * ho * wo
    p = ConvParams(fake, fake if c1 else None, c0p, c1, batch, h, w, ho, wo, k, stride, int(upsample), fake, n,
                   _kpad(k * k * (c0p + c1)), fake if geglu_bias else None, fake if temb else None, n if temb else 0,
                   fake if residual else None, fake, out_layout, act, dtype_code(dtype), 0, None, 0,
                   fake if gn_stats else None, 0, gn_unit_for(n) if gn_stats else 0,
                   gn_slots_for(ho * wo) if gn_stats else 0, fake if row_stats else None, fake if ln else None,
                   fake if ln else None, 1.0 / (c0p + c1) if ln else 0.0, 1e-5 if ln else 0.0)
    out = (ctypes.c_int * 5)()
    _check(lib.ldm_conv2d_describe_plan(ctypes.byref(p), out), "ldm_conv2d_describe_plan")
    kind, bm, bn, ks, st = list(out)
    if kind == 0 or kind == 4:
        blocks = -(-M // bm) * -(-n // bn) * ks
    elif kind == 1:
        blocks = M // bm * (n // bn) * ks
    else:
        blocks = -(-M // bm) * (n // bn) if bn else None
    return {"kind": PLAN_KINDS[kind], "bm": bm, "bn": bn, "ksplit": ks, "stages": st, "blocks": blocks}


def softmax_rows(s, n, scale, dtype):
    """s fp32 [rows, stride] (GPU) -> softmax over the first n columns of scale * s, zeros in
    columns [n, stride); output dtype fp32 or bf16."""
    lib = load_library()
    _gpu(s)
    if s.dtype != torch.float32 or s.ndim != 2 or not s.is_contiguous():
        raise TypeError("softmax_rows: s must be a contiguous fp32 [rows, stride] tensor")
    rows, stride = s.shape
    p = torch.empty(rows, stride, dtype=dtype, device=s.device)
    _check(lib.ldm_softmax_rows(_ptr(s), rows, int(n), stride, float(scale), _ptr(p), dtype_code(dtype), _stream(s)),
           "ldm_softmax_rows")
    return p


def set_attention_waves(waves=0):
    """Tuning hook: 4 or 8 waves per flash-attention block (8: every K/V tile serves twice the
    queries); 0 = automatic (8 when that still gives >= 256 blocks)."""
    load_library().ldm_attention_set_waves(int(waves))


def set_attention_maxcol(mode=2):
    """Tuning hook (head_dim 40): 2 the 32x32x16 kernel (default), 1 the 16x16x32 kernel with the
    scale and running max in the Q.K^T padding, 0 the 16x16x32 kernel with an FMA per score."""
    load_library().ldm_attention_set_maxcol(int(mode))


FP8_SCALED_HEAD_DIMS = (40,)     # ldm_attention_fp8's block-scaled MFMA kernel (others: non-scaled P.V)


def set_attention_fp8_scaled(enabled=True):
    """Tuning / A-B hook: head_dim 40 fp8 attention on the block-scaled MFMA kernel (default) or on the
    non-scaled P.V path."""
    load_library().ldm_attention_set_fp8_scaled(int(bool(enabled)))


def set_wgrad_ring(ring=True):
    """Tuning / A-B hook: bf16 weight gradient on four 32-pixel LDS stages (default) or two 64-pixel."""
    load_library().ldm_conv2d_wgrad_set_ring(int(ring))


def set_wgrad_reduce3(enabled=True):
    """A-B hook: the 3x3 weight gradient's slab sum by wave-owned channel x tap blocks (default) or
    one packed element per thread."""
    load_library().ldm_conv2d_wgrad_set_reduce3(int(bool(enabled)))


def set_wgrad_fast_loader(enabled=True):
    """A-B hook: the weight gradient's pointer-walk operand loader for stride-1 convs (default) or
    the general pixel-decoding loader everywhere."""
    load_library().ldm_conv2d_wgrad_set_fast_loader(int(bool(enabled)))


def set_attention_bwd32(enabled=True):
    """Tuning / A-B hook: the bf16 attention backward (head_dim <= 64) on the 32x32x16 MFMA kernels
    (default) or the 16x16x16 ones."""
    load_library().ldm_attention_set_bwd32(int(bool(enabled)))


def set_attention_d80(enabled=True):
    """Tuning / A-B hook: head_dim 80 on the 32x32x16 kernel (default) or the 16x16x32 one."""
    load_library().ldm_attention_set_d80(int(bool(enabled)))


def set_attention_qs2(mode=1):
    """Tuning / A-B hook for head_dim 40: 0 the default kernel (32 queries per wave, two 8-wave
    blocks per CU); 1 two 32-query subtiles per wave sharing each K / V fragment read (one block per
    CU); 2 the tile loop software-pipelined inside each wave (attn_d40p_kernel)."""
    load_library().ldm_attention_set_qs2(int(mode))


def set_attention_il(enabled=True):
    """A/B hook for head_dim 40 with >= 256 blocks of 64 queries: the two-subtile kernel whose MFMA and
    softmax phases interleave inside each wave (default on) or the 32-query kernel; bit-identical.
    The interleaved kernel runs 128-key tiles; ``enabled=2`` / ``3``: on 64- / 256-key tiles (A/B)."""
    load_library().ldm_attention_set_il(int(enabled) if enabled in (2, 3) else int(bool(enabled)))


def set_attention_skew(mode=0):
    """Tuning / A-B hook for head_dim 40 / 80 on the 32x32x16 kernel: 0 planner, 1 off, 2 the block's
    waves in two phases half an iteration apart (bit-identical)."""
    load_library().ldm_attention_set_skew(int(mode))


def set_attention_d160(enabled=False):
    """Tuning / A-B hook: head_dim 160 on the 32x32x16 kernel, or (default) the 16x16x32 one."""
    load_library().ldm_attention_set_d160(1 if enabled else 0)


def set_attention_pair(enabled=True):
    """Tuning / A-B hook: the head_dim 80 kernel's key-tile loop unrolled by two (default; bit-identical).
    ``enabled=2`` / ``3``: 128-key tiles without / with the unrolled loop (A/B)."""
    load_library().ldm_attention_set_pair(int(enabled) if enabled in (2, 3) else (1 if enabled else 0))


def set_attention_kvsplit(splits=-1):
    """Tuning / A-B hook for head_dim 40 bf16 split-KV (ldm_attention_ws): -1 planner, 0 / 1 off,
    k >= 2 forced."""
    load_library().ldm_attention_set_kvsplit(int(splits))


def force_attention_legacy(legacy=True):
    """Tuning hook: route bf16 attention through the 16x16x16-MFMA kernel (A/B only)."""
    load_library().ldm_attention_force_legacy(int(bool(legacy)))


def force_conv_stages(stages=0):
    """Tuning hook: LDS ring depth of the 128x160 tile (3 / 4), 0 = planner."""
    load_library().ldm_conv2d_force_stages(int(stages))


def set_conv_raster_group(group_m=8):
    """Tuning hook: M panels per tile-raster group (1 = row-major tile order)."""
    load_library().ldm_conv2d_set_raster_group(int(group_m))


def set_conv_halo(mode=0):
    """Tuning hook: halo-tiled 3x3 kernel — 0 planner, 1 never, 2 whenever legal."""
    load_library().ldm_conv2d_set_halo(int(mode))


def set_conv_halo_split(ks=0):
    """Tuning hook: split-K factor of the 16x16 whole-image halo tiles (0 = planner)."""
    load_library().ldm_conv2d_set_halo_split(int(ks))


def set_conv_halo_rows32(rows=0):
    """Tuning / A-B hook: output rows per halo tile at the 32x32 level: 0 the planner (8 for >= 1280
    input channels, else 4), 4 or 8 forced (8: 256-row tiles, K split over channel blocks as at the
    16x16 level)."""
    load_library().ldm_conv2d_set_halo_rows32(int(rows))


def set_conv_ars(mode=0):
    """Tuning hook: A-register-stationary short-K 1x1 GEMM — 0 planner, 1 never, 2 whenever legal."""
    load_library().ldm_conv2d_set_ars(int(mode))


def set_conv_wide(mode=0):
    """Tuning hook: wide-tile persistent 1x1 GEMM — 0 planner, 1 never, 2 whenever legal (256-row
    tiles), 3 whenever legal (128-row tiles)."""
    load_library().ldm_conv2d_set_wide(int(mode))


def set_conv_ring(mode=0):
    """Tuning hook: deep-ring 1x1 GEMM of the 16x16 / 8x8 levels — 0 planner, 1 never, 2 whenever
    legal."""
    load_library().ldm_conv2d_set_ring(int(mode))


def set_conv_ring_split(ks=0):
    """Tuning hook: K splits of the deep-ring kernel (its 3x3 conv form; > 0 forces every ring call)."""
    load_library().ldm_conv2d_set_ring_split(int(ks))


def set_conv_splitk_cols(cols=0):
    """Tuning hook: split-K reduction tile width — 0 planner, 64 or 128 forced."""
    load_library().ldm_conv2d_set_splitk_cols(int(cols))


def set_conv_fast_addressing(mode=4):
    """A/B hook: the tile kernel's fast operand addressing — 4 planner (default), 1 / True everywhere it
    applies, 2 convs only, 3 1x1 only, 0 / False off (bit-identical in every mode)."""
    load_library().ldm_conv2d_set_fast_addressing(int(mode))


def set_conv_fewblock_ring(enabled=True):
    """A/B hook: 4-stage LDS ring for <= 256-block 64-row tile plans (default on)."""
    load_library().ldm_conv2d_set_fewblock_ring(int(bool(enabled)))


def set_conv_splitk_rows(rows=0):
    """Tuning hook: split-K reduction tile rows — 0 planner, 16, 32 or 64 forced."""
    load_library().ldm_conv2d_set_splitk_rows(int(rows))


def set_conv_epilogue(mode=0):
    """Tuning hook: 0 bf16 pre-activated staging epilogue (default), 1 fp32 staging."""
    load_library().ldm_conv2d_set_epilogue(int(mode))


def force_conv_plan(bm=0, bn=0, ksplit=1):
    """Tuning hook: force ldm_conv2d's tile plan (bm=256 -> large-tile bf16 kernel); bm=0 resets."""
    load_library().ldm_conv2d_force_plan(int(bm), int(bn), int(ksplit))


def linear(pc: PackedConv, x, **kw):
    """x [..., K] rows -> [..., N] (a 1x1 conv over rows)."""
    rows = x.numel() // x.shape[-1]
    y = conv2d(pc, x, rows, 1, 1, **kw)
    if kw.get("out_layout", OUT_NHWC) == OUT_GEGLU:
        v = y.view(*x.shape[:-1], pc.n // 2)
    else:
        v = y.view(*x.shape[:-1], y.shape[-1])
    setattr(v, GN_PART_ATTR, gn_stats_of(y))
    return v


FF_WIDTH = 320             # ldm_feedforward's model width (the 64x64 UNet level)
FF_MIN_TILES = 256         # 128-row tiles below which the fused kernel leaves CUs idle (one per CU)


def feedforward_ok(pc1: PackedConv, pc2: PackedConv, x):
    """Whether ldm_feedforward takes this FeedForward: bf16, width 320, hidden F % 64 == 0 and
    <= 1280, and enough rows for one 128-row tile per CU (fewer run the two-launch form)."""
    rows = x.numel() // x.shape[-1]
    F = pc2.kpad
    return (x.dtype == torch.bfloat16 and pc1.dtype == torch.bfloat16 and pc2.dtype == torch.bfloat16
            and x.shape[-1] == FF_WIDTH and pc1.geglu and pc1.ksize == 1 and pc2.ksize == 1 and pc1.kpad == FF_WIDTH
            and pc2.n == FF_WIDTH and pc1.n == 2 * F and pc2.cin == F and F % 64 == 0 and F <= 1280
            and -(-rows // 128) >= FF_MIN_TILES)


def feedforward(pc1: PackedConv, pc2: PackedConv, x, *, ln=None, residual=None, out=None, row_stats=None,
                proj_out=None):
    """FeedForward(GEGLU) in one launch (ldm_feedforward): out = Linear2(h * gelu(g)) (+ residual)
    with [h | g] = Linear1(x) (LayerNorm-folded when ln = (rows, eps) and pc1 is a packed_ln_fold
    weight).  Equal bit for bit to linear(pc2, linear(pc1, x, out_layout=OUT_GEGLU, ln=ln),
    residual=residual, out=out, row_stats=row_stats); x [..., 320].

    proj_out = (pc_po, x_in, batch, h, w, gn_stats): Transformer2DModel.proj_out applied behind it
    in the same launch (h never stored): returns conv2d(pc_po, ff_out, batch, h, w, residual=x_in,
    gn_stats=gn_stats) instead, as NHWC [batch, h, w, 320] with the GroupNorm accumulators attached."""
    lib = load_library()
    _gpu(x, pc1.w, pc2.w, residual, out, row_stats)
    _contig(x, "x")
    _contig(residual, "residual")
    rows = x.numel() // x.shape[-1]
    C, F = x.shape[-1], pc2.kpad
    if not (pc1.geglu and pc1.n == 2 * F and pc1.kpad == C and pc2.n == C and pc2.cin == F):
        raise ValueError("feedforward: pc1 must be the GEGLU pack [2F][C] and pc2 the [C][F] pack")
    if x.dtype != pc1.dtype:
        raise TypeError("feedforward: x dtype != packed weight dtype")
    po_params, po_out, part = None, None, None
    if proj_out is not None:
        pc3, x_in, pb, ph, pw, gn_stats = proj_out
        _gpu(pc3.w, x_in)
        if pc3.ksize != 1 or pc3.n != C or pc3.kpad != C or pc3.dtype != x.dtype or pb * ph * pw != rows:
            raise ValueError("feedforward: proj_out must be a 1x1 [320][320] pack over the same rows")
        if out is not None or row_stats is not None:
            raise ValueError("feedforward: with proj_out the feed-forward's output is not stored")
        if x_in is not None and (x_in.numel() != rows * C or x_in.dtype != x.dtype or not x_in.is_contiguous()):
            raise ValueError("feedforward: proj_out residual must match the output")
        po_out = torch.empty(pb, ph, pw, C, dtype=x.dtype, device=x.device)
        unit, slots = 0, 0
        if gn_stats and rows % 64 == 0 and (ph * pw) % 64 == 0:
            unit, slots = gn_unit_for(C), gn_slots_for(ph * pw)
            part = _gn_accumulators(pb, slots, C // unit, x.device)
        po_params = ConvParams(None, None, C, 0, pb, ph, pw, ph, pw, 1, 1, 0, _ptr(pc3.w), C, C, _ptr(pc3.bias),
                               None, 0, _ptr(x_in), _ptr(po_out), OUT_NHWC, ACT_NONE, dtype_code(x.dtype), 0, None,
                               0, _ptr(part), 0, unit, slots, None, None, None, 0.0, 0.0)
    elif out is None:
        out = torch.empty(x.shape[:-1] + (C,), dtype=x.dtype, device=x.device)
    elif out.numel() != rows * C or out.dtype != x.dtype or not out.is_contiguous():
        raise ValueError("feedforward: preallocated out has the wrong size / dtype / layout")
    if residual is not None and (residual.numel() != rows * C or residual.dtype != x.dtype):
        raise ValueError("feedforward: residual must match the output")
    if row_stats is not None and (row_stats.dtype != torch.float64 or row_stats.numel() != 2 * rows
                                  or not row_stats.is_contiguous()):
        raise ValueError("row_stats must be a contiguous fp64 [M, 2] tensor")
    ln_rows, ln_c1, inv_k, eps = None, None, 0.0, 0.0
    if ln is not None:
        ln_rows, eps = ln
        if getattr(pc1, "ln_c1", None) is None:
            raise ValueError("ln needs a packed_ln_fold weight")
        if ln_rows.dtype != torch.float64 or ln_rows.numel() != 2 * rows or not ln_rows.is_contiguous():
            raise ValueError("ln rows must be a contiguous fp64 [M, 2] tensor")
        ln_c1, inv_k = pc1.ln_c1, 1.0 / C
    dt = dtype_code(x.dtype)
    g = ConvParams(_ptr(x), None, C, 0, rows, 1, 1, 1, 1, 1, 1, 0, _ptr(pc1.w), pc1.n, pc1.kpad, _ptr(pc1.bias),
                   None, 0, None, None, OUT_GEGLU, ACT_NONE, dt, 0, None, 0, None, 0, 0, 0, None, _ptr(ln_rows),
                   _ptr(ln_c1), float(inv_k), float(eps))
    f = ConvParams(None, None, F, 0, rows, 1, 1, 1, 1, 1, 1, 0, _ptr(pc2.w), C, F, _ptr(pc2.bias), None, 0,
                   _ptr(residual), _ptr(out), OUT_NHWC, ACT_NONE, dt, 0, None, 0, None, 0, 0, 0, _ptr(row_stats),
                   None, None, 0.0, 0.0)
    ev = _prof_start()
    _check(lib.ldm_feedforward(ctypes.byref(g), ctypes.byref(f), None if po_params is None else ctypes.byref(po_params),
                               _stream(x)), "ldm_feedforward")
    if po_out is not None:
        out = po_out
    setattr(out, GN_PART_ATTR, part)
    if ev is not None:
        flops = 2.0 * rows * (2 * F * C + C * F + (C * C if po_out is not None else 0))
        nbytes = (x.numel() + out.numel() + (0 if residual is None else residual.numel())) * x.element_size() + \
            (pc1.w.numel() + pc2.w.numel()) * pc1.w.element_size()
        _prof_stop(ev, "igemm", flops, nbytes, f"ff M={rows} C={C} F={F}")
    return out


TIN_WIDTH = 320            # ldm_transformer_in's model width (the 64x64 UNet level)


def transformer_in_ok(pc_in: PackedConv, pc_qkv: PackedConv, x, batch, hw, groups):
    """Whether ldm_transformer_in takes this Transformer2DModel input: bf16, width 320, a
    LayerNorm-folded QKV pack, whole 128-row tiles per image, producer GroupNorm statistics on x
    in a layout the kernel stages, and one 128-row tile per CU (fewer run the three-launch form)."""
    C = x.shape[-1]
    if not (x.dtype == torch.bfloat16 and pc_in.dtype == torch.bfloat16 and pc_qkv.dtype == torch.bfloat16
            and C == TIN_WIDTH and pc_in.ksize == 1 and pc_qkv.ksize == 1 and pc_in.n == C and pc_in.kpad == C
            and pc_qkv.n == 3 * C and pc_qkv.kpad == C and getattr(pc_qkv, "ln_c1", None) is not None
            and hw % 128 == 0 and batch * hw // 128 >= FF_MIN_TILES and 0 < groups <= 64 and C % groups == 0):
        return False
    s0, _, unit, slots = _gn_sources(x, None, batch, C, 0, groups)
    return s0 is not None and slots * (C // unit) <= 256


def set_transformer_in_mode(mode):
    """Tuning / A-B hook: ldm_transformer_in kernel variant (1 = default)."""
    load_library().ldm_transformer_in_set_mode(int(mode))


def transformer_in(pc_in: PackedConv, pc_qkv: PackedConv, x, batch, hw, groups, gamma, beta, gn_eps, ln_eps):
    """Transformer2DModel's input half in one launch (ldm_transformer_in): returns (h, qkv) with
    h = linear(pc_in, group_norm(x, ...)) and qkv = linear(pc_qkv, h, ln=(row_stats(h), ln_eps)) —
    equal bit for bit to the three separate calls; x [batch, hw, 320] with producer statistics."""
    lib = load_library()
    _gpu(x, pc_in.w, pc_qkv.w, gamma, beta)
    _contig(x, "x")
    C = x.shape[-1]
    if not transformer_in_ok(pc_in, pc_qkv, x, batch, hw, groups):
        raise ValueError("transformer_in: call outside ldm_transformer_in's scope (see transformer_in_ok)")
    if gamma.numel() != C or beta.numel() != C or gamma.dtype != torch.float32 or beta.dtype != torch.float32:
        raise ValueError("gamma/beta must be fp32 [C]")
    s0, _, unit, slots = _gn_sources(x, None, batch, C, 0, groups)
    h = torch.empty(batch, hw, C, dtype=x.dtype, device=x.device)
    qkv = torch.empty(batch, hw, 3 * C, dtype=x.dtype, device=x.device)
    gn = GnFold(_ptr(s0), unit, slots, groups, float(gn_eps), _ptr(gamma), _ptr(beta))
    dt = dtype_code(x.dtype)
    pi = ConvParams(_ptr(x), None, C, 0, batch, hw, 1, hw, 1, 1, 1, 0, _ptr(pc_in.w), C, C, _ptr(pc_in.bias),
                    None, 0, None, _ptr(h), OUT_NHWC, ACT_NONE, dt, 0, None, 0, None, 0, 0, 0, None, None, None,
                    0.0, 0.0)
    pq = ConvParams(None, None, C, 0, batch, hw, 1, hw, 1, 1, 1, 0, _ptr(pc_qkv.w), 3 * C, C, _ptr(pc_qkv.bias),
                    None, 0, None, _ptr(qkv), OUT_NHWC, ACT_NONE, dt, 0, None, 0, None, 0, 0, 0, None, None,
                    _ptr(pc_qkv.ln_c1), 1.0 / C, float(ln_eps))
    ev = _prof_start()
    _check(lib.ldm_transformer_in(ctypes.byref(gn), ctypes.byref(pi), ctypes.byref(pq), _stream(x)),
           "ldm_transformer_in")
    if ev is not None:
        rows = batch * hw
        flops = 2.0 * rows * C * 4 * C
        nbytes = (x.numel() + h.numel() + qkv.numel()) * x.element_size() + \
            (pc_in.w.numel() + pc_qkv.w.numel()) * pc_in.w.element_size()
        _prof_stop(ev, "igemm", flops, nbytes, f"tin M={rows} C={C}")
    return h, qkv


# ======================================================================================
# attention / norms
# ======================================================================================
def attention(q, k, v, batch, heads, head_dim, n_q, n_kv, q_stride, k_stride, v_stride, out=None, scale=None,
              fp8=False):
    """fp8=True: ldm_attention_fp8 (head_dim 40: Q.K^T and P.V on the block-scaled e4m3 MFMA; other
    head dims: P.V on the non-scaled e4m3 MFMA; bf16 inputs only)."""
    lib = load_library()
    _gpu(q, k, v, out)
    C = heads * head_dim
    if out is None:
        out = torch.empty(batch, n_q, C, dtype=q.dtype, device=q.device)
    if not (q.dtype == k.dtype == v.dtype == out.dtype):
        raise TypeError("q/k/v/out dtypes differ")
    for t, stride, n in ((q, q_stride, n_q), (k, k_stride, n_kv), (v, v_stride, n_kv)):
        need = ((batch - 1) * n + (n - 1)) * stride + C
        if t.storage_offset() + need > t.untyped_storage().nbytes() // t.element_size():
            raise ValueError("attention operand too small for the given strides")
    p = AttnParams(_ptr(q), _ptr(k), _ptr(v), _ptr(out), q_stride, k_stride, v_stride, C, batch, heads, head_dim,
                   n_q, n_kv, float(scale if scale is not None else head_dim ** -0.5), dtype_code(q.dtype))
    ev = _prof_start()
    if fp8:
        if q.dtype != torch.bfloat16:
            raise TypeError("fp8 attention takes bf16 q/k/v")
        wsb = int(lib.ldm_attention_fp8_workspace_bytes(ctypes.byref(p)))
        ws = torch.empty(wsb, dtype=torch.uint8, device=q.device) if wsb else None
        _check(lib.ldm_attention_fp8(ctypes.byref(p), _ptr(ws), wsb, _stream(q)), "ldm_attention_fp8")
    else:
        wsb = int(lib.ldm_attention_workspace_bytes(ctypes.byref(p)))
        if wsb:
            ws = torch.empty(wsb, dtype=torch.uint8, device=q.device)
            _check(lib.ldm_attention_ws(ctypes.byref(p), _ptr(ws), wsb, _stream(q)), "ldm_attention_ws")
        else:
            _check(lib.ldm_attention(ctypes.byref(p), _stream(q)), "ldm_attention")
    _prof_stop(ev, "attention", 4.0 * batch * heads * n_q * n_kv * head_dim,
               (2 * batch * n_q * C + 2 * batch * n_kv * C) * q.element_size(), f"N={n_q} L={n_kv} d={head_dim}")
    return out


def _gn_checked(x, batch, c):
    s = gn_stats_of(x)
    if s is not None and (s.dtype != torch.float64 or s.ndim != 4 or s.shape[0] != batch or s.shape[3] != 2
                          or s.shape[2] == 0 or c % s.shape[2] or not s.is_contiguous()):
        raise ValueError("attached GroupNorm accumulators do not match the tensor")
    return s


def _gn_sources(x0, x1, batch, c0, c1, groups):
    """(stats0, stats1, unit, slots) the kernel can consume, or (None, None, 0, 0): one unit and
    slot count for both sources, the unit dividing the group size and the concat offset (else the
    kernel recomputes the statistics)."""
    s0, s1 = _gn_checked(x0, batch, c0), _gn_checked(x1, batch, c1)
    if s0 is None or (c1 and s1 is None):
        return None, None, 0, 0
    unit, slots = c0 // s0.shape[2], s0.shape[1]
    if c1 and (c1 // s1.shape[2] != unit or s1.shape[1] != slots):
        return None, None, 0, 0
    if (c0 + c1) % groups or ((c0 + c1) // groups) % unit or slots * (c0 + c1) // unit > 2560:
        return None, None, 0, 0                   # (the kernel stages slots x units in <= 40 KB of LDS)
    return s0, s1, unit, slots


GN_MAX_GROUPS = 64        # ldm_group_norm_ex: per-group statistics staged in LDS (gst[64])
GN_MAX_CHANNELS = 2560    # GN_MAXC: the UNet's widest concat (csrc/norms.hip)


def group_norm(x0, batch, hw, groups, gamma, beta, eps, act=ACT_NONE, x1=None, out=None):
    """GroupNorm over NHWC [batch, hw, c0 (+c1)] -> contiguous NHWC [batch, hw, c0+c1].

    The one-launch kernel stages <= 64 groups and <= 2560 channels in LDS (every SD-1.x UNet,
    seg-VAE and PoseExpNet width fits); wider calls are refused here, before any launch."""
    done = getattr(x0, GN_DONE_ATTR, None)
    if done is not None and x1 is None and out is None and done[0] == gn_key(groups, gamma, beta, eps, act):
        return done[1]                    # applied by the producing conv's split-K reduction
    c_all = (x0.numel() + (0 if x1 is None else x1.numel())) // max(1, batch * hw)
    if groups > GN_MAX_GROUPS or c_all > GN_MAX_CHANNELS or groups <= 0 or c_all % groups:
        raise ValueError(f"group_norm: {groups} groups over {c_all} channels is outside the HIP kernel's range "
                         f"(groups <= {GN_MAX_GROUPS} dividing C, C <= {GN_MAX_CHANNELS})")
    lib = load_library()
    _gpu(x0, x1, gamma, beta, out)
    _contig(x0, "x0")
    _contig(x1, "x1")
    c0 = x0.numel() // (batch * hw)
    c1 = 0 if x1 is None else x1.numel() // (batch * hw)
    C = c0 + c1
    if gamma.numel() != C or beta.numel() != C or gamma.dtype != torch.float32 or beta.dtype != torch.float32:
        raise ValueError("gamma/beta must be fp32 [C]")
    if out is None:
        out = torch.empty(batch, hw, C, dtype=x0.dtype, device=x0.device)
    ws = torch.empty(int(lib.ldm_group_norm_workspace_bytes(batch, hw, C)), dtype=torch.uint8, device=x0.device)
    s0, s1, unit, slots = _gn_sources(x0, x1, batch, c0, c1, groups)
    ev = _prof_start()
    _check(lib.ldm_group_norm(_ptr(x0), _ptr(x1), c0, c1, batch, hw, groups, _ptr(gamma), _ptr(beta), float(eps),
                              act, _ptr(out), _ptr(s0), _ptr(s1), unit, slots, _ptr(ws), dtype_code(x0.dtype),
                              _stream(x0)), "ldm_group_norm")
    passes = 2.0 + (s0 is None) * 1.0
    _prof_stop(ev, "group_norm", 0.0, passes * out.numel() * out.element_size(),
               f"hw={hw} C={c0}+{c1} fused_stats={s0 is not None}")
    return out


def layer_norm(x, gamma, beta, eps, act=ACT_NONE, out=None):
    lib = load_library()
    _gpu(x, gamma, beta, out)
    _contig(x, "x")
    C = x.shape[-1]
    rows = x.numel() // C
    if out is None:
        out = torch.empty_like(x)
    ev = _prof_start()
    _check(lib.ldm_layer_norm(_ptr(x), rows, C, _ptr(gamma), _ptr(beta), float(eps), act, _ptr(out),
                              dtype_code(x.dtype), _stream(x)), "ldm_layer_norm")
    _prof_stop(ev, "layer_norm", 0.0, 2.0 * out.numel() * out.element_size())
    return out


def linear_rows_ok(pc: PackedConv, rows, x=None, sinusoid=False):
    """ldm_linear_rows takes this bf16 linear over `rows` (<= 16) rows (sinusoid input: k <= 512)."""
    k = pc.cin
    return (pc.dtype == torch.bfloat16 and pc.ksize == 1 and 0 < rows <= 16 and pc.n % 16 == 0 and k % 32 == 0
            and k <= (512 if sinusoid else 1536) and (x is None or (x.dtype == torch.bfloat16 and x.is_contiguous())))


def linear_rows(pc: PackedConv, x, rows, *, act=ACT_NONE, out_dtype=None, t=None, freqs=None, flip_sin_to_cos=True):
    """out [rows, n] = act(x @ W^T + b) for a handful of rows (ldm_linear_rows: the time-embedding
    MLP); x=None with (t, freqs): the input row is the sinusoidal timestep projection of t."""
    lib = load_library()
    dev = pc.w.device
    _gpu(pc.w, x, t, freqs)
    if x is not None and x.numel() != rows * pc.cin:
        raise ValueError("x must be [rows, cin]")
    out_dtype = out_dtype or pc.dtype
    out = torch.empty(rows, pc.n, dtype=out_dtype, device=dev)
    ev = _prof_start()
    _check(lib.ldm_linear_rows(_ptr(x), _ptr(t), 0 if t is None else t.numel(), _ptr(freqs), int(flip_sin_to_cos),
                               _ptr(pc.w), pc.kpad, pc.cin, pc.n, _ptr(pc.bias), rows, act, _ptr(out),
                               dtype_code(out_dtype), _stream(pc.w)), "ldm_linear_rows")
    _prof_stop(ev, "linear_rows", 2.0 * rows * pc.n * pc.cin_real, pc.w.numel() * pc.w.element_size() +
               rows * (pc.cin * (0 if x is None else x.element_size()) + pc.n * out.element_size()),
               f"rows={rows} N={pc.n} K={pc.cin_real}")
    return out


def unet_tail_ok(x, batch, h, w, groups, pc: PackedConv):
    """ldm_unet_tail takes this GroupNorm -> SiLU -> conv_out (bf16 input with producer statistics)."""
    st = gn_stats_of(x)
    if x.dtype != torch.bfloat16 or pc.dtype != torch.bfloat16 or pc.ksize != 3 or pc.n > 4 or st is None:
        return False
    c = pc.cin
    unit, slots = c // st.shape[2], st.shape[1]
    return (x.is_contiguous() and x.numel() == batch * h * w * c and h % 2 == 0 and w % 16 == 0 and w <= 64
            and c % 64 == 0 and c <= 640 and 0 < groups <= 64 and c % groups == 0 and (c // groups) % unit == 0
            and slots * (c // unit) <= 1024 and pc.bias is not None)


def unet_tail(x, batch, h, w, groups, gamma, beta, eps, pc: PackedConv, eps_dtype, ddim=None, want_eps=True):
    """GroupNorm(conv_norm_out) -> SiLU -> conv_out in one launch (ldm_unet_tail), x NHWC [batch, h, w, c]
    with producer GroupNorm statistics.  Returns the NCHW model output [batch, cout, h, w] in eps_dtype,
    or with ``ddim`` = dict(sample, t, alphas_cumprod, final_alpha, step_ratio, prediction_type,
    clip_sample, clip_range, use_clipped, out_dtype) the DDIM step on it fused: (eps | None, prev, x0)."""
    lib = load_library()
    st = gn_stats_of(x)
    _gpu(x, gamma, beta, pc.w, st)
    c = pc.cin
    unit, slots = c // st.shape[2], st.shape[1]
    eps_out = torch.empty(batch, pc.n, h, w, dtype=eps_dtype, device=x.device) if (want_eps or ddim is None) else None
    prev = x0 = None
    d = ddim or {}
    if ddim is not None:
        smp = d["sample"]
        _gpu(smp, d["t"], d["alphas_cumprod"])
        _contig(smp, "sample")
        if smp.shape != (batch, pc.n, h, w) or d["t"].dtype != torch.int64 or d["t"].numel() != 1:
            raise ValueError("ddim sample must be NCHW [batch, cout, h, w] and t one int64 device element")
        prev = d.get("prev_out")
        if prev is None:
            prev = torch.empty(smp.shape, dtype=d["out_dtype"], device=x.device)
        elif prev.shape != smp.shape or prev.dtype != d["out_dtype"] or not prev.is_contiguous():
            raise ValueError("ddim prev_out must be a contiguous tensor of the sample's shape and the output dtype")
        # (prev_out may be the sample itself: every element is read and written by the same thread)
        x0 = torch.empty(smp.shape, dtype=d["out_dtype"], device=x.device)
    p = UnetTailParams(_ptr(x), batch, h, w, c, _ptr(st), unit, slots, groups, float(eps), _ptr(gamma), _ptr(beta),
                       _ptr(pc.w), pc.kpad, pc.n, _ptr(pc.bias), _ptr(eps_out), dtype_code(eps_dtype),
                       _ptr(d.get("sample")), dtype_code(d["sample"].dtype) if ddim else 0, _ptr(d.get("t")),
                       _ptr(d.get("alphas_cumprod")), float(d.get("final_alpha", 0.0)), int(d.get("step_ratio", 0)),
                       PRED[d.get("prediction_type", "epsilon")], int(d.get("clip_sample", 0)),
                       float(d.get("clip_range", 0.0)), int(d.get("use_clipped", 0)),
                       d["alphas_cumprod"].numel() if ddim else 0, _ptr(prev), _ptr(x0),
                       dtype_code(d["out_dtype"]) if ddim else 0)
    ev = _prof_start()
    _check(lib.ldm_unet_tail(ctypes.byref(p), _stream(x)), "ldm_unet_tail")
    _prof_stop(ev, "igemm", 2.0 * batch * h * w * pc.n * 9 * c, x.numel() * x.element_size(),
               f"tail M={batch * h * w} C={c} N={pc.n}")
    if ddim is None:
        return eps_out
    return eps_out, prev, x0


def timestep_proj(t_f32, batch, freqs, dim, flip_sin_to_cos, dtype):
    lib = load_library()
    _gpu(t_f32, freqs)
    if t_f32.dtype != torch.float32 or t_f32.numel() not in (1, batch):
        raise ValueError("timesteps must be fp32 with 1 or batch elements")
    out = torch.empty(batch, dim, dtype=dtype, device=t_f32.device)
    _check(lib.ldm_timestep_proj(_ptr(t_f32), t_f32.numel(), batch, _ptr(freqs), dim, int(flip_sin_to_cos),
                                 _ptr(out), dtype_code(dtype), _stream(t_f32)), "ldm_timestep_proj")
    return out


# ======================================================================================
# DDIM, codec, layout helpers
# ======================================================================================
def ddim_step(model_output, sample, t_dev, alphas_cumprod_dev, final_alpha, step_ratio, prediction_type,
              clip_sample, clip_range, use_clipped, out_dtype, want_prev=True, want_x0=True):
    lib = load_library()
    _gpu(model_output, sample, t_dev, alphas_cumprod_dev)
    _contig(model_output, "model_output")
    _contig(sample, "sample")
    if model_output.numel() != sample.numel():
        raise ValueError("model_output and sample sizes differ")
    if t_dev.dtype != torch.int64 or t_dev.numel() != 1:
        raise ValueError("t must be a single int64 device element")
    prev = torch.empty(sample.shape, dtype=out_dtype, device=sample.device) if want_prev else None
    x0 = torch.empty(sample.shape, dtype=out_dtype, device=sample.device) if want_x0 else None
    p = DdimParams(_ptr(model_output), dtype_code(model_output.dtype), _ptr(sample), dtype_code(sample.dtype),
                   _ptr(prev), _ptr(x0), dtype_code(out_dtype), sample.numel(), _ptr(t_dev), _ptr(alphas_cumprod_dev),
                   float(final_alpha), int(step_ratio), PRED[prediction_type], int(clip_sample), float(clip_range),
                   int(use_clipped), alphas_cumprod_dev.numel())
    _check(lib.ldm_ddim_step(ctypes.byref(p), _stream(sample)), "ldm_ddim_step")
    return prev, x0


def ddim_add_noise(x0, noise, t_dev, ac_dev, scale):
    lib = load_library()
    _gpu(x0, noise, t_dev, ac_dev)
    _contig(x0, "x0")
    _contig(noise, "noise")
    B = x0.shape[0]
    if t_dev.numel() != B or t_dev.dtype != torch.int64 or noise.shape != x0.shape or noise.dtype != x0.dtype:
        raise ValueError("add_noise: timesteps must be int64 [B]; noise must match x0")
    out = torch.empty_like(x0)
    _check(lib.ldm_ddim_add_noise(_ptr(x0), _ptr(noise), _ptr(t_dev), _ptr(ac_dev), ac_dev.numel(), float(scale), B,
                                  x0.numel() // B, _ptr(out), dtype_code(x0.dtype), _stream(x0)), "ldm_ddim_add_noise")
    return out


def ddim_remove_noise(xt, noise, t_dev, ac_dev, scale):
    lib = load_library()
    _gpu(xt, noise, t_dev, ac_dev)
    _contig(xt, "xt")
    _contig(noise, "noise")
    B = xt.shape[0]
    if t_dev.numel() != B or t_dev.dtype != torch.int64 or noise.shape != xt.shape or noise.dtype != xt.dtype:
        raise ValueError("remove_noise: timesteps must be int64 [B]; noise must match xt")
    out = torch.empty_like(xt)
    _check(lib.ldm_ddim_remove_noise(_ptr(xt), _ptr(noise), _ptr(t_dev), _ptr(ac_dev), ac_dev.numel(), float(scale), B,
                                     xt.numel() // B, _ptr(out), dtype_code(xt.dtype), _stream(xt)),
           "ldm_ddim_remove_noise")
    return out


def bit_encode(ids, n, ignore_label, fill_value):
    """ids int64 [..., H, W] (GPU) -> (planes fp32 [..., n, H, W], ignore mask bool [..., H, W])."""
    lib = load_library()
    _gpu(ids)
    if ids.dtype != torch.int64:
        raise TypeError("ids must be int64")
    ids = ids.contiguous()
    H, W = ids.shape[-2], ids.shape[-1]
    batch = math.prod(ids.shape[:-2])
    planes = torch.empty(*ids.shape[:-2], n, H, W, dtype=torch.float32, device=ids.device)
    mask = torch.empty(ids.shape, dtype=torch.bool, device=ids.device)
    _check(lib.ldm_bit_encode(_ptr(ids), batch, H * W, n, int(ignore_label), float(fill_value), _ptr(planes),
                              _ptr(mask), _stream(ids)), "ldm_bit_encode")
    return planes, mask


def bit_decode(planes, drop_31=True):
    """planes [..., n, H, W] (GPU, fp32/bf16) -> ids int64 [..., H, W]."""
    lib = load_library()
    _gpu(planes)
    planes = planes.contiguous()
    n, H, W = planes.shape[-3], planes.shape[-2], planes.shape[-1]
    batch = math.prod(planes.shape[:-3]) if planes.ndim > 3 else 1
    ids = torch.empty(*planes.shape[:-3], H, W, dtype=torch.int64, device=planes.device)
    _check(lib.ldm_bit_decode(_ptr(planes), batch, n, H * W, int(drop_31), _ptr(ids), dtype_code(planes.dtype),
                              _stream(planes)), "ldm_bit_decode")
    return ids


CONF_MODE = {"none": 0, "max": 1, "topk_diff": 2}


def panoptic_pixels(logits, mask_th, ignore_label, conf_mode="max"):
    """logits fp32 NCHW [B, K, H, W] (GPU) -> (pred int32 [B, H, W], counts int32 [B, K],
    mask_counts int32 [B, K]) — argmax + confidence threshold + the per-label histograms."""
    lib = load_library()
    _gpu(logits)
    if logits.dtype != torch.float32 or logits.ndim != 4:
        raise TypeError("panoptic_pixels: logits must be fp32 [B, K, H, W]")
    logits = logits.contiguous()
    B, Kc, H, W = logits.shape
    dev = logits.device
    pred = torch.empty(B, H, W, dtype=torch.int32, device=dev)
    counts = torch.empty(B, Kc, dtype=torch.int32, device=dev)
    mcounts = torch.empty(B, Kc, dtype=torch.int32, device=dev)
    _check(lib.ldm_panoptic_pixels(_ptr(logits), B, Kc, H * W, CONF_MODE[conf_mode], float(mask_th), int(ignore_label),
                                   _ptr(pred), _ptr(counts), _ptr(mcounts), _stream(logits)), "ldm_panoptic_pixels")
    return pred, counts, mcounts


def panoptic_finalize(pred, counts, mask_counts, count_th, overlap_th, ignore_label):
    """-> (panoptic int32 [B, H, W] = cleaned_pred + 1, keep int32 [B, K])."""
    lib = load_library()
    for t in (pred, counts, mask_counts):
        _gpu(t)
        if t.dtype != torch.int32 or not t.is_contiguous():
            raise TypeError("panoptic_finalize: int32 contiguous tensors expected")
    B, H, W = pred.shape
    Kc = counts.shape[1]
    if counts.shape != (B, Kc) or mask_counts.shape != (B, Kc):
        raise ValueError("panoptic_finalize: counts must be [B, K]")
    out = torch.empty_like(pred)
    keep = torch.empty_like(counts)
    _check(lib.ldm_panoptic_finalize(_ptr(pred), _ptr(counts), _ptr(mask_counts), B, Kc, H * W, int(count_th),
                                     float(overlap_th), int(ignore_label), _ptr(keep), _ptr(out), _stream(pred)),
           "ldm_panoptic_finalize")
    return out, keep


def nchw_to_nhwc(sources, c_pad, dtype):
    """Gather up to three NCHW tensors [B, c_i, H, W] into one NHWC [B, H, W, c_pad] tensor."""
    lib = load_library()
    srcs = [s.contiguous() for s in sources if s is not None]
    _gpu(*srcs)
    if not 1 <= len(srcs) <= 3:
        raise ValueError("1..3 sources")
    B, _, H, W = srcs[0].shape
    for s in srcs:
        if s.shape[0] != B or s.shape[2:] != (H, W):
            raise ValueError("sources must share batch and spatial size")
    args = []
    for i in range(3):
        if i < len(srcs):
            s = srcs[i]
            args += [_ptr(s), s.shape[1], dtype_code(s.dtype)]
        else:
            args += [None, 0, 0]
    out = torch.empty(B, H, W, c_pad, dtype=dtype, device=srcs[0].device)
    _check(lib.ldm_nchw_to_nhwc(*args, B, H * W, c_pad, _ptr(out), dtype_code(dtype), _stream(srcs[0])),
           "ldm_nchw_to_nhwc")
    return out


CONV_IN_MIN_ROWS = 256    # ldm_conv_in blocks (output rows) below which the two launches are faster


def conv_in_ok(pc: PackedConv, sources, batch, h, w):
    """ldm_conv_in takes this conv_in: bf16 3x3 pack over 16 padded channels, n % 64 == 0 (<= 320),
    width % 16 == 0 (<= 64), the sources' channels <= 16, and >= 256 output rows (one block each: a
    single 64x64 frame's 64 blocks lose to the two launches, 16.4 vs 15.1 us; at B = 8 24.6 vs 27.7)."""
    srcs = [t for t in sources if t is not None]
    return (pc.dtype == torch.bfloat16 and batch * h >= CONV_IN_MIN_ROWS and pc.ksize == 3 and pc.cin == 16 and pc.n % 64 == 0 and pc.n <= 320
            and pc.bias is not None and w % 16 == 0 and w <= 64 and 1 <= len(srcs) <= 3
            and sum(t.shape[1] for t in srcs) <= 16
            and all(t.dtype in (torch.float32, torch.bfloat16) and t.shape[0] == batch and t.shape[2:] == (h, w)
                    for t in srcs))


def conv_in(pc: PackedConv, sources, batch, h, w, gn_stats=True):
    """The UNet's conv_in on the channel concatenation of up to three NCHW sources, one launch
    (ldm_conv_in: replaces nchw_to_nhwc + conv2d).  NHWC bf16 [batch, h, w, n] with the GroupNorm
    accumulators attached as conv2d(gn_stats=True) attaches them."""
    lib = load_library()
    srcs = [t.contiguous() for t in sources if t is not None]
    _gpu(pc.w, *srcs)
    out = torch.empty(batch, h, w, pc.n, dtype=torch.bfloat16, device=pc.w.device)
    part, unit, slots = None, 0, 0
    if gn_stats and (h * w) % 64 == 0:
        unit, slots = gn_unit_for(pc.n), gn_slots_for(h * w)
        part = _gn_accumulators(batch, slots, pc.n // unit, pc.w.device)
    p = ConvInParams()
    for i, t in enumerate(srcs):
        p.src[i], p.c[i], p.src_dtype[i] = _ptr(t), t.shape[1], dtype_code(t.dtype)
    p.batch, p.height, p.width, p.dtype = batch, h, w, dtype_code(torch.bfloat16)
    p.w, p.n, p.kpad, p.bias, p.out = _ptr(pc.w), pc.n, pc.kpad, _ptr(pc.bias), _ptr(out)
    p.gn_partial, p.gn_unit, p.gn_slots = _ptr(part), unit, slots
    ev = _prof_start()
    _check(lib.ldm_conv_in(ctypes.byref(p), _stream(pc.w)), "ldm_conv_in")
    setattr(out, GN_PART_ATTR, part)
    setattr(out, GN_DONE_ATTR, None)
    _prof_stop(ev, "igemm", 2.0 * batch * h * w * pc.n * 9 * pc.cin_real,
               sum(t.numel() * t.element_size() for t in srcs) + pc.w.numel() * 2 + out.numel() * 2,
               f"conv_in M={batch * h * w} N={pc.n} Cin={pc.cin_real}")
    return out


def resize_bilinear(x, size=None, scale_factor=None, mul=1.0, add=0.0, out_dtype=None):
    """F.interpolate(x, size|scale_factor, mode='bilinear', align_corners=False) * mul + add (NCHW)."""
    lib = load_library()
    _gpu(x)
    x = x.contiguous()
    B, C, H, W = x.shape
    if size is not None:
        ho, wo = (size, size) if isinstance(size, int) else tuple(size)
        sh, sw = H / ho, W / wo
    else:
        sfh, sfw = (scale_factor, scale_factor) if not isinstance(scale_factor, (tuple, list)) else scale_factor
        ho, wo = int(math.floor(H * sfh)), int(math.floor(W * sfw))
        sh, sw = 1.0 / sfh, 1.0 / sfw
    odt = out_dtype or x.dtype
    out = torch.empty(B, C, ho, wo, dtype=odt, device=x.device)
    _check(lib.ldm_resize_bilinear(_ptr(x), B * C, H, W, ho, wo, float(sh), float(sw), float(mul), float(add),
                                   _ptr(out), dtype_code(x.dtype), dtype_code(odt), _stream(x)), "ldm_resize_bilinear")
    return out


def gaussian_posterior(moments, clamp_output, act_fn):
    """NCHW moments [B, 2L, H, W] -> (mean, logvar, std, var) fp32 [B, L, H, W]."""
    lib = load_library()
    _gpu(moments)
    moments = moments.contiguous()
    B, C2, H, W = moments.shape
    L = C2 // 2
    outs = [torch.empty(B, L, H, W, dtype=torch.float32, device=moments.device) for _ in range(4)]
    _check(lib.ldm_gaussian_posterior(_ptr(moments), B, H * W, L, int(clamp_output), POST_ACT[act_fn],
                                      *[_ptr(o) for o in outs], dtype_code(moments.dtype), _stream(moments)),
           "ldm_gaussian_posterior")
    return tuple(outs)


# ======================================================================================
# training path (backward kernels + optimizer)
# ======================================================================================
def conv2d_wgrad(pc: PackedConv, x0, batch, h, w, dy, *, x1=None, stride=1, upsample=False, dw=None,
                 accumulate=False):
    """Weight gradient of conv2d(pc, x0[, x1]) given dy (NHWC [batch, ho, wo, n], compute dtype).

    Returns dw fp32 in the TORCH layout of the packed weight's source ([n][cin_real][k][k] or
    [n][cin_real] for 1x1), GEGLU rows un-interleaved.  dw may be a preallocated view."""
    lib = load_library()
    _gpu(x0, x1, dy, dw)
    for t, nm in ((x0, "x0"), (x1, "x1"), (dy, "dy")):
        _contig(t, nm)
    if pc.shuffle2:
        raise NotImplementedError("ConvTranspose weight gradient is not on the UNet training path")
    c0 = x0.numel() // (batch * h * w)
    c1 = 0 if x1 is None else x1.numel() // (batch * h * w)
    if c0 + c1 != pc.cin:
        raise ValueError(f"wgrad expects {pc.cin} input channels, got {c0}+{c1}")
    if pc.ksize == 1:
        ho, wo = h, w
    elif upsample:
        ho, wo = 2 * h, 2 * w
    else:
        ho, wo = (h + 2 - 3) // stride + 1, (w + 2 - 3) // stride + 1
    n = pc.n
    if dy.numel() != batch * ho * wo * n or dy.dtype != pc.dtype or x0.dtype != pc.dtype:
        raise ValueError("dy must be [batch, ho, wo, n] in the compute dtype")
    shape = (n, pc.cin_real) if pc.ksize == 1 else (n, pc.cin_real, pc.ksize, pc.ksize)
    if dw is None:
        dw = torch.empty(shape, dtype=torch.float32, device=x0.device)
        accumulate = False
    elif dw.numel() != math.prod(shape) or dw.dtype != torch.float32 or not dw.is_contiguous():
        raise ValueError("dw must be a contiguous fp32 tensor of the weight's size")
    p = WgradParams(_ptr(x0), _ptr(x1), c0, c1, batch, h, w, ho, wo, pc.ksize, stride, int(upsample), _ptr(dy), n,
                    pc.kpad, pc.cin_real, int(pc.geglu), _ptr(dw), int(accumulate), dtype_code(pc.dtype), None, 0)
    ws_bytes = int(lib.ldm_conv2d_wgrad_workspace_bytes(ctypes.byref(p)))
    if ws_bytes == 0:
        raise ValueError("ldm_conv2d_wgrad rejected the configuration")
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x0.device)
    p.workspace, p.workspace_bytes = _ptr(ws), ws_bytes
    ev = _prof_start()
    _check(lib.ldm_conv2d_wgrad(ctypes.byref(p), _stream(x0)), "ldm_conv2d_wgrad")
    _prof_stop(ev, "wgrad", 2.0 * batch * ho * wo * n * pc.ksize * pc.ksize * pc.cin_real,
               (x0.numel() + (0 if x1 is None else x1.numel()) + dy.numel()) * x0.element_size() + ws_bytes * 2,
               f"k{pc.ksize} M={batch * ho * wo} N={n} Cin={c0}+{c1}")
    return dw


def colsum(x, rows, c, segments=1, geglu=False, out=None, accumulate=False):
    """fp32 [segments, c] column sums of x viewed as [rows, c]."""
    lib = load_library()
    _gpu(x, out)
    _contig(x, "x")
    if x.numel() != rows * c:
        raise ValueError("colsum: numel != rows * c")
    if out is None:
        out = torch.empty(segments, c, dtype=torch.float32, device=x.device)
        accumulate = False
    elif out.numel() != segments * c or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("colsum: bad out")
    ws = torch.empty(int(lib.ldm_colsum_workspace_bytes(rows, c, segments)), dtype=torch.uint8, device=x.device)
    _check(lib.ldm_colsum(_ptr(x), rows, c, segments, int(geglu), _ptr(out), int(accumulate), _ptr(ws),
                          dtype_code(x.dtype), _stream(x)), "ldm_colsum")
    return out


def group_norm_train(x0, batch, hw, groups, gamma, beta, eps, act=ACT_NONE, x1=None):
    """group_norm() that also returns the per-(batch, group) (mean, rstd) for the backward."""
    lib = load_library()
    _gpu(x0, x1, gamma, beta)
    _contig(x0, "x0")
    _contig(x1, "x1")
    c0 = x0.numel() // (batch * hw)
    c1 = 0 if x1 is None else x1.numel() // (batch * hw)
    C = c0 + c1
    out = torch.empty(batch, hw, C, dtype=x0.dtype, device=x0.device)
    mr = torch.empty(batch, groups, 2, dtype=torch.float32, device=x0.device)
    ws = torch.empty(int(lib.ldm_group_norm_workspace_bytes(batch, hw, C)), dtype=torch.uint8, device=x0.device)
    s0, s1, unit, slots = _gn_sources(x0, x1, batch, c0, c1, groups)
    _check(lib.ldm_group_norm_ex(_ptr(x0), _ptr(x1), c0, c1, batch, hw, groups, _ptr(gamma), _ptr(beta), float(eps),
                                 act, _ptr(out), _ptr(s0), _ptr(s1), unit, slots, _ptr(ws), _ptr(mr),
                                 dtype_code(x0.dtype), _stream(x0)), "ldm_group_norm_ex")
    return out, mr


def group_norm_bwd(x0, batch, hw, groups, mean_rstd, gamma, beta, act, dy, *, x1=None, add_src=None, dx0=None,
                   dx1=None, acc0=False, acc1=False, dgamma=None, dbeta=None, acc_params=False):
    lib = load_library()
    _gpu(x0, x1, dy, add_src, dx0, dx1)
    for t, nm in ((x0, "x0"), (x1, "x1"), (dy, "dy"), (add_src, "add_src")):
        _contig(t, nm)
    c0 = x0.numel() // (batch * hw)
    c1 = 0 if x1 is None else x1.numel() // (batch * hw)
    C = c0 + c1
    if dy.numel() != batch * hw * C or dy.dtype != x0.dtype:
        raise ValueError("group_norm_bwd: dy must be [batch, hw, c0 + c1] in the compute dtype")
    if dx0 is None:
        dx0, acc0 = torch.empty_like(x0), False
    if c1 and dx1 is None:
        dx1, acc1 = torch.empty_like(x1), False
    ws = torch.empty(int(lib.ldm_group_norm_bwd_workspace_bytes(batch, hw, C, groups)), dtype=torch.uint8,
                     device=x0.device)
    _check(lib.ldm_group_norm_bwd(_ptr(x0), _ptr(x1), c0, c1, batch, hw, groups, _ptr(mean_rstd), _ptr(gamma),
                                  _ptr(beta), act, _ptr(dy), _ptr(add_src), _ptr(dx0), _ptr(dx1), int(acc0), int(acc1),
                                  _ptr(dgamma), _ptr(dbeta), int(acc_params), _ptr(ws), dtype_code(x0.dtype),
                                  _stream(x0)), "ldm_group_norm_bwd")
    return dx0, dx1


def layer_norm_bwd(x, dy, gamma, eps, add_src=None, dx=None, dgamma=None, dbeta=None, acc_params=False):
    lib = load_library()
    _gpu(x, dy, add_src, dx)
    for t, nm in ((x, "x"), (dy, "dy"), (add_src, "add_src")):
        _contig(t, nm)
    C = x.shape[-1]
    rows = x.numel() // C
    if dx is None:
        dx = torch.empty_like(x)
    ws = torch.empty(int(lib.ldm_layer_norm_bwd_workspace_bytes(rows, C)), dtype=torch.uint8, device=x.device)
    _check(lib.ldm_layer_norm_bwd(_ptr(x), _ptr(dy), rows, C, _ptr(gamma), float(eps), _ptr(add_src), _ptr(dx),
                                  _ptr(dgamma), _ptr(dbeta), int(acc_params), _ptr(ws), dtype_code(x.dtype),
                                  _stream(x)), "ldm_layer_norm_bwd")
    return dx


def geglu_fwd(hg):
    """[..., 2F] packed GEGLU pre-activation -> [..., F] h * gelu(g)."""
    lib = load_library()
    _gpu(hg)
    _contig(hg, "hg")
    F2 = hg.shape[-1]
    rows = hg.numel() // F2
    out = torch.empty(*hg.shape[:-1], F2 // 2, dtype=hg.dtype, device=hg.device)
    _check(lib.ldm_geglu(_ptr(hg), None, rows, F2 // 2, _ptr(out), None, dtype_code(hg.dtype), _stream(hg)),
           "ldm_geglu")
    return out


def geglu_bwd(hg, dout):
    lib = load_library()
    _gpu(hg, dout)
    _contig(hg, "hg")
    _contig(dout, "dout")
    F2 = hg.shape[-1]
    rows = hg.numel() // F2
    dhg = torch.empty_like(hg)
    _check(lib.ldm_geglu(_ptr(hg), _ptr(dout), rows, F2 // 2, None, _ptr(dhg), dtype_code(hg.dtype), _stream(hg)),
           "ldm_geglu")
    return dhg


def sum_pool2(x, batch, h_out, w_out, out=None, accumulate=False):
    lib = load_library()
    _gpu(x, out)
    _contig(x, "x")
    C = x.numel() // (batch * 4 * h_out * w_out)
    if out is None:
        out = torch.empty(batch, h_out, w_out, C, dtype=x.dtype, device=x.device)
        accumulate = False
    _check(lib.ldm_sum_pool2(_ptr(x), batch, h_out, w_out, C, _ptr(out), int(accumulate), dtype_code(x.dtype),
                             _stream(x)), "ldm_sum_pool2")
    return out


def mse_loss(pred, target, mask=None, t=None, weights=None, grad_scale=1.0, want_grad=True):
    """Returns (loss_sum fp64 device scalar, dpred or None)."""
    lib = load_library()
    _gpu(pred, target, mask, t, weights)
    pred = pred.contiguous()
    target = target.float().contiguous()
    B, Cc, H, W = pred.shape
    if mask is not None:
        mask = mask.float().contiguous()
        if mask.numel() != B * H * W:
            raise ValueError("mask must be [B, H, W]")
    if weights is not None:
        if t is None or t.dtype != torch.int64 or t.numel() != B:
            raise ValueError("per-sample int64 timesteps are needed with weights")
        weights = weights.float().contiguous()
    dpred = torch.empty_like(pred) if want_grad else None
    total = torch.empty((), dtype=torch.float64, device=pred.device)
    ws = torch.empty(int(lib.ldm_reduce_workspace_bytes()), dtype=torch.uint8, device=pred.device)
    _check(lib.ldm_mse_loss(_ptr(pred), _ptr(target), _ptr(mask), _ptr(t), _ptr(weights),
                            0 if weights is None else weights.numel(), B, Cc, H * W, float(grad_scale), _ptr(dpred),
                            _ptr(total), _ptr(ws), dtype_code(pred.dtype), _stream(pred)), "ldm_mse_loss")
    return total, dpred


def sq_norm(g, out=None, accumulate=False):
    lib = load_library()
    _gpu(g)
    if g.dtype != torch.float32 or not g.is_contiguous():
        raise ValueError("sq_norm takes a contiguous fp32 buffer")
    if out is None:
        out = torch.empty((), dtype=torch.float64, device=g.device)
        accumulate = False
    ws = torch.empty(int(lib.ldm_reduce_workspace_bytes()), dtype=torch.uint8, device=g.device)
    _check(lib.ldm_sq_norm(_ptr(g), g.numel(), _ptr(out), int(accumulate), _ptr(ws), _stream(g)), "ldm_sq_norm")
    return out


def repack(table, ndesc, total_chunks, device):
    """ldm_repack over a device byte table of ndesc ldm_repack_desc records (models/repack.py)."""
    lib = load_library()
    _gpu(table)
    _check(lib.ldm_repack(_ptr(table), int(ndesc), int(total_chunks),
                          ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)), "ldm_repack")


def adamw(param, grad, exp_avg, exp_avg_sq, segments, nseg, step, beta1=0.9, beta2=0.999, eps=1e-8, sqsum=None,
          max_norm=0.0):
    """segments: device byte tensor of nseg packed {int64 begin, end; float lr, wd} records."""
    lib = load_library()
    _gpu(param, grad, exp_avg, exp_avg_sq, segments, sqsum)
    n = param.numel()
    for t in (grad, exp_avg, exp_avg_sq):
        if t.numel() != n or t.dtype != torch.float32:
            raise ValueError("adamw buffers must be fp32 of equal size")
    _check(lib.ldm_adamw(_ptr(param), _ptr(grad), _ptr(exp_avg), _ptr(exp_avg_sq), _ptr(segments), int(nseg), n,
                         float(beta1), float(beta2), float(eps), int(step), _ptr(sqsum), float(max_norm),
                         _stream(param)), "ldm_adamw")


def attention_fwd_lse(q, k, v, batch, heads, head_dim, n_q, n_kv, q_stride, k_stride, v_stride, scale=None):
    """attention() that also returns the log2-domain LSE [batch, heads, n_q] for the backward."""
    lib = load_library()
    _gpu(q, k, v)
    C = heads * head_dim
    out = torch.empty(batch, n_q, C, dtype=q.dtype, device=q.device)
    lse = torch.empty(batch, heads, n_q, dtype=torch.float32, device=q.device)
    p = AttnParams(_ptr(q), _ptr(k), _ptr(v), _ptr(out), q_stride, k_stride, v_stride, C, batch, heads, head_dim,
                   n_q, n_kv, float(scale if scale is not None else head_dim ** -0.5), dtype_code(q.dtype))
    ev = _prof_start()
    _check(lib.ldm_attention_fwd_lse(ctypes.byref(p), _ptr(lse), _stream(q)), "ldm_attention_fwd_lse")
    _prof_stop(ev, "attention", 4.0 * batch * heads * n_q * n_kv * head_dim,
               (2 * batch * n_q * C + 2 * batch * n_kv * C) * q.element_size(), f"N={n_q} L={n_kv} d={head_dim}")
    return out, lse


def attention_bwd(q, k, v, o, d_o, lse, batch, heads, head_dim, n_q, n_kv, q_stride, k_stride, v_stride, dq, dk, dv,
                  dq_stride, dkv_stride, scale=None):
    lib = load_library()
    _gpu(q, k, v, o, d_o, lse, dq, dk, dv)
    _contig(d_o, "d_o")
    C = heads * head_dim
    p = AttnParams(_ptr(q), _ptr(k), _ptr(v), _ptr(o), q_stride, k_stride, v_stride, C, batch, heads, head_dim,
                   n_q, n_kv, float(scale if scale is not None else head_dim ** -0.5), dtype_code(q.dtype))
    ws = torch.empty(int(lib.ldm_attention_bwd_workspace_bytes(ctypes.byref(p))), dtype=torch.uint8, device=q.device)
    ev = _prof_start()
    _check(lib.ldm_attention_bwd(ctypes.byref(p), _ptr(o), _ptr(d_o), C, _ptr(lse), _ptr(dq), _ptr(dk), _ptr(dv),
                                 dq_stride, dkv_stride, _ptr(ws), _stream(q)), "ldm_attention_bwd")
    _prof_stop(ev, "attention_bwd", 10.0 * batch * heads * n_q * n_kv * head_dim,
               (4 * batch * n_q * C + 4 * batch * n_kv * C) * q.element_size(), f"N={n_q} L={n_kv} d={head_dim}")


# ======================================================================================
# AE training (row a16): point losses + VAE-backward helpers
# ======================================================================================
def _coords(c, boxes):
    if c.dtype != torch.float32 or c.ndim != 3 or c.shape[0] != boxes or c.shape[2] != 2 or not c.is_contiguous():
        raise ValueError("coords must be contiguous fp32 [boxes, P, 2]")
    return c.shape[1]


def point_sample(x, coords, planes=None):
    """x fp32 NCHW [N, C, H, W]; boxes = N (C planes each) or len(planes) (one plane each, index
    into the flattened N*C planes) -> [boxes, C or 1, P]."""
    lib = load_library()
    _gpu(x, coords, planes)
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise TypeError("point_sample: x must be contiguous fp32 NCHW")
    N, C, H, W = x.shape
    boxes = N if planes is None else planes.numel()
    P = _coords(coords, boxes)
    cc = C if planes is None else 1
    out = torch.empty(boxes, cc, P, dtype=torch.float32, device=x.device)
    _check(lib.ldm_point_sample(_ptr(x), boxes, cc, H, W, _ptr(planes), _ptr(coords), P, _ptr(out), _stream(x)),
           "ldm_point_sample")
    return out


def point_sample_bwd(dout, coords, din, planes=None, scale_t=None, scale=1.0):
    """din (fp32 NCHW, accumulated in place) += adjoint of point_sample applied to dout * scale * scale_t."""
    lib = load_library()
    _gpu(dout, coords, din, planes, scale_t)
    N, C, H, W = din.shape
    boxes, cc, P = dout.shape
    if _coords(coords, boxes) != P or cc != (C if planes is None else 1):
        raise ValueError("point_sample_bwd: shapes do not match")
    _check(lib.ldm_point_sample_bwd(_ptr(dout), boxes, cc, H, W, _ptr(planes), _ptr(coords), P, _ptr(scale_t),
                                    float(scale), _ptr(din), _stream(din)), "ldm_point_sample_bwd")


def point_labels_nearest(targets, coords):
    lib = load_library()
    _gpu(targets, coords)
    B, H, W = targets.shape
    P = _coords(coords, B)
    lab = torch.empty(B, P, dtype=torch.int64, device=targets.device)
    _check(lib.ldm_point_labels(_ptr(targets.contiguous()), H, W, None, None, _ptr(coords), B, P, 0, _ptr(lab), None,
                                _stream(targets)), "ldm_point_labels")
    return lab


def point_labels_mask(targets, img, cls, coords):
    lib = load_library()
    _gpu(targets, img, cls, coords)
    B, H, W = targets.shape
    boxes = img.numel()
    P = _coords(coords, boxes)
    val = torch.empty(boxes, P, dtype=torch.float32, device=targets.device)
    _check(lib.ldm_point_labels(_ptr(targets.contiguous()), H, W, _ptr(img), _ptr(cls), _ptr(coords), boxes, P, 1,
                                None, _ptr(val), _stream(targets)), "ldm_point_labels")
    return val


def point_uncertainty(x):
    lib = load_library()
    _gpu(x)
    boxes, C, P = x.shape
    u = torch.empty(boxes, P, dtype=torch.float32, device=x.device)
    _check(lib.ldm_point_uncertainty(_ptr(x), boxes, C, P, _ptr(u), _stream(x)), "ldm_point_uncertainty")
    return u


def topk_select(u, k, coords=None):
    lib = load_library()
    _gpu(u, coords)
    rows, n = u.shape
    idx = torch.empty(rows, k, dtype=torch.int32, device=u.device)
    co = None if coords is None else torch.empty(rows, k, 2, dtype=torch.float32, device=u.device)
    _check(lib.ldm_topk_select(_ptr(u.contiguous()), rows, n, k, _ptr(coords), _ptr(idx), _ptr(co), _stream(u)),
           "ldm_topk_select")
    return idx, co


def point_ce(x, labels, temperature, ignore_label):
    lib = load_library()
    _gpu(x, labels)
    B, C, P = x.shape
    acc = torch.empty(2, dtype=torch.float64, device=x.device)
    grad = torch.empty_like(x)
    _check(lib.ldm_point_ce(_ptr(x), _ptr(labels), B, C, P, float(temperature), int(ignore_label), _ptr(acc),
                            _ptr(grad), _stream(x)), "ldm_point_ce")
    return acc, grad


def point_bce_dice(x, y):
    lib = load_library()
    _gpu(x, y)
    M, P = x.shape
    acc = torch.empty(2, dtype=torch.float64, device=x.device)
    grad = torch.empty_like(x)
    _check(lib.ldm_point_bce_dice(_ptr(x), _ptr(y), M, P, _ptr(acc), _ptr(grad), _stream(x)), "ldm_point_bce_dice")
    return acc, grad


def silu(z, dy=None):
    lib = load_library()
    _gpu(z, dy)
    out = torch.empty_like(z)
    _check(lib.ldm_silu(_ptr(z), _ptr(dy), z.numel(), _ptr(out), dtype_code(z.dtype), _stream(z)), "ldm_silu")
    return out


def space_to_depth2(d, batch, h, w):
    """d NHWC [batch, 2h, 2w, c] -> [batch, h, w, 4c] in (dy, dx, c) order."""
    lib = load_library()
    _gpu(d)
    c = d.numel() // (batch * 4 * h * w)
    out = torch.empty(batch, h, w, 4 * c, dtype=d.dtype, device=d.device)
    _check(lib.ldm_space_to_depth2(_ptr(d.contiguous()), batch, h, w, c, _ptr(out), dtype_code(d.dtype), _stream(d)),
           "ldm_space_to_depth2")
    return out


def posterior_sample(moments, eps):
    lib = load_library()
    _gpu(moments, eps)
    B, C2, H, W = moments.shape
    z = torch.empty(B, C2 // 2, H, W, dtype=torch.float32, device=moments.device)
    _check(lib.ldm_posterior_sample(_ptr(moments), _ptr(eps), B, C2 // 2, H * W, _ptr(z), _stream(moments)),
           "ldm_posterior_sample")
    return z


def posterior_bwd(moments, eps, dz_nhwc):
    lib = load_library()
    _gpu(moments, eps, dz_nhwc)
    B, C2, H, W = moments.shape
    cs = dz_nhwc.shape[-1]
    dm = torch.empty_like(moments)
    _check(lib.ldm_posterior_bwd(_ptr(moments), _ptr(eps), _ptr(dz_nhwc), cs, B, C2 // 2, H * W, _ptr(dm),
                                 dtype_code(dz_nhwc.dtype), _stream(moments)), "ldm_posterior_bwd")
    return dm
