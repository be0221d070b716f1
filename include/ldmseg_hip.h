/*
 * ldmseg_hip.h — C ABI of the MI355X (gfx950) kernels behind the latent-diffusion
 * denoising path of weentiaan/Video-latent-diffusion-panoptic-segmentation.
 *
 * The reference has no FFI: its hot path is the nn.Module / scheduler Python API, whose
 * arithmetic is dispatched implicitly to stock PyTorch / diffusers kernels.
 * Each entry point below replaces one family of those implicit op sites; the drop-in
 * Python modules (ldmseg.models.UNet / GeneralVAESeg, ldmseg.schedulers.DDIMNoiseScheduler)
 * bind them with ctypes.
 *
 * Conventions
 *  - All pointers are DEVICE pointers owned by the caller (PyTorch caching allocator); no
 *    entry point allocates, frees or synchronises, so every call is hipGraph-capturable.
 *  - Activations inside the UNet/VAE are NHWC ("rows" = pixels or tokens, channels
 *    contiguous).  Boundary tensors (UNet sample/output, VAE input/logits) are NCHW.
 *  - dtype codes: LDM_F32 (exact fp32 path, the 1e-3 parity gate) or LDM_BF16 (fp32
 *    accumulation, bf16 storage — the performance path).
 *  - Return value: LDM_OK or an LDM_ERR_* code (ldm_status_string() describes it); shape
 *    and alignment preconditions are checked on the host before any launch.
 */
#ifndef LDMSEG_HIP_H
#define LDMSEG_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* ldm_stream_t; /* == hipStream_t */

enum { LDM_F32 = 0, LDM_BF16 = 1 };
enum {
  LDM_OK = 0,
  LDM_ERR_ARG = 1,     /* bad argument / unsupported configuration */
  LDM_ERR_ALIGN = 2,   /* pointer or channel count violates the vector-width requirement */
  LDM_ERR_LAUNCH = 3,  /* hipLaunchKernel failed */
};

/* ---------------------------------------------------------------------------------------
 * ldm_conv2d — implicit-GEMM convolution / GEMM on MFMA.
 * Replaces: every nn.Conv2d (3x3 stride 1/2, 1x1), nn.Linear and ConvTranspose2d(k2,s2)
 * site of the path — diffusers ResnetBlock2D conv1/conv2/conv_shortcut, Transformer2DModel
 * proj_in/proj_out, Attention to_q/k/v/to_out, FeedForward GEGLU + net.2,
 * TimestepEmbedding linear_1/2, time_emb_proj, Down/Upsample2D conv
 * (reached via ldmseg/models/unet.py:305-307,357,361-431) and GeneralVAESeg encoder/decoder
 * convs (ldmseg/models/vae.py:134-173,191-245).
 *
 *   out[m, n] = epilogue( sum_k A[m, k] * W[n, k] )
 * A rows m = (b, oy, ox) over batch x h_out x w_out; k = (ky, kx, c) tap-major over the
 * channel concatenation [a0 (c0 ch) || a1 (c1 ch)] of the NHWC input, zero padded by
 * ksize/2 (optionally read through a nearest-2x upsample, Upsample2D).
 * W is pre-packed [n_alloc][kpad] (K = ksize*ksize*(c0+c1) padded with zeros to kpad).
 * ------------------------------------------------------------------------------------- */
enum { LDM_OUT_NHWC = 0, LDM_OUT_NCHW = 1, LDM_OUT_GEGLU = 2, LDM_OUT_SHUFFLE2 = 3 };
enum { LDM_ACT_NONE = 0, LDM_ACT_SILU = 1, LDM_ACT_RELU = 2, LDM_ACT_SIGMOID = 3 };

typedef struct {
  const void* a0;          /* NHWC [batch][h_in][w_in][c0] */
  const void* a1;          /* NHWC [batch][h_in][w_in][c1] or NULL (c1 == 0) */
  int c0, c1;
  int batch, h_in, w_in;
  int h_out, w_out;
  int ksize;               /* 1 or 3 */
  int stride;              /* 1 or 2 */
  int upsample;            /* 1: input is nearest-upsampled x2 before the conv */
  const void* w;           /* [n_alloc][kpad] */
  int n;                   /* GEMM N (for GEGLU: 2 x output channels, for SHUFFLE2: 4 x Cout) */
  int kpad;                /* multiple of 64 */
  const float* bias;       /* [n] or NULL (packed like W for GEGLU / SHUFFLE2) */
  const float* temb;       /* per-(batch, n) additive term: temb[b * temb_stride + n], or NULL */
  int temb_stride;
  const void* residual;    /* same layout/dtype as out, added after activation; may alias out */
  void* out;
  int out_layout;          /* LDM_OUT_* */
  int act;                 /* LDM_ACT_* applied after bias/temb, before residual */
  int dtype;               /* A / W / residual dtype */
  int out_f32;             /* 1: out is fp32 regardless of dtype */
  void* workspace;         /* split-K fp32 slab, >= ldm_conv2d_workspace_bytes(p) bytes (or NULL if 0) */
  int64_t workspace_bytes;
  double* gn_partial;      /* optional: GroupNorm statistics of the output, [batch][gn_slots][n / gn_unit][2]
                              fp64 (sum, sumsq) accumulators, one per gn_unit consecutive channels,
                              that the epilogue ADDS to (atomically, one fp32 partial per unit and
                              tile, spread over gn_slots copies by tile row): zero them first
                              (NHWC, h_out*w_out % 64 == 0) */
  int pad_mode;            /* 0: zero padding ksize/2 on every side; 1: diffusers Downsample2D(padding=0):
                              F.pad (0, 1, 0, 1) then an unpadded conv (AutoencoderKL encoder) */
  int gn_unit;             /* channels per gn_partial accumulator (n % gn_unit == 0; 0 means 1).  Any
                              GroupNorm whose group size and concat offset are multiples of it can
                              consume them — 10 serves every SD UNet GroupNorm, concats included */
  int gn_slots;            /* copies of the accumulators (0 means 1): same-address atomics serialise,
                              so the row tiles of one batch are spread over the slots */
  /* LayerNorm folded into 1x1 GEMMs (bf16, NHWC or GEGLU output, no time embedding, no
   * gn_partial; the transformer block's norm1 -> QKV and norm3 -> ff.net.0, unet.py:83-105):
   *   row_stats  optional OUTPUT: [M][2] fp64 (sum, sumsq) of each stored output row, ADDED
   *              atomically (zero it first) — the statistics of the next LayerNorm's input.  The
   *              per-tile partials are fp32 and their fp64 sum is exact, so the result does not
   *              depend on the order the tiles land in (run-to-run deterministic), and the fold's
   *              E[x^2] - mean^2 is taken in fp64 (no cancellation for rows with |mean| >> std);
   *   ln_rows    optional INPUT: [M][2] (sum, sumsq) of each row of a0 (a row_stats), with
   *              ln_c1 [n] = sum_k W'[n][k] (W' = W diag(gamma), the packed weight) and bias =
   *              W beta + b: out = rstd (acc - mean c1) + bias = Linear(LayerNorm(a0)), where
   *              mean = sum * ln_inv_k, rstd = 1 / sqrt(sumsq * ln_inv_k - mean^2 + ln_eps).
   * Either forces an unsplit 1x1 tile plan of the 2-blocks-per-CU kernel. */
  double* row_stats;
  const double* ln_rows;
  const float* ln_c1;
  float ln_inv_k;
  float ln_eps;
  /* GroupNorm(+activation) of the output applied by the split-K reduction in the same launch
   * (ldm_conv2d_gn_fusable says whether a call takes it; ldm_conv2d refuses gn_out otherwise).
   * Replaces: ldm_conv2d (split K, ResnetBlock2D conv1 / conv2 / Downsample2D at the 16x16 / 8x8 /
   * mid levels, unet.py:361-425) + the ldm_group_norm of its output (ResnetBlock2D norm2 / the next
   * block's norm1 / Transformer2DModel.norm).  One reduction block owns one image's 40-channel
   * segment (whole groups), sums the K slabs in split order, applies the epilogue, rounds to bf16,
   * takes exact fp64 per-unit (gn_unit channels) sums of the rounded values and forms each group's
   * (mean, rstd) from them exactly as ldm_group_norm does from a producer's accumulators — so gn_out
   * equals ldm_group_norm(out, those accumulators) bit for bit.  gn_partial, when set, receives the
   * same unit sums (slot 0; the other slots stay zero).
   * Scope: bf16, NHWC, no phase upsample, h_out * w_out in {32, 64, 128, 256}, n % 40 == 0,
   * group size n / gn_groups in {4, 8, 20, 40}, gn_unit dividing the group size. */
  void* gn_out;            /* NHWC bf16 [M][n] or NULL (off) */
  const float* gn_gamma;   /* [n] */
  const float* gn_beta;    /* [n] */
  int gn_groups;
  int gn_act;              /* LDM_ACT_NONE or LDM_ACT_SILU */
  float gn_eps;
  int gn_skip_out;         /* 1: `out` is not written (the pre-norm tensor is dead; out may alias gn_out) */
} ldm_conv_params;

/* Deep-K / few-tile shapes are split over K into an fp32 slab; this returns its size (0: none). */
size_t ldm_conv2d_workspace_bytes(const ldm_conv_params* p);
int ldm_conv2d(const ldm_conv_params* p, ldm_stream_t stream);
/* The kernel and tile plan ldm_conv2d would run for p (host only, no launch): out[0] kind
 * (0 tile kernel, 1 halo 3x3, 2 wide persistent 1x1, 3 A-register-stationary 1x1, 4 large
 * 256x160 tile), out[1] bm, out[2] bn, out[3] ksplit, out[4] LDS stages.  LDM_OK or the
 * validation error ldm_conv2d would return. */
int ldm_conv2d_describe_plan(const ldm_conv_params* p, int* out);
/* 1 when ldm_conv2d(p) with gn_out / gn_gamma / gn_beta / gn_groups set applies the GroupNorm in the
 * split-K reduction's launch (the plan splits K and the shape is in the fused kernel's scope), else 0
 * (host only, no launch). */
int ldm_conv2d_gn_fusable(const ldm_conv_params* p);
/* Tuning hook: the fewest reduction blocks (images x 40-channel segments) the fused GroupNorm takes
 * (default 16: every in-scope call; smaller grids keep the two launches). */
void ldm_conv2d_set_gn_fuse_min_blocks(int n);
/* Tuning hook (benchmarks and tests only, not thread-safe): force the tile plan of every
 * following ldm_conv2d call where it is legal — bm in {32, 64, 128} x bn in {32, 64, 128},
 * or bm = 256 for the large-tile bf16 kernel (bn 160); ksplit >= 1 (clamped).  bm = 0
 * restores the built-in heuristic.  Query ldm_conv2d_workspace_bytes after forcing. */
void ldm_conv2d_force_plan(int bm, int bn, int ksplit);
/* Tuning hook: LDS ring depth (3 or 4; 0 = planner's choice) of the 128x160 bf16 tile. */
void ldm_conv2d_force_stages(int stages);
/* Tuning hook: M panels per tile-raster group of ldm_conv2d (default 8; 1 = row-major tiles). */
void ldm_conv2d_set_raster_group(int group_m);
/* Tuning hook: the halo-tiled 3x3 kernel (bf16, stride 1, 64-channel-aligned sources, output
 * width 64 or 32: 4-row tiles; 16x16 images: whole-image tiles with K split over channel blocks
 * into an fp32 slab): 0 = planner's choice, 1 = never, 2 = whenever legal. */
void ldm_conv2d_set_halo(int mode);
/* Tuning hook: force the split-K factor of the 16x16 whole-image halo tiles (0 = planner). */
void ldm_conv2d_set_halo_split(int ksplit);
/* tuning hook: output rows per halo tile at the 32x32 level: 0 planner (8 for >= 1280 input channels,
 * else 4), 4 or 8 forced (8: 256-row tiles, K split over channel blocks as at the 16x16 level) */
void ldm_conv2d_set_halo_rows32(int rows);
/* Tuning hook: the A-register-stationary bf16 1x1 GEMM (K = 320, N a multiple of 160, NHWC or
 * GEGLU, no time embedding / GroupNorm partials): 0 = planner's choice (the 64x64 UNet level),
 * 1 = never, 2 = whenever legal. */
void ldm_conv2d_set_ars(int mode);
/* Tuning hook: the wide-tile persistent bf16 1x1 GEMM (256 x 320 tiles, one 8-wave block per CU
 * walking its tiles; N a multiple of 320, NHWC or GEGLU, no time embedding / split-K):
 * 0 = planner's choice (>= 256 tiles), 1 = never, 2 = whenever legal (256-row tiles),
 * 3 = whenever legal with 128-row tiles. */
void ldm_conv2d_set_wide(int mode);
/* Tuning hook: the deep-ring 1x1 GEMM of the 16x16 / 8x8 levels (csrc/gemm_ring.hip): 0 planner, 1 never,
   2 whenever legal. */
void ldm_conv2d_set_ring(int mode);
/* Tuning hook: K splits of the deep-ring kernel's implicit-GEMM 3x3 conv form (and, when > 0, of
   every ring call): 0 planner (toward one block per CU), > 0 forced (at most 16). */
void ldm_conv2d_set_ring_split(int ks);
/* Tuning hook: column width of the split-K reduction kernel's tiles — 0 = planner's choice
 * (64 when 128-wide tiles give fewer than 512 blocks), 64 or 128 forced. */
/* A/B hook: the tile kernel's fast operand addressing (per-row offsets computed once, the K position
 * as one wave-uniform add per K tile; tap-major 64-aligned K tiles or 64-aligned 1x1 convs with >= 8
 * K tiles, no upsampled gather): 4 = planner (default: convs, and 1x1 GEMMs of <= 320 blocks),
 * 1 = wherever it applies, 2 = convs only, 3 = 1x1 only, 0 = the general per-K-tile address walk.
 * Bit-identical in every mode. */
void ldm_conv2d_set_fast_addressing(int mode);
/* A/B hook: plans of 64-row tiles that give <= 256 blocks (config 2's deep levels) run the 4-stage LDS
 * ring (three K tiles in flight per block): 1 = on (default), 0 = two stages. */
void ldm_conv2d_set_fewblock_ring(int enabled);
void ldm_conv2d_set_splitk_cols(int cols);
/* Tuning hook: row count of the split-K reduction kernel's tiles — 0 = planner's choice (64, halved
 * down to 16 while the 64-column tiles give fewer than 512 blocks), 16, 32 or 64 forced (16 with
 * 128 columns runs 32). */
void ldm_conv2d_set_splitk_rows(int rows);
/* Tuning hook: bf16 NHWC epilogue of the 2-blocks-per-CU tiles — 0 = bias / time embedding /
 * activation applied from the accumulators and the tile staged once as bf16 (default),
 * 1 = fp32 staging in row halves (the round-1 form). */
void ldm_conv2d_set_epilogue(int mode);

/* ---------------------------------------------------------------------------------------
 * ldm_feedforward — the transformer block's FeedForward(GEGLU) as ONE launch: the two
 * ldm_conv2d calls it replaces, passed as they would be passed separately, with the [M][F]
 * GEGLU intermediate kept on chip (never written).
 * Replaces: diffusers BasicTransformerBlock  hidden = ff(norm3(hidden)) + hidden  —
 * ff.net.0 GEGLU proj + gelu gate, ff.net.2 Linear (unet.py:83-105 via 361-425).
 *   geglu: the ff.net.0 call — 1x1, a0 = x [M][320] bf16, w = GEGLU-packed [2F][320] (16-column
 *          hidden/gate interleave), bias packed likewise, out_layout LDM_OUT_GEGLU, out ignored
 *          (may be NULL); optional LayerNorm fold (ln_rows / ln_c1 / ln_inv_k / ln_eps);
 *   ff2:   the ff.net.2 call — 1x1, w = [320][F] (kpad = F = c0), bias, residual (may alias a0
 *          and out), out [M][320], optional row_stats; a0 ignored (the intermediate).
 * Scope: bf16, model width 320 (the 64x64 UNet level), F a multiple of 64 up to 1280; no time
 * embedding, activation, GroupNorm partials, split-K or fp32 output.  Results equal the two
 * separate calls bit for bit (same MFMA sequence per element, same bf16 rounding points).
 *   proj_out: optional (NULL = none) — Transformer2DModel.proj_out applied to the feed-forward's
 *          output as a third 1x1 call (320 -> 320, bias, residual = the transformer input,
 *          out, optional gn_partial / gn_unit / gn_slots; batch / h_out / w_out give the image
 *          of each row for the GroupNorm partials).  The feed-forward's output h then never
 *          reaches HBM: ff2's out may be NULL and its row_stats must be. */
int ldm_feedforward(const ldm_conv_params* geglu, const ldm_conv_params* ff2, const ldm_conv_params* proj_out,
                    ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_transformer_in — the input half of a Transformer2DModel as ONE launch: the GroupNorm
 * (Transformer2DModel.norm, from the producer's unit accumulators), proj_in, and norm1 folded
 * into the fused to_q/k/v GEMM.
 * Replaces: diffusers Transformer2DModel  h = proj_in(norm(x));  qkv = to_qkv(norm1(h))
 * (unet.py:361-425) — i.e. ldm_group_norm + ldm_conv2d(proj_in, row_stats) + ldm_conv2d(qkv, ln_rows).
 *   gn:      the GroupNorm: acc = the fp64 [batch][slots][C / unit][2] unit accumulators the
 *            producer's epilogue summed (ldm_conv2d gn_partial), groups, eps, gamma / beta [C];
 *            no activation (the transformer's GroupNorm has none);
 *   proj_in: 1x1, a0 = x [M][320] bf16 (the raw, un-normalised input), w [320][320], bias, out = h
 *            [M][320] (to_out's residual); batch / h_out / w_out: the images (h_out * w_out % 128 == 0);
 *   qkv:     1x1, w = the packed_ln_fold [960][320] weight, bias, ln_c1, ln_inv_k, ln_eps, out =
 *            qkv [M][960]; a0 and ln_rows are ignored (h and its row statistics stay on chip).
 * Scope: bf16, width 320 (the 64x64 UNet level).  h and qkv equal the three separate calls bit
 * for bit (same GroupNorm arithmetic, MFMA sequence per element, row-statistics summation order
 * and bf16 rounding points). */
typedef struct {
  const double* acc;       /* [batch][slots][C / unit][2] fp64 (sum, sumsq) */
  int unit, slots, groups;
  float eps;
  const float* gamma;      /* [C] */
  const float* beta;       /* [C] */
} ldm_gn_fold;
int ldm_transformer_in(const ldm_gn_fold* gn, const ldm_conv_params* proj_in, const ldm_conv_params* qkv,
                       ldm_stream_t stream);
/* Tuning / A-B hook: kernel variant of ldm_transformer_in (1 = default; see csrc/transformer_in.hip). */
void ldm_transformer_in_set_mode(int mode);

/* ---------------------------------------------------------------------------------------
 * ldm_conv_in — the UNet's conv_in straight from the sampler's NCHW sources, in one launch.
 * Replaces: ldm_nchw_to_nhwc([x_t || rgb (|| cond)], trainers_ldm_cond.py:1134-1141) + ldm_conv2d of
 * the 8 / 12-channel conv_in (unet.py:357, built by modify_encoder :178-233).
 *   src[i], c[i], src_dtype[i]: up to three NCHW [batch][c_i][height][width] tensors (fp32 or bf16),
 *     concatenated over channels (<= 16 in all), each value rounded to bf16 as ldm_nchw_to_nhwc stores it;
 *   w: ldm_conv2d's packed [n][kpad] bf16 weight of the 3x3 conv with 16 (zero-padded) input channels
 *     (k = (ky, kx, c)), bias [n] fp32; out: NHWC bf16 [batch][height][width][n];
 *   gn_partial / gn_unit / gn_slots: as ldm_conv2d's (the zeroed fp64 GroupNorm accumulators the
 *     next ldm_group_norm consumes; each output row adds to slot row % gn_slots), or NULL.
 * Scope: dtype bf16, width <= 64 and % 16 == 0, n % 64 == 0 and <= 320. */
typedef struct {
  const void* src[3];
  int c[3];
  int src_dtype[3];
  int batch, height, width;
  int dtype;                   /* LDM_BF16 */
  const void* w;
  int n, kpad;
  const float* bias;
  void* out;
  double* gn_partial;
  int gn_unit, gn_slots;
} ldm_conv_in_params;
int ldm_conv_in(const ldm_conv_in_params* p, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_attention — fused multi-head scaled-dot-product attention (online softmax, MFMA).
 * Replaces: diffusers Attention(AttnProcessor) self-attention attn1 (and cross-attention
 * attn2 when not removed, unet.py:83-105): softmax(Q K^T * scale) V per (batch, head).
 * Row r of batch b, head h lives at ptr + (b * n + r) * stride + h * head_dim.
 * ------------------------------------------------------------------------------------- */
typedef struct {
  const void* q; const void* k; const void* v; void* o;
  int q_stride, k_stride, v_stride, o_stride;  /* elements between consecutive rows */
  int batch, heads, head_dim;                   /* head_dim <= 160 */
  int n_q, n_kv;
  float scale;
  int dtype;
} ldm_attn_params;

int ldm_attention(const ldm_attn_params* p, ldm_stream_t stream);
/* As ldm_attention, with a caller workspace that lets the bf16 head_dim-40 / 80 / 160 paths split the keys
 * when the (batch, heads, n_q) grid alone would leave the GPU under-occupied (a single frame of the
 * 64x64 level: 128 eight-wave query blocks; of the 32x32 level: 32; of the 16x16 level: 32 four-wave
 * blocks of the 16x16x32 head_dim-160 kernel): each split writes a normalised fp32 partial and its
 * log-sum-exp to the workspace and a merge kernel combines them (same math, different fp32
 * summation order).  ldm_attention_workspace_bytes returns 0 when no split applies; then the call
 * is exactly ldm_attention and the workspace may be NULL. */
size_t ldm_attention_workspace_bytes(const ldm_attn_params* p);
int ldm_attention_ws(const ldm_attn_params* p, void* workspace, int64_t workspace_bytes, ldm_stream_t stream);
/* Tuning / A-B hook for the split: -1 planner (default), 0 or 1 off, k >= 2 forced (at most 8 and
 * n_kv / 128 splits). */
void ldm_attention_set_kvsplit(int splits);
/* Tuning / A-B hook: 1 (default) runs the head_dim-80 32x32x16 kernel with the key-tile loop unrolled
 * by two (compile-time K / V buffer per tile; bit-identical), 0 the one-tile loop; 2 / 3: 128-key
 * tiles without / with the unrolled loop (A/B). */
void ldm_attention_set_pair(int enabled);
/* BASELINE config 5 ("fp8 MFMA attention", pose-conditioned video LDM at T=16): as ldm_attention
 * (bf16 inputs and output).
 *   head_dim 40 (16-byte row strides): BOTH products on the block-scaled
 *     v_mfma_scale_f32_32x32x64_f8f6f4 (2x the bf16 MFMA rate) — Q * scale * log2(e), K, V and P
 *     rounded to OCP e4m3 (unit E8M0 scales), fp32 accumulation, softmax in fp32.  K and V are
 *     quantized once per call into the caller's workspace (ldm_attention_fp8_workspace_bytes).
 *   other head dims: P.V on the non-scaled e4m3 MFMA (issues at the bf16 rate on gfx950; an
 *     accuracy mode), Q.K^T bf16; the workspace is unused (may be NULL). */
size_t ldm_attention_fp8_workspace_bytes(const ldm_attn_params* p);
int ldm_attention_fp8(const ldm_attn_params* p, void* workspace, int64_t workspace_bytes, ldm_stream_t stream);
/* Tuning / A-B hook: 0 sends head_dim 40 to the non-scaled P.V path as well (default 1). */
void ldm_attention_set_fp8_scaled(int enabled);
/* Tuning hook (benchmarks / tests only): 1 routes bf16 through the 16x16x16-MFMA kernel
 * instead of the 16x16x32 one; 0 restores the default. */
void ldm_attention_force_legacy(int legacy);
/* Tuning / A-B hook: 1 (default) runs head_dim 80 on the 32x32x16 kernel of head_dim 40, 0 on the
 * 16x16x32 one. */
void ldm_attention_set_d80(int enabled);
/* Tuning / A-B hook: 1 runs head_dim 160 on the 32x32x16 kernel of head_dim 40 (4 waves, 376
 * registers per lane: one block per CU; split-KV through ldm_attention_ws), 0 (default: measured
 * faster in the step) on the 16x16x32 one. */
void ldm_attention_set_d160(int enabled);
/* tuning / A-B hook: head_dim 40 with 64 queries per wave (two 32-query subtiles sharing every
 * K / V fragment read; 8 waves, one block per CU) */
void ldm_attention_set_qs2(int enabled);
/* A/B hook: head_dim 40 with >= 256 blocks of 64 queries (the headline's and config 5's top level) on the
 * two-subtile kernel whose subtiles' MFMA and softmax phases interleave inside each wave (1, default),
 * or on the 32-query kernel (0); the interleaved kernel runs 128-key tiles (two 64-key halves per
 * barrier); 2 / 3: on 64- / 256-key tiles (A/B); all bit-identical. */
void ldm_attention_set_il(int enabled);
/* Tuning / A-B hook: the head_dim 40 / 80 kernels with the block's waves in two phases half an
 * iteration apart (the upper half runs softmax + P.V of tile t - 1, then Q.K^T of tile t, beside the
 * lower half's tile t; three K/V buffers; bit-identical): 0 = planner's choice, 1 = off, 2 = on,
 * 3 = the default head_dim-40 kernel held to one block per CU (the equal-occupancy reference). */
void ldm_attention_set_skew(int mode);
/* Tuning / A-B hook: 1 (default) runs the bf16 backward for head_dim <= 64 on the 32x32x16 MFMA
 * kernels, 0 on the 16x16x16 ones. */
void ldm_attention_set_bwd32(int enabled);
/* Tuning hook (A/B only), head_dim 40: 2 (default) the 32x32x16-MFMA kernel; 1 the 16x16x32 kernel
 * with the softmax scale and running max carried in the Q.K^T head-dim padding; 0 the 16x16x32
 * kernel with one FMA per score. */
void ldm_attention_set_maxcol(int mode);
/* Tuning hook: waves per block of the bf16 flash-attention kernel (4 or 8; 0 = automatic). */
void ldm_attention_set_waves(int waves);
/* Training forward: as ldm_attention, and also stores lse[(b * heads + h) * n_q + q] =
 * log2-domain row log-sum-exp of the scaled scores (max2 + log2(l)), consumed by the backward. */
int ldm_attention_fwd_lse(const ldm_attn_params* p, float* lse, ldm_stream_t stream);
/* Backward of ldm_attention (the autograd of diffusers Attention's softmax(QK^T s)V that the
 * reference training step differentiates, trainers_ldm_cond.py:851-856): given o, do and lse,
 * writes dq/dk/dv (same row layout/strides as q/k/v; may be column slices of one [N][3C]
 * tensor).  workspace: >= ldm_attention_bwd_workspace_bytes(p) bytes. */
size_t ldm_attention_bwd_workspace_bytes(const ldm_attn_params* p);
int ldm_attention_bwd(const ldm_attn_params* p, const void* o, const void* d_o, int do_stride, const float* lse,
                      void* dq, void* dk, void* dv, int dq_stride, int dkv_stride, void* workspace,
                      ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_group_norm — GroupNorm (+ optional SiLU) over NHWC rows of one or two channel-
 * concatenated sources (the up-block [hidden || skip] concat is never materialised).
 * Replaces: ResnetBlock2D norm1/norm2 + SiLU (eps 1e-5), Transformer2DModel.norm (eps 1e-6),
 * conv_norm_out + conv_act (unet.py:428-430), GeneralVAESeg GroupNorm (vae.py:163,235).
 * stats0/stats1: the fp64 (sum, sumsq) accumulators [batch][stats_slots][c_i / stats_unit][2]
 * that ldm_conv2d's epilogue summed for x0 / x1 (gn_partial, gn_unit = stats_unit, gn_slots =
 * stats_slots), or NULL to compute them here (an extra read of the tensor).  stats_unit must
 * divide c0 and the group size.
 * One kernel when both are given: every block reduces its batch's accumulators to per-group
 * mean / rstd in LDS while its first rows are in flight, then streams its rows.
 * workspace: >= ldm_group_norm_workspace_bytes(batch, hw, c0 + c1) bytes of device memory.
 * ------------------------------------------------------------------------------------- */
size_t ldm_group_norm_workspace_bytes(int batch, int hw, int channels);
int ldm_group_norm(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups,
                   const float* gamma, const float* beta, float eps, int act, void* out,
                   const double* stats0, const double* stats1, int stats_unit, int stats_slots, void* workspace,
                   int dtype, ldm_stream_t stream);
/* Training forward: also stores (mean, rstd) per (batch, group) [batch][groups] float2. */
int ldm_group_norm_ex(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups,
                      const float* gamma, const float* beta, float eps, int act, void* out,
                      const double* stats0, const double* stats1, int stats_unit, int stats_slots,
                      void* workspace, float* save_mean_rstd, int dtype, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_layer_norm — LayerNorm over the channel dimension of [rows][c] (NHWC pixels or tokens).
 * Replaces: BasicTransformerBlock norm1/norm2/norm3 (eps 1e-5) and LayerNorm2d
 * (vae.py:310-323, eps 1e-6), optionally followed by SiLU (vae.py:158).
 * ------------------------------------------------------------------------------------- */
int ldm_layer_norm(const void* x, int rows, int c, const float* gamma, const float* beta,
                   float eps, int act, void* out, int dtype, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_unet_tail — the UNet tail in one launch (unet.py:428-431): GroupNorm(conv_norm_out) ->
 * SiLU -> conv_out (3x3, pad 1, c -> cout <= 4) -> NCHW model output, optionally followed by the
 * sampler's DDIM step on it (ddim_scheduler.py:218-269; the ldm_ddim_step arithmetic).
 * h: bf16 NHWC [batch][height][width][c] with its producer's GroupNorm accumulators (ldm_conv2d
 * gn_partial: fp64 [batch][gn_slots][c / gn_unit][2]); height % 2 == 0, width % 16 == 0,
 * width <= 64, c % 64 == 0, c <= 640, groups <= 64.  w: the conv_out weight packed as ldm_conv2d
 * takes it (bf16 [cout][kpad], k = (ky, kx, c)).  eps_out (optional when the DDIM step is fused):
 * NCHW [batch][cout][height][width] in eps_dtype; the model output is rounded to eps_dtype
 * before the DDIM step, as the unfused path stores it.  prev / x0 (either may be NULL; both
 * NULL: no DDIM step): NCHW in out_dtype; sample NCHW in sample_dtype.
 * ------------------------------------------------------------------------------------- */
typedef struct {
  const void* h;
  int batch, height, width, c;
  const double* gn_acc;
  int gn_unit, gn_slots, groups;
  float eps;
  const float* gamma;
  const float* beta;
  const void* w;
  int kpad, cout;
  const float* bias;
  void* eps_out;
  int eps_dtype;
  const void* sample;
  int sample_dtype;
  const int64_t* t;                      /* device int64 [1] */
  const float* alphas_cumprod;
  float final_alpha_cumprod;
  int step_ratio, prediction_type, clip_sample;
  float clip_range;
  int use_clipped_model_output, num_train_timesteps;
  void* prev;
  void* x0;
  int out_dtype;
} ldm_unet_tail_params;

int ldm_unet_tail(const ldm_unet_tail_params* p, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_linear_rows — out[m][:] = act(x[m] . W^T + bias) for rows <= 16 (the time-embedding MLP:
 * diffusers TimestepEmbedding linear_1 / linear_2 and the batched ResnetBlock2D time_emb_proj,
 * unet.py:301-307 and every resnet's temb input).  x bf16 [rows][k]; x == NULL takes the row
 * as the sinusoidal projection of t (the ldm_timestep_proj values rounded to bf16, dim = k <= 512).
 * W packed bf16 [n][kpad] (n % 16 == 0, k % 32 == 0, k <= 1536), bias fp32 [n] or NULL,
 * out [rows][n] fp32 or bf16 (16-byte aligned).
 * ------------------------------------------------------------------------------------- */
int ldm_linear_rows(const void* x, const float* t, int n_t, const float* freqs, int flip_sin_to_cos,
                    const void* w, int kpad, int k, int n, const float* bias, int rows, int act, void* out,
                    int out_dtype, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_timestep_proj — sinusoidal timestep projection (diffusers Timesteps, unet.py:305):
 * out[b, :] = flip? [cos(t_b f) || sin(t_b f)] : [sin || cos],  f = freqs[0..dim/2).
 * t is read on the device (fp32 [n_t], n_t == 1 broadcasts over batch: unet.py:303), so
 * the DDIM loop never syncs to the host.
 * ------------------------------------------------------------------------------------- */
int ldm_timestep_proj(const float* t, int n_t, int batch, const float* freqs, int dim,
                      int flip_sin_to_cos, void* out, int dtype, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_ddim_step — fused DDIM reverse step (ldmseg/schedulers/ddim_scheduler.py:218-269).
 * Coefficients are derived on the device from t (int64, device) and the alphas_cumprod
 * table (fp32, device), so a device-resident timestep costs no host sync (the reference
 * indexes a CPU table with a device scalar every step).
 * Tensors: model_output (mo_dtype), sample (x_dtype) -> prev, x0 (out_dtype); n elements.
 * ------------------------------------------------------------------------------------- */
enum { LDM_PRED_EPSILON = 0, LDM_PRED_SAMPLE = 1, LDM_PRED_V = 2 };
typedef struct {
  const void* model_output; int mo_dtype;
  const void* sample; int x_dtype;
  void* prev; void* x0; int out_dtype;   /* either may be NULL */
  int64_t n;
  const int64_t* t;                      /* device scalar */
  const float* alphas_cumprod;           /* device [num_train_timesteps] */
  float final_alpha_cumprod;
  int step_ratio;                        /* num_train_timesteps // num_inference_steps */
  int prediction_type;
  int clip_sample; float clip_range;
  int use_clipped_model_output;
  int num_train_timesteps;               /* table length; an out-of-range t yields NaN, never an OOB read */
} ldm_ddim_step_params;

int ldm_ddim_step(const ldm_ddim_step_params* p, ldm_stream_t stream);

/* add_noise (:155-187) / remove_noise (:189-216): per-sample timesteps t[batch], device. */
int ldm_ddim_add_noise(const void* x0, const void* noise, const int64_t* t, const float* alphas_cumprod,
                       int num_train_timesteps, float scale, int batch, int64_t per_sample, void* out,
                       int dtype, ldm_stream_t stream);
int ldm_ddim_remove_noise(const void* xt, const void* noise, const int64_t* t, const float* alphas_cumprod,
                          int num_train_timesteps, float scale, int batch, int64_t per_sample, void* out,
                          int dtype, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Bit-channel mask codec (bit-exact). Replaces Cityscapes/KITTI encode_bitmap /
 * decode_bitmap (ldmseg/data/cityscapes.py:256-270, kitti.py:292-306, coco.py:378-391).
 * encode: ids int64 [batch][hw] -> planes fp32 [batch][n][hw] (+ ignore mask uint8 [batch][hw])
 * decode: planes [batch][n][hw] (dtype) -> ids int64 [batch][hw]; drop_31: v == 31 -> 0.
 * ------------------------------------------------------------------------------------- */
int ldm_bit_encode(const int64_t* ids, int batch, int64_t hw, int n, int64_t ignore_label,
                   float fill_value, float* planes, uint8_t* ignore_mask, ldm_stream_t stream);
int ldm_bit_decode(const void* planes, int batch, int n, int64_t hw, int drop_31, int64_t* ids,
                   int dtype, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * ldm_softmax_rows — p[r][j] = softmax_j(scale * s[r][j]) over the first n of `stride` columns
 * (fp32 in, fp32 math — diffusers upcast_softmax), written with zeros in columns [n, stride) so
 * p can be the K-padded A operand of the following P.V GEMM.  Replaces the softmax of the
 * AutoencoderKL mid-block attention (single head, head_dim 512 > the flash kernel's 160).
 * n <= 8192.
 * ------------------------------------------------------------------------------------- */
int ldm_softmax_rows(const float* s, int rows, int n, int stride, float scale, void* p, int dtype,
                     ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * AE training (row a16): the point losses of SegmentationLosses.point_loss
 * (ldmseg/trainers/losses.py:117-395, detectron2_utils.py:20-100) and VAE-backward helpers.
 * A "box" is one image (C planes, planes == NULL) or one mask (the single plane planes[box]).
 * coords: [boxes][p] float2 in [0, 1]^2 (x, y), as point_sample takes them.
 * ldm_point_sample:      out[box][c][p] = grid_sample(bilinear, zeros, align_corners=False).
 * ldm_point_sample_bwd:  din += adjoint (atomic), point gradients scaled by scale * *scale_ptr.
 * ldm_point_labels:      mode 0: int64 labels by nearest sampling of targets [img][h][w] (zeros
 *                        padding); mode 1: fp32 bilinear sample of (targets[img[box]] == cls[box]).
 * ldm_point_uncertainty: u = top2[1] - top2[0] over c (c > 1) or -|x| (c == 1).
 * ldm_topk_select:       idx[row][k] = indices of the k largest u[row][:n] (ties at the k-th value in
 *                        index order; the set, not the order, is specified); coords_out[row][k] the
 *                        gathered coords (optional).
 * ldm_point_ce:          acc = (sum of CE over non-ignored points, their count) as doubles; grad =
 *                        (softmax(x / T) - onehot) / T (0 at ignored points), unscaled by the count.
 * ldm_point_bce_dice:    acc = (sum over masks of mean BCE, sum of dice); grad = d(bce_mean + dice)/dx.
 * ldm_silu:              out = silu(z) (dy == NULL) or dy * silu'(z).
 * ldm_space_to_depth2:   [b][2h][2w][c] -> [b][h][w][(dy, dx, c)] (ConvTranspose k2s2 backward).
 * ldm_posterior_sample / _bwd: z = mean + exp(clamp(logvar, -30, 20) / 2) * eps from NCHW fp32
 *                        moments; the backward reads dz from NHWC rows of c_stride channels.
 * ------------------------------------------------------------------------------------- */
int ldm_point_sample(const float* in, int boxes, int c, int h, int w, const int32_t* planes, const float* coords,
                     int p, float* out, ldm_stream_t stream);
int ldm_point_sample_bwd(const float* dout, int boxes, int c, int h, int w, const int32_t* planes,
                         const float* coords, int p, const float* scale_ptr, float scale, float* din,
                         ldm_stream_t stream);
int ldm_point_labels(const int64_t* targets, int h, int w, const int32_t* img, const int32_t* cls,
                     const float* coords, int boxes, int p, int mode, int64_t* labels, float* values,
                     ldm_stream_t stream);
int ldm_point_uncertainty(const float* x, int boxes, int c, int p, float* u, ldm_stream_t stream);
int ldm_topk_select(const float* u, int rows, int n, int k, const float* coords, int32_t* idx, float* coords_out,
                    ldm_stream_t stream);
int ldm_point_ce(const float* x, const int64_t* labels, int boxes, int c, int p, float temperature,
                 int64_t ignore_label, double* acc, float* grad, ldm_stream_t stream);
int ldm_point_bce_dice(const float* x, const float* y, int masks, int p, double* acc, float* grad,
                       ldm_stream_t stream);
int ldm_silu(const void* z, const void* dy, int64_t n, void* out, int dtype, ldm_stream_t stream);
int ldm_space_to_depth2(const void* d, int batch, int h, int w, int c, void* out, int dtype, ldm_stream_t stream);
int ldm_posterior_sample(const float* moments, const float* eps, int batch, int latent, int hw, float* z,
                         ldm_stream_t stream);
int ldm_posterior_bwd(const float* moments, const float* eps, const void* dz, int c_stride, int batch, int latent,
                      int hw, float* dmoments, int dtype, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Panoptic head (config 4 post-processing).
 * Replaces: the per-image CPU loop of TrainerDiffusion.compute_pq
 * (ldmseg/trainers/trainers_ldm_cond.py:1287-1330) and the argmax / confidence threshold of
 * decode_latents (:426-435).  logits: NCHW fp32 [batch][k][hw].
 * ldm_panoptic_pixels: pred[b][p] = argmax_k (first maximal index), set to ignore_label where
 *   the confidence (conf_mode 1: max softmax prob, 2: top1 - top2 prob; 0: no threshold)
 *   is < mask_th; counts[b][k] = #(pred == k); mask_counts[b][k] = #(sigmoid(logit_k) >= mask_th).
 *   counts / mask_counts are zeroed here (async memset on `stream`).
 * ldm_panoptic_finalize: keep[b][k] = k != ignore_label && counts >= count_th &&
 *   !(counts / mask_counts < overlap_th) (float64; a zero mask count keeps the label, as
 *   numpy's inf does); out[b][p] = keep[pred] ? pred + 1 : 0  (the reference's cleaned_pred + 1).
 * k <= 1024.
 * ------------------------------------------------------------------------------------- */
int ldm_panoptic_pixels(const float* logits, int batch, int k, int hw, int conf_mode, float mask_th,
                        int ignore_label, int32_t* pred, int32_t* counts, int32_t* mask_counts,
                        ldm_stream_t stream);
int ldm_panoptic_finalize(const int32_t* pred, const int32_t* counts, const int32_t* mask_counts,
                          int batch, int k, int hw, int count_th, double overlap_th, int ignore_label,
                          int32_t* keep, int32_t* out, ldm_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * Layout / resampling helpers on the path boundary.
 * ldm_nchw_to_nhwc: gathers up to 3 NCHW sources (the sampler's [x_t || rgb || cond] concat,
 * trainers_ldm_cond.py:1134-1141) into one NHWC tensor with c_pad channels (zero filled).
 * ldm_resize_bilinear: F.interpolate(mode='bilinear', align_corners=False) on NCHW
 * (vae.py:271, trainers_ldm_cond.py:343,380-392); optional affine y = x*mul + add.
 * ldm_gaussian_posterior: DiagonalGaussianDistribution (vae.py:371-415) from NHWC moments.
 * ------------------------------------------------------------------------------------- */
int ldm_nchw_to_nhwc(const void* s0, int c0, int dt0, const void* s1, int c1, int dt1,
                     const void* s2, int c2, int dt2, int batch, int hw, int c_pad,
                     void* out, int dtype, ldm_stream_t stream);
int ldm_resize_bilinear(const void* x, int planes, int h_in, int w_in, int h_out, int w_out,
                        float scale_h, float scale_w, float mul, float add, void* out,
                        int in_dtype, int out_dtype, ldm_stream_t stream);
enum { LDM_POST_NONE = 0, LDM_POST_TANH = 1, LDM_POST_SIGMOID = 2, LDM_POST_CLIP = 3 };
int ldm_gaussian_posterior(const void* moments, int batch, int hw, int latent_channels,
                           int clamp_output, int act_fn, float* mean, float* logvar, float* std,
                           float* var, int dtype, ldm_stream_t stream);


/* =======================================================================================
 * Training path: backward of the fused forward ops and the
 * optimizer step.  Replaces the torch autograd backward + AdamW of the reference training
 * step (trainers_ldm_cond.py:792-900: compute_loss :530-619, loss.backward :851-856,
 * update_weights :769-781 = clip_grad_norm_ + AdamW from trainers/optim.py:53-82).
 * Gradients of weights / affine params are fp32; activation gradients use the compute dtype.
 * ======================================================================================= */

/* ldm_conv2d_wgrad — weight gradient of ldm_conv2d: dW[n][k] = sum_m dY[m][n] * A[m][k] with the
 * same implicit im2col A as the forward (geometry fields as ldm_conv_params; upsample 0/1).
 * dy: NHWC [batch*h_out*w_out][n] (compute dtype, n % 8 == 0 for bf16).  dw: fp32 in the torch
 * layout [n][cin_real][ksize][ksize] (ksize 1: [n][cin_real]); geglu: dy columns are the packed
 * GEGLU interleave and dw rows are written un-interleaved; accumulate: dw += instead of =. */
typedef struct {
  const void* a0; const void* a1; int c0, c1;
  int batch, h_in, w_in, h_out, w_out, ksize, stride, upsample;
  const void* dy; int n; int kpad;
  int cin_real, geglu;
  float* dw; int accumulate;
  int dtype;
  void* workspace; int64_t workspace_bytes;
} ldm_wgrad_params;
size_t ldm_conv2d_wgrad_workspace_bytes(const ldm_wgrad_params* p);
int ldm_conv2d_wgrad(const ldm_wgrad_params* p, ldm_stream_t stream);
/* Tuning / A-B hook: 1 (default) runs the bf16 weight gradient on a ring of four 32-pixel LDS
 * stages (three in flight), 0 on two 64-pixel stages, 2 on five 32-pixel stages (stride-1 convs). */
void ldm_conv2d_wgrad_set_ring(int ring);
/* A-B hook: 1 (default) = stride-1 weight gradients load their operands by per-lane pointers
 * advanced 16 rows per DMA (branch-free); 0 = the general pixel-decoding loader everywhere. */
void ldm_conv2d_wgrad_set_fast_loader(int on);
/* A-B hook: 1 (default) = 3x3 slab sums by wave-owned [64 channel][9 tap] blocks written as
 * contiguous runs; 0 = one packed element per thread (stores 36 bytes apart). */
void ldm_conv2d_wgrad_set_reduce3(int on);

/* ldm_colsum — out[s][c] (+)= sum over the rows of segment s of x[rows][c] (segments split the
 * rows evenly).  Bias gradients (1 segment) and per-batch time-embedding gradients (batch
 * segments).  geglu: columns are the packed GEGLU interleave, out is un-interleaved. fp32 out.
 * Deterministic: 128-row chunks write an fp32 slab (workspace, ldm_colsum_workspace_bytes)
 * that a second pass sums in chunk order — no atomics, bit-identical run to run. */
size_t ldm_colsum_workspace_bytes(int rows, int c, int segments);
int ldm_colsum(const void* x, int rows, int c, int segments, int geglu, float* out, int accumulate,
               void* workspace, int dtype, ldm_stream_t stream);

/* ldm_group_norm_bwd — backward of ldm_group_norm_ex (act NONE or SILU) given the saved
 * (mean, rstd).  dx of the two sources goes to dx0 [rows][c0] / dx1 [rows][c1]; acc0/acc1 add
 * into what they hold; add_src (optional, [rows][c0+c1]) is added too (a parallel branch's
 * gradient, e.g. a conv_shortcut dgrad).  dgamma/dbeta fp32 [C] (accumulated if acc_params). */
size_t ldm_group_norm_bwd_workspace_bytes(int batch, int hw, int channels, int groups);
int ldm_group_norm_bwd(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups,
                       const float* mean_rstd, const float* gamma, const float* beta, int act,
                       const void* dy, const void* add_src, void* dx0, void* dx1, int acc0, int acc1,
                       float* dgamma, float* dbeta, int acc_params, void* workspace, int dtype,
                       ldm_stream_t stream);

/* ldm_layer_norm_bwd — LayerNorm backward over [rows][c]; dx = LN'(dy) + add_src (the residual
 * stream's gradient).  dgamma/dbeta fp32 [c] (acc_params: +=).  Deterministic: per-block partials
 * to a slab (workspace, ldm_layer_norm_bwd_workspace_bytes) summed in block order. */
size_t ldm_layer_norm_bwd_workspace_bytes(int rows, int c);
int ldm_layer_norm_bwd(const void* x, const void* dy, int rows, int c, const float* gamma, float eps,
                       const void* add_src, void* dx, float* dgamma, float* dbeta, int acc_params,
                       void* workspace, int dtype, ldm_stream_t stream);

/* ldm_geglu — diffusers GEGLU on the packed GEMM output hg [rows][2f] ([h16 | g16] blocks):
 * dout == NULL: out[rows][f] = h * gelu(g);  else dhg[rows][2f] = (dout gelu(g), dout h gelu'(g)). */
int ldm_geglu(const void* hg, const void* dout, int rows, int f, void* out, void* dhg, int dtype,
              ldm_stream_t stream);

/* ldm_sum_pool2 — NHWC 2x2 sum pooling [batch][2h][2w][c] -> [batch][h][w][c] (data gradient of
 * the Upsample2D nearest-2x); accumulate: out +=. */
int ldm_sum_pool2(const void* x, int batch, int h_out, int w_out, int c, void* out, int accumulate, int dtype,
                  ldm_stream_t stream);

/* ldm_mse_loss — trainers_ldm_cond.py:592-604 (l2, ohem_ratio 1): per element
 * l = (pred - target)^2 * mask[b][pix] * weights[t[b]]; *loss_sum = sum l (fp64, device);
 * dpred = 2 (pred - target) mask w * grad_scale (NULL: loss only).  pred/dpred NCHW in dtype,
 * target fp32 NCHW, mask fp32 [batch][hw] or NULL, weights fp32 [num_weights] or NULL. */
int ldm_mse_loss(const void* pred, const float* target, const float* mask, const int64_t* t,
                 const float* weights, int num_weights, int batch, int ch, int hw, float grad_scale,
                 void* dpred, double* loss_sum, void* workspace, int dtype, ldm_stream_t stream);

/* ldm_sq_norm — *sum (+)= sum g^2 over a flat fp32 buffer (fp64 accumulation, device). */
int ldm_sq_norm(const float* g, int64_t n, double* sum, int accumulate, void* workspace, ldm_stream_t stream);

/* ldm_repack — refresh packed weights in place from their fp32 source parameters (the training
 * step, after each optimizer update), one launch over a device array of descriptors.  Tile index
 * space: descriptor i covers tiles [chunk0_i, chunk0_{i+1}) (chunk0 ascending, starting at 0);
 * modes 0 / 1 have ceil(rows / 16) * ceil(cpad / 64) tiles (16 destination rows x 64 channels,
 * every tap), mode 2 ceil(rows / 2048).
 *   mode 0: forward pack, bf16 dst[row0 + r][kpad], r < rows: dst[..][(ky*ks + kx)*cpad + c] =
 *           W[r'][c][ky][kx] (W fp32 [co][ci][ks][ks]; r' = r, or the GEGLU 16-interleave's source
 *           row when geglu; zero where r' >= co, c >= ci or the tap is past ks*ks)
 *   mode 1: data-gradient pack (ldmseg packed_dgrad): dst[row0 + r][(ky*ks + kx)*cpad + c] =
 *           W[c'][r][ks-1-ky][ks-1-kx], r < rows = ci, c' = c or its GEGLU source row, c < co
 *   mode 2: fp32 vector dst[row0 + j] = src[j'] for j < rows (j' = j or its GEGLU source row,
 *           co = the vector length).  rows = elements.
 * ks <= 3; cpad a multiple of 8.  f32: modes 0 / 1 write fp32 packs (the exact-fp32 compute path)
 * instead of bf16.  Replaces the torch re-pack of every trainable weight after
 * trainers_ldm_cond.py:769-781's optimizer step. */
typedef struct {
  const float* src;
  void* dst;
  int64_t chunk0;
  int rows, row0, kpad, co, ci, ks, cpad, mode, geglu, f32;
} ldm_repack_desc;
int ldm_repack(const ldm_repack_desc* descs, int ndesc, int64_t total_tiles, ldm_stream_t stream);

/* Workspace of ldm_mse_loss / ldm_sq_norm: per-block fp64 partials, summed in a fixed order by a
 * second one-block pass (deterministic; no atomics). */
size_t ldm_reduce_workspace_bytes(void);

/* ldm_adamw — torch.optim.AdamW step over flat fp32 buffers (param, grad, exp_avg, exp_avg_sq).
 * segments: device array of {int64 begin, int64 end, float lr, float weight_decay} (24 B each,
 * sorted, per-parameter hyper-parameters of trainers/optim.py get_optimizer_params);
 * sqsum (device, may be NULL) + max_norm > 0 applies clip_grad_norm_'s coefficient. */
int ldm_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const void* segments, int nseg,
              int64_t n, float beta1, float beta2, float eps, int step, const double* sqsum, float max_norm,
              ldm_stream_t stream);

const char* ldm_status_string(int status);
int ldm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LDMSEG_HIP_H */
