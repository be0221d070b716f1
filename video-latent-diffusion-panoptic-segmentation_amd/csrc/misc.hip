// Elementwise / boundary kernels of the denoising path: timestep projection, fused DDIM
// step / add_noise / remove_noise, bit-channel mask codec, NCHW->NHWC input gather,
// bilinear resize and the seg-VAE gaussian posterior.  All HBM-bound; one thread per
// element (or per pixel), grid-stride, no host synchronisation (graph-capturable).
#include "common.h"

namespace {

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline unsigned grid_for(int64_t n, int64_t cap = 256 * 32) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  return (unsigned)std::min<int64_t>(b, cap);
}

template <typename T>
__device__ __forceinline__ float ld(const void* p, int64_t i) {
  return to_f(reinterpret_cast<const T*>(p)[i]);
}
__device__ __forceinline__ float ld_dt(const void* p, int64_t i, int dt) {
  return dt == LDM_BF16 ? ld<bf16_t>(p, i) : ld<float>(p, i);
}
__device__ __forceinline__ void st_dt(void* p, int64_t i, float v, int dt) {
  if (dt == LDM_BF16) reinterpret_cast<bf16_t*>(p)[i] = f2bf(v);
  else reinterpret_cast<float*>(p)[i] = v;
}
// torch semantics: a fp32 table cast to the sample dtype before use (ddim_scheduler.py:168,202)
__device__ __forceinline__ float table_in_dtype(float a, int dt) { return dt == LDM_BF16 ? bf2f(f2bf(a)) : a; }

// ------------------------------------------------------------------ timestep projection
__global__ void tproj_kernel(const float* __restrict__ t, int n_t, int batch, const float* __restrict__ freqs,
                             int dim, int flip, void* out, int dtype) {
  const int half = dim / 2;
  const int64_t total = (int64_t)batch * dim;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int b = (int)(i / dim), j = (int)(i - (int64_t)b * dim);
    const float tv = t[n_t == 1 ? 0 : b];
    const int f = j < half ? j : j - half;
    const float arg = tv * freqs[f];
    const bool first = j < half;
    // layout [sin || cos], flipped to [cos || sin] when flip_sin_to_cos
    const bool use_cos = flip ? first : !first;
    st_dt(out, i, use_cos ? cosf(arg) : sinf(arg), dtype);
  }
}


// ------------------------------------------------------------------ few-row linear (time embedding)
// out[m][n] = act(x[m] . W[n] + bias[n]) for rows <= 16: the time-embedding MLP (diffusers
// TimestepEmbedding linear_1 / linear_2, unet.py:305-307) and the batched time_emb_proj of every
// ResNet — GEMV-shaped (B = 8 rows), bound by streaming the packed weight once.  One 16-column group
// per block; the block's four waves split K into k32 steps and issue every weight / input load of
// their share before the first MFMA (v_mfma_f32_16x16x32_bf16, rows padded to 16); the four partial
// tiles are summed in a fixed order through LDS.  x == NULL: the input row is the sinusoidal timestep
// projection (diffusers Timesteps, the tproj_kernel values rounded to bf16) computed in place.
constexpr int LR_MAXS = 12;   // k32 steps per wave held in registers (K <= 4 * 32 * 12 = 1536)
constexpr int LR_SIN_MAXK = 512;   // sinusoid width formed in LDS

__global__ __launch_bounds__(256) void linear_rows_kernel(const bf16_t* __restrict__ x, const float* __restrict__ t,
                                                          int n_t, const float* __restrict__ freqs, int flip,
                                                          const bf16_t* __restrict__ w, int kpad, int k, int n,
                                                          const float* __restrict__ bias, int rows, int act, void* out,
                                                          int out_dt) {
  __shared__ f32x4_t part[3][64];
  __shared__ __attribute__((aligned(16))) bf16_t xs[16 * LR_SIN_MAXK];   // the sinusoid rows (x == NULL)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int nk = k / 32;
  const int s0 = nk * wave / 4, s1 = nk * (wave + 1) / 4;
  uint4 wb[LR_MAXS], xa[LR_MAXS];
  const bf16_t* wrow = w + (int64_t)(n0 + lr) * kpad + 8 * g;
#pragma unroll
  for (int i = 0; i < LR_MAXS; ++i)
    if (s0 + i < s1) wb[i] = *reinterpret_cast<const uint4*>(wrow + (s0 + i) * 32);
  if (x) {
#pragma unroll
    for (int i = 0; i < LR_MAXS; ++i)
      if (s0 + i < s1)
        xa[i] = lr < rows ? *reinterpret_cast<const uint4*>(x + (int64_t)lr * k + (s0 + i) * 32 + 8 * g)
                          : make_uint4(0u, 0u, 0u, 0u);
  } else {
    // the sinusoid rows, one value per thread at a time into LDS (sin / cos of arguments up to ~1e3
    // take ocml's slow range reduction: 24 of them serially per lane cost ~12 us), then the fragments
    const int half = k / 2;
    for (int e = threadIdx.x; e < rows * k; e += 256) {
      const int r = e / k, j = e - r * k;
      const bool first = j < half;
      const float arg = t[n_t == 1 ? 0 : r] * freqs[first ? j : j - half];
      const bool use_cos = flip ? first : !first;            // [sin || cos], flipped to [cos || sin]
      xs[e] = f2bf(use_cos ? cosf(arg) : sinf(arg));
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < LR_MAXS; ++i)
      if (s0 + i < s1)
        xa[i] = lr < rows ? *reinterpret_cast<const uint4*>(xs + lr * k + (s0 + i) * 32 + 8 * g)
                          : make_uint4(0u, 0u, 0u, 0u);
  }
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < LR_MAXS; ++i) {
    if (s0 + i >= s1) continue;
    Frag8<bf16_t> a, b;
    a.v = wb[i];
    b.v = xa[i];
    mma_k32(acc, a, b);                  // D[n][m]: lane (g, lr) holds columns 4g..4g+3 of row lr
  }
  if (wave > 0) part[wave - 1][lane] = acc;
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int q = 0; q < 3; ++q) acc += part[q][lane];
  if (lr >= rows) return;
  const int nc = n0 + 4 * g;
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = act_f(acc[r] + (bias ? bias[nc + r] : 0.f), act);
  if (out_dt == LDM_F32) {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + (int64_t)lr * n + nc) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    bf16_t h[4] = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(out) + (int64_t)lr * n + nc) = *reinterpret_cast<const uint2*>(h);
  }
}

// ------------------------------------------------------------------ DDIM
struct DdimArgs {
  const void* mo; int mo_dt;
  const void* x; int x_dt;
  void* prev; void* x0; int out_dt;
  int64_t n;
  const int64_t* t;
  const float* ac;
  float final_ac;
  int step_ratio, pred, clip;
  float clip_range;
  int use_clipped;
  int ntrain;
};

__device__ __forceinline__ float table_at(const float* ac, int64_t t, int ntrain) { return ddim_table_at(ac, t, ntrain); }

__global__ void ddim_step_kernel(const DdimArgs a) {
  const DdimCoef c = ddim_coef(a.ac, *a.t, a.step_ratio, a.final_ac, a.ntrain);
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * 256) {
    const float2 r = ddim_apply(c, ld_dt(a.mo, i, a.mo_dt), ld_dt(a.x, i, a.x_dt), a.pred, a.clip, a.clip_range,
                                a.use_clipped);
    if (a.prev) st_dt(a.prev, i, r.x, a.out_dt);
    if (a.x0) st_dt(a.x0, i, r.y, a.out_dt);
  }
}

__global__ void add_noise_kernel(const void* x0, const void* noise, const int64_t* t, const float* ac, int ntrain,
                                 float scale, int64_t per, int64_t n, void* out, int dt) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / per;
    const float a = table_in_dtype(table_at(ac, t[b], ntrain), dt);
    const float c0 = sqrtf(a) * scale, c1 = sqrtf(1.0f - a);
    st_dt(out, i, c0 * ld_dt(x0, i, dt) + c1 * ld_dt(noise, i, dt), dt);
  }
}

__global__ void remove_noise_kernel(const void* xt, const void* noise, const int64_t* t, const float* ac,
                                    int ntrain, float scale, int64_t per, int64_t n, void* out, int dt) {
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / per;
    const float a = table_in_dtype(table_at(ac, t[b], ntrain), dt);
    st_dt(out, i, (ld_dt(xt, i, dt) - sqrtf(1.0f - a) * ld_dt(noise, i, dt)) / (sqrtf(a) * scale), dt);
  }
}

// ------------------------------------------------------------------ bit codec
__global__ void bit_encode_kernel(const int64_t* __restrict__ ids, int batch, int64_t hw, int n, int64_t ignore,
                                  float fill, float* __restrict__ planes, uint8_t* __restrict__ mask) {
  const int64_t total = (int64_t)batch * hw;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / hw, pix = i - b * hw;
    const int64_t id = ids[i];
    const bool ign = id == ignore;
    if (mask) mask[i] = ign ? 1 : 0;
    float* pl = planes + b * n * hw + pix;
    for (int j = 0; j < n; ++j) pl[(int64_t)j * hw] = ign ? fill : (float)((id >> j) & 1);
  }
}

template <typename T>
__global__ void bit_decode_kernel(const T* __restrict__ planes, int batch, int n, int64_t hw, int drop31,
                                  int64_t* __restrict__ ids) {
  const int64_t total = (int64_t)batch * hw;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / hw, pix = i - b * hw;
    const T* pl = planes + b * n * hw + pix;
    int64_t v = 0;
    for (int j = 0; j < n; ++j) v |= (int64_t)(to_f(pl[(int64_t)j * hw]) > 0.f) << j;
    if (drop31 && v == 31) v = 0;
    ids[i] = v;
  }
}

// ------------------------------------------------------------------ NCHW sources -> NHWC
__global__ void nchw_to_nhwc_kernel(const void* s0, int c0, int d0, const void* s1, int c1, int d1, const void* s2,
                                    int c2, int d2, int batch, int hw, int cpad, void* out, int dt) {
  const int64_t total = (int64_t)batch * hw;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / hw, pix = i - b * hw;
    int c = 0;
    for (int k = 0; k < c0; ++k, ++c) st_dt(out, i * cpad + c, ld_dt(s0, (b * c0 + k) * hw + pix, d0), dt);
    for (int k = 0; k < c1; ++k, ++c) st_dt(out, i * cpad + c, ld_dt(s1, (b * c1 + k) * hw + pix, d1), dt);
    for (int k = 0; k < c2; ++k, ++c) st_dt(out, i * cpad + c, ld_dt(s2, (b * c2 + k) * hw + pix, d2), dt);
    for (; c < cpad; ++c) st_dt(out, i * cpad + c, 0.f, dt);
  }
}

// ------------------------------------------------------------------ bilinear (align_corners=False)
__global__ void resize_bilinear_kernel(const void* x, int64_t planes, int hi, int wi, int ho, int wo, float sh,
                                       float sw, float mul, float add, void* out, int idt, int odt) {
  const int64_t total = planes * ho * wo;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t pl = i / ((int64_t)ho * wo);
    const int r = (int)(i - pl * ho * wo);
    const int oy = r / wo, ox = r - oy * wo;
    float fy = fmaxf((oy + 0.5f) * sh - 0.5f, 0.f);
    float fx = fmaxf((ox + 0.5f) * sw - 0.5f, 0.f);
    const int y0 = min((int)fy, hi - 1), x0 = min((int)fx, wi - 1);
    const int y1 = y0 + (y0 < hi - 1 ? 1 : 0), x1 = x0 + (x0 < wi - 1 ? 1 : 0);
    const float ly = fy - y0, lx = fx - x0;
    const float hy = 1.f - ly, hx = 1.f - lx;
    const int64_t base = pl * hi * wi;
    const float v00 = ld_dt(x, base + (int64_t)y0 * wi + x0, idt), v01 = ld_dt(x, base + (int64_t)y0 * wi + x1, idt);
    const float v10 = ld_dt(x, base + (int64_t)y1 * wi + x0, idt), v11 = ld_dt(x, base + (int64_t)y1 * wi + x1, idt);
    const float v = hy * (hx * v00 + lx * v01) + ly * (hx * v10 + lx * v11);
    st_dt(out, i, v * mul + add, odt);
  }
}

// ------------------------------------------------------------------ gaussian posterior (NCHW moments)
__global__ void posterior_kernel(const void* mom, int batch, int hw, int L, int clampo, int act, float* mean,
                                 float* logvar, float* stdv, float* var, int dt) {
  const int64_t total = (int64_t)batch * L * hw;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / ((int64_t)L * hw);
    const int64_t r = i - b * L * hw;  // (l, pix)
    float mu = ld_dt(mom, b * 2 * L * hw + r, dt);
    float lv = ld_dt(mom, b * 2 * L * hw + (int64_t)L * hw + r, dt);
    if (clampo) { mu = fminf(fmaxf(mu, -5.f), 5.f); lv = fminf(fmaxf(lv, -5.f), 5.f); }
    if (act == LDM_POST_TANH) mu = tanhf(mu);
    else if (act == LDM_POST_SIGMOID) mu = 2.f / (1.f + expf(-mu)) - 1.f;
    else if (act == LDM_POST_CLIP) mu = fminf(fmaxf(mu, -1.f), 1.f);
    lv = fminf(fmaxf(lv, -30.f), 20.f);
    if (mean) mean[i] = mu;
    if (logvar) logvar[i] = lv;
    if (stdv) stdv[i] = expf(0.5f * lv);
    if (var) var[i] = expf(lv);
  }
}

}  // namespace

extern "C" int ldm_timestep_proj(const float* t, int n_t, int batch, const float* freqs, int dim, int flip,
                                 void* out, int dtype, ldm_stream_t stream) {
  if (!t || !freqs || !out || batch <= 0 || dim <= 0 || dim % 2 || (n_t != 1 && n_t != batch)) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  hipLaunchKernelGGL(tproj_kernel, dim3(grid_for((int64_t)batch * dim)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), t, n_t, batch, freqs, dim, flip, out, dtype);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_linear_rows(const void* x, const float* t, int n_t, const float* freqs, int flip, const void* w,
                               int kpad, int k, int n, const float* bias, int rows, int act, void* out, int out_dtype,
                               ldm_stream_t stream) {
  if (!w || !out || rows <= 0 || rows > 16 || n <= 0 || n % 16 || k <= 0 || k % 32 || k > kpad || kpad % 8) return LDM_ERR_ARG;
  if (k > 4 * 32 * LR_MAXS || (out_dtype != LDM_F32 && out_dtype != LDM_BF16)) return LDM_ERR_ARG;
  if (act < LDM_ACT_NONE || act > LDM_ACT_SIGMOID) return LDM_ERR_ARG;
  if (!x && (!t || !freqs || k % 2 || k > LR_SIN_MAXK || (n_t != 1 && n_t != rows))) return LDM_ERR_ARG;
  if ((x && !aligned16(x)) || !aligned16(w) || !aligned16(out) || (reinterpret_cast<uintptr_t>(out) & 15)) return LDM_ERR_ALIGN;
  hipLaunchKernelGGL(linear_rows_kernel, dim3(n / 16), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const bf16_t*>(x), t, n_t, freqs, flip, reinterpret_cast<const bf16_t*>(w), kpad,
                     k, n, bias, rows, act, out, out_dtype);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_ddim_step(const ldm_ddim_step_params* p, ldm_stream_t stream) {
  if (!p || !p->model_output || !p->sample || !p->t || !p->alphas_cumprod || p->n < 0) return LDM_ERR_ARG;
  if (!p->prev && !p->x0) return LDM_ERR_ARG;
  if (p->prediction_type < 0 || p->prediction_type > 2 || p->step_ratio <= 0) return LDM_ERR_ARG;
  if (p->n == 0) return LDM_OK;
  DdimArgs a;
  a.mo = p->model_output; a.mo_dt = p->mo_dtype; a.x = p->sample; a.x_dt = p->x_dtype;
  a.prev = p->prev; a.x0 = p->x0; a.out_dt = p->out_dtype; a.n = p->n; a.t = p->t; a.ac = p->alphas_cumprod;
  a.final_ac = p->final_alpha_cumprod; a.step_ratio = p->step_ratio; a.pred = p->prediction_type;
  a.clip = p->clip_sample; a.clip_range = p->clip_range; a.use_clipped = p->use_clipped_model_output;
  a.ntrain = p->num_train_timesteps;
  if (a.ntrain <= 0) return LDM_ERR_ARG;
  hipLaunchKernelGGL(ddim_step_kernel, dim3(grid_for(p->n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_ddim_add_noise(const void* x0, const void* noise, const int64_t* t, const float* ac, int ntrain,
                                  float scale, int batch, int64_t per, void* out, int dtype, ldm_stream_t stream) {
  if (!x0 || !noise || !t || !ac || !out || batch <= 0 || per < 0 || ntrain <= 0) return LDM_ERR_ARG;
  const int64_t n = (int64_t)batch * per;
  if (n == 0) return LDM_OK;
  hipLaunchKernelGGL(add_noise_kernel, dim3(grid_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), x0,
                     noise, t, ac, ntrain, scale, per, n, out, dtype);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_ddim_remove_noise(const void* xt, const void* noise, const int64_t* t, const float* ac, int ntrain,
                                     float scale, int batch, int64_t per, void* out, int dtype, ldm_stream_t stream) {
  if (!xt || !noise || !t || !ac || !out || batch <= 0 || per < 0 || ntrain <= 0) return LDM_ERR_ARG;
  const int64_t n = (int64_t)batch * per;
  if (n == 0) return LDM_OK;
  hipLaunchKernelGGL(remove_noise_kernel, dim3(grid_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), xt,
                     noise, t, ac, ntrain, scale, per, n, out, dtype);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_bit_encode(const int64_t* ids, int batch, int64_t hw, int n, int64_t ignore_label,
                              float fill_value, float* planes, uint8_t* ignore_mask, ldm_stream_t stream) {
  if (batch < 0 || hw < 0 || n <= 0 || n > 62) return LDM_ERR_ARG;
  const int64_t total = (int64_t)batch * hw;
  if (total == 0) return LDM_OK;
  if (!ids || !planes) return LDM_ERR_ARG;
  hipLaunchKernelGGL(bit_encode_kernel, dim3(grid_for(total)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     ids, batch, hw, n, ignore_label, fill_value, planes, ignore_mask);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_bit_decode(const void* planes, int batch, int n, int64_t hw, int drop_31, int64_t* ids, int dtype,
                              ldm_stream_t stream) {
  if (batch < 0 || hw < 0 || n <= 0 || n > 62) return LDM_ERR_ARG;
  const int64_t total = (int64_t)batch * hw;
  if (total == 0) return LDM_OK;
  if (!planes || !ids) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == LDM_BF16)
    hipLaunchKernelGGL((bit_decode_kernel<bf16_t>), dim3(grid_for(total)), dim3(256), 0, s,
                       (const bf16_t*)planes, batch, n, hw, drop_31, ids);
  else if (dtype == LDM_F32)
    hipLaunchKernelGGL((bit_decode_kernel<float>), dim3(grid_for(total)), dim3(256), 0, s, (const float*)planes,
                       batch, n, hw, drop_31, ids);
  else return LDM_ERR_ARG;
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_nchw_to_nhwc(const void* s0, int c0, int dt0, const void* s1, int c1, int dt1, const void* s2,
                                int c2, int dt2, int batch, int hw, int c_pad, void* out, int dtype,
                                ldm_stream_t stream) {
  if (!s0 || !out || c0 <= 0 || c1 < 0 || c2 < 0 || batch <= 0 || hw <= 0) return LDM_ERR_ARG;
  if ((c1 && !s1) || (c2 && !s2) || c_pad < c0 + c1 + c2) return LDM_ERR_ARG;
  const int64_t total = (int64_t)batch * hw;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(total)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     s0, c0, dt0, s1, c1, dt1, s2, c2, dt2, batch, hw, c_pad, out, dtype);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_resize_bilinear(const void* x, int planes, int h_in, int w_in, int h_out, int w_out, float scale_h,
                                   float scale_w, float mul, float add, void* out, int in_dtype, int out_dtype,
                                   ldm_stream_t stream) {
  if (!x || !out || planes <= 0 || h_in <= 0 || w_in <= 0 || h_out <= 0 || w_out <= 0) return LDM_ERR_ARG;
  const int64_t total = (int64_t)planes * h_out * w_out;
  hipLaunchKernelGGL(resize_bilinear_kernel, dim3(grid_for(total)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, (int64_t)planes, h_in, w_in, h_out, w_out, scale_h,
                     scale_w, mul, add, out, in_dtype, out_dtype);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_gaussian_posterior(const void* moments, int batch, int hw, int latent_channels, int clamp_output,
                                      int act_fn, float* mean, float* logvar, float* stdv, float* var, int dtype,
                                      ldm_stream_t stream) {
  if (!moments || batch <= 0 || hw <= 0 || latent_channels <= 0) return LDM_ERR_ARG;
  const int64_t total = (int64_t)batch * latent_channels * hw;
  hipLaunchKernelGGL(posterior_kernel, dim3(grid_for(total)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     moments, batch, hw, latent_channels, clamp_output, act_fn, mean, logvar, stdv, var, dtype);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" const char* ldm_status_string(int status) {
  switch (status) {
    case LDM_OK: return "ok";
    case LDM_ERR_ARG: return "invalid argument or unsupported configuration";
    case LDM_ERR_ALIGN: return "pointer / channel alignment violates the 16-byte vector requirement";
    case LDM_ERR_LAUNCH: return "kernel launch failed";
    default: return "unknown status";
  }
}

extern "C" int ldm_abi_version(void) { return 1; }

// ---------------------------------------------------------------------------------------
// ldm_softmax_rows: one wave per row, the row held in registers (<= 128 values per lane), fp32
// max / exp / sum, output bf16 or fp32 with zero fill of the padding columns.
// ---------------------------------------------------------------------------------------
namespace {
template <typename T, int VPL>
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ s, int rows, int n, int stride,
                                                           float scale, T* __restrict__ p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* sr = s + (int64_t)row * stride;
  float v[VPL];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int j = lane + 64 * i;
    v[i] = j < n ? sr[j] * scale : -INFINITY;
    m = fmaxf(m, v[i]);
  }
  m = wave_max(m);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    v[i] = lane + 64 * i < n ? __expf(v[i] - m) : 0.f;
    sum += v[i];
  }
  const float inv = 1.0f / wave_sum(sum);
  T* pr = p + (int64_t)row * stride;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int j = lane + 64 * i;
    if (j < stride) pr[j] = from_f<T>(v[i] * inv);
  }
}

template <typename T>
int softmax_launch(const float* s, int rows, int n, int stride, float scale, void* p, hipStream_t st) {
  const int vpl = (stride + 63) / 64;
  const dim3 grid((rows + 3) / 4);
#define SM_CASE(V)                                                                                        \
  if (vpl <= V) {                                                                                         \
    hipLaunchKernelGGL((softmax_rows_kernel<T, V>), grid, dim3(256), 0, st, s, rows, n, stride, scale,   \
                       static_cast<T*>(p));                                                               \
    return LDM_OK;                                                                                        \
  }
  SM_CASE(4) SM_CASE(16) SM_CASE(64) SM_CASE(128)
#undef SM_CASE
  return LDM_ERR_ARG;
}
}  // namespace

extern "C" int ldm_softmax_rows(const float* s, int rows, int n, int stride, float scale, void* p, int dtype,
                                ldm_stream_t stream) {
  if (!s || !p || rows <= 0 || n <= 0 || stride < n || stride > 8192) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int r = dtype == LDM_BF16 ? softmax_launch<bf16_t>(s, rows, n, stride, scale, p, st)
                                  : softmax_launch<float>(s, rows, n, stride, scale, p, st);
  if (r != LDM_OK) return r;
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

// ======================================================================================
// Packed-weight refresh (the training step's per-iteration repack, trainers/ldm.py): after the
// fused AdamW updates the fp32 master weights, every bf16 [n][kpad] forward pack, every flipped /
// transposed data-gradient pack and every concatenated / interleaved fp32 bias vector is rewritten
// in place from its source parameters by ONE launch over a descriptor table — instead of ~1200
// torch permute / pad / cast kernels per iteration (profiles/r02d_train_kernel_stats.csv).
// Layouts are those of ldmseg.ops.native.PackedConv and models.unet_train.packed_dgrad.
// ======================================================================================
namespace {
__device__ __forceinline__ int geglu_src_row(int p, int half) {   // packed (interleaved) row -> source row
  const int blk = p >> 5, w = p & 31;
  return w < 16 ? blk * 16 + w : half + blk * 16 + (w - 16);
}

// One block per tile of one descriptor (tile0 = the descriptor's first block): a tile is 16
// destination rows x 64 channels over every tap.  The tile's source floats are read as contiguous
// runs into LDS (a run per source row: 64 channels x taps, or 16 rows x taps), then written as
// 16-byte rows of 8 consecutive destination elements — both the fp32 reads and the packed writes
// are coalesced (the earlier element-per-chunk gather read the data-gradient packs' sources at a
// stride of ci * 9 floats: 9.4 ms of a 142 ms training iteration, profiles/r03a_train_*).
constexpr int RP_R = 16, RP_C = 64, RP_MAXT = 9, RP_VEC = 2048;
__global__ __launch_bounds__(256) void repack_kernel(const ldm_repack_desc* __restrict__ d, int nd, int64_t total) {
  __shared__ __attribute__((aligned(16))) float lds[RP_R * RP_C * RP_MAXT];
  const int64_t q = blockIdx.x;
  if (q >= total) return;
  int lo = 0, hi = nd - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].chunk0 <= q) lo = mid; else hi = mid - 1;
  }
  const ldm_repack_desc e = d[lo];
  const int64_t local = q - e.chunk0;
  const float* src = e.src;
  const int tid = threadIdx.x;
  if (e.mode == 2) {                                   // fp32 vector [row0 + j] = src[perm j]
    float* dst = static_cast<float*>(e.dst);
    for (int j = (int)local * RP_VEC + tid; j < e.rows && j < ((int)local + 1) * RP_VEC; j += 256)
      dst[e.row0 + j] = src[e.geglu ? geglu_src_row(j, e.co >> 1) : j];
    return;
  }
  const int T = e.ks * e.ks;
  const int nct = (e.cpad + RP_C - 1) / RP_C;
  const int r0 = (int)(local / nct) * RP_R, c0 = (int)(local % nct) * RP_C;
  const bool fwd = e.mode == 0;
  // LDS image: fwd  lds[i][jj * T + t] = W[row'(r0 + i)][c0 + jj][t]        (run 64 T per source row)
  //            dgrad lds[jj][i * T + t] = W[c'(c0 + jj)][r0 + i][t]          (run 16 T per source row)
  const int nsrc = fwd ? RP_R : RP_C, run = fwd ? RP_C * T : RP_R * T;
  // source row sr's run starts at run_base(sr) (float index, or -1: a zero row) and holds `lim`
  // valid floats (the channel range is clipped at ci)
  auto run_base = [&](int sr, int& lim) -> int64_t {
    if (fwd) {
      const int r = r0 + sr;
      const int co = e.geglu ? geglu_src_row(r, e.co >> 1) : r;
      lim = (e.ci - c0) * T;
      return (r < e.rows && co < e.co) ? ((int64_t)co * e.ci + c0) * T : -1;
    }
    const int c = c0 + sr;
    const int co = e.geglu ? geglu_src_row(c, e.co >> 1) : c;
    lim = (e.ci - r0) * T;
    return c < e.co ? ((int64_t)co * e.ci + r0) * T : -1;
  };
  if ((e.ci * T) % 4 == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    // 16-byte loads: every run starts 16-byte aligned (a 16-byte aligned source; c0 * T, r0 * T and
    // ci * T are multiples of 4) and is a whole number of float4; independent loads, all in flight.
    // A source that is not 16-byte aligned (FlatParams aligns its offsets, other callers may not)
    // takes the scalar loop below
    const int run4 = run / 4;
    for (int idx = tid; idx < nsrc * run4; idx += 256) {
      const int sr = idx / run4, x = 4 * (idx - sr * run4);
      int lim;
      const int64_t b = run_base(sr, lim);
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (b >= 0 && x < lim) v = *reinterpret_cast<const float4*>(src + b + x);
      *reinterpret_cast<float4*>(lds + sr * run + x) = v;
    }
  } else {
    for (int idx = tid; idx < nsrc * run; idx += 256) {
      const int sr = idx / run, x = idx - sr * run;
      int lim;
      const int64_t b = run_base(sr, lim);
      lds[idx] = (b >= 0 && x < lim) ? src[b + x] : 0.f;
    }
  }
  __syncthreads();
  // writes: item (i, tap, g) = destination row r0 + i, columns tap * cpad + c0 + 8 g .. + 7
  for (int w = tid; w < RP_R * T * (RP_C / 8); w += 256) {
    const int i = w / (T * 8), rem = w - i * (T * 8), tap = rem >> 3, g = rem & 7;
    const int row = r0 + i, c = c0 + 8 * g;
    if (row >= e.rows || c >= e.cpad) continue;
    float v8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      v8[k] = fwd ? lds[i * run + (8 * g + k) * T + tap] : lds[(8 * g + k) * run + i * T + (T - 1 - tap)];
    const int64_t o = (int64_t)(e.row0 + row) * e.kpad + tap * e.cpad + c;
    if (e.f32) {
      float* dst = static_cast<float*>(e.dst) + o;
      reinterpret_cast<float4*>(dst)[0] = make_float4(v8[0], v8[1], v8[2], v8[3]);
      reinterpret_cast<float4*>(dst)[1] = make_float4(v8[4], v8[5], v8[6], v8[7]);
    } else {
      bf16_t h[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) h[k] = f2bf(v8[k]);
      *reinterpret_cast<uint4*>(static_cast<bf16_t*>(e.dst) + o) = *reinterpret_cast<const uint4*>(h);
    }
  }
  // the K padding past the last tap (kpad > T * cpad) stays zero: rewritten by the first column tile
  if (c0 == 0 && e.kpad > T * e.cpad) {
    const int pad = e.kpad - T * e.cpad;
    for (int w = tid; w < RP_R * pad; w += 256) {
      const int i = w / pad, k = T * e.cpad + (w - i * pad);
      if (r0 + i >= e.rows) continue;
      const int64_t o = (int64_t)(e.row0 + r0 + i) * e.kpad + k;
      if (e.f32) static_cast<float*>(e.dst)[o] = 0.f;
      else static_cast<bf16_t*>(e.dst)[o] = f2bf(0.f);
    }
  }
}
}  // namespace

extern "C" int ldm_repack(const ldm_repack_desc* descs, int ndesc, int64_t total_tiles, ldm_stream_t stream) {
  if (!descs || ndesc <= 0 || total_tiles <= 0 || total_tiles >= (1LL << 31)) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(repack_kernel, dim3((unsigned)total_tiles), dim3(256), 0, s, descs, ndesc, total_tiles);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
