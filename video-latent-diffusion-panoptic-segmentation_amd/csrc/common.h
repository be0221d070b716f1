// Shared device helpers for the ldmseg HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ldmseg_hip.h"

typedef unsigned short bf16_t;  // storage type; arithmetic always in fp32

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
// round-to-nearest-even via v_cvt_pk_bf16_f32 (keeps NaN a NaN)
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float load(const float* p) { return *p; }
  static __device__ __forceinline__ void store(float* p, float v) { *p = v; }
  static constexpr int kSize = 4;
};
template <> struct Elem<bf16_t> {
  static __device__ __forceinline__ float load(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void store(bf16_t* p, float v) { *p = f2bf(v); }
  static constexpr int kSize = 2;
};

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<bf16_t>(bf16_t v) { return bf2f(v); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) { return f2bf(v); }

// x * sigmoid(x) with v_exp + v_rcp (1 ulp) instead of an IEEE division sequence
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// epilogue activation (LDM_ACT_*): SiLU (the UNet), ReLU / sigmoid (PoseExpNet, posenet.py:7-19,76-79)
__device__ __forceinline__ float act_f(float x, int act) {
  if (act == LDM_ACT_SILU) return silu_f(x);
  if (act == LDM_ACT_RELU) return fmaxf(x, 0.f);
  if (act == LDM_ACT_SIGMOID) return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
  return x;
}
// erf via Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 absolute): one v_rcp, one v_exp and a
// degree-5 Horner chain instead of ocml erff's ~40-instruction path.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y *= t;
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  return copysignf(fmaf(-y, e, 1.0f), x);
}
__device__ __forceinline__ float gelu_f(float x) {  // exact-form (erf) GELU, torch approximate='none'
#ifdef LDM_ABLATE_GELU   // ablation builds only (tools/ablate.sh)
  return x;
#endif
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------------------
// MFMA tiles with one code path for bf16 and exact fp32.
//
// mma_k32: D[16x16] += A[16 x 32] * B[32 x 16].  Lane l (g = l>>4) supplies the 8 K-values
//   k = 8g + j (j = 0..7) of A row (l&15) and of B column (l&15).  bf16: one
//   v_mfma_f32_16x16x32_bf16.  fp32: eight v_mfma_f32_16x16x4_f32, step j feeding k-slot g
//   with element j — i.e. the same set of products summed in a different (exact fp32) order.
// mma_k16: same with 4 K-values per lane (k = 4g + j); bf16 v_mfma_f32_16x16x16_bf16.
// C/D layout (both): row = 4g + r (register r), col = l & 15.
// ---------------------------------------------------------------------------------------
template <typename T> struct Frag8;
template <> struct Frag8<bf16_t> { uint4 v; };
template <> struct Frag8<float> { uint4 v[2]; };
template <typename T> struct Frag4;
template <> struct Frag4<bf16_t> { uint2 v; };
template <> struct Frag4<float> { uint4 v; };

__device__ __forceinline__ void mma_k32(f32x4_t& acc, const Frag8<bf16_t>& a, const Frag8<bf16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a.v),
                                                __builtin_bit_cast(bf16x8_t, b.v), acc, 0, 0, 0);
}
__device__ __forceinline__ void mma_k32(f32x4_t& acc, const Frag8<float>& a, const Frag8<float>& b) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float* pa = reinterpret_cast<const float*>(&a.v[h]);
    const float* pb = reinterpret_cast<const float*>(&b.v[h]);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[j], pb[j], acc, 0, 0, 0);
  }
}
__device__ __forceinline__ void mma_k16(f32x4_t& acc, const Frag4<bf16_t>& a, const Frag4<bf16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(short4_t, a.v),
                                                  __builtin_bit_cast(short4_t, b.v), acc, 0, 0, 0);
}
__device__ __forceinline__ void mma_k16(f32x4_t& acc, const Frag4<float>& a, const Frag4<float>& b) {
  const float* pa = reinterpret_cast<const float*>(&a.v);
  const float* pb = reinterpret_cast<const float*>(&b.v);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[j], pb[j], acc, 0, 0, 0);
}

// 16 B per lane global -> LDS at M0 + 16 * lane (LDS-DMA, per-lane 64-bit source).
// Inline asm so that hipcc does not drain every in-flight DMA before the next ds_read; the
// consumer owns the wait (explicit `s_waitcnt vmcnt` + barrier).  M0 is saved and restored.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}

// DDIM step arithmetic (ddim_scheduler.py:218-269), shared by ldm_ddim_step and the fused UNet tail:
// coefficients of timestep t (ac = alphas_cumprod, NaN for an out-of-range t, never an OOB read) and
// the per-element update.
struct DdimCoef { float sa, sb, sap, sbp; };
__device__ __forceinline__ float ddim_table_at(const float* ac, int64_t t, int ntrain) {
  return (t >= 0 && t < ntrain) ? ac[t] : __int_as_float(0x7fc00000);
}
__device__ __forceinline__ DdimCoef ddim_coef(const float* ac, int64_t t, int step_ratio, float final_ac, int ntrain) {
  const int64_t pt = t - step_ratio;
  const float at = ddim_table_at(ac, t, ntrain);
  const float ap = pt >= 0 ? ddim_table_at(ac, pt, ntrain) : final_ac;
  const float bt = 1.0f - at;
  return DdimCoef{sqrtf(at), sqrtf(bt), sqrtf(ap), sqrtf(1.0f - ap)};
}
// m = model output, x = sample -> (prev_sample, pred_original_sample)
__device__ __forceinline__ float2 ddim_apply(const DdimCoef& c, float m, float x, int pred, int clip, float clip_range,
                                             int use_clipped) {
  float x0, eps;
  if (pred == LDM_PRED_EPSILON) { x0 = (x - c.sb * m) / c.sa; eps = m; }
  else if (pred == LDM_PRED_SAMPLE) { x0 = m; eps = (x - c.sa * x0) / c.sb; }
  else { x0 = c.sa * x - c.sb * m; eps = c.sa * m + c.sb * x; }
  if (clip) x0 = fminf(fmaxf(x0, -clip_range), clip_range);
  if (use_clipped) eps = (x - c.sa * x0) / c.sb;
  return make_float2(c.sap * x0 + c.sbp * eps, x0);
}

#define LDM_CHECK_LAUNCH()                                   \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return LDM_ERR_LAUNCH;             \
  } while (0)
