// GroupNorm(+SiLU) and LayerNorm over NHWC rows (ldm_group_norm / ldm_layer_norm).
//
// GroupNorm is HBM-bound: one read and one write of the tensor, in ONE launch.  Its statistics
// arrive as fp64 (sum, sumsq) accumulators per (batch, unit of U consecutive channels), summed
// by the producing conv's epilogue (ldm_conv2d gn_partial / gn_unit), so the tensor is not
// re-read for them (gn_stats computes them, U = 1, when no producer did).  Units, not groups:
// one tensor feeds GroupNorms of different groupings (a skip is normalised alone in the down
// path and at an offset inside an up-block concat) and U = 10 divides all of them.
//   gn_apply  grid (row blocks, batch); issues its first UNR rows of loads, then reduces its
//             batch's <= C / U accumulators to per-group (mean, rstd) in LDS while they are in
//             flight (no separate finalize launch); every thread owns fixed 16-B channel columns,
//             so its scale / shift live in registers, and streams y = silu?(x * scale + shift).
// Inputs may be the channel concatenation of two NHWC tensors (up-block [hidden || skip]),
// read in place.
#include "common.h"

#include <algorithm>

namespace {

constexpr int GN_MAXC = 2560;        // channels per GroupNorm (the UNet's largest concat)
constexpr int GN_STATS_SLOTS = 4;    // accumulator copies written by the fallback statistics kernel
#ifndef GN_TARGET_BLOCKS
#define GN_TARGET_BLOCKS 1024        // apply grid size (ablation builds vary it)
#endif
#ifndef GN_UNR
#define GN_UNR 8                     // rows in flight per apply thread
#endif

// fallback statistics (no producer accumulators): grid (row blocks, batch); a block sums its
// rows for every channel (column passes of <= 256 vectors, RB rows in parallel, fp32 over the
// block's <= rows_per_block rows) and adds them to slot blockIdx.x % slots of the zeroed fp64
// accumulators [batch][slots][C][2] (unit 1).
template <typename T>
__global__ __launch_bounds__(256) void gn_stats(const T* __restrict__ x, int C, int hw, int rows_per_block,
                                                int slots, double* __restrict__ acc) {
  constexpr int EPC = 16 / sizeof(T);
  __shared__ float red[256 * EPC * 2];
  const int V = C / EPC;
  const int b = blockIdx.y;
  const int r_beg = blockIdx.x * rows_per_block, r_end = min(hw, r_beg + rows_per_block);
  double* dst = acc + ((int64_t)b * slots + blockIdx.x % slots) * C * 2;
  for (int v0 = 0; v0 < V; v0 += 256) {
    const int vn = min(256, V - v0);
    const int rb = 256 / vn;
    const int tx = threadIdx.x % vn, ty = threadIdx.x / vn;
    float sm[EPC], sq[EPC];
#pragma unroll
    for (int k = 0; k < EPC; ++k) { sm[k] = 0.f; sq[k] = 0.f; }
    if (ty < rb)
      for (int r = r_beg + ty; r < r_end; r += rb) {
        const uint4 raw = *reinterpret_cast<const uint4*>(x + ((int64_t)b * hw + r) * C + (v0 + tx) * EPC);
        const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
          const float f = to_f(e[k]);
          sm[k] += f;
          sq[k] += f * f;
        }
      }
    __syncthreads();                                   // the previous pass's reads of red are done
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      red[(threadIdx.x * EPC + k) * 2] = sm[k];
      red[(threadIdx.x * EPC + k) * 2 + 1] = sq[k];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < vn * EPC; e += 256) {
      const int col = e / EPC, k = e % EPC;
      float a = 0.f, q = 0.f;
      for (int j = 0; j < rb; ++j) {
        a += red[((j * vn + col) * EPC + k) * 2];
        q += red[((j * vn + col) * EPC + k) * 2 + 1];
      }
      double* d = dst + (int64_t)((v0 + col) * EPC + k) * 2;
      unsafeAtomicAdd(d, (double)a);
      unsafeAtomicAdd(d + 1, (double)q);
    }
  }
}

// y = silu?(x * scale + shift).  Block = BX x RB threads: tx owns vector columns tx + BX * k
// (k < NCOL) for all its rows, ty strides rows by RB; grid (row blocks, batch).  Dynamic LDS:
// the batch's slots x C / unit accumulators (double2 each, <= 40 KB).
template <typename T, int NCOL>
__global__ __launch_bounds__(256) void gn_apply(const T* __restrict__ x0, const T* __restrict__ x1, int c0, int c1,
                                                int hw, int rows_per_block, const double* __restrict__ acc0,
                                                const double* __restrict__ acc1, int unit, int slots, int groups,
                                                float eps,
                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                int act, T* __restrict__ out, float2* __restrict__ save) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int UNR = GN_UNR;
  extern __shared__ double2 ured[];
  __shared__ float2 gst[64];
  const int C = c0 + c1, V = C / EPC, cpg = C / groups;
  const int BX = blockDim.x, RB = blockDim.y;
  const int tx = threadIdx.x, ty = threadIdx.y;
  const int tid = ty * BX + tx, nt = BX * RB;
  const int b = blockIdx.y;
  const int r_beg = blockIdx.x * rows_per_block;
  const int r_end = min(hw, r_beg + rows_per_block);
  const int64_t rowb = (int64_t)b * hw;
  const T* src[NCOL];
  int ld[NCOL], cc[NCOL];
  bool on[NCOL];
#pragma unroll
  for (int k = 0; k < NCOL; ++k) {
    const int v = tx + BX * k;
    on[k] = v < V;
    const int c = min(v, V - 1) * EPC;
    cc[k] = c;
    src[k] = c < c0 ? x0 + c : x1 + (c - c0);
    ld[k] = c < c0 ? c0 : c1;
  }
  uint4 raw[NCOL][UNR];
  auto load = [&](int r0) {
#pragma unroll
    for (int k = 0; k < NCOL; ++k)
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * RB;
        if (on[k] && r < r_end) raw[k][u] = *reinterpret_cast<const uint4*>(src[k] + (rowb + r) * ld[k]);
      }
  };
  load(r_beg + ty);                 // the first pass's rows are in flight during the statistics
  // accumulators -> LDS (all loads in flight), then thread per group: mean / rstd in fp64
  const int u0 = c0 / unit, u1 = c1 / unit, upg = cpg / unit;
  const int un = u0 + u1;
  for (int i = tid; i < slots * un; i += nt) {              // entry (slot, unit): all loads in flight
    const int sl = i / un, u = i - sl * un;
    ured[i] = u < u0 ? *reinterpret_cast<const double2*>(acc0 + (((int64_t)b * slots + sl) * u0 + u) * 2)
                     : *reinterpret_cast<const double2*>(acc1 + (((int64_t)b * slots + sl) * u1 + (u - u0)) * 2);
  }
  __syncthreads();
  for (int gi = tid; gi < groups; gi += nt) {
    double sa = 0.0, sq = 0.0;
    for (int sl = 0; sl < slots; ++sl)
      for (int k = 0; k < upg; ++k) {
        const double2 v = ured[sl * un + gi * upg + k];
        sa += v.x;
        sq += v.y;
      }
    const double cnt = (double)hw * cpg;
    const double mean = sa / cnt;
    double var = sq / cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    const float2 ms = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)eps)));
    gst[gi] = ms;
    if (save && blockIdx.x == 0) save[b * groups + gi] = ms;   // training: kept for the backward
  }
  __syncthreads();
  float sc[NCOL][EPC], sh[NCOL][EPC];
#pragma unroll
  for (int k = 0; k < NCOL; ++k) {
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      const int c = cc[k] + e;
      const float2 ms = gst[c / cpg];
      sc[k][e] = ms.y * gamma[c];
      sh[k][e] = fmaf(-ms.x, sc[k][e], beta[c]);   // explicit FMAs: ldm_transformer_in repeats them
    }
  }
  for (int r0 = r_beg + ty; r0 < r_end; r0 += UNR * RB) {
    if (r0 != r_beg + ty) load(r0);
#pragma unroll
    for (int k = 0; k < NCOL; ++k) {
      if (!on[k]) continue;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * RB;
        if (r >= r_end) break;
        const T* e = reinterpret_cast<const T*>(&raw[k][u]);
        uint4 res;
        T* o = reinterpret_cast<T*>(&res);
#pragma unroll
        for (int j = 0; j < EPC; ++j) {
          float y = fmaf(to_f(e[j]), sc[k][j], sh[k][j]);
          if (act == LDM_ACT_SILU) y = silu_f(y);
          o[j] = from_f<T>(y);
        }
        *reinterpret_cast<uint4*>(out + (rowb + r) * C + cc[k]) = res;
      }
    }
  }
}

// Small images without producer statistics (config 5's 4x8 level: hw = 32, C = 1280, where a 64-row
// conv tile spans two images so the producer cannot sum per-image units): one 512-thread block per
// image stages the whole [hw][C] slab in LDS (<= GNS_MAX_BYTES) and takes EXACT two-pass group
// statistics from it in a fixed order (per-channel partials of row phases, then per group), then
// writes y — one launch instead of memset + statistics + apply (33 -> ~5 us per launch).
constexpr int GNS_MAX_BYTES = 96 * 1024;
template <typename T>
__global__ __launch_bounds__(512) void gn_small(const T* __restrict__ x0, const T* __restrict__ x1, int c0, int c1,
                                                int hw, int groups, float eps, const float* __restrict__ gamma,
                                                const float* __restrict__ beta, int act, T* __restrict__ out,
                                                float2* __restrict__ save) {
  constexpr int EPC = 16 / sizeof(T);
  extern __shared__ uint4 img[];                       // [hw][V] vectors, then [nph][C] fp32 partials
  __shared__ float2 gst[64];
  const int C = c0 + c1, V = C / EPC, cpg = C / groups;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int nph = 512 / V;                             // row phases of the per-channel partials
  float* part = reinterpret_cast<float*>(img + (int64_t)hw * V);
  for (int e = tid; e < hw * V; e += 512) {
    const int r = e / V, v = e - r * V, c = v * EPC;
    img[e] = c < c0 ? *reinterpret_cast<const uint4*>(x0 + ((int64_t)b * hw + r) * c0 + c)
                    : *reinterpret_cast<const uint4*>(x1 + ((int64_t)b * hw + r) * c1 + (c - c0));
  }
  __syncthreads();
  const int v = tid % V, ph = tid / V;
  for (int pass = 0; pass < 2; ++pass) {               // 0: sums -> mean; 1: centred squares -> var
    if (ph < nph) {
      float acc[EPC], mu[EPC];
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        acc[k] = 0.f;
        mu[k] = pass ? gst[(v * EPC + k) / cpg].x : 0.f;
      }
      for (int r = ph; r < hw; r += nph) {
        const uint4 raw = img[r * V + v];
        const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
          const float f = to_f(e[k]) - mu[k];
          acc[k] += pass ? f * f : f;
        }
      }
#pragma unroll
      for (int k = 0; k < EPC; ++k) part[ph * C + v * EPC + k] = acc[k];
    }
    __syncthreads();
    if (tid < groups) {
      float a = 0.f;
      for (int q = 0; q < nph; ++q)
        for (int c = tid * cpg; c < (tid + 1) * cpg; ++c) a += part[q * C + c];
      const float n = (float)hw * cpg;
      if (pass == 0) gst[tid].x = a / n;
      else gst[tid].y = 1.0f / sqrtf(a / n + eps);
    }
    __syncthreads();
  }
  if (save && tid < groups) save[b * groups + tid] = gst[tid];
  for (int e = tid; e < hw * V; e += 512) {
    const int r = e / V, vv = e - r * V;
    const uint4 raw = img[e];
    const T* x = reinterpret_cast<const T*>(&raw);
    uint4 res;
    T* o = reinterpret_cast<T*>(&res);
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      const int c = vv * EPC + k;
      const float2 ms = gst[c / cpg];
      const float sc = ms.y * gamma[c];
      float y = to_f(x[k]) * sc + (beta[c] - ms.x * sc);
      if (act == LDM_ACT_SILU) y = silu_f(y);
      o[k] = from_f<T>(y);
    }
    *reinterpret_cast<uint4*>(out + ((int64_t)b * hw + r) * C + vv * EPC) = res;
  }
}

// LayerNorm over the last dim, two-pass (mean, then centred variance) in fp32 registers.
// G lanes per row (G | 64): a wave normalises 64/G rows at once, each lane holding NV 16-byte
// chunks (chunk v = lane_in_row + G * i), so C = 320 bf16 (40 chunks) runs 8 rows per wave
// with every lane busy; reductions are xor-shuffles within the G-lane group.  Grid-stride
// over row groups.
template <typename T, int G, int NV>
__global__ __launch_bounds__(256) void ln_kernel(const T* __restrict__ x, int rows, int C,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 float eps, int act, T* __restrict__ out) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int RPW = 64 / G;                      // rows per wave
  const int lane = threadIdx.x & 63;
  const int gl = lane % G;
  const int V = C / EPC;
  const float inv_c = 1.0f / (float)C;
  const int stride = gridDim.x * 4 * RPW;
  for (int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / G; row - lane / G < rows; row += stride) {
    const bool rv = row < rows;
    const T* xr = x + (int64_t)row * C;
    float vals[NV][EPC];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = gl + G * i;
      if (rv && v < V) {
        const uint4 raw = *reinterpret_cast<const uint4*>(xr + v * EPC);
        const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int k = 0; k < EPC; ++k) { vals[i][k] = to_f(e[k]); s += vals[i][k]; }
      }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * inv_c;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (rv && gl + G * i < V) {
#pragma unroll
        for (int k = 0; k < EPC; ++k) { const float d = vals[i][k] - mean; q += d * d; }
      }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q * inv_c + eps);
    T* orow = out + (int64_t)row * C;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = gl + G * i;
      if (rv && v < V) {
        float gm[EPC], bt[EPC];
#pragma unroll
        for (int k = 0; k < EPC; k += 4) {
          const float4 g4 = *reinterpret_cast<const float4*>(gamma + v * EPC + k);
          const float4 b4 = *reinterpret_cast<const float4*>(beta + v * EPC + k);
          gm[k] = g4.x; gm[k + 1] = g4.y; gm[k + 2] = g4.z; gm[k + 3] = g4.w;
          bt[k] = b4.x; bt[k + 1] = b4.y; bt[k + 2] = b4.z; bt[k + 3] = b4.w;
        }
        uint4 res;
        T* r = reinterpret_cast<T*>(&res);
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
          float y = (vals[i][k] - mean) * rstd * gm[k] + bt[k];
          if (act == LDM_ACT_SILU) y = silu_f(y);
          r[k] = from_f<T>(y);
        }
        *reinterpret_cast<uint4*>(orow + v * EPC) = res;
      }
    }
  }
}

template <typename T, int G>
int ln_launch_g(const void* x, int rows, int c, const float* gamma, const float* beta, float eps, int act, void* out,
                hipStream_t s) {
  constexpr int EPC = 16 / sizeof(T);
  const int V = c / EPC;
  const int nv = (V + G - 1) / G;
  const int rpb = 4 * (64 / G);
  const int grid = std::min((rows + rpb - 1) / rpb, 256 * 16);
#define LN_CASE(NVC)                                                                                       \
  if (nv <= NVC) {                                                                                         \
    hipLaunchKernelGGL((ln_kernel<T, G, NVC>), dim3(grid), dim3(256), 0, s, (const T*)x, rows, c, gamma, beta, \
                       eps, act, (T*)out);                                                                 \
    return LDM_OK;                                                                                         \
  }
  LN_CASE(1) LN_CASE(2) LN_CASE(4) LN_CASE(5) LN_CASE(8) LN_CASE(16)
#undef LN_CASE
  return LDM_ERR_ARG;
}

template <typename T>
int ln_launch(const void* x, int rows, int c, const float* gamma, const float* beta, float eps, int act, void* out,
              hipStream_t s) {
  constexpr int EPC = 16 / sizeof(T);
  const int V = c / EPC;
  // the smallest lane group that keeps <= 8 chunks per lane
  if (V <= 8 * 8) return ln_launch_g<T, 8>(x, rows, c, gamma, beta, eps, act, out, s);
  if (V <= 16 * 8) return ln_launch_g<T, 16>(x, rows, c, gamma, beta, eps, act, out, s);
  if (V <= 32 * 8) return ln_launch_g<T, 32>(x, rows, c, gamma, beta, eps, act, out, s);
  return ln_launch_g<T, 64>(x, rows, c, gamma, beta, eps, act, out, s);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline size_t round16(size_t x) { return (x + 15) & ~(size_t)15; }

template <typename T>
int gn_launch(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups, const float* gamma,
              const float* beta, float eps, int act, void* out, const double* a0, const double* a1, int unit,
              int slots, void* ws, float* save, hipStream_t s) {
  constexpr int EPC = 16 / sizeof(T);
  const int C = c0 + c1, V = C / EPC;
  if ((a0 && !a1 && c1 > 0) || (!a0 && a1)) a0 = a1 = nullptr;     // one layout for both: recompute both
  const size_t small_lds = (size_t)hw * C * sizeof(T) + (size_t)(512 / std::max(1, V)) * C * sizeof(float);
  if (!a0 && V <= 512 && (size_t)hw * C * sizeof(T) <= GNS_MAX_BYTES && small_lds <= 128 * 1024) {
    static bool attr_set = false;                    // > 64 KB of dynamic LDS: raise the kernel's cap once
    if (!attr_set) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gn_small<T>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              128 * 1024) != hipSuccess)
        return LDM_ERR_LAUNCH;
      attr_set = true;
    }
    hipLaunchKernelGGL((gn_small<T>), dim3(batch), dim3(512), small_lds, s, static_cast<const T*>(x0),
                       static_cast<const T*>(x1), c0, c1, hw, groups, eps, gamma, beta, act, static_cast<T*>(out),
                       reinterpret_cast<float2*>(save));
    LDM_CHECK_LAUNCH();
    return LDM_OK;
  }
  if (!a0) {
    unit = 1;
    slots = std::max(1, std::min(GN_STATS_SLOTS, GN_MAXC / C));    // slots x C entries fit the LDS
    double* w = static_cast<double*>(ws);
    if (hipMemsetAsync(w, 0, (size_t)batch * slots * C * 2 * sizeof(double), s) != hipSuccess) return LDM_ERR_LAUNCH;
    const int rpb = std::max(64, (int)(((int64_t)hw * batch + 1023) / 1024));
    const dim3 grid((hw + rpb - 1) / rpb, batch);
    hipLaunchKernelGGL((gn_stats<T>), grid, dim3(256), 0, s, static_cast<const T*>(x0), c0, hw, rpb, slots, w);
    LDM_CHECK_LAUNCH();
    a0 = w;
    if (c1 > 0) {
      w += (size_t)batch * slots * c0 * 2;
      hipLaunchKernelGGL((gn_stats<T>), grid, dim3(256), 0, s, static_cast<const T*>(x1), c1, hw, rpb, slots, w);
      LDM_CHECK_LAUNCH();
      a1 = w;
    }
  }
  // columns: NCOL per thread so BX <= 256; rows: RB per pass, ~1024 blocks in all (one pass of
  // UNR rows per thread at the 64x64 / 32x32 levels: every load in flight at once)
  const int ncol = (V + 255) / 256;
  const int bx = (V + ncol - 1) / ncol;
  const int rb = std::max(1, 256 / bx);
  const int per_b = std::max(1, std::min((hw + rb - 1) / rb, (GN_TARGET_BLOCKS + batch - 1) / batch));
  const int rpb = (hw + per_b - 1) / per_b;
  const int nb = (hw + rpb - 1) / rpb;
  const dim3 grid(nb, batch), block(bx, rb);
  const size_t lds = (size_t)slots * (C / unit) * sizeof(double2);
  if (lds > GN_MAXC * sizeof(double2)) return LDM_ERR_ARG;
#define GN_APPLY(NC)                                                                                        \
  hipLaunchKernelGGL((gn_apply<T, NC>), grid, block, lds, s, static_cast<const T*>(x0),                     \
                     static_cast<const T*>(x1), c0, c1, hw, rpb, a0, a1, unit, slots, groups, eps, gamma, beta, \
                     act, static_cast<T*>(out), reinterpret_cast<float2*>(save))
  if (ncol == 1) GN_APPLY(1);
  else if (ncol == 2) GN_APPLY(2);
  else if (ncol == 3) GN_APPLY(3);
  else return LDM_ERR_ARG;
#undef GN_APPLY
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

}  // namespace

extern "C" size_t ldm_group_norm_workspace_bytes(int batch, int hw, int channels) {
  (void)hw;
  return round16((size_t)batch * GN_STATS_SLOTS * channels * 2 * sizeof(double)) + 64;   // fallback accumulators
}

extern "C" int ldm_group_norm_ex(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups,
                                 const float* gamma, const float* beta, float eps, int act, void* out,
                                 const double* stats0, const double* stats1, int stats_unit, int stats_slots,
                                 void* workspace, float* save_mean_rstd, int dtype, ldm_stream_t stream) {
  if (!x0 || !out || !workspace || !gamma || !beta) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  if (batch <= 0 || hw <= 0 || c0 <= 0 || c1 < 0 || (c1 > 0 && !x1) || groups <= 0 || groups > 64) return LDM_ERR_ARG;
  const int C = c0 + c1;
  if (C % groups || C > GN_MAXC) return LDM_ERR_ARG;
  if ((stats0 || stats1) && (stats_unit <= 0 || stats_slots <= 0 || c0 % stats_unit || c1 % stats_unit ||
                             (C / groups) % stats_unit))
    return LDM_ERR_ARG;
  const int epc = dtype == LDM_F32 ? 4 : 8;
  if (c0 % epc || c1 % epc) return LDM_ERR_ALIGN;
  if (!aligned16(x0) || (x1 && !aligned16(x1)) || !aligned16(out) || !aligned16(workspace)) return LDM_ERR_ALIGN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == LDM_BF16)
    return gn_launch<bf16_t>(x0, x1, c0, c1, batch, hw, groups, gamma, beta, eps, act, out, stats0, stats1,
                             stats_unit, stats_slots, workspace, save_mean_rstd, s);
  return gn_launch<float>(x0, x1, c0, c1, batch, hw, groups, gamma, beta, eps, act, out, stats0, stats1, stats_unit,
                          stats_slots, workspace, save_mean_rstd, s);
}

extern "C" int ldm_group_norm(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups,
                              const float* gamma, const float* beta, float eps, int act, void* out,
                              const double* stats0, const double* stats1, int stats_unit, int stats_slots,
                              void* workspace, int dtype, ldm_stream_t stream) {
  return ldm_group_norm_ex(x0, x1, c0, c1, batch, hw, groups, gamma, beta, eps, act, out, stats0, stats1, stats_unit,
                           stats_slots, workspace, nullptr, dtype, stream);
}

extern "C" int ldm_layer_norm(const void* x, int rows, int c, const float* gamma, const float* beta, float eps,
                              int act, void* out, int dtype, ldm_stream_t stream) {
  if (!x || !out || !gamma || !beta || rows <= 0 || c <= 0) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  const int epc = dtype == LDM_F32 ? 4 : 8;
  if (c % epc) return LDM_ERR_ALIGN;
  if (!aligned16(x) || !aligned16(out)) return LDM_ERR_ALIGN;
  if (!aligned16(gamma) || !aligned16(beta)) return LDM_ERR_ALIGN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int st = dtype == LDM_BF16 ? ln_launch<bf16_t>(x, rows, c, gamma, beta, eps, act, out, s)
                                   : ln_launch<float>(x, rows, c, gamma, beta, eps, act, out, s);
  if (st != LDM_OK) return st;
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
