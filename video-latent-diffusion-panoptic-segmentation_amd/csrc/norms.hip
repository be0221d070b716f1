// GroupNorm(+SiLU) and LayerNorm over NHWC rows (ldm_group_norm / ldm_layer_norm).
//
// GroupNorm is HBM-bound.  Statistics come as per-channel (sum, sumsq) partials over 64-pixel
// chunks — normally written by the producing conv's epilogue (ldm_conv2d gn_partial), so the
// tensor is NOT re-read for them; otherwise gn_partial computes them here.
//   gn_finalize: per (batch, group) fp64 reduction -> per-(batch, channel) scale/shift table
//   gn_apply   : y = silu?(x * scale + shift), one 16-B vector per thread, one read + one write
// Inputs may be the channel concatenation of two NHWC tensors (up-block [hidden || skip]),
// read in place.
#include "common.h"

#include <algorithm>

namespace {

constexpr int GN_PPC = 64;  // pixels per partial chunk (== the conv epilogue's 64-row chunks)

template <typename T>
__global__ __launch_bounds__(256) void gn_partial(const T* __restrict__ x, int C, int hw, int chunks,
                                                  float2* __restrict__ part) {
  constexpr int EPC = 16 / sizeof(T);
  const int V = C / EPC;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int v = blockIdx.x * 64 + tx;
  const int chunk = blockIdx.y, b = blockIdx.z;
  float s[EPC], ss[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) { s[e] = 0.f; ss[e] = 0.f; }
  if (v < V) {
    const int p0 = chunk * GN_PPC, p1 = min(hw, p0 + GN_PPC);
    for (int pix = p0 + ty; pix < p1; pix += 4) {
      const uint4 raw = *reinterpret_cast<const uint4*>(x + ((int64_t)b * hw + pix) * C + v * EPC);
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        const float f = to_f(e[k]);
        s[k] += f;
        ss[k] += f * f;
      }
    }
  }
  __shared__ float red[4][64][EPC][2];
#pragma unroll
  for (int k = 0; k < EPC; ++k) { red[ty][tx][k][0] = s[k]; red[ty][tx][k][1] = ss[k]; }
  __syncthreads();
  if (ty == 0 && v < V) {
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      float a = 0.f, q = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) { a += red[j][tx][k][0]; q += red[j][tx][k][1]; }
      part[((int64_t)b * chunks + chunk) * C + v * EPC + k] = make_float2(a, q);
    }
  }
}

// one 256-thread block per (batch, group): fp64 sum of the partials (each thread's loads are
// unrolled 4-wide so they are in flight together — the partials are L2-resident, so this is a
// latency problem, not a bandwidth one), then the group's scale/shift entries
__global__ __launch_bounds__(256) void gn_finalize(const float2* __restrict__ part0, const float2* __restrict__ part1,
                                                   int c0, int c1, int hw, int chunks, int groups, float eps,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   float2* __restrict__ table, float2* __restrict__ save) {
  const int b = blockIdx.x;
  const int gi = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = c0 + c1, cpg = C / groups;
  const int n = chunks * cpg;
  double a = 0.0, q = 0.0;
  for (int i0 = tid; i0 < n; i0 += 4 * 256) {
    float2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 256;
      v[u] = make_float2(0.f, 0.f);
      if (i < n) {
        const int ch = i / cpg, c = gi * cpg + (i - ch * cpg);
        const int64_t row = (int64_t)b * chunks + ch;
        v[u] = c < c0 ? part0[row * c0 + c] : part1[row * c1 + (c - c0)];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { a += v[u].x; q += v[u].y; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o, 64); q += __shfl_xor(q, o, 64); }
  __shared__ double red[4][2];
  if (lane == 0) { red[wave][0] = a; red[wave][1] = q; }
  __syncthreads();
  a = red[0][0] + red[1][0] + red[2][0] + red[3][0];
  q = red[0][1] + red[1][1] + red[2][1] + red[3][1];
  const double cnt = (double)hw * cpg;
  const double mean = a / cnt;
  double var = q / cnt - mean * mean;
  if (var < 0.0) var = 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  if (save && tid == 0) save[(int64_t)b * groups + gi] = make_float2((float)mean, rstd);   // for the backward
  for (int k = tid; k < cpg; k += 256) {
    const int c = gi * cpg + k;
    const float sc = rstd * gamma[c];
    table[(int64_t)b * C + c] = make_float2(sc, beta[c] - (float)mean * sc);
  }
}

// y = silu?(x * scale[b, c] + shift[b, c]) over 16-byte vectors; each thread takes UNR
// vectors a grid-stride apart and issues all their loads before any math (HBM latency
// overlaps), with 32-bit index math (nvec < 2^31 is checked on the host).
template <typename T>
__global__ __launch_bounds__(256) void gn_apply(const T* __restrict__ x0, const T* __restrict__ x1, int c0, int c1,
                                                int hw, int nvec, const float2* __restrict__ table, int act,
                                                T* __restrict__ out) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int UNR = 4;
  const int C = c0 + c1, V = C / EPC;
  const int step = gridDim.x * 256;
  for (int i0 = blockIdx.x * 256 + threadIdx.x; i0 < nvec; i0 += UNR * step) {
    uint4 raw[UNR];
    int mm[UNR], cc[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int i = i0 + u * step;
      const int m = i / V;
      const int c = (i - m * V) * EPC;
      mm[u] = m;
      cc[u] = c;
      if (i < nvec)
        raw[u] = (c < c0) ? *reinterpret_cast<const uint4*>(x0 + (int64_t)m * c0 + c)
                          : *reinterpret_cast<const uint4*>(x1 + (int64_t)m * c1 + (c - c0));
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (i0 + u * step >= nvec) break;
      const int b = mm[u] / hw, c = cc[u];
      const T* e = reinterpret_cast<const T*>(&raw[u]);
      const float4* tb = reinterpret_cast<const float4*>(table + (int64_t)b * C + c);
      uint4 res;
      T* r = reinterpret_cast<T*>(&res);
#pragma unroll
      for (int k = 0; k < EPC; k += 2) {
        const float4 st = tb[k >> 1];   // (scale_k, shift_k, scale_k+1, shift_k+1)
        float y0 = to_f(e[k]) * st.x + st.y;
        float y1 = to_f(e[k + 1]) * st.z + st.w;
        if (act == LDM_ACT_SILU) { y0 = silu_f(y0); y1 = silu_f(y1); }
        r[k] = from_f<T>(y0);
        r[k + 1] = from_f<T>(y1);
      }
      *reinterpret_cast<uint4*>(out + (int64_t)mm[u] * C + c) = res;
    }
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
              const float* beta, float eps, int act, void* out, const float* p0, const float* p1, void* ws,
              float* save, hipStream_t s) {
  constexpr int EPC = 16 / sizeof(T);
  const int C = c0 + c1;
  const int chunks = (hw + GN_PPC - 1) / GN_PPC;
  char* w = static_cast<char*>(ws);
  float2* table = reinterpret_cast<float2*>(w);
  w += round16((size_t)batch * C * sizeof(float2));
  const float2* part0 = reinterpret_cast<const float2*>(p0);
  const float2* part1 = reinterpret_cast<const float2*>(p1);
  if (!part0) {
    float2* dst = reinterpret_cast<float2*>(w);
    w += round16((size_t)batch * chunks * c0 * sizeof(float2));
    hipLaunchKernelGGL((gn_partial<T>), dim3((c0 / EPC + 63) / 64, chunks, batch), dim3(256), 0, s,
                       static_cast<const T*>(x0), c0, hw, chunks, dst);
    LDM_CHECK_LAUNCH();
    part0 = dst;
  }
  if (c1 > 0 && !part1) {
    float2* dst = reinterpret_cast<float2*>(w);
    hipLaunchKernelGGL((gn_partial<T>), dim3((c1 / EPC + 63) / 64, chunks, batch), dim3(256), 0, s,
                       static_cast<const T*>(x1), c1, hw, chunks, dst);
    LDM_CHECK_LAUNCH();
    part1 = dst;
  }
  hipLaunchKernelGGL(gn_finalize, dim3(batch, groups), dim3(256), 0, s, part0, part1, c0, c1, hw, chunks,
                     groups, eps, gamma, beta, table, reinterpret_cast<float2*>(save));
  LDM_CHECK_LAUNCH();
  const int64_t nvec = (int64_t)batch * hw * (C / EPC);
  if (nvec >= (1LL << 31) - 4 * 256 * 2048) return LDM_ERR_ARG;
  const int64_t blocks = std::min<int64_t>((nvec + 4 * 256 - 1) / (4 * 256), 256 * 8);
  hipLaunchKernelGGL((gn_apply<T>), dim3((unsigned)blocks), dim3(256), 0, s, static_cast<const T*>(x0),
                     static_cast<const T*>(x1), c0, c1, hw, (int)nvec, table, act, static_cast<T*>(out));
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

}  // namespace

extern "C" size_t ldm_group_norm_workspace_bytes(int batch, int hw, int channels) {
  const size_t chunks = (hw + GN_PPC - 1) / GN_PPC;
  return round16((size_t)batch * channels * sizeof(float2)) + 2 * round16((size_t)batch * chunks * channels *
                                                                          sizeof(float2)) + 64;
}

extern "C" int ldm_group_norm_ex(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups,
                                 const float* gamma, const float* beta, float eps, int act, void* out,
                                 const float* stats0, const float* stats1, void* workspace, float* save_mean_rstd,
                                 int dtype, ldm_stream_t stream) {
  if (!x0 || !out || !workspace || !gamma || !beta) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  if (batch <= 0 || hw <= 0 || c0 <= 0 || c1 < 0 || (c1 > 0 && !x1) || groups <= 0) return LDM_ERR_ARG;
  const int C = c0 + c1;
  if (C % groups) return LDM_ERR_ARG;
  if ((stats0 || stats1) && hw % GN_PPC) return LDM_ERR_ARG;   // producer partials use 64-row chunks
  const int epc = dtype == LDM_F32 ? 4 : 8;
  if (c0 % epc || c1 % epc) return LDM_ERR_ALIGN;
  if (!aligned16(x0) || (x1 && !aligned16(x1)) || !aligned16(out) || !aligned16(workspace)) return LDM_ERR_ALIGN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == LDM_BF16)
    return gn_launch<bf16_t>(x0, x1, c0, c1, batch, hw, groups, gamma, beta, eps, act, out, stats0, stats1,
                             workspace, save_mean_rstd, s);
  return gn_launch<float>(x0, x1, c0, c1, batch, hw, groups, gamma, beta, eps, act, out, stats0, stats1, workspace,
                          save_mean_rstd, s);
}

extern "C" int ldm_group_norm(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups,
                              const float* gamma, const float* beta, float eps, int act, void* out,
                              const float* stats0, const float* stats1, void* workspace, int dtype,
                              ldm_stream_t stream) {
  return ldm_group_norm_ex(x0, x1, c0, c1, batch, hw, groups, gamma, beta, eps, act, out, stats0, stats1, workspace,
                           nullptr, dtype, stream);
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
