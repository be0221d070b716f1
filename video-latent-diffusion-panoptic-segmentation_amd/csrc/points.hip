// AE training (row a16): PointRend-style point losses of SegmentationLosses.point_loss
// (ldmseg/trainers/losses.py:117-395 via detectron2_utils.py:20-100) and the elementwise
// pieces of the VAE backward that the conv / norm kernels do not cover.
//
//  ldm_point_sample      grid_sample(bilinear, zeros, align_corners=False) of NCHW fp32 planes at
//                        [0,1]^2 points (point_sample, detectron2_utils.py:75-100); a "box" reads
//                        C consecutive planes, or the one plane planes[box] (mask losses).
//  ldm_point_sample_bwd  its adjoint: atomic scatter-add of the point gradients into the planes.
//  ldm_point_labels      targets sampled at the points: nearest (CE labels, rint like grid_sample)
//                        or bilinear of (target == cls[box]) (the mask targets of loss_masks).
//  ldm_point_uncertainty top2[1] - top2[0] over C (calculate_uncertainty_seg) or -|x| (C == 1).
//  ldm_topk_select       per row, the indices of the k largest values (radix select on
//                        order-preserving keys; ties at the threshold taken in index order) and
//                        the gathered coordinates (get_uncertain_point_coords_with_randomness).
//  ldm_point_ce          cross entropy over C at every point with ignore_index (F.cross_entropy,
//                        mean over the non-ignored points) and its gradient.
//  ldm_point_bce_dice    per mask: mean BCE-with-logits + dice (losses.py:187-247) and gradient.
//  ldm_silu_fwd/_bwd     SiLU and its derivative from the pre-activation.
//  ldm_space_to_depth2   dOut [B,2H,2W,C] -> [B,H,W,4C] ((dy,dx,c) order): ConvTranspose k2s2 backward.
//  ldm_posterior_sample / _bwd  z = mean + exp(logvar/2) * eps with logvar clamped to [-30, 20]
//                        (DiagonalGaussianDistribution.sample, vae.py:371-405) and its backward.
#include "common.h"

#include <algorithm>
#include <math.h>

namespace {

// grid_sample source coordinate, align_corners=False: ((g + 1) * size - 1) / 2, g = 2p - 1
__device__ __forceinline__ float src_coord(float p, int size) { return ((2.f * p - 1.f + 1.f) * size - 1.f) * 0.5f; }

struct Bilin {
  int x0, y0;
  float wx1, wy1;
};
__device__ __forceinline__ Bilin bilin(float px, float py, int H, int W) {
  const float ix = src_coord(px, W), iy = src_coord(py, H);
  Bilin b;
  b.x0 = (int)floorf(ix);
  b.y0 = (int)floorf(iy);
  b.wx1 = ix - (float)b.x0;
  b.wy1 = iy - (float)b.y0;
  return b;
}
__device__ __forceinline__ float tap(const float* pl, int x, int y, int H, int W) {
  return (x >= 0 && x < W && y >= 0 && y < H) ? pl[(int64_t)y * W + x] : 0.f;
}

__global__ __launch_bounds__(256) void point_sample_kernel(const float* __restrict__ in, int C, int H, int W,
                                                           const int32_t* __restrict__ planes,
                                                           const float* __restrict__ coords, int P,
                                                           float* __restrict__ out) {
  const int box = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const float2 c = reinterpret_cast<const float2*>(coords)[(int64_t)box * P + p];
  const Bilin b = bilin(c.x, c.y, H, W);
  const float w00 = (1.f - b.wx1) * (1.f - b.wy1), w01 = b.wx1 * (1.f - b.wy1);
  const float w10 = (1.f - b.wx1) * b.wy1, w11 = b.wx1 * b.wy1;
  const int64_t hw = (int64_t)H * W;
  const float* base = in + (planes ? (int64_t)planes[box] * hw : (int64_t)box * C * hw);
  for (int ch = 0; ch < C; ++ch) {
    const float* pl = base + ch * hw;
    // torch's grid_sampler_2d sums the four taps in this order (nw, ne, sw, se)
    const float v = tap(pl, b.x0, b.y0, H, W) * w00 + tap(pl, b.x0 + 1, b.y0, H, W) * w01 +
                    tap(pl, b.x0, b.y0 + 1, H, W) * w10 + tap(pl, b.x0 + 1, b.y0 + 1, H, W) * w11;
    out[((int64_t)box * C + ch) * P + p] = v;
  }
}

__device__ __forceinline__ void scatter(float* pl, int x, int y, int H, int W, float v) {
  if (x >= 0 && x < W && y >= 0 && y < H && v != 0.f) atomicAdd(pl + (int64_t)y * W + x, v);
}

__global__ __launch_bounds__(256) void point_sample_bwd_kernel(const float* __restrict__ dout, int C, int H, int W,
                                                               const int32_t* __restrict__ planes,
                                                               const float* __restrict__ coords, int P,
                                                               const float* __restrict__ scale_ptr, float scale,
                                                               float* __restrict__ din) {
  const int box = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const float s = scale * (scale_ptr ? *scale_ptr : 1.f);
  const float2 c = reinterpret_cast<const float2*>(coords)[(int64_t)box * P + p];
  const Bilin b = bilin(c.x, c.y, H, W);
  const float w00 = (1.f - b.wx1) * (1.f - b.wy1), w01 = b.wx1 * (1.f - b.wy1);
  const float w10 = (1.f - b.wx1) * b.wy1, w11 = b.wx1 * b.wy1;
  const int64_t hw = (int64_t)H * W;
  float* base = din + (planes ? (int64_t)planes[box] * hw : (int64_t)box * C * hw);
  for (int ch = 0; ch < C; ++ch) {
    const float g = dout[((int64_t)box * C + ch) * P + p] * s;
    float* pl = base + ch * hw;
    scatter(pl, b.x0, b.y0, H, W, g * w00);
    scatter(pl, b.x0 + 1, b.y0, H, W, g * w01);
    scatter(pl, b.x0, b.y0 + 1, H, W, g * w10);
    scatter(pl, b.x0 + 1, b.y0 + 1, H, W, g * w11);
  }
}

// mode 0: nearest label (int64 out); mode 1: bilinear of (target == cls[box]) (fp32 out)
__global__ __launch_bounds__(256) void point_labels_kernel(const int64_t* __restrict__ tgt, int H, int W,
                                                           const int32_t* __restrict__ img,
                                                           const int32_t* __restrict__ cls,
                                                           const float* __restrict__ coords, int P, int mode,
                                                           int64_t* __restrict__ lab, float* __restrict__ val) {
  const int box = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const float2 c = reinterpret_cast<const float2*>(coords)[(int64_t)box * P + p];
  const int64_t* t = tgt + (int64_t)(img ? img[box] : box) * H * W;
  if (mode == 0) {
    const int x = (int)rintf(src_coord(c.x, W)), y = (int)rintf(src_coord(c.y, H));
    const bool in = x >= 0 && x < W && y >= 0 && y < H;
    // grid_sample(targets.float(), mode='nearest') -> .long(): zeros padding gives label 0
    lab[(int64_t)box * P + p] = in ? (int64_t)(float)t[(int64_t)y * W + x] : 0;
    return;
  }
  const int64_t k = cls[box];
  const Bilin b = bilin(c.x, c.y, H, W);
  auto m = [&](int x, int y) -> float {
    return (x >= 0 && x < W && y >= 0 && y < H && t[(int64_t)y * W + x] == k) ? 1.f : 0.f;
  };
  val[(int64_t)box * P + p] = m(b.x0, b.y0) * ((1.f - b.wx1) * (1.f - b.wy1)) + m(b.x0 + 1, b.y0) * (b.wx1 * (1.f - b.wy1)) +
                              m(b.x0, b.y0 + 1) * ((1.f - b.wx1) * b.wy1) + m(b.x0 + 1, b.y0 + 1) * (b.wx1 * b.wy1);
}

__global__ __launch_bounds__(256) void point_uncertainty_kernel(const float* __restrict__ x, int C, int P,
                                                                float* __restrict__ u) {
  const int box = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const float* xb = x + (int64_t)box * C * P + p;
  if (C == 1) {
    u[(int64_t)box * P + p] = -fabsf(xb[0]);
    return;
  }
  float m1 = -INFINITY, m2 = -INFINITY;
  for (int ch = 0; ch < C; ++ch) {
    const float v = xb[(int64_t)ch * P];
    if (v > m1) { m2 = m1; m1 = v; }
    else if (v > m2) m2 = v;
  }
  u[(int64_t)box * P + p] = m2 - m1;
}

// order-preserving float -> uint32 (larger float -> larger key)
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// one 1024-thread block per row: 4 radix passes (8 bits) find the k-th largest key, then the
// selection: every key above it, then keys equal to it in index order until k are taken.
__global__ __launch_bounds__(1024) void topk_select_kernel(const float* __restrict__ u, int n, int k,
                                                           const float* __restrict__ coords,
                                                           int32_t* __restrict__ idx_out,
                                                           float* __restrict__ coords_out) {
  __shared__ int hist[256];
  __shared__ uint32_t s_prefix;
  __shared__ int s_need, s_gt, s_eqtaken;
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* ur = u + (int64_t)row * n;
  uint32_t prefix = 0, mask = 0;
  int need = k;                         // how many still to pick among keys matching the prefix
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += 1024) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
      const uint32_t key = fkey(ur[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1);
    }
    __syncthreads();
    if (tid == 0) {
      int acc = 0, d = 255;
      for (; d > 0; --d) {
        if (acc + hist[d] >= need) break;
        acc += hist[d];
      }
      s_prefix = prefix | ((uint32_t)d << shift);
      s_need = need - acc;
    }
    __syncthreads();
    prefix = s_prefix;
    need = s_need;
    mask |= 0xFFu << shift;
    __syncthreads();
  }
  const uint32_t kth = prefix;          // the k-th largest key; `need` of the keys == kth are taken
  if (tid == 0) { s_gt = 0; s_eqtaken = 0; }
  __syncthreads();
  // keys > kth: k - need of them, in any order (the loss sums over points)
  for (int i = tid; i < n; i += 1024) {
    const uint32_t key = fkey(ur[i]);
    if (key > kth) {
      const int slot = atomicAdd(&s_gt, 1);
      idx_out[(int64_t)row * k + slot] = i;
    }
  }
  __syncthreads();
  const int base = s_gt;                // == k - need
  // keys == kth: the first `need` in index order (a block-wide ordered scan, 1024 at a time)
  __shared__ int scan[1024];
  for (int i0 = 0; i0 < n && s_eqtaken < need; i0 += 1024) {
    const int i = i0 + tid;
    const int f = (i < n && fkey(ur[i]) == kth) ? 1 : 0;
    scan[tid] = f;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int v = tid >= o ? scan[tid - o] : 0;
      __syncthreads();
      scan[tid] += v;
      __syncthreads();
    }
    const int rank = s_eqtaken + scan[tid] - f;
    if (f && rank < need) idx_out[(int64_t)row * k + base + rank] = i;
    __syncthreads();
    if (tid == 1023) s_eqtaken += scan[1023];
    __syncthreads();
  }
  __syncthreads();
  if (coords_out) {
    for (int j = tid; j < k; j += 1024) {
      const int i = idx_out[(int64_t)row * k + j];
      reinterpret_cast<float2*>(coords_out)[(int64_t)row * k + j] =
          reinterpret_cast<const float2*>(coords)[(int64_t)row * n + i];
    }
  }
}

// cross entropy over C at each point; sums into acc[0] (loss) / acc[1] (count), fp64 atomics;
// grad (unscaled by the count) = (softmax - onehot) / T
__global__ __launch_bounds__(256) void point_ce_kernel(const float* __restrict__ x, const int64_t* __restrict__ lab,
                                                       int C, int P, float inv_t, int64_t ignore,
                                                       double* __restrict__ acc, float* __restrict__ grad) {
  const int box = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  const bool ok = p < P;
  double l = 0.0, cnt = 0.0;
  if (ok) {
    const float* xb = x + (int64_t)box * C * P + p;
    float* gb = grad + (int64_t)box * C * P + p;
    const int64_t y = lab[(int64_t)box * P + p];
    if (y == ignore) {
      for (int ch = 0; ch < C; ++ch) gb[(int64_t)ch * P] = 0.f;
    } else {
      float m = -INFINITY;
      for (int ch = 0; ch < C; ++ch) m = fmaxf(m, xb[(int64_t)ch * P] * inv_t);
      float s = 0.f;
      for (int ch = 0; ch < C; ++ch) s += expf(xb[(int64_t)ch * P] * inv_t - m);
      const float lse = m + logf(s);
      const float xy = (y >= 0 && y < C) ? xb[(int64_t)y * P] * inv_t : 0.f;
      l = (double)(lse - xy);
      cnt = 1.0;
      const float is = 1.f / s;
      for (int ch = 0; ch < C; ++ch) {
        const float pr = expf(xb[(int64_t)ch * P] * inv_t - m) * is;
        gb[(int64_t)ch * P] = (pr - (ch == y ? 1.f : 0.f)) * inv_t;
      }
    }
  }
  l = wave_sum_d(l);
  cnt = wave_sum_d(cnt);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(acc, l);
    atomicAdd(acc + 1, cnt);
  }
}

// one block per mask: BCE mean over P + dice; loss sums into acc[0] (bce) and acc[1] (dice);
// grad = d(bce_mean + dice) / dx (the caller scales by 1 / num_masks)
__global__ __launch_bounds__(256) void point_bce_dice_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                             int P, double* __restrict__ acc,
                                                             float* __restrict__ grad) {
  __shared__ float red[3][4];
  const int box = blockIdx.x, tid = threadIdx.x;
  const float* xb = x + (int64_t)box * P;
  const float* yb = y + (int64_t)box * P;
  float bce = 0.f, sy = 0.f, ss = 0.f, ssy = 0.f;
  for (int p = tid; p < P; p += 256) {
    const float v = xb[p], t = yb[p];
    bce += fmaxf(v, 0.f) - v * t + log1pf(expf(-fabsf(v)));
    const float s = 1.f / (1.f + expf(-v));
    ss += s;
    sy += t;
    ssy += s * t;
  }
  bce = wave_sum(bce); ss = wave_sum(ss); sy = wave_sum(sy); ssy = wave_sum(ssy);
  __shared__ float r4[4][4];
  if ((tid & 63) == 0) { r4[tid >> 6][0] = bce; r4[tid >> 6][1] = ss; r4[tid >> 6][2] = sy; r4[tid >> 6][3] = ssy; }
  __syncthreads();
  bce = r4[0][0] + r4[1][0] + r4[2][0] + r4[3][0];
  ss = r4[0][1] + r4[1][1] + r4[2][1] + r4[3][1];
  sy = r4[0][2] + r4[1][2] + r4[2][2] + r4[3][2];
  ssy = r4[0][3] + r4[1][3] + r4[2][3] + r4[3][3];
  const float num = 2.f * ssy + 1.f, den = ss + sy + 1.f;
  if (tid == 0) {
    atomicAdd(acc, (double)(bce / (float)P));
    atomicAdd(acc + 1, (double)(1.f - num / den));
  }
  (void)red;
  const float invp = 1.f / (float)P;
  for (int p = tid; p < P; p += 256) {
    const float v = xb[p], t = yb[p];
    const float s = 1.f / (1.f + expf(-v));
    const float ddice_ds = -(2.f * t * den - num) / (den * den);
    grad[(int64_t)box * P + p] = (s - t) * invp + ddice_ds * s * (1.f - s);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void silu_kernel(const T* __restrict__ z, const T* __restrict__ dy, int64_t n,
                                                   T* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = to_f(z[i]);
    const float s = 1.f / (1.f + expf(-v));
    out[i] = from_f<T>(dy ? to_f(dy[i]) * s * (1.f + v * (1.f - s)) : v * s);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void s2d_kernel(const T* __restrict__ d, int B, int H, int W, int C,
                                                  T* __restrict__ out) {
  const int64_t n = (int64_t)B * H * W * 4 * C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C);
    int64_t r = i / C;
    const int q = (int)(r % 4);
    r /= 4;
    const int x = (int)(r % W);
    r /= W;
    const int y = (int)(r % H);
    const int b = (int)(r / H);
    const int yy = 2 * y + (q >> 1), xx = 2 * x + (q & 1);
    out[i] = d[(((int64_t)b * 2 * H + yy) * 2 * W + xx) * C + c];
  }
}

// moments NCHW fp32 [B, 2L, HW]; eps [B, L, HW]; z [B, L, HW]
__global__ __launch_bounds__(256) void posterior_sample_kernel(const float* __restrict__ mom, const float* __restrict__ eps,
                                                               int L, int hw, int64_t n, float* __restrict__ z) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / ((int64_t)L * hw), r = i - b * L * hw;
    const float mean = mom[b * 2 * L * hw + r];
    const float lv = fminf(fmaxf(mom[b * 2 * L * hw + (int64_t)L * hw + r], -30.f), 20.f);
    z[i] = mean + expf(0.5f * lv) * eps[i];
  }
}

// dz read from NHWC rows with c_stride channels (the decoder's dgrad output); dmom NCHW fp32
template <typename T>
__global__ __launch_bounds__(256) void posterior_bwd_kernel(const float* __restrict__ mom, const float* __restrict__ eps,
                                                            const T* __restrict__ dz, int c_stride, int L, int hw,
                                                            int64_t n, float* __restrict__ dmom) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / ((int64_t)L * hw), r = i - b * L * hw;
    const int c = (int)(r / hw), pix = (int)(r - (int64_t)c * hw);
    const float g = to_f(dz[((int64_t)b * hw + pix) * c_stride + c]);
    const float raw = mom[b * 2 * L * hw + (int64_t)L * hw + r];
    const float lv = fminf(fmaxf(raw, -30.f), 20.f);
    dmom[b * 2 * L * hw + r] = g;
    dmom[b * 2 * L * hw + (int64_t)L * hw + r] = (raw > -30.f && raw < 20.f) ? g * eps[i] * 0.5f * expf(0.5f * lv) : 0.f;
  }
}

unsigned grid_for(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 16)); }

}  // namespace

extern "C" int ldm_point_sample(const float* in, int boxes, int c, int h, int w, const int32_t* planes,
                                const float* coords, int p, float* out, ldm_stream_t stream) {
  if (!in || !coords || !out || boxes <= 0 || c <= 0 || h <= 0 || w <= 0 || p <= 0) return LDM_ERR_ARG;
  hipLaunchKernelGGL(point_sample_kernel, dim3((p + 255) / 256, boxes), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), in, c, h, w, planes, coords, p, out);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_point_sample_bwd(const float* dout, int boxes, int c, int h, int w, const int32_t* planes,
                                    const float* coords, int p, const float* scale_ptr, float scale, float* din,
                                    ldm_stream_t stream) {
  if (!dout || !coords || !din || boxes <= 0 || c <= 0 || h <= 0 || w <= 0 || p <= 0) return LDM_ERR_ARG;
  hipLaunchKernelGGL(point_sample_bwd_kernel, dim3((p + 255) / 256, boxes), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), dout, c, h, w, planes, coords, p, scale_ptr, scale, din);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_point_labels(const int64_t* targets, int h, int w, const int32_t* img, const int32_t* cls,
                                const float* coords, int boxes, int p, int mode, int64_t* labels, float* values,
                                ldm_stream_t stream) {
  if (!targets || !coords || boxes <= 0 || p <= 0 || h <= 0 || w <= 0) return LDM_ERR_ARG;
  if ((mode == 0 && !labels) || (mode == 1 && (!values || !cls)) || mode < 0 || mode > 1) return LDM_ERR_ARG;
  hipLaunchKernelGGL(point_labels_kernel, dim3((p + 255) / 256, boxes), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), targets, h, w, img, cls, coords, p, mode, labels, values);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_point_uncertainty(const float* x, int boxes, int c, int p, float* u, ldm_stream_t stream) {
  if (!x || !u || boxes <= 0 || c <= 0 || p <= 0) return LDM_ERR_ARG;
  hipLaunchKernelGGL(point_uncertainty_kernel, dim3((p + 255) / 256, boxes), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), x, c, p, u);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_topk_select(const float* u, int rows, int n, int k, const float* coords, int32_t* idx,
                               float* coords_out, ldm_stream_t stream) {
  if (!u || !idx || rows <= 0 || n <= 0 || k <= 0 || k > n || (coords_out && !coords)) return LDM_ERR_ARG;
  hipLaunchKernelGGL(topk_select_kernel, dim3(rows), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream), u, n, k,
                     coords, idx, coords_out);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_point_ce(const float* x, const int64_t* labels, int boxes, int c, int p, float temperature,
                            int64_t ignore_label, double* acc, float* grad, ldm_stream_t stream) {
  if (!x || !labels || !acc || !grad || boxes <= 0 || c <= 0 || p <= 0 || !(temperature > 0.f)) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(acc, 0, 2 * sizeof(double), s) != hipSuccess) return LDM_ERR_LAUNCH;
  hipLaunchKernelGGL(point_ce_kernel, dim3((p + 255) / 256, boxes), dim3(256), 0, s, x, labels, c, p,
                     1.f / temperature, ignore_label, acc, grad);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_point_bce_dice(const float* x, const float* y, int masks, int p, double* acc, float* grad,
                                  ldm_stream_t stream) {
  if (!x || !y || !acc || !grad || masks <= 0 || p <= 0) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(acc, 0, 2 * sizeof(double), s) != hipSuccess) return LDM_ERR_LAUNCH;
  hipLaunchKernelGGL(point_bce_dice_kernel, dim3(masks), dim3(256), 0, s, x, y, p, acc, grad);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_silu(const void* z, const void* dy, int64_t n, void* out, int dtype, ldm_stream_t stream) {
  if (!z || !out || n <= 0 || (dtype != LDM_F32 && dtype != LDM_BF16)) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == LDM_BF16)
    hipLaunchKernelGGL((silu_kernel<bf16_t>), dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)z, (const bf16_t*)dy,
                       n, (bf16_t*)out);
  else
    hipLaunchKernelGGL((silu_kernel<float>), dim3(grid_for(n)), dim3(256), 0, s, (const float*)z, (const float*)dy, n,
                       (float*)out);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_space_to_depth2(const void* d, int batch, int h, int w, int c, void* out, int dtype,
                                   ldm_stream_t stream) {
  if (!d || !out || batch <= 0 || h <= 0 || w <= 0 || c <= 0 || (dtype != LDM_F32 && dtype != LDM_BF16))
    return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = (int64_t)batch * h * w * 4 * c;
  if (dtype == LDM_BF16)
    hipLaunchKernelGGL((s2d_kernel<bf16_t>), dim3(grid_for(n)), dim3(256), 0, s, (const bf16_t*)d, batch, h, w, c,
                       (bf16_t*)out);
  else
    hipLaunchKernelGGL((s2d_kernel<float>), dim3(grid_for(n)), dim3(256), 0, s, (const float*)d, batch, h, w, c,
                       (float*)out);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_posterior_sample(const float* moments, const float* eps, int batch, int latent, int hw, float* z,
                                    ldm_stream_t stream) {
  if (!moments || !eps || !z || batch <= 0 || latent <= 0 || hw <= 0) return LDM_ERR_ARG;
  const int64_t n = (int64_t)batch * latent * hw;
  hipLaunchKernelGGL(posterior_sample_kernel, dim3(grid_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     moments, eps, latent, hw, n, z);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_posterior_bwd(const float* moments, const float* eps, const void* dz, int c_stride, int batch,
                                 int latent, int hw, float* dmoments, int dtype, ldm_stream_t stream) {
  if (!moments || !eps || !dz || !dmoments || batch <= 0 || latent <= 0 || hw <= 0 || c_stride < latent)
    return LDM_ERR_ARG;
  const int64_t n = (int64_t)batch * latent * hw;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == LDM_BF16)
    hipLaunchKernelGGL((posterior_bwd_kernel<bf16_t>), dim3(grid_for(n)), dim3(256), 0, s, moments, eps,
                       (const bf16_t*)dz, c_stride, latent, hw, n, dmoments);
  else if (dtype == LDM_F32)
    hipLaunchKernelGGL((posterior_bwd_kernel<float>), dim3(grid_for(n)), dim3(256), 0, s, moments, eps,
                       (const float*)dz, c_stride, latent, hw, n, dmoments);
  else
    return LDM_ERR_ARG;
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
