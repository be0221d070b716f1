// Training-path kernels: the backward pass of the denoiser and the optimizer step.
//
// The reference trains the UNet with torch autograd + AdamW (trainers_ldm_cond.py:792-900,
// update_weights :769-781; optimizer trainers/optim.py:53-82).  Here the backward of every
// fused forward op is hand-written:
//   ldm_conv2d_wgrad     dW[n][k] = sum_m dY[m][n] A[m][k]: implicit GEMM over the pixel axis,
//                        both operands staged by LDS-DMA into XOR-swizzled [64 m][256 B] images
//                        and read TRANSPOSED (ds_read_b64_tr_b16) as MFMA fragments; the pixel
//                        axis is split over blocks into an fp32 slab that a second kernel sums
//                        straight into the torch weight layout ([n][c][ky][kx], GEGLU rows
//                        un-interleaved).  (The data gradient is ldm_conv2d itself with the
//                        transposed/flipped weight; stride 2 via its zero-insert gather.)
//   ldm_colsum           per-segment column sums (bias grads; per-batch time-embedding grads)
//   ldm_group_norm_bwd   GroupNorm(+SiLU) backward from the forward's saved (mean, rstd)
//   ldm_layer_norm_bwd   LayerNorm backward (+ the residual-stream gradient add)
//   ldm_geglu_fwd/bwd    h * gelu(g) on the interleaved [h16 | g16] GEMM output
//   ldm_sum_pool2        dgrad of the nearest-2x upsample (2x2 sum)
//   ldm_mse_loss         masked, SNR-weighted L2 loss + its gradient (trainers_ldm_cond.py:592-604)
//   ldm_sq_norm / ldm_adamw   global grad norm (clip_grad_norm_) and a fused AdamW over flat
//                        fp32 master buffers (per-parameter lr / weight decay segments)
#include "common.h"

#include <algorithm>

namespace {

__device__ const uint4 kZero16 = {0u, 0u, 0u, 0u};

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ======================================================================================
// weight gradient
// ======================================================================================
struct WgArgs {
  const char* a0; const char* a1;
  int c0, c1, cin;
  int h_in, w_in, h_out, w_out, hw_out, ksize, stride, upsample, pad;
  const char* dy;
  int n, kpad, K, M;
  int tiles_n, splits;
  float* part;                  // [splits][n][kpad]
  float inv_hw, inv_w;          // 1 / hw_out, 1 / w_out (pixel decode by reciprocal, M < 2^24)
};

// q = x / d, r = x % d for 0 <= x < 2^24 from a float reciprocal (|x * inv - x / d| < 1, one
// correction step): ~8 VALU instead of an integer division's ~30 — the wgrad loader decodes 4
// pixels per lane per 64-pixel stage
__device__ __forceinline__ void fdivmod(int x, int d, float inv, int& q, int& r) {
  q = (int)((float)x * inv);
  r = x - q * d;
  if (r < 0) { --q; r += d; }
  else if (r >= d) { ++q; r -= d; }
}


// XOR swizzle of the 16 16-byte chunks of a 256-byte row: serves the transposed fragment
// reads (and row reads) conflict-free (cdna_hip_programming.md T10 image (b)).
__device__ __forceinline__ int wg_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// MFMA 16x16x32 fragment of a [rows = reduction][cols] image, read transposed: lane (g, lr)
// gets column col0 + lr of rows r0 + 8g + j, j = 0..7 (the A map with A[row=col][k=row] and
// the B map with B[k=row][col]).
template <typename T> __device__ __forceinline__ Frag8<T> wg_frag(const char* img, int r0, int col0, int lane);
template <>
__device__ __forceinline__ Frag8<bf16_t> wg_frag<bf16_t>(const char* img, int r0, int col0, int lane) {
  typedef __attribute__((ext_vector_type(4))) short s4_t;
  typedef __attribute__((address_space(3))) s4_t lds_s4_t;
  const int g = lane >> 4, lr = lane & 15, q = lr >> 2, pp = lr & 3;
  const int chunk = (col0 >> 3) + (pp >> 1);
  uint2 h[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int row = r0 + 8 * g + 4 * hh + q;
    const char* addr = img + row * 256 + 16 * (chunk ^ wg_swz(row)) + 8 * (pp & 1);
    const s4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(addr));
    h[hh] = __builtin_bit_cast(uint2, x);
  }
  Frag8<bf16_t> f;
  f.v = make_uint4(h[0].x, h[0].y, h[1].x, h[1].y);
  return f;
}
template <>
__device__ __forceinline__ Frag8<float> wg_frag<float>(const char* img, int r0, int col0, int lane) {
  const int g = lane >> 4, lr = lane & 15;
  const int col = col0 + lr;
  Frag8<float> f;
  float* e = reinterpret_cast<float*>(&f.v[0]);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = r0 + 8 * g + j;
    e[j] = *reinterpret_cast<const float*>(img + row * 256 + 16 * ((col >> 2) ^ wg_swz(row)) + 4 * (col & 3));
  }
  return f;
}

// One block = one [TE n] x [TE k] tile of dW over one pixel range.  TE = 128 (bf16) / 64 (fp32),
// i.e. 256-byte image rows.  4 waves as 2 (n) x 2 (k), wave tile TE/2 x TE/2.
// Stages of MB pixels in an NS-slot LDS ring.  The main loop is bound by operand latency, not by
// the MFMA or the LDS reads (ablation builds, profiles/r03_r3j_wgrad.txt: loads removed 410 -> 152
// us, MFMAs removed 410 -> 364 us at the 64x64-level 3x3 320): with one 32-KB 64-pixel stage in
// flight per block (NS = 2) every stage waits out a memory round trip.  The bf16 default is a ring of
// four 32-pixel stages (16 KB each, three in flight, counted vmcnt and a raw barrier per stage).
// Loader modes (block-uniform, chosen on the host): WG_GENERAL walks (b, y, x) and decodes every
// source pixel (stride 2, upsample); WG_1X1 (1x1, stride 1) and WG_PLAIN (k x k, stride 1, same
// size, 16 / w_out < h_out) keep one pointer per operand that advances by 16 rows per DMA and test
// the tap's bounds with a wrap-by-one-subtraction (x, y) walker: straight-line selects, no
// divergent branches (the branchy general form cost 6.7 VALU + 5.6 SALU per MFMA, r04k PMC).
enum { WG_GENERAL = 0, WG_1X1 = 1, WG_PLAIN = 2 };

template <typename T, int MB, int NS, int MODE = WG_GENERAL>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(const WgArgs p) {
  constexpr int ES = sizeof(T), EPC = 16 / ES;
  constexpr int TE = 256 / ES, WT = TE / 2, NF = WT / 16;
  constexpr int IMG = MB * 256;                  // bytes per operand image of one stage
  constexpr int PER = 2 * (MB / 16);             // DMA instructions per wave and stage
  __shared__ uint4 smem[NS * 2 * IMG / 16];
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const char* sbase = reinterpret_cast<const char*>(smem);

  // XCD-contiguous ids (block b runs on XCD b mod 8), tiles fastest: an XCD works through one or two
  // M ranges (splits) for all of their output tiles, so their dy / x rows are shared in its L2.
  // (split fastest spread every XCD over all splits whenever splits != 8: L2 hit rate 0.21 / 0.51,
  // 1.4 / 2.9 GB fetched for the GEGLU 320 / up-block 960 weight gradients, r04k PMC)
  int split, tile;
  {
    const int bid = blockIdx.x, nblk = gridDim.x;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    const int t = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
    const int ntile = nblk / p.splits;
    split = t / ntile;
    tile = t - split * ntile;
  }
  const int tn = tile % p.tiles_n, tk = tile / p.tiles_n;
  const int n0 = tn * TE, k0 = tk * TE;
  const int m_lo = (int)((int64_t)p.M * split / p.splits);
  const int m_hi = (int)((int64_t)p.M * (split + 1) / p.splits);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // loader: wave-instruction i of wave w fills image rows 16 i + 4 w .. +3 lane-linearly;
  // lane -> (row 16 i + 4 w + (lane >> 4), physical chunk lane & 15) -> logical chunk
  const int rlow = 4 * wave + (lane >> 4);
  const int ch = (lane & 15) ^ wg_swz(rlow);
  const int ncol = n0 + ch * EPC;
  const bool nval = ncol < p.n;
  const int kk = k0 + ch * EPC;
  const bool kval = kk < p.K;
  const int tap = kval ? kk / p.cin : 0;
  const int c = kk - tap * p.cin;
  const int ky = tap / p.ksize, kx = tap - ky * p.ksize;
  const bool s1 = c >= p.c0;
  const T* xs = reinterpret_cast<const T*>(s1 ? p.a1 : p.a0);
  const int cs = s1 ? p.c1 : p.c0;
  const int cof = s1 ? c - p.c0 : c;
  const int hin_v = p.upsample ? 2 * p.h_in : p.h_in, win_v = p.upsample ? 2 * p.w_in : p.w_in;

  // Row walker: the lane's pixel rows are m_lo + rlow + 16 j, visited in order by successive issue()
  // calls (4 per 64-pixel stage), so (b, oy, ox) advances by a precomputed (q16, r16) = divmod(16,
  // w_out) instead of being decoded per row (the per-row decode was the loader's VALU bound: ~45
  // VALU per row, more issue cycles than the stage's MFMAs).  Stride 1 without upsampling (the
  // 3x3 / 1x1 convs but Downsample / Upsample) keeps the source pixel = row + a per-lane constant,
  // so both operand addresses advance by one add per row.
  int wb, wy, wx;
  fdivmod(m_lo + rlow, p.hw_out, p.inv_hw, wb, wy);
  { int q; fdivmod(wy, p.w_out, p.inv_w, q, wx); wy = q; }
  const int q16 = 16 / p.w_out, r16 = 16 - q16 * p.w_out;
  const bool plain = p.stride == 1 && !p.upsample && p.h_in == p.h_out && p.w_in == p.w_out;
  const bool noborder = plain && p.ksize == 1;
  // plain: source pixel = m + (ky - pad) * w_in + (kx - pad) (valid only when in bounds)
  const int pix_shift = (ky - p.pad) * p.w_in + (kx - p.pad);
  int mrow = m_lo + rlow;
  // fast modes: per-lane operand pointers (unused lanes are redirected to kZero16 by a select)
  const char* dyp = p.dy + ((int64_t)mrow * p.n + ncol) * ES;
  const char* xp = reinterpret_cast<const char*>(xs + ((int64_t)mrow + (MODE == WG_PLAIN ? pix_shift : 0)) * cs + cof);
  const int64_t dystep = (int64_t)16 * p.n * ES, xstep = (int64_t)16 * cs * ES;
  const int dyk = ky - p.pad, dxk = kx - p.pad;
  auto issue = [&](int mb, int slot) {
    (void)mb;
#ifdef LDM_ABL_NO_LOADS
    return;
#endif
    const unsigned dyb = lds0 + (unsigned)(slot * 2 * IMG);
    const unsigned xb = dyb + IMG;
    if constexpr (MODE != WG_GENERAL) {
#pragma unroll
      for (int i = 0; i < MB / 16; ++i) {
        const bool mok = mrow < m_hi;
        bool xok = mok && kval;
        if constexpr (MODE == WG_PLAIN)
          xok = xok && (unsigned)(wy + dyk) < (unsigned)p.h_in && (unsigned)(wx + dxk) < (unsigned)p.w_in;
        const void* sd = (mok && nval) ? (const void*)dyp : (const void*)&kZero16;
        const void* sx = xok ? (const void*)xp : (const void*)&kZero16;
        const unsigned off = (unsigned)((16 * i + 4 * wave) * 256);
        glds16(sd, __builtin_amdgcn_readfirstlane(dyb + off));
        glds16(sx, __builtin_amdgcn_readfirstlane(xb + off));
        mrow += 16;
        dyp += dystep;
        xp += xstep;
        if constexpr (MODE == WG_PLAIN) {
          wx += r16;
          const int c = wx >= p.w_out;
          wx -= c ? p.w_out : 0;
          wy += q16 + c;
          wy -= wy >= p.h_out ? p.h_out : 0;
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < MB / 16; ++i) {
      const int m = mrow;
      const bool mok = m < m_hi;
      const void* sd = (mok && nval) ? (const void*)(p.dy + ((int64_t)m * p.n + ncol) * ES) : (const void*)&kZero16;
      const void* sx = &kZero16;
      if (mok && kval && noborder) {
        sx = xs + (int64_t)m * cs + cof;                  // 1x1, stride 1: the source row is the row
      } else if (mok && kval) {
        const int uy = (p.upsample ? wy : wy * p.stride) - p.pad + ky;
        const int ux = (p.upsample ? wx : wx * p.stride) - p.pad + kx;
        if ((unsigned)uy < (unsigned)hin_v && (unsigned)ux < (unsigned)win_v) {
          int64_t pix;
          if (plain) pix = (int64_t)m + pix_shift;
          else pix = ((int64_t)wb * p.h_in + (p.upsample ? (uy >> 1) : uy)) * p.w_in + (p.upsample ? (ux >> 1) : ux);
          sx = xs + pix * cs + cof;
        }
      }
      const unsigned off = (unsigned)((16 * i + 4 * wave) * 256);
      glds16(sd, __builtin_amdgcn_readfirstlane(dyb + off));
      glds16(sx, __builtin_amdgcn_readfirstlane(xb + off));
      // advance the walker by 16 rows
      mrow += 16;
      if (!noborder) {
        wx += r16;
        wy += q16;
        if (wx >= p.w_out) { wx -= p.w_out; ++wy; }
        while (wy >= p.h_out) { wy -= p.h_out; ++wb; }
      }
    }
  };

  const int wn = wave & 1, wk = wave >> 1;
  f32x4_t acc[NF][NF];
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int slot) {
    const char* dyi = sbase + slot * 2 * IMG;
    const char* xi = dyi + IMG;
#pragma unroll
    for (int s = 0; s < MB / 32; ++s) {
      Frag8<T> af[NF], bf[NF];
#pragma unroll
      for (int i = 0; i < NF; ++i) af[i] = wg_frag<T>(dyi, 32 * s, wn * WT + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < NF; ++j) bf[j] = wg_frag<T>(xi, 32 * s, wk * WT + 16 * j, lane);
#ifdef LDM_ABL_NO_MFMA
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int i = 0; i < NF; ++i) asm volatile("" ::"v"(af[i].v.x), "v"(bf[i].v.x));
        continue;
      }
#endif
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) mma_k32(acc[i][j], af[i], bf[j]);
    }
  };

  if (m_lo < m_hi) {
    const int nst = (m_hi - m_lo + MB - 1) / MB;
    if constexpr (NS == 2) {
      issue(m_lo, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int st = 0; st < nst; ++st) {
        const int slot = st & 1;
        if (st + 1 < nst) issue(m_lo + (st + 1) * MB, slot ^ 1);
        compute(slot);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    } else {
      static_assert(NS == 4 || NS == 5, "ring depth");
#pragma unroll
      for (int i = 0; i < NS - 1; ++i)
        if (i < nst) issue(m_lo + i * MB, i);
      for (int st = 0; st < nst; ++st) {
        // stage st landed for this wave; the (up to NS - 2) younger stages may stay in flight
        const int ahead = min(NS - 2, nst - 1 - st);
        if (NS == 5 && ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER) : "memory");
        else if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // raw barrier (__syncthreads would drain the stages in flight): every wave's part of stage st
        // is in LDS and every wave is done with the slot stage st + 3 reuses (stage st - 1's)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (st + NS - 1 < nst) issue(m_lo + (st + NS - 1) * MB, (st + NS - 1) % NS);
        compute(st % NS);
      }
      __syncthreads();
    }
  }
  // C/D: row = n (4g + r), col = k (lane & 15)
  const int g = lane >> 4, lr = lane & 15;
  float* part = p.part + (int64_t)split * p.n * p.kpad;
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int k = k0 + wk * WT + 16 * j + lr;
      if (k >= p.kpad) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * WT + 16 * i + 4 * g + r;
        if (n < p.n) part[(int64_t)n * p.kpad + k] = acc[i][j][r];
      }
    }
}

// packed GEGLU row (hidden/gate interleaved in 16-row blocks) of torch row nt
__device__ __forceinline__ int geglu_packed_row(int nt, int half) {
  const int hi = nt >= half;
  const int i = hi ? nt - half : nt;
  return (i >> 4) * 32 + 16 * hi + (i & 15);
}

// 3x3 form: the torch layout puts a channel's 9 taps together, so the element-per-thread form's
// stores land 36 bytes apart.  Here a wave owns one packed row and 64 channels: lane c sums its 9
// taps over the splits (9 coalesced 256-byte reads per split, splits in order as above), the wave
// stages the [64 c][9 taps] block in LDS and writes it back as 9 contiguous 256-byte runs.
__global__ __launch_bounds__(256) void wgrad_reduce3(const float* __restrict__ part, int splits, int n, int kpad,
                                                     int cin_pad, int cin_real, int geglu, float* __restrict__ dst,
                                                     int accumulate) {
  __shared__ float st[4][64 * 9];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ncb = (cin_real + 63) / 64;
  const int item = blockIdx.x * 4 + w;
  if (item >= n * ncb) return;   // wave-uniform; no block barrier below
  const int np = item / ncb, c0 = (item - np * ncb) * 64;
  const int c = c0 + lane;
  const int total = n * kpad;
  float sum[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) sum[t] = 0.f;
  if (c < cin_real) {
    const float* src = part + (int64_t)np * kpad + c;
    for (int sp = 0; sp < splits; ++sp) {
      float v[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) v[t] = src[(int64_t)sp * total + t * cin_pad];
#pragma unroll
      for (int t = 0; t < 9; ++t) sum[t] += v[t];
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) st[w][lane * 9 + t] = sum[t];
  // the wave's own LDS rows: a wavefront-scope fence orders the stores before the transposed reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  int nt = np;
  if (geglu) {  // inverse of geglu_packed_row
    const int blk = np >> 5, r = np & 31, half = n >> 1;
    nt = (r < 16) ? blk * 16 + r : half + blk * 16 + (r - 16);
  }
  const int nc = min(64, cin_real - c0);
  float* out = dst + ((int64_t)nt * cin_real + c0) * 9;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int o = j * 64 + lane;
    if (o < nc * 9) {
      const float v = st[w][o];
      out[o] = accumulate ? out[o] + v : v;
    }
  }
}

// Sum the split slab into the torch weight layout.  Thread per packed element (coalesced slab
// reads).  dst[nt][c][ky][kx] (ksize 3) or dst[nt][c] (ksize 1), c < cin_real.
__global__ __launch_bounds__(256) void wgrad_reduce(const float* __restrict__ part, int splits, int n, int kpad,
                                                    int ksize, int cin_pad, int cin_real, int geglu,
                                                    float* __restrict__ dst, int accumulate) {
  const int total = n * kpad;   // < 2^31 (checked by the launcher)
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int np = (int)((unsigned)idx / (unsigned)kpad), k = idx - np * kpad;
  const int taps = ksize * ksize;
  const int tap = k / cin_pad, c = k - tap * cin_pad;
  if (tap >= taps || c >= cin_real) return;
  int nt = np;
  if (geglu) {  // inverse of geglu_packed_row
    const int blk = np >> 5, w = np & 31, half = n >> 1;
    nt = (w < 16) ? blk * 16 + w : half + blk * 16 + (w - 16);
  }
  // the splits in order, eight loads in flight (a load-add loop waits out the latency per split)
  float s = 0.f;
  int sp = 0;
  for (; sp + 8 <= splits; sp += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(sp + u) * total + idx];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; sp < splits; ++sp) s += part[(int64_t)sp * total + idx];
  const int64_t o = ((int64_t)nt * cin_real + c) * taps + tap;
  dst[o] = accumulate ? dst[o] + s : s;
}

// ======================================================================================
// column sums: out[seg][c] (+)= sum_{rows of seg} x[row][c]
// ======================================================================================
// Deterministic: every (row chunk, segment) block writes its column sums to its own row of the
// fp32 slab part[chunk][segment][C] (no atomics); slab_reduce then sums the chunks in order.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ x, int C, int rows_per_seg, int rchunk,
                                                     int geglu, float* __restrict__ part) {
  constexpr int EPC = 16 / sizeof(T);
  const int V = C / EPC;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int v = blockIdx.x * 64 + tx;
  const int seg = blockIdx.z;
  const int r0 = blockIdx.y * rchunk, r1 = min(rows_per_seg, r0 + rchunk);
  float s[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) s[e] = 0.f;
  if (v < V) {
    const T* base = x + (int64_t)seg * rows_per_seg * C + v * EPC;
    int r = r0 + ty;
    // eight rows in flight per thread (a single-load loop waits out the memory latency per row)
    for (; r + 28 < r1; r += 32) {
      uint4 raw[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) raw[u] = *reinterpret_cast<const uint4*>(base + (int64_t)(r + 4 * u) * C);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const T* e = reinterpret_cast<const T*>(&raw[u]);
#pragma unroll
        for (int k = 0; k < EPC; ++k) s[k] += to_f(e[k]);
      }
    }
    for (; r < r1; r += 4) {
      const uint4 raw = *reinterpret_cast<const uint4*>(base + (int64_t)r * C);
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int k = 0; k < EPC; ++k) s[k] += to_f(e[k]);
    }
  }
  __shared__ float red[4][64][EPC];
#pragma unroll
  for (int k = 0; k < EPC; ++k) red[ty][tx][k] = s[k];
  __syncthreads();
  if (ty == 0 && v < V) {
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      const float t = red[0][tx][k] + red[1][tx][k] + red[2][tx][k] + red[3][tx][k];
      int c = v * EPC + k;
      if (geglu) {
        const int blk = c >> 5, w = c & 31, half = C >> 1;
        c = (w < 16) ? blk * 16 + w : half + blk * 16 + (w - 16);
      }
      part[((int64_t)blockIdx.y * gridDim.z + seg) * C + c] = t;
    }
  }
}

// out[i] (+)= sum_{q < nparts} part[q * stride + i], i < width (the deterministic second pass of
// the slab reductions: column sums, LayerNorm / GroupNorm dgamma / dbeta).  Parts-parallel: a block
// owns 32 columns; its 8 part groups g sum parts q = g, g + 8, ... in order (four loads in flight),
// then the 8 group sums combine in the fixed order g = 0 .. 7 — deterministic, and a column's
// parts are walked by 8 threads instead of one (the serial form ran 128-512 dependent parts on
// 2-20 blocks: ~17.5 us per launch, latency-bound)
__global__ __launch_bounds__(256) void slab_reduce(const float* __restrict__ part, int nparts, int64_t stride,
                                                   int64_t width, float* __restrict__ out, int accumulate) {
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t i = (int64_t)blockIdx.x * 32 + cl;
  float s = 0.f;
  if (i < width) {
    int q = g;
    for (; q + 24 < nparts; q += 32) {       // four loads in flight, summed in order
      const float a = part[(int64_t)q * stride + i], b = part[(int64_t)(q + 8) * stride + i];
      const float c = part[(int64_t)(q + 16) * stride + i], d = part[(int64_t)(q + 24) * stride + i];
      s += a; s += b; s += c; s += d;
    }
    for (; q < nparts; q += 8) s += part[(int64_t)q * stride + i];
  }
  __shared__ float red[8][32];
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && i < width) {
    float t = red[0][cl];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += red[k][cl];
    out[i] = accumulate ? out[i] + t : t;
  }
}

// *sum (+)= sum_{q < n} part[q] (fp64), one block, fixed-order tree: the deterministic second pass of
// the loss and gradient-norm reductions
__global__ __launch_bounds__(256) void dsum_final(const double* __restrict__ part, int n, double* __restrict__ sum,
                                                  int accumulate) {
  __shared__ double red[256];
  double a = 0.0;
  for (int q = threadIdx.x; q < n; q += 256) a += part[q];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *sum = accumulate ? *sum + red[0] : red[0];
}

// ======================================================================================
// GroupNorm backward.  z = x_hat * gamma + beta, y = act(z); with dz = dy * act'(z):
//   dbeta_c = sum dz, dgamma_c = sum dz x_hat
//   dx = rstd * (gamma dz - mean_g(gamma dz) - x_hat * mean_g(gamma dz x_hat))
// ======================================================================================
constexpr int GNB_PPC = 64;

__device__ __forceinline__ float silu_grad(float z) {
  const float s = 1.0f / (1.0f + __expf(-z));
  return s * (1.0f + z * (1.0f - s));
}

template <typename T>
__device__ __forceinline__ uint4 load_cat(const T* x0, const T* x1, int c0, int c1, int64_t m, int c) {
  return (c < c0) ? *reinterpret_cast<const uint4*>(x0 + m * c0 + c)
                  : *reinterpret_cast<const uint4*>(x1 + m * c1 + (c - c0));
}

// partials per (b, 64-pixel chunk, channel): (sum dz, sum dz * x_hat)
template <typename T>
__global__ __launch_bounds__(256) void gnb_partial(const T* __restrict__ x0, const T* __restrict__ x1, int c0, int c1,
                                                   const T* __restrict__ dy, int hw, int chunks, int groups,
                                                   const float2* __restrict__ mr, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, int act,
                                                   float2* __restrict__ part) {
  constexpr int EPC = 16 / sizeof(T);
  const int C = c0 + c1, V = C / EPC, cpg = C / groups;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int v = blockIdx.x * 64 + tx;
  const int chunk = blockIdx.y, b = blockIdx.z;
  float s[EPC], sx[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) { s[e] = 0.f; sx[e] = 0.f; }
  if (v < V) {
    const int cb = v * EPC;
    float mean[EPC], rstd[EPC], gm[EPC], bt[EPC];
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      const float2 q = mr[(int64_t)b * groups + (cb + k) / cpg];
      mean[k] = q.x; rstd[k] = q.y; gm[k] = gamma[cb + k]; bt[k] = beta[cb + k];
    }
    const int p0 = chunk * GNB_PPC, p1 = min(hw, p0 + GNB_PPC);
    auto accum = [&](const uint4& rx, const uint4& rd) {
      const T* ex = reinterpret_cast<const T*>(&rx);
      const T* ed = reinterpret_cast<const T*>(&rd);
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        const float xh = (to_f(ex[k]) - mean[k]) * rstd[k];
        float dz = to_f(ed[k]);
        if (act == LDM_ACT_SILU) dz *= silu_grad(xh * gm[k] + bt[k]);
        s[k] += dz;
        sx[k] += dz * xh;
      }
    };
    int pix = p0 + ty;
    // four pixels' loads in flight per thread, then the same sums in pixel order
    for (; pix + 12 < p1; pix += 16) {
      uint4 rx[4], rd[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t m = (int64_t)b * hw + pix + 4 * u;
        rx[u] = load_cat(x0, x1, c0, c1, m, cb);
        rd[u] = *reinterpret_cast<const uint4*>(dy + m * C + cb);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) accum(rx[u], rd[u]);
    }
    for (; pix < p1; pix += 4) {
      const int64_t m = (int64_t)b * hw + pix;
      accum(load_cat(x0, x1, c0, c1, m, cb), *reinterpret_cast<const uint4*>(dy + m * C + cb));
    }
  }
  __shared__ float red[4][64][EPC][2];
#pragma unroll
  for (int k = 0; k < EPC; ++k) { red[ty][tx][k][0] = s[k]; red[ty][tx][k][1] = sx[k]; }
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

// per (b, group): coefficients k1 = -rstd * mean(gamma dz), k2 = -rstd * mean(gamma dz x_hat)
__global__ __launch_bounds__(256) void gnb_finalize(const float2* __restrict__ part, int C, int hw, int chunks,
                                                    int groups, const float2* __restrict__ mr,
                                                    const float* __restrict__ gamma, float2* __restrict__ coef) {
  const int b = blockIdx.x;
  const int gi = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (gi >= groups) return;
  const int cpg = C / groups;
  const int n = chunks * cpg;
  double a = 0.0, q = 0.0;
  for (int i = lane; i < n; i += 64) {
    const int ch = i / cpg, c = gi * cpg + (i - ch * cpg);
    const float2 v = part[((int64_t)b * chunks + ch) * C + c];
    a += (double)gamma[c] * v.x;
    q += (double)gamma[c] * v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o, 64); q += __shfl_xor(q, o, 64); }
  if (lane == 0) {
    const double cnt = (double)hw * cpg;
    const float rstd = mr[(int64_t)b * groups + gi].y;
    coef[(int64_t)b * groups + gi] = make_float2((float)(-rstd * a / cnt), (float)(-rstd * q / cnt));
  }
}

// per channel: dbeta, dgamma (+)= sum over (b, chunk)
// dgamma / dbeta from the per-(row chunk, channel) partials: a block owns 16 channels and splits
// the rows over 16 lanes per channel (eight loads in flight each), fp64 sums combined in LDS in a
// fixed order.  (One thread per channel summing every row serially was latency-bound: ~84 us per
// launch in the training profile.)
__global__ __launch_bounds__(256) void gnb_param(const float2* __restrict__ part, int C, int rows,
                                                 float* __restrict__ dgamma, float* __restrict__ dbeta, int accumulate) {
  constexpr int CH = 16, SL = 16, U = 8;
  __shared__ double2 red[SL][CH];
  const int cl = threadIdx.x % CH, sl = threadIdx.x / CH;
  const int c = blockIdx.x * CH + cl;
  double a = 0.0, q = 0.0;
  if (c < C) {
    int r = sl;
    for (; r + (U - 1) * SL < rows; r += U * SL) {
      float2 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = part[(int64_t)(r + u * SL) * C + c];
#pragma unroll
      for (int u = 0; u < U; ++u) { a += v[u].x; q += v[u].y; }
    }
    for (; r < rows; r += SL) {
      const float2 v = part[(int64_t)r * C + c];
      a += v.x;
      q += v.y;
    }
  }
  red[sl][cl] = make_double2(a, q);
  __syncthreads();
  if (sl == 0 && c < C) {
    for (int k = 1; k < SL; ++k) { a += red[k][cl].x; q += red[k][cl].y; }
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)a : (float)a;
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)q : (float)q;
  }
}

// dx = rstd gamma dz + k1 + k2 x_hat (+ add_src) (+ existing dst), split into the two sources
template <typename T>
__global__ __launch_bounds__(256) void gnb_apply(const T* __restrict__ x0, const T* __restrict__ x1, int c0, int c1,
                                                 const T* __restrict__ dy, int hw, int groups, int nvec,
                                                 const float2* __restrict__ mr, const float2* __restrict__ coef,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 int act, const T* __restrict__ add_src, T* dx0, T* dx1, int acc0,
                                                 int acc1) {
  constexpr int EPC = 16 / sizeof(T);
  const int C = c0 + c1, V = C / EPC, cpg = C / groups;
  const bool vec = cpg >= EPC && !(reinterpret_cast<uintptr_t>(gamma) & 15) &&
                   (act != LDM_ACT_SILU || !(reinterpret_cast<uintptr_t>(beta) & 15));
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += gridDim.x * 256) {
    const int mi = (int)((unsigned)i / (unsigned)V);   // 32-bit: nvec < 2^31 (launcher)
    const int64_t m = mi;
    const int cb = (i - mi * V) * EPC;
    const int b = (int)((unsigned)mi / (unsigned)hw);
    const uint4 rx = load_cat(x0, x1, c0, c1, m, cb);
    const uint4 rd = *reinterpret_cast<const uint4*>(dy + m * C + cb);
    const T* ex = reinterpret_cast<const T*>(&rx);
    const T* ed = reinterpret_cast<const T*>(&rd);
    float ad[EPC];
    if (add_src) {
      const uint4 ra = *reinterpret_cast<const uint4*>(add_src + m * C + cb);
      const T* ea = reinterpret_cast<const T*>(&ra);
#pragma unroll
      for (int k = 0; k < EPC; ++k) ad[k] = to_f(ea[k]);
    } else {
#pragma unroll
      for (int k = 0; k < EPC; ++k) ad[k] = 0.f;
    }
    const bool first = cb < c0;
    T* dst = first ? dx0 + m * c0 + cb : dx1 + m * c1 + (cb - c0);
    const bool acc = first ? acc0 : acc1;
    float prev[EPC];
    if (acc) {
      const uint4 rp = *reinterpret_cast<const uint4*>(dst);
      const T* ep = reinterpret_cast<const T*>(&rp);
#pragma unroll
      for (int k = 0; k < EPC; ++k) prev[k] = to_f(ep[k]);
    } else {
#pragma unroll
      for (int k = 0; k < EPC; ++k) prev[k] = 0.f;
    }
    uint4 res;
    T* r = reinterpret_cast<T*>(&res);
    if (vec) {
      // a vector spans at most two groups: both groups' statistics loaded once, selected per
      // channel (no per-channel division or scalar stat loads); gamma / beta as vectors
      const int gi0 = cb / cpg, bnd = (gi0 + 1) * cpg, gi1 = min(gi0 + 1, groups - 1);
      const float2 q0 = mr[b * groups + gi0], q1 = mr[b * groups + gi1];
      const float2 f0 = coef[b * groups + gi0], f1 = coef[b * groups + gi1];
      float gm[EPC], bt[EPC];
#pragma unroll
      for (int k = 0; k < EPC; k += 4) {
        const float4 g4 = *reinterpret_cast<const float4*>(gamma + cb + k);
        gm[k] = g4.x; gm[k + 1] = g4.y; gm[k + 2] = g4.z; gm[k + 3] = g4.w;
        if (act == LDM_ACT_SILU) {
          const float4 b4 = *reinterpret_cast<const float4*>(beta + cb + k);
          bt[k] = b4.x; bt[k + 1] = b4.y; bt[k + 2] = b4.z; bt[k + 3] = b4.w;
        }
      }
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        const bool hi = cb + k >= bnd;
        const float qx = hi ? q1.x : q0.x, qy = hi ? q1.y : q0.y;
        const float cx = hi ? f1.x : f0.x, cy = hi ? f1.y : f0.y;
        const float xh = (to_f(ex[k]) - qx) * qy;
        float dz = to_f(ed[k]);
        if (act == LDM_ACT_SILU) dz *= silu_grad(xh * gm[k] + bt[k]);
        r[k] = from_f<T>(qy * gm[k] * dz + cx + cy * xh + ad[k] + prev[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        const int gi = (cb + k) / cpg;
        const float2 q = mr[(int64_t)b * groups + gi];
        const float2 cf = coef[(int64_t)b * groups + gi];
        const float xh = (to_f(ex[k]) - q.x) * q.y;
        const float gm = gamma[cb + k];
        float dz = to_f(ed[k]);
        if (act == LDM_ACT_SILU) dz *= silu_grad(xh * gm + beta[cb + k]);
        r[k] = from_f<T>(q.y * gm * dz + cf.x + cf.y * xh + ad[k] + prev[k]);
      }
    }
    *reinterpret_cast<uint4*>(dst) = res;
  }
}

// ======================================================================================
// LayerNorm backward: one wave-group of G lanes per row (as the forward), stats recomputed.
//   dx = rstd (g - mean(g) - x_hat mean(g x_hat)),  g = gamma dy;  + add_src
//   dgamma += dy x_hat, dbeta += dy  (block partials to a slab, summed in order by slab_reduce)
// ======================================================================================
template <typename T, int G, int NV>
__global__ __launch_bounds__(256) void lnb_kernel(const T* __restrict__ x, const T* __restrict__ dy, int rows, int C,
                                                  const float* __restrict__ gamma, float eps,
                                                  const T* __restrict__ add_src, T* __restrict__ dx,
                                                  float* __restrict__ part) {
  constexpr int EPC = 16 / sizeof(T);
  constexpr int RPW = 64 / G;
  const int lane = threadIdx.x & 63;
  const int gl = lane % G;
  const int V = C / EPC;
  const float inv_c = 1.0f / (float)C;
  float pg[NV][EPC], pb[NV][EPC];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < EPC; ++k) { pg[i][k] = 0.f; pb[i][k] = 0.f; }
  const int stride = gridDim.x * 4 * RPW;
  for (int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / G; row - lane / G < rows; row += stride) {
    const bool rv = row < rows;
    float xv[NV][EPC], dv[NV][EPC];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = gl + G * i;
      if (rv && v < V) {
        const uint4 r1 = *reinterpret_cast<const uint4*>(x + (int64_t)row * C + v * EPC);
        const uint4 r2 = *reinterpret_cast<const uint4*>(dy + (int64_t)row * C + v * EPC);
        const T* e1 = reinterpret_cast<const T*>(&r1);
        const T* e2 = reinterpret_cast<const T*>(&r2);
#pragma unroll
        for (int k = 0; k < EPC; ++k) { xv[i][k] = to_f(e1[k]); dv[i][k] = to_f(e2[k]); s += xv[i][k]; }
      }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * inv_c;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (rv && gl + G * i < V) {
#pragma unroll
        for (int k = 0; k < EPC; ++k) { const float d = xv[i][k] - mean; q += d * d; }
      }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q * inv_c + eps);
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = gl + G * i;
      if (rv && v < V) {
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
          const float xh = (xv[i][k] - mean) * rstd;
          xv[i][k] = xh;
          const float gdy = gamma[v * EPC + k] * dv[i][k];
          sg += gdy;
          sgx += gdy * xh;
          pg[i][k] += dv[i][k] * xh;
          pb[i][k] += dv[i][k];
        }
      }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) { sg += __shfl_xor(sg, o, 64); sgx += __shfl_xor(sgx, o, 64); }
    const float mg = sg * inv_c, mgx = sgx * inv_c;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = gl + G * i;
      if (rv && v < V) {
        float ad[EPC];
        if (add_src) {
          const uint4 ra = *reinterpret_cast<const uint4*>(add_src + (int64_t)row * C + v * EPC);
          const T* ea = reinterpret_cast<const T*>(&ra);
#pragma unroll
          for (int k = 0; k < EPC; ++k) ad[k] = to_f(ea[k]);
        } else {
#pragma unroll
          for (int k = 0; k < EPC; ++k) ad[k] = 0.f;
        }
        uint4 res;
        T* r = reinterpret_cast<T*>(&res);
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
          const float gdy = gamma[v * EPC + k] * dv[i][k];
          r[k] = from_f<T>(rstd * (gdy - mg - xv[i][k] * mgx) + ad[k]);
        }
        *reinterpret_cast<uint4*>(dx + (int64_t)row * C + v * EPC) = res;
      }
    }
  }
  // dgamma / dbeta: lanes with the same gl share channels; reduce over the wave's row groups
  // with shuffles, then one atomic per channel per wave
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < EPC; ++k) {
      float a = pg[i][k], b2 = pb[i][k];
#pragma unroll
      for (int o = G; o < 64; o <<= 1) { a += __shfl_xor(a, o, 64); b2 += __shfl_xor(b2, o, 64); }
      pg[i][k] = a; pb[i][k] = b2;
    }
  // then the block's 4 waves are summed in LDS (one wave after the other, fixed order) and the
  // block writes its row of the [grid][2][C] slab (per-wave atomics had put 4096 contended adds on
  // every channel address, ~1 ms per launch, profiles/r02d_train_kernel_stats.csv; one atomic per
  // block left the sum order to the hardware)
  constexpr int CMAX = G * NV * EPC;
  __shared__ float red[2 * CMAX];
  const int wave = threadIdx.x >> 6;
  for (int w = 0; w < 4; ++w) {
    if (wave == w && lane < G) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int v = gl + G * i;
        if (v < V) {
#pragma unroll
          for (int k = 0; k < EPC; ++k) {
            const int c = v * EPC + k;
            red[c] = (w == 0 ? 0.f : red[c]) + pg[i][k];
            red[CMAX + c] = (w == 0 ? 0.f : red[CMAX + c]) + pb[i][k];
          }
        }
      }
    }
    __syncthreads();
  }
  float* row = part + (int64_t)blockIdx.x * 2 * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    row[c] = red[c];
    row[C + c] = red[CMAX + c];
  }
}

// ======================================================================================
// GEGLU on the interleaved GEMM output hg [rows][2F] (16-column blocks: [h16 | g16]):
//   fwd  out[r][j] = h * gelu(g)
//   bwd  dh = dout * gelu(g), dg = dout * h * gelu'(g)   -> dhg in the same interleaved layout
// ======================================================================================
__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.0f + erf_fast(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __builtin_amdgcn_exp2f(-0.5f * x * x * 1.4426950408889634f);
  return cdf + x * pdf;
}

template <typename T>
__global__ __launch_bounds__(256) void geglu_kernel(const T* __restrict__ hg, const T* __restrict__ dout, int rows,
                                                    int F, T* __restrict__ out, T* __restrict__ dhg) {
  // thread per (row, 4 output columns)
  const int64_t total = (int64_t)rows * (F / 4);
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t r = t / (F / 4);
    const int j = (int)(t - r * (F / 4)) * 4;
    const int pc = (j >> 4) * 32 + (j & 15);
    const T* row = hg + r * 2 * F;
    float h[4], g[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { h[k] = to_f(row[pc + k]); g[k] = to_f(row[pc + 16 + k]); }
    if (!dout) {
#pragma unroll
      for (int k = 0; k < 4; ++k) out[r * F + j + k] = from_f<T>(h[k] * gelu_f(g[k]));
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d = to_f(dout[r * F + j + k]);
        dhg[r * 2 * F + pc + k] = from_f<T>(d * gelu_f(g[k]));
        dhg[r * 2 * F + pc + 16 + k] = from_f<T>(d * h[k] * gelu_grad(g[k]));
      }
    }
  }
}

// ======================================================================================
// 2x2 sum pool over NHWC (data gradient of the nearest-2x upsample)
// ======================================================================================
template <typename T>
__global__ __launch_bounds__(256) void sum_pool2_kernel(const T* __restrict__ x, int batch, int h, int w, int C,
                                                        T* __restrict__ out, int accumulate) {
  constexpr int EPC = 16 / sizeof(T);
  const int V = C / EPC;
  const int64_t total = (int64_t)batch * h * w * V;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int v = (int)(t % V);
    const int64_t pix = t / V;
    const int xo = (int)(pix % w);
    const int64_t t2 = pix / w;
    const int yo = (int)(t2 % h);
    const int b = (int)(t2 / h);
    float s[EPC];
#pragma unroll
    for (int k = 0; k < EPC; ++k) s[k] = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int yi = 2 * yo + (a >> 1), xi = 2 * xo + (a & 1);
      const uint4 raw = *reinterpret_cast<const uint4*>(x + (((int64_t)b * 2 * h + yi) * 2 * w + xi) * C + v * EPC);
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int k = 0; k < EPC; ++k) s[k] += to_f(e[k]);
    }
    T* dst = out + pix * C + v * EPC;
    if (accumulate) {
      const uint4 raw = *reinterpret_cast<const uint4*>(dst);
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int k = 0; k < EPC; ++k) s[k] += to_f(e[k]);
    }
    uint4 res;
    T* r = reinterpret_cast<T*>(&res);
#pragma unroll
    for (int k = 0; k < EPC; ++k) r[k] = from_f<T>(s[k]);
    *reinterpret_cast<uint4*>(dst) = res;
  }
}

// ======================================================================================
// loss: l = (pred - target)^2 * mask[b, pix] * w[t_b]; loss_sum += l; dpred = 2 (pred - target)
// * mask * w * grad_scale.  pred/target/dpred NCHW [batch][ch][hw]; mask [batch][hw] or NULL.
// ======================================================================================
template <typename T>
__global__ __launch_bounds__(256) void mse_kernel(const T* __restrict__ pred, const float* __restrict__ target,
                                                  const float* __restrict__ mask, const int64_t* __restrict__ t,
                                                  const float* __restrict__ wtab, int ntab, int batch, int ch, int hw,
                                                  float grad_scale, T* __restrict__ dpred, double* __restrict__ part) {
  const int64_t total = (int64_t)batch * ch * hw;
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / ((int64_t)ch * hw);
    const int pix = (int)(i % hw);
    float w = 1.0f;
    if (wtab) {
      const int64_t tb = t[b];
      w = (tb >= 0 && tb < ntab) ? wtab[tb] : __builtin_nanf("");
    }
    if (mask) w *= mask[b * hw + pix];
    const float d = to_f(pred[i]) - target[i];
    acc += (double)(d * d * w);
    if (dpred) dpred[i] = from_f<T>(2.0f * d * w * grad_scale);
  }
  __shared__ double red[4];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ======================================================================================
// optimizer: sum of squares (fp64 accumulation) and fused AdamW over flat fp32 buffers
// ======================================================================================
__global__ __launch_bounds__(256) void sqnorm_kernel(const float* __restrict__ g, int64_t n, double* __restrict__ part) {
  double acc = 0.0;
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    acc += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += (double)g[i] * g[i];
  __shared__ double red[4];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

struct AdamSeg {
  int64_t begin, end;
  float lr, wd;
};

// torch.optim.AdamW (decoupled weight decay, bias-corrected, amsgrad off, maximize off):
//   p *= 1 - lr wd;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;
//   p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
// g is first multiplied by the clip coefficient min(1, max_norm / (||g|| + 1e-6)) computed on
// the device from `sqsum` (clip_grad_norm_, trainers_ldm_cond.py:769-781), so no host sync.
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const AdamSeg* __restrict__ segs, int nseg, int64_t chunk,
                                                    float beta1, float beta2, float eps, float bc1, float bc2_sqrt,
                                                    const double* __restrict__ sqsum, float max_norm) {
  float clip = 1.0f;
  if (sqsum && max_norm > 0.f) {
    const float norm = (float)sqrt(*sqsum);
    clip = fminf(1.0f, max_norm / (norm + 1e-6f));
  }
  // block -> segment by binary search on the block's first element
  const int64_t i0 = (int64_t)blockIdx.x * chunk;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].begin <= i0) lo = mid; else hi = mid - 1;
  }
  int s = lo;
  const int64_t i1 = i0 + chunk;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
    while (s < nseg && i >= segs[s].end) ++s;
    if (s >= nseg) break;
    if (i < segs[s].begin) continue;
    const float lr = segs[s].lr, wd = segs[s].wd;
    const float gi = g[i] * clip;
    float pi = p[i] * (1.0f - lr * wd);
    const float mi = beta1 * m[i] + (1.0f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.0f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= (lr / bc1) * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[i] = pi;
  }
}

constexpr int DSUM_MAX_PARTS = 2048;   // per-block fp64 partials of the loss / norm reductions

int grid_for(int64_t work, int per_block, int cap) {
  const int64_t b = (work + per_block - 1) / per_block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

constexpr int LNB_MAX_GRID = 512;
int lnb_params(const float* part, int grid, int c, float* dg, float* db, int acc, hipStream_t s) {
  if (hipGetLastError() != hipSuccess) return LDM_ERR_LAUNCH;
  if (dg) hipLaunchKernelGGL(slab_reduce, dim3((unsigned)((c + 31) / 32)), dim3(256), 0, s, part, grid, (int64_t)2 * c,
                             (int64_t)c, dg, acc);
  if (db) hipLaunchKernelGGL(slab_reduce, dim3((unsigned)((c + 31) / 32)), dim3(256), 0, s, part + c, grid,
                             (int64_t)2 * c, (int64_t)c, db, acc);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

template <typename T, int G>
int lnb_launch_g(const void* x, const void* dy, int rows, int c, const float* gamma, float eps, const void* add,
                 void* dx, float* dg, float* db, int acc, float* part, hipStream_t s) {
  constexpr int EPC = 16 / sizeof(T);
  const int V = c / EPC;
  const int nv = (V + G - 1) / G;
  const int rpb = 4 * (64 / G);
  const int grid = std::min((rows + rpb - 1) / rpb, LNB_MAX_GRID);
#define LNB_CASE(NVC)                                                                                      \
  if (nv <= NVC) {                                                                                         \
    hipLaunchKernelGGL((lnb_kernel<T, G, NVC>), dim3(grid), dim3(256), 0, s, (const T*)x, (const T*)dy, rows, c, \
                       gamma, eps, (const T*)add, (T*)dx, part);                                           \
    return lnb_params(part, grid, c, dg, db, acc, s);                                                      \
  }
  LNB_CASE(1) LNB_CASE(2) LNB_CASE(4) LNB_CASE(5) LNB_CASE(8)
#undef LNB_CASE
  return LDM_ERR_ARG;
}

template <typename T>
int lnb_launch(const void* x, const void* dy, int rows, int c, const float* gamma, float eps, const void* add,
               void* dx, float* dg, float* db, int acc, float* part, hipStream_t s) {
  constexpr int EPC = 16 / sizeof(T);
  const int V = c / EPC;
  // the smallest lane group that keeps <= 4 chunks per lane (x, dy and two partial sets live
  // in registers per chunk)
  if (V <= 8 * 4) return lnb_launch_g<T, 8>(x, dy, rows, c, gamma, eps, add, dx, dg, db, acc, part, s);
  if (V <= 16 * 4) return lnb_launch_g<T, 16>(x, dy, rows, c, gamma, eps, add, dx, dg, db, acc, part, s);
  if (V <= 32 * 4) return lnb_launch_g<T, 32>(x, dy, rows, c, gamma, eps, add, dx, dg, db, acc, part, s);
  return lnb_launch_g<T, 64>(x, dy, rows, c, gamma, eps, add, dx, dg, db, acc, part, s);
}

size_t round16(size_t x) { return (x + 15) & ~(size_t)15; }

// Pixel-axis splits: the makespan in block-work units, per XCD (blocks go round-robin to the 8 XCDs;
// 32 CUs x 2 resident blocks each), divided by the splits (a block's work is M / splits).  A round of
// two blocks per CU costs 2 units, a last partial round of at most one block per CU ~1.6 (a lone
// block issues faster).  The old rule (>= 512 blocks) left e.g. 552 blocks for the 3x3 320 at 64x64
// (69 tiles x 8): a second round of 40 lone blocks, ~45 % of the kernel.  Each split adds a
// [n][kpad] fp32 slab to write and reduce: ~33 ns per tile at HBM rate against ~9 ns per pixel
// row for one unit, i.e. 3.7 tiles / M units per split.
int wgrad_splits(const ldm_wgrad_params* q, int M, int tiles) {
  (void)q;
  const int max_sp = std::max(1, std::min(M / 256, 64));
  int best = 1;
  double best_cost = 1e30;
  for (int sp = 1; sp <= max_sp; ++sp) {
    const int per_xcd = (tiles * sp + 7) / 8;
    const int full = per_xcd / 64, rem = per_xcd % 64;
    const double units = 2.0 * full + (rem == 0 ? 0.0 : rem > 32 ? 2.0 : 1.6);
    const double cost = units / sp + sp * 3.7 * tiles / M;
    if (cost < best_cost) { best_cost = cost; best = sp; }
  }
  return best;
}

int wgrad_validate(const ldm_wgrad_params* q, int* es_out, int* M_out) {
  if (!q || !q->a0 || !q->dy || !q->dw) return LDM_ERR_ARG;
  if (q->dtype != LDM_F32 && q->dtype != LDM_BF16) return LDM_ERR_ARG;
  const int es = q->dtype == LDM_F32 ? 4 : 2, ce = 16 / es;
  if (q->ksize != 1 && q->ksize != 3) return LDM_ERR_ARG;
  if (q->stride != 1 && q->stride != 2) return LDM_ERR_ARG;
  if (q->upsample && q->stride != 1) return LDM_ERR_ARG;
  if (q->batch <= 0 || q->h_in <= 0 || q->w_in <= 0 || q->h_out <= 0 || q->w_out <= 0) return LDM_ERR_ARG;
  if (q->c0 <= 0 || q->c1 < 0 || (q->c1 > 0 && !q->a1)) return LDM_ERR_ARG;
  if (q->c0 % ce || q->c1 % ce || q->n % ce) return LDM_ERR_ALIGN;
  if ((int64_t)q->batch * q->h_out * q->w_out >= (1 << 24)) return LDM_ERR_ARG;   // reciprocal pixel decode
  const int cin = q->c0 + q->c1;
  if (q->kpad % 64 || q->ksize * q->ksize * cin > q->kpad || q->n <= 0) return LDM_ERR_ARG;
  if ((int64_t)q->n * q->kpad >= (1LL << 31)) return LDM_ERR_ARG;   // 32-bit slab indexing
  if (q->cin_real <= 0 || q->cin_real > cin) return LDM_ERR_ARG;
  if (q->geglu && q->n % 32) return LDM_ERR_ARG;
  if (!aligned16(q->a0) || (q->a1 && !aligned16(q->a1)) || !aligned16(q->dy)) return LDM_ERR_ALIGN;
  const int pad = q->ksize / 2;
  const int hin_eff = q->upsample ? 2 * q->h_in : q->h_in, win_eff = q->upsample ? 2 * q->w_in : q->w_in;
  if (q->h_out != (hin_eff + 2 * pad - q->ksize) / q->stride + 1) return LDM_ERR_ARG;
  if (q->w_out != (win_eff + 2 * pad - q->ksize) / q->stride + 1) return LDM_ERR_ARG;
  const int64_t M = (int64_t)q->batch * q->h_out * q->w_out;
  if (M >= (1LL << 31)) return LDM_ERR_ARG;
  *es_out = es;
  *M_out = (int)M;
  return LDM_OK;
}

}  // namespace

namespace {
int g_wgrad_ring = 1;   // tuning / A-B hook (ldm_conv2d_wgrad_set_ring): 0 = two 64-pixel stages,
                        // 2 = a five-slot ring (four stages in flight; stride-1 modes only)
int g_wgrad_reduce3 = 1;   // A-B hook (ldm_conv2d_wgrad_set_reduce3): 0 = element-per-thread 3x3 slab sum
int g_wgrad_fast = 1;   // A-B hook (ldm_conv2d_wgrad_set_fast_loader): 0 = the general loader everywhere
}  // namespace
extern "C" void ldm_conv2d_wgrad_set_ring(int ring) { g_wgrad_ring = ring < 0 ? 0 : ring > 2 ? 2 : ring; }
extern "C" void ldm_conv2d_wgrad_set_fast_loader(int on) { g_wgrad_fast = on ? 1 : 0; }
extern "C" void ldm_conv2d_wgrad_set_reduce3(int on) { g_wgrad_reduce3 = on ? 1 : 0; }

extern "C" size_t ldm_conv2d_wgrad_workspace_bytes(const ldm_wgrad_params* q) {
  int es = 0, M = 0;
  if (wgrad_validate(q, &es, &M) != LDM_OK) return 0;
  const int te = 256 / es;
  const int tiles = ((q->n + te - 1) / te) * ((q->kpad + te - 1) / te);
  const int sp = wgrad_splits(q, M, tiles);
  return (size_t)sp * q->n * q->kpad * sizeof(float);
}

extern "C" int ldm_conv2d_wgrad(const ldm_wgrad_params* q, ldm_stream_t stream) {
  int es = 0, M = 0;
  const int st = wgrad_validate(q, &es, &M);
  if (st != LDM_OK) return st;
  const int te = 256 / es;
  const int tiles_n = (q->n + te - 1) / te, tiles_k = (q->kpad + te - 1) / te;
  const int sp = wgrad_splits(q, M, tiles_n * tiles_k);
  const size_t need = (size_t)sp * q->n * q->kpad * sizeof(float);
  if (!q->workspace || q->workspace_bytes < (int64_t)need || !aligned16(q->workspace)) return LDM_ERR_ARG;
  WgArgs a;
  a.a0 = static_cast<const char*>(q->a0);
  a.a1 = static_cast<const char*>(q->a1);
  a.c0 = q->c0; a.c1 = q->c1; a.cin = q->c0 + q->c1;
  a.h_in = q->h_in; a.w_in = q->w_in; a.h_out = q->h_out; a.w_out = q->w_out; a.hw_out = q->h_out * q->w_out;
  a.ksize = q->ksize; a.stride = q->stride; a.upsample = q->upsample; a.pad = q->ksize / 2;
  a.dy = static_cast<const char*>(q->dy);
  a.n = q->n; a.kpad = q->kpad; a.K = q->ksize * q->ksize * a.cin; a.M = M;
  a.tiles_n = tiles_n; a.splits = sp;
  a.inv_hw = 1.0f / (float)a.hw_out;
  a.inv_w = 1.0f / (float)a.w_out;
  a.part = static_cast<float*>(q->workspace);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int blocks = tiles_n * tiles_k * sp;
  const bool plain = q->stride == 1 && !q->upsample && q->h_in == q->h_out && q->w_in == q->w_out;
  const int mode = !g_wgrad_fast || !plain ? WG_GENERAL
                   : q->ksize == 1          ? WG_1X1
                   : 16 / q->w_out < q->h_out ? WG_PLAIN : WG_GENERAL;
  if (q->dtype == LDM_BF16 && g_wgrad_ring == 2 && mode == WG_1X1)
    hipLaunchKernelGGL((wgrad_kernel<bf16_t, 32, 5, WG_1X1>), dim3(blocks), dim3(256), 0, s, a);
  else if (q->dtype == LDM_BF16 && g_wgrad_ring == 2 && mode == WG_PLAIN)
    hipLaunchKernelGGL((wgrad_kernel<bf16_t, 32, 5, WG_PLAIN>), dim3(blocks), dim3(256), 0, s, a);
  else if (q->dtype == LDM_BF16 && g_wgrad_ring && mode == WG_1X1)
    hipLaunchKernelGGL((wgrad_kernel<bf16_t, 32, 4, WG_1X1>), dim3(blocks), dim3(256), 0, s, a);
  else if (q->dtype == LDM_BF16 && g_wgrad_ring && mode == WG_PLAIN)
    hipLaunchKernelGGL((wgrad_kernel<bf16_t, 32, 4, WG_PLAIN>), dim3(blocks), dim3(256), 0, s, a);
  else if (q->dtype == LDM_BF16 && g_wgrad_ring) hipLaunchKernelGGL((wgrad_kernel<bf16_t, 32, 4>), dim3(blocks), dim3(256), 0, s, a);
  else if (q->dtype == LDM_BF16) hipLaunchKernelGGL((wgrad_kernel<bf16_t, 64, 2>), dim3(blocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((wgrad_kernel<float, 64, 2>), dim3(blocks), dim3(256), 0, s, a);
  LDM_CHECK_LAUNCH();
  const int64_t total = (int64_t)q->n * q->kpad;
  if (q->ksize == 3 && g_wgrad_reduce3) {
    const int items = q->n * ((q->cin_real + 63) / 64);
    hipLaunchKernelGGL(wgrad_reduce3, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s, a.part, sp, q->n, q->kpad,
                       a.cin, q->cin_real, q->geglu, q->dw, q->accumulate);
  } else {
    hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a.part, sp, q->n,
                       q->kpad, q->ksize, a.cin, q->cin_real, q->geglu, q->dw, q->accumulate);
  }
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

constexpr int COLSUM_RCHUNK = 128;
extern "C" size_t ldm_colsum_workspace_bytes(int rows, int c, int segments) {
  if (rows <= 0 || c <= 0 || segments <= 0) return 0;
  const int rps = rows / segments;
  return (size_t)((rps + COLSUM_RCHUNK - 1) / COLSUM_RCHUNK) * segments * c * sizeof(float);
}

extern "C" int ldm_colsum(const void* x, int rows, int c, int segments, int geglu, float* out, int accumulate,
                          void* workspace, int dtype, ldm_stream_t stream) {
  if (!x || !out || !workspace || rows <= 0 || c <= 0 || segments <= 0 || rows % segments) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  const int epc = dtype == LDM_F32 ? 4 : 8;
  if (c % epc || !aligned16(x) || !aligned16(workspace)) return LDM_ERR_ALIGN;
  if (geglu && c % 32) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int rps = rows / segments;
  const int chunks = (rps + COLSUM_RCHUNK - 1) / COLSUM_RCHUNK;
  float* part = static_cast<float*>(workspace);
  dim3 grid((c / epc + 63) / 64, chunks, segments);
  if (dtype == LDM_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, c, rps, COLSUM_RCHUNK, geglu,
                       part);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, s, (const float*)x, c, rps, COLSUM_RCHUNK, geglu,
                       part);
  LDM_CHECK_LAUNCH();
  const int64_t width = (int64_t)segments * c;
  hipLaunchKernelGGL(slab_reduce, dim3((unsigned)((width + 31) / 32)), dim3(256), 0, s, part, chunks, width, width,
                     out, accumulate);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" size_t ldm_group_norm_bwd_workspace_bytes(int batch, int hw, int channels, int groups) {
  const size_t chunks = (hw + GNB_PPC - 1) / GNB_PPC;
  return round16((size_t)batch * chunks * channels * sizeof(float2)) + round16((size_t)batch * groups * sizeof(float2)) +
         64;
}

extern "C" int ldm_group_norm_bwd(const void* x0, const void* x1, int c0, int c1, int batch, int hw, int groups,
                                  const float* mean_rstd, const float* gamma, const float* beta, int act,
                                  const void* dy, const void* add_src, void* dx0, void* dx1, int acc0, int acc1,
                                  float* dgamma, float* dbeta, int acc_params, void* workspace, int dtype,
                                  ldm_stream_t stream) {
  if (!x0 || !dy || !mean_rstd || !gamma || !beta || !dx0 || !workspace) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  if (batch <= 0 || hw <= 0 || c0 <= 0 || c1 < 0 || (c1 > 0 && (!x1 || !dx1)) || groups <= 0) return LDM_ERR_ARG;
  const int C = c0 + c1;
  if (C % groups) return LDM_ERR_ARG;
  const int epc = dtype == LDM_F32 ? 4 : 8;
  if (c0 % epc || c1 % epc) return LDM_ERR_ALIGN;
  if (!aligned16(x0) || (x1 && !aligned16(x1)) || !aligned16(dy) || !aligned16(dx0) || (dx1 && !aligned16(dx1)) ||
      (add_src && !aligned16(add_src)) || !aligned16(workspace))
    return LDM_ERR_ALIGN;
  const int chunks = (hw + GNB_PPC - 1) / GNB_PPC;
  char* w = static_cast<char*>(workspace);
  float2* part = reinterpret_cast<float2*>(w);
  w += round16((size_t)batch * chunks * C * sizeof(float2));
  float2* coef = reinterpret_cast<float2*>(w);
  const float2* mr = reinterpret_cast<const float2*>(mean_rstd);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t nvec = (int64_t)batch * hw * (C / epc);
  if (nvec >= (1LL << 31)) return LDM_ERR_ARG;
  const dim3 pg((C / epc + 63) / 64, chunks, batch);
  const int ablocks = grid_for(nvec, 256, 256 * 8);
  if (dtype == LDM_BF16) {
    hipLaunchKernelGGL(gnb_partial<bf16_t>, pg, dim3(256), 0, s, (const bf16_t*)x0, (const bf16_t*)x1, c0, c1,
                       (const bf16_t*)dy, hw, chunks, groups, mr, gamma, beta, act, part);
  } else {
    hipLaunchKernelGGL(gnb_partial<float>, pg, dim3(256), 0, s, (const float*)x0, (const float*)x1, c0, c1,
                       (const float*)dy, hw, chunks, groups, mr, gamma, beta, act, part);
  }
  LDM_CHECK_LAUNCH();
  hipLaunchKernelGGL(gnb_finalize, dim3(batch, (groups + 3) / 4), dim3(256), 0, s, part, C, hw, chunks, groups, mr,
                     gamma, coef);
  LDM_CHECK_LAUNCH();
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(gnb_param, dim3((C + 15) / 16), dim3(256), 0, s, part, C, batch * chunks, dgamma, dbeta,
                       acc_params);
    LDM_CHECK_LAUNCH();
  }
  if (dtype == LDM_BF16) {
    hipLaunchKernelGGL(gnb_apply<bf16_t>, dim3(ablocks), dim3(256), 0, s, (const bf16_t*)x0, (const bf16_t*)x1, c0,
                       c1, (const bf16_t*)dy, hw, groups, (int)nvec, mr, coef, gamma, beta, act,
                       (const bf16_t*)add_src, (bf16_t*)dx0, (bf16_t*)dx1, acc0, acc1);
  } else {
    hipLaunchKernelGGL(gnb_apply<float>, dim3(ablocks), dim3(256), 0, s, (const float*)x0, (const float*)x1, c0, c1,
                       (const float*)dy, hw, groups, (int)nvec, mr, coef, gamma, beta, act, (const float*)add_src,
                       (float*)dx0, (float*)dx1, acc0, acc1);
  }
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" size_t ldm_layer_norm_bwd_workspace_bytes(int rows, int c) {
  if (rows <= 0 || c <= 0) return 0;
  return (size_t)LNB_MAX_GRID * 2 * c * sizeof(float);
}

extern "C" int ldm_layer_norm_bwd(const void* x, const void* dy, int rows, int c, const float* gamma, float eps,
                                  const void* add_src, void* dx, float* dgamma, float* dbeta, int acc_params,
                                  void* workspace, int dtype, ldm_stream_t stream) {
  if (!x || !dy || !dx || !gamma || !workspace || rows <= 0 || c <= 0) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  const int epc = dtype == LDM_F32 ? 4 : 8;
  if (c % epc) return LDM_ERR_ALIGN;
  if (c / epc > 64 * 8) return LDM_ERR_ARG;
  if (!aligned16(x) || !aligned16(dy) || !aligned16(dx) || (add_src && !aligned16(add_src))) return LDM_ERR_ALIGN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(workspace);
  const int acc = acc_params ? 1 : 0;
  const int st = dtype == LDM_BF16
                     ? lnb_launch<bf16_t>(x, dy, rows, c, gamma, eps, add_src, dx, dgamma, dbeta, acc, part, s)
                     : lnb_launch<float>(x, dy, rows, c, gamma, eps, add_src, dx, dgamma, dbeta, acc, part, s);
  if (st != LDM_OK) return st;
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_geglu(const void* hg, const void* dout, int rows, int f, void* out, void* dhg, int dtype,
                         ldm_stream_t stream) {
  if (!hg || rows <= 0 || f <= 0 || f % 16) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  if (dout ? !dhg : !out) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int blocks = grid_for((int64_t)rows * (f / 4), 256, 256 * 16);
  if (dtype == LDM_BF16)
    hipLaunchKernelGGL(geglu_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)hg, (const bf16_t*)dout, rows,
                       f, (bf16_t*)out, (bf16_t*)dhg);
  else
    hipLaunchKernelGGL(geglu_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)hg, (const float*)dout, rows, f,
                       (float*)out, (float*)dhg);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_sum_pool2(const void* x, int batch, int h_out, int w_out, int c, void* out, int accumulate,
                             int dtype, ldm_stream_t stream) {
  if (!x || !out || batch <= 0 || h_out <= 0 || w_out <= 0 || c <= 0) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  const int epc = dtype == LDM_F32 ? 4 : 8;
  if (c % epc || !aligned16(x) || !aligned16(out)) return LDM_ERR_ALIGN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int blocks = grid_for((int64_t)batch * h_out * w_out * (c / epc), 256, 256 * 16);
  if (dtype == LDM_BF16)
    hipLaunchKernelGGL(sum_pool2_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)x, batch, h_out, w_out,
                       c, (bf16_t*)out, accumulate);
  else
    hipLaunchKernelGGL(sum_pool2_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, batch, h_out, w_out, c,
                       (float*)out, accumulate);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_mse_loss(const void* pred, const float* target, const float* mask, const int64_t* t,
                            const float* weights, int num_weights, int batch, int ch, int hw, float grad_scale,
                            void* dpred, double* loss_sum, void* workspace, int dtype, ldm_stream_t stream) {
  if (!pred || !target || !loss_sum || !workspace || batch <= 0 || ch <= 0 || hw <= 0) return LDM_ERR_ARG;
  if (weights && (!t || num_weights <= 0)) return LDM_ERR_ARG;
  if (dtype != LDM_F32 && dtype != LDM_BF16) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(workspace);
  const int blocks = grid_for((int64_t)batch * ch * hw, 256 * 4, DSUM_MAX_PARTS);
  if (dtype == LDM_BF16)
    hipLaunchKernelGGL(mse_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, (const bf16_t*)pred, target, mask, t, weights,
                       num_weights, batch, ch, hw, grad_scale, (bf16_t*)dpred, part);
  else
    hipLaunchKernelGGL(mse_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)pred, target, mask, t, weights,
                       num_weights, batch, ch, hw, grad_scale, (float*)dpred, part);
  LDM_CHECK_LAUNCH();
  hipLaunchKernelGGL(dsum_final, dim3(1), dim3(256), 0, s, part, blocks, loss_sum, 0);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" size_t ldm_reduce_workspace_bytes(void) { return DSUM_MAX_PARTS * sizeof(double); }

extern "C" int ldm_sq_norm(const float* g, int64_t n, double* sum, int accumulate, void* workspace,
                           ldm_stream_t stream) {
  if (!g || !sum || !workspace || n < 0) return LDM_ERR_ARG;
  if (!aligned16(g)) return LDM_ERR_ALIGN;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) {
    if (!accumulate && hipMemsetAsync(sum, 0, sizeof(double), s) != hipSuccess) return LDM_ERR_LAUNCH;
    return LDM_OK;
  }
  double* part = static_cast<double*>(workspace);
  const int blocks = grid_for(n / 4 + 1, 256 * 8, DSUM_MAX_PARTS);
  hipLaunchKernelGGL(sqnorm_kernel, dim3(blocks), dim3(256), 0, s, g, n, part);
  LDM_CHECK_LAUNCH();
  hipLaunchKernelGGL(dsum_final, dim3(1), dim3(256), 0, s, part, blocks, sum, accumulate);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const void* segments,
                         int nseg, int64_t n, float beta1, float beta2, float eps, int step, const double* sqsum,
                         float max_norm, ldm_stream_t stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !segments || nseg <= 0 || n <= 0 || step <= 0) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t chunk = 256 * 16;
  const float bc1 = 1.0f - powf(beta1, (float)step);
  const float bc2 = 1.0f - powf(beta2, (float)step);
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)((n + chunk - 1) / chunk)), dim3(256), 0, s, param, grad, exp_avg,
                     exp_avg_sq, static_cast<const AdamSeg*>(segments), nseg, chunk, beta1, beta2, eps, bc1,
                     sqrtf(bc2), sqsum, max_norm);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
