// Fused multi-head attention forward (ldm_attention): softmax(Q K^T * scale) V, online softmax.
//
// Orientation ("swapped" products, so the softmax reduction axis stays inside one lane):
//   S^T[kv][q] = K[kv][:] . Q[q][:]       mfma A = K tile (LDS, ds_read_b64), B = Q (registers)
//   O^T[d][q] += V^T[d][kv] . P^T[kv][q]   mfma A = V^T fragment read TRANSPOSED from the row-major
//                                           V tile (ds_read_b64_tr_b16), B = P: the S^T accumulator
//                                           registers converted in place (no LDS round trip)
// With the 16x16x16 MFMA the accumulator of one 16-kv S^T fragment (a lane holds kv = 4g+r of
// its q column) is exactly the B operand of P.V, and a row max needs two cross-lane shuffles.
// K/V tiles (64 keys) arrive by LDS-DMA (global_load_lds_dwordx4, per-lane source: rows past
// n_kv and the head-dim padding read a zero constant), double buffered; row pitch 4*odd
// dwords (conflict-free ds_read_b64).  Softmax VALU per score: max, fma+exp2, cvt.
//   - the scale is folded into the exp2 FMA (p = 2^(s*c - m)); masking only on a partial tile;
//   - lazy rescale: O/l are rescaled only when a row max grows by > 8 (log2 units);
//   - head_dim 40 (padded to 48): the padding column d = 40 of V is a column of ONES, so the
//     P.V MFMA produces the softmax denominator for free (same bf16 P as the numerator).
// bf16: v_mfma_f32_16x16x16_bf16; fp32: v_mfma_f32_16x16x4_f32 (exact), V^T via scalar reads.
#include "common.h"

namespace {

struct AttnArgs {
  const char* q; const char* k; const char* v; char* o;
  int qs, ks, vs, os;
  int heads, d, nq, nkv;
  float scale_log2;
  float* lse;         // optional [batch][heads][nq]: log2-domain log-sum-exp (training forward)
  int kvsplit;        // > 1: attn_d40_kernel<..., KVS> splits the keys; partials in opart / lsepart
  int batch;
  float* opart;       // [kvsplit][batch][heads][nq][d] normalised fp32 partial outputs
  float* lsepart;     // [kvsplit][batch][heads][nq] their log2-domain log-sum-exp
};

__device__ const uint4 kZeros16 = {0u, 0u, 0u, 0u};
__device__ const uint4 kOnesBf16 = {0x3f80u, 0u, 0u, 0u};       // bf16 1.0 then zeros
__device__ const uint4 kOnesF32 = {0x3f800000u, 0u, 0u, 0u};    // fp32 1.0 then zeros

constexpr int KVT = 64;        // keys per tile
constexpr float kRescaleThr = 8.0f;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

template <typename T, int DP, int QSUB, bool ONES>
__global__ __launch_bounds__(256, 2) void attn_kernel(const AttnArgs p) {
  constexpr int ES = sizeof(T);
  constexpr int EPC = 16 / ES;          // elements per 16-B chunk
  constexpr int ND = DP / 16;
  constexpr int CPR = DP / EPC;         // data chunks per row (incl. zero head-dim padding)
  constexpr int RCH = CPR + 1;          // + one pad chunk: pitch = 4*odd dwords
  constexpr int ROW = RCH * EPC;        // row pitch in elements
  constexpr int TILE = KVT * ROW;       // elements per K (or V) tile
  constexpr int NBUF = (2 * 2 * TILE * ES <= 96 * 1024) ? 2 : 1;   // fp32 at d=160: single buffer
  __shared__ uint4 smem[NBUF * 2 * TILE * ES / 16];
  T* const lds = reinterpret_cast<T*>(smem);
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const int qbase = blockIdx.x * (64 * QSUB) + wave * 16 * QSUB;

  const T* qp = reinterpret_cast<const T*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * p.d;
  const T* kp = reinterpret_cast<const T*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * p.d;
  const T* vp = reinterpret_cast<const T*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * p.d;
  const void* ones = (ES == 2) ? (const void*)&kOnesBf16 : (const void*)&kOnesF32;
  const int ones_chunk = ONES ? p.d / EPC : -1;

  // ---- K/V tile DMA: per matrix RCH wave-instructions of 64 lanes x 16 B (lane-linear rows)
  auto issue_tile = [&](int kv0, int buf) {
    const unsigned kb = lds0 + (unsigned)(buf * 2 * TILE * ES);
    const unsigned vb = kb + TILE * ES;
    for (int i = wave; i < RCH; i += 4) {
      const int L = i * 64 + lane;
      const int row = L / RCH, c = L - row * RCH;
      const int kv = kv0 + row, d = c * EPC;
      const bool ok = kv < p.nkv && c < CPR && d < p.d;
      const void* ks = ok ? (const void*)(kp + (int64_t)kv * p.ks + d) : (const void*)&kZeros16;
      const void* vs = ok ? (const void*)(vp + (int64_t)kv * p.vs + d)
                          : (c == ones_chunk ? ones : (const void*)&kZeros16);
      const unsigned off = __builtin_amdgcn_readfirstlane(i * 64 * 16);
      glds16(ks, kb + off);
      glds16(vs, vb + off);
    }
  };

  // ---- Q fragments (B operand): lane holds Q[q = qbase + 16 s + lr][d = 16 ds + 4g .. +3]
  Frag4<T> qf[QSUB][ND];
#pragma unroll
  for (int s = 0; s < QSUB; ++s) {
    const int qi = qbase + 16 * s + lr;
#pragma unroll
    for (int ds = 0; ds < ND; ++ds) {
      const int dd = 16 * ds + 4 * g;
      if (qi < p.nq && dd < p.d) qf[s][ds] = *reinterpret_cast<const Frag4<T>*>(qp + (int64_t)qi * p.qs + dd);
      else qf[s][ds] = Frag4<T>{};
    }
  }

  f32x4_t oacc[ND][QSUB];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int s = 0; s < QSUB; ++s) oacc[i][s] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float mrun[QSUB], lrun[QSUB];
#pragma unroll
  for (int s = 0; s < QSUB; ++s) { mrun[s] = -INFINITY; lrun[s] = 0.f; }
  const float c2 = p.scale_log2;

  auto compute = [&](int buf, int kv0, bool masked) {
    const T* Ks = lds + buf * 2 * TILE;
    const T* Vs = Ks + TILE;
    // S^T = K Q^T
    f32x4_t sacc[4][QSUB];
#pragma unroll
    for (int js = 0; js < 4; ++js)
#pragma unroll
      for (int s = 0; s < QSUB; ++s) sacc[js][s] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < ND; ++ds) {
#pragma unroll
      for (int js = 0; js < 4; ++js) {
        const Frag4<T> ka = *reinterpret_cast<const Frag4<T>*>(Ks + (16 * js + lr) * ROW + 16 * ds + 4 * g);
#pragma unroll
        for (int s = 0; s < QSUB; ++s) mma_k16(sacc[js][s], ka, qf[s][ds]);
      }
    }
    // online softmax in log2 units; P packed as the P.V B operand
    Frag4<T> pf[4][QSUB];
#pragma unroll
    for (int s = 0; s < QSUB; ++s) {
      if (masked) {
#pragma unroll
        for (int js = 0; js < 4; ++js)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kv0 + 16 * js + 4 * g + r >= p.nkv) sacc[js][s][r] = -INFINITY;
      }
      float mx = fmaxf(fmaxf(sacc[0][s][0], sacc[0][s][1]), fmaxf(sacc[0][s][2], sacc[0][s][3]));
#pragma unroll
      for (int js = 1; js < 4; ++js)
        mx = fmaxf(mx, fmaxf(fmaxf(sacc[js][s][0], sacc[js][s][1]), fmaxf(sacc[js][s][2], sacc[js][s][3])));
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float ms = mx * c2;
      if (__any(ms > mrun[s] + kRescaleThr)) {       // lazy rescale (whole wave, per-lane factor)
        const float mnew = fmaxf(mrun[s], ms);
        const float alpha = __builtin_amdgcn_exp2f(mrun[s] - mnew);
        mrun[s] = mnew;
        if (!ONES) lrun[s] *= alpha;
#pragma unroll
        for (int i = 0; i < ND; ++i) oacc[i][s] *= alpha;
      }
      const float mneg = -mrun[s];
      float lsum = 0.f;
#pragma unroll
      for (int js = 0; js < 4; ++js) {
        float pv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#if ATTN_ABL == 1   // ablation: no transcendental
          pv[r] = fmaf(sacc[js][s][r], c2, mneg);
#else
          pv[r] = __builtin_amdgcn_exp2f(fmaf(sacc[js][s][r], c2, mneg));
#endif
          if (!ONES) lsum += pv[r];
        }
        if constexpr (ES == 2) {
          bf16_t hb[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) hb[r] = f2bf(pv[r]);
          pf[js][s].v = *reinterpret_cast<const uint2*>(hb);
        } else {
          pf[js][s].v = *reinterpret_cast<const uint4*>(pv);
        }
      }
      if (!ONES) lrun[s] += lsum;
    }
    // O^T += V^T P^T
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
#pragma unroll
      for (int js = 0; js < 4; ++js) {
        Frag4<T> va;
        if constexpr (ES == 2) {
          // lane 4q+p of each 16-lane group addresses row kv = 16js + 4g + q, cols 16dd + 4p..+3;
          // lane i of the group receives column 16dd + i of those 4 rows
          typedef __attribute__((ext_vector_type(4))) short s4_t;
          typedef __attribute__((address_space(3))) s4_t lds_s4_t;
          const T* addr = Vs + (16 * js + 4 * g + (lr >> 2)) * ROW + 16 * dd + 4 * (lr & 3);
          const s4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(addr));
          va.v = __builtin_bit_cast(uint2, x);
        } else {
          float* f = reinterpret_cast<float*>(&va.v);
#pragma unroll
          for (int j = 0; j < 4; ++j) f[j] = to_f(Vs[(16 * js + 4 * g + j) * ROW + 16 * dd + lr]);
        }
#pragma unroll
        for (int s = 0; s < QSUB; ++s) mma_k16(oacc[dd][s], va, pf[js][s]);
      }
    }
  };

  const int ntiles = (p.nkv + KVT - 1) / KVT;
  issue_tile(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = NBUF == 2 ? (t & 1) : 0;
    if (NBUF == 2 && t + 1 < ntiles) issue_tile((t + 1) * KVT, buf ^ 1);   // prefetch under compute
    const int kv0 = t * KVT;
    if (kv0 + KVT > p.nkv) compute(buf, kv0, true);
    else compute(buf, kv0, false);
    if (NBUF == 1 && t + 1 < ntiles) {
      __syncthreads();
      issue_tile((t + 1) * KVT, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- normalise and store O[q][h*d + d]
  T* op = reinterpret_cast<T*>(p.o) + (int64_t)b * p.nq * p.os + (int64_t)h * p.d;
#pragma unroll
  for (int s = 0; s < QSUB; ++s) {
    float lt;
    if constexpr (ONES) {
      // the denominator sits in O^T row d = DP - 8 (subtile ND-1, lane group g = 2, register 0)
      lt = __shfl(oacc[ND - 1][s][0], 32 + lr, 64);
    } else {
      lt = lrun[s] + __shfl_xor(lrun[s], 16, 64);
      lt += __shfl_xor(lt, 32, 64);
    }
    const float inv = 1.0f / lt;
    const int qi = qbase + 16 * s + lr;
    if (qi >= p.nq) continue;
    if (p.lse && g == 0) p.lse[((int64_t)b * p.heads + h) * p.nq + qi] = mrun[s] + __log2f(lt);
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
      const int d = 16 * dd + 4 * g;
      if (d >= p.d) continue;
      if constexpr (ES == 2) {
        bf16_t hb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) hb[r] = f2bf(oacc[dd][s][r] * inv);
        *reinterpret_cast<uint2*>(op + (int64_t)qi * p.os + d) = *reinterpret_cast<const uint2*>(hb);
      } else {
        float fv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) fv[r] = oacc[dd][s][r] * inv;
        *reinterpret_cast<uint4*>(op + (int64_t)qi * p.os + d) = *reinterpret_cast<const uint4*>(fv);
      }
    }
  }
}

template <typename T, int DP, int QSUB, bool ONES>
int launch_cfg(const AttnArgs& a, int batch, hipStream_t s) {
  dim3 grid((a.nq + 64 * QSUB - 1) / (64 * QSUB), a.heads, batch);
  hipLaunchKernelGGL((attn_kernel<T, DP, QSUB, ONES>), grid, dim3(256), 0, s, a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

template <typename T, int DP>
int launch_dp(const AttnArgs& a, int batch, hipStream_t s) {
  constexpr int QS = DP <= 64 ? 4 : 2;
  if (a.d == DP - 8) return launch_cfg<T, DP, QS, true>(a, batch, s);
  return launch_cfg<T, DP, QS, false>(a, batch, s);
}

template <typename T>
int launch_t(const AttnArgs& a, int batch, hipStream_t s) {
  const int dp = (a.d + 15) / 16 * 16;
  switch (dp) {
    case 16: return launch_dp<T, 16>(a, batch, s);
    case 32: return launch_dp<T, 32>(a, batch, s);
    case 48: return launch_dp<T, 48>(a, batch, s);
    case 64: return launch_dp<T, 64>(a, batch, s);
    case 80: return launch_dp<T, 80>(a, batch, s);
    case 96: return launch_dp<T, 96>(a, batch, s);
    case 128: return launch_dp<T, 128>(a, batch, s);
    case 160: return launch_dp<T, 160>(a, batch, s);
    default: return LDM_ERR_ARG;
  }
}


// ======================================================================================
// bf16 forward on the full-rate v_mfma_f32_16x16x32_bf16 (the 16x16x16 form above issues at
// half the FLOP rate on gfx950: 16 busy cycles for half the work).
//   S^T[kv][q]: per 16-key fragment, one x32 MFMA per 32 head-dim columns, the head dim
//               zero-padded to a multiple of 32 (d = 40 -> 64: a 16x16x16 remainder would cost
//               the same 16 cycles as the padded x32);  A = K rows (ds_read_b128), B = Q.
//   O^T[d][q] += V^T P^T over 32 keys per MFMA: the B operand concatenates the bf16-packed S^T
//               accumulators of key fragments 2t and 2t+1 (k order kv = 32t + 16(j>>2) + 4g +
//               (j&3)), and the A operand concatenates the two matching ds_read_b64_tr_b16 reads
//               of V, so the permuted k order is the same on both sides and nothing moves
//               between lanes.
// Softmax VALU per score: max3 (half), fma + exp2, half a cvt_pk.
// ======================================================================================
// max over the 4 lanes {l, l^16, l^32, l^48} with the gfx950 row-swap permutes (VALU, no LDS
// round trip as ds_bpermute would take)
__device__ __forceinline__ float max_over_groups(float v) {
  unsigned u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  u = __float_as_uint(v);
  const auto b = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// IEEE maximum (NaN-propagating) needs no operand canonicalisation and folds to v_maximum3_f32
// on gfx950; inline asm would hide the MFMA-result read hazard from the compiler
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}

__device__ __forceinline__ float max_over_groups_raw(float v) {
  unsigned u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = vmax3(__uint_as_float(a[0]), __uint_as_float(a[1]), __uint_as_float(a[1]));
  u = __float_as_uint(v);
  const auto b = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return vmax3(__uint_as_float(b[0]), __uint_as_float(b[1]), __uint_as_float(b[1]));
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

#ifndef ATTN_ABL
#define ATTN_ABL 0   // ablation builds only (tools/attn_ablate.sh): 1 no exp2, 2 no QK MFMA, 3 no PV MFMA
#endif

// fp8 P.V (BASELINE config 5, "fp8 MFMA attention"): P (<= 2^8 under the lazy rescale) and V are
// rounded to OCP e4m3 (v_cvt_pk_fp8_f32; V saturated to +-448) and multiplied on
// v_mfma_f32_16x16x32_fp8_fp8 with fp32 accumulation; Q.K^T and the softmax stay bf16 / fp32.  The
// ones column of V is exactly 1.0 in e4m3, so the denominator sums the same rounded P as the
// numerator.  NB: the non-scaled fp8 MFMA issues at the bf16 rate on gfx950 (MI355X_MICROARCH.md,
// Matrix cores), so this path trades accuracy for no MFMA time; it exists for config 5's numerics.
__device__ __forceinline__ uint32_t pack_fp8x4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
__device__ __forceinline__ float sat448(float x) { return __builtin_amdgcn_fmed3f(x, -448.f, 448.f); }
__device__ __forceinline__ uint32_t bf16x4_to_fp8x4(uint2 v) {
  return pack_fp8x4(sat448(__uint_as_float(v.x << 16)), sat448(__uint_as_float(v.x & 0xffff0000u)),
                    sat448(__uint_as_float(v.y << 16)), sat448(__uint_as_float(v.y & 0xffff0000u)));
}

// MC ("max column", head_dim % 32 != 0 and % 8 == 0): the softmax's scale and running max ride
// in the Q.K^T MFMA's head-dim padding instead of one FMA per score.  Q is prescaled by
// scale * log2(e) (bf16), Q[:, d] = -m (m bf16-exact) and K[:, d] = 1, so the accumulator is
// already s * c - m and p = exp2(acc).  When the max grows past the lazy-rescale threshold the
// tile's accumulators are shifted once and the Q column rewritten; numerator and denominator
// (ones column of V) see the same m, so its bf16 rounding cancels.
__device__ __forceinline__ float bf16_rne(float x) {
  const unsigned u = __float_as_uint(x);
  return __uint_as_float((u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u);
}
__device__ __forceinline__ uint4 scale_bf16x8(uint4 v, float c) {
  unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = pack_bf16x2(__uint_as_float(w[i] << 16) * c, __uint_as_float(w[i] & 0xffff0000u) * c);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// KVS: split-KV as in attn_d40_kernel (block id = (query block, split), key tiles [t0, t1), fp32
// partials + log-sum-exp for attn_kv_combine)
template <int DP, int QSUB, bool ONES, int NW = 4, int OCC = 8 / NW, bool F8 = false, bool MC = false,
          bool KVS = false>
__global__ __launch_bounds__(64 * NW, OCC) void attn32_kernel(const AttnArgs p) {
  typedef bf16_t T;
  constexpr int ES = 2, EPC = 8;
  constexpr int ND = DP / 16;           // 16-row O^T fragments (P.V covers DP columns)
  constexpr int DPK = (DP + 31) / 32 * 32;   // Q.K^T head dim, zero-padded to whole x32 chunks
  constexpr int NC = DPK / 32;
  constexpr int CPR = DPK / EPC;
  constexpr int RCH = CPR + 1;
  constexpr int ROW = RCH * EPC;
  constexpr int TILE = KVT * ROW;
  __shared__ uint4 smem[2 * 2 * TILE * ES / 16];
  T* const lds = reinterpret_cast<T*>(smem);
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  // 1-D grid, XCD-aware: blocks b and b+8 share an XCD, so each XCD gets a contiguous run of
  // (batch, head, q-block) ids and the q-blocks of one head read its K/V from one L2 (with the
  // 3-D grid the 8 q-blocks of a head landed on 8 XCDs: 8x the K/V misses)
  int qb, h, b, split = 0;
  {
    const int nqb = (p.nq + 16 * QSUB * NW - 1) / (16 * QSUB * NW);
    const int bid = blockIdx.x, nblk = gridDim.x;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    int t = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
    if constexpr (KVS) {
      split = t % p.kvsplit;
      t /= p.kvsplit;
    }
    qb = t % nqb;
    const int hb = t / nqb;
    h = hb % p.heads;
    b = hb / p.heads;
  }
  const int qbase = qb * (16 * QSUB * NW) + wave * 16 * QSUB;
  const int ntiles_all = (p.nkv + KVT - 1) / KVT;
  const int t0 = KVS ? ntiles_all * split / p.kvsplit : 0;               // this block's key tiles
  const int t1 = KVS ? ntiles_all * (split + 1) / p.kvsplit : ntiles_all;

  const T* qp = reinterpret_cast<const T*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * p.d;
  const T* kp = reinterpret_cast<const T*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * p.d;
  const T* vp = reinterpret_cast<const T*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * p.d;
  const int ones_chunk = ONES ? p.d / EPC : -1;

  auto issue_tile = [&](int kv0, int buf) {
    const unsigned kb = lds0 + (unsigned)(buf * 2 * TILE * ES);
    const unsigned vb = kb + TILE * ES;
    for (int i = wave; i < RCH; i += NW) {
      const int L = i * 64 + lane;
      const int row = L / RCH, c = L - row * RCH;
      const int kv = kv0 + row, d = c * EPC;
      const bool ok = kv < p.nkv && c < CPR && d < p.d;
      const bool kone = MC && c == p.d / EPC && kv < p.nkv;      // K[:, d] = 1 (max column)
      const void* ks = ok ? (const void*)(kp + (int64_t)kv * p.ks + d)
                          : (kone ? (const void*)&kOnesBf16 : (const void*)&kZeros16);
      const void* vs = ok ? (const void*)(vp + (int64_t)kv * p.vs + d)
                          : (c == ones_chunk ? (const void*)&kOnesBf16 : (const void*)&kZeros16);
      const unsigned off = __builtin_amdgcn_readfirstlane(i * 64 * 16);
      glds16(ks, kb + off);
      glds16(vs, vb + off);
    }
  };
  // full tiles from per-lane pointers advanced by one tile of rows (attn_d40_kernel's form)
  constexpr int NSL = (RCH + NW - 1) / NW;
  const char* kq[NSL];
  const char* vq[NSL];
  int64_t kstep[NSL], vstep[NSL];
#pragma unroll
  for (int s2 = 0; s2 < NSL; ++s2) {
    const int i = wave + NW * s2;
    const int L = i * 64 + lane;
    const int row = L / RCH, c = L - row * RCH;
    const bool dat = i < RCH && c < CPR && c * EPC < p.d;
    const bool kone = MC && c == p.d / EPC;
    const bool vone = c == ones_chunk;
    kq[s2] = dat ? reinterpret_cast<const char*>(kp + (int64_t)((t0 + 1) * KVT + row) * p.ks + c * EPC)
                 : reinterpret_cast<const char*>(kone ? (const void*)&kOnesBf16 : (const void*)&kZeros16);
    vq[s2] = dat ? reinterpret_cast<const char*>(vp + (int64_t)((t0 + 1) * KVT + row) * p.vs + c * EPC)
                 : reinterpret_cast<const char*>(vone ? (const void*)&kOnesBf16 : (const void*)&kZeros16);
    kstep[s2] = dat ? (int64_t)KVT * p.ks * ES : 0;
    vstep[s2] = dat ? (int64_t)KVT * p.vs * ES : 0;
  }
  auto issue_full = [&](int buf) {   // the next full tile (tiles 1, 2, ... in order)
    const unsigned kb = lds0 + (unsigned)(buf * 2 * TILE * ES);
    const unsigned vb = kb + TILE * ES;
#pragma unroll
    for (int s2 = 0; s2 < NSL; ++s2) {
      const int i = wave + NW * s2;
      if (i >= RCH) break;
      const unsigned off = __builtin_amdgcn_readfirstlane(i * 64 * 16);
      glds16(kq[s2], kb + off);
      glds16(vq[s2], vb + off);
      kq[s2] += kstep[s2];
      vq[s2] += vstep[s2];
    }
  };
  const float c2 = p.scale_log2;

  // Q fragments: x32 chunk c: lane holds Q[q][32c + 8g .. +8] (zero past head_dim; MC: * c2,
  // and column d = -m, initially 0)
  Frag8<T> q32[QSUB][NC];
#pragma unroll
  for (int s = 0; s < QSUB; ++s) {
    const int qi = qbase + 16 * s + lr;
    const T* qrow = qp + (int64_t)qi * p.qs;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int dd = 32 * c + 8 * g;
      if (qi < p.nq && dd < p.d) {
        const uint4 raw = *reinterpret_cast<const uint4*>(qrow + dd);
        q32[s][c].v = MC ? scale_bf16x8(raw, c2) : raw;
      } else {
        q32[s][c].v = make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
  const int gq = (p.d & 31) >> 3;                       // MC: lane group holding Q column d

  f32x4_t oacc[ND][QSUB];
#pragma unroll
  for (int i = 0; i < ND; ++i)
#pragma unroll
    for (int s = 0; s < QSUB; ++s) oacc[i][s] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float mrun[QSUB], lrun[QSUB];
#pragma unroll
  for (int s = 0; s < QSUB; ++s) { mrun[s] = MC ? 0.f : -INFINITY; lrun[s] = 0.f; }

  auto compute = [&](int buf, int kv0, bool masked, bool first) {
    const T* Ks = lds + buf * 2 * TILE;
    const T* Vs = Ks + TILE;
    f32x4_t sacc[4][QSUB];
#pragma unroll
    for (int js = 0; js < 4; ++js)
#pragma unroll
      for (int s = 0; s < QSUB; ++s) sacc[js][s] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int js = 0; js < 4; ++js) {
      const T* krow = Ks + (16 * js + lr) * ROW;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        Frag8<T> ka;
        ka.v = *reinterpret_cast<const uint4*>(krow + 32 * c + 8 * g);
#pragma unroll
        for (int s = 0; s < QSUB; ++s) {
#if ATTN_ABL == 2   // ablation: no Q.K^T MFMA
          sacc[js][s][c & 3] += __uint_as_float(ka.v.x ^ q32[s][c].v.y);
#else
          mma_k32(sacc[js][s], ka, q32[s][c]);
#endif
        }
      }
    }
    uint2 pk[4][QSUB];                      // bf16 P^T, (kv 4g .. 4g+3 of fragment js) per lane
    uint32_t pk8[4][QSUB];                  // F8: the same four values as e4m3 bytes
#pragma unroll
    for (int s = 0; s < QSUB; ++s) {
      if (masked) {
#pragma unroll
        for (int js = 0; js < 4; ++js)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kv0 + 16 * js + 4 * g + r >= p.nkv) sacc[js][s][r] = -INFINITY;
      }
      // maximum3 straight on the MFMA results (fmaxf would canonicalise every operand first)
      float m0 = vmax3(sacc[0][s][0], sacc[0][s][1], sacc[0][s][2]);
      float m1 = vmax3(sacc[0][s][3], sacc[1][s][0], sacc[1][s][1]);
      float m2 = vmax3(sacc[1][s][2], sacc[1][s][3], sacc[2][s][0]);
      float m3 = vmax3(sacc[2][s][1], sacc[2][s][2], sacc[2][s][3]);
      float m4 = vmax3(sacc[3][s][0], sacc[3][s][1], sacc[3][s][2]);
      float mx = vmax3(m0, m1, m2);
      mx = vmax3(mx, m3, m4);
      mx = max_over_groups_raw(vmax3(mx, sacc[3][s][3], sacc[3][s][3]));
      if constexpr (MC) {
        // accumulators are s * c2 - m already; the first tile always sets m (from m = 0)
        if (first || __any(mx > kRescaleThr)) {
          const float tgt = mrun[s] + mx;
          const float mn = bf16_rne(first ? tgt : fmaxf(mrun[s], tgt));
          const float delta = mn - mrun[s];
          const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-delta);   // (O = 0 on the first tile)
          mrun[s] = mn;
          if (!ONES) lrun[s] *= alpha;
#pragma unroll
          for (int i = 0; i < ND; ++i) oacc[i][s] *= alpha;
#pragma unroll
          for (int js = 0; js < 4; ++js) sacc[js][s] -= delta;
          if (g == gq) q32[s][NC - 1].v.x = (q32[s][NC - 1].v.x & 0xffff0000u) | (__float_as_uint(-mn) >> 16);
        }
        float lsum = 0.f;
#pragma unroll
        for (int js = 0; js < 4; ++js) {
          float pv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pv[r] = __builtin_amdgcn_exp2f(sacc[js][s][r]);
            if (!ONES) lsum += pv[r];
          }
          if constexpr (F8) pk8[js][s] = pack_fp8x4(pv[0], pv[1], pv[2], pv[3]);
          else pk[js][s] = make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
        }
        if (!ONES) lrun[s] += lsum;
        continue;
      }
      const float ms = mx * c2;
      if (__any(ms > mrun[s] + kRescaleThr)) {
        const float mnew = fmaxf(mrun[s], ms);
        const float alpha = __builtin_amdgcn_exp2f(mrun[s] - mnew);
        mrun[s] = mnew;
        if (!ONES) lrun[s] *= alpha;
#pragma unroll
        for (int i = 0; i < ND; ++i) oacc[i][s] *= alpha;
      }
      const float mneg = -mrun[s];
      float lsum = 0.f;
#pragma unroll
      for (int js = 0; js < 4; ++js) {
        float pv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#if ATTN_ABL == 1   // ablation: no transcendental
          pv[r] = fmaf(sacc[js][s][r], c2, mneg);
#else
          pv[r] = __builtin_amdgcn_exp2f(fmaf(sacc[js][s][r], c2, mneg));
#endif
          if (!ONES) lsum += pv[r];
        }
        if constexpr (F8) pk8[js][s] = pack_fp8x4(pv[0], pv[1], pv[2], pv[3]);
        else pk[js][s] = make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
      }
      if (!ONES) lrun[s] += lsum;
    }
    // O^T += V^T P^T, 32 keys per MFMA
    typedef __attribute__((ext_vector_type(4))) short s4_t;
    typedef __attribute__((address_space(3))) s4_t lds_s4_t;
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const T* a0 = Vs + (32 * t + 4 * g + (lr >> 2)) * ROW + 16 * dd + 4 * (lr & 3);
        const uint2 lo = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0)));
        const uint2 hi = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0 + 16 * ROW)));
        if constexpr (F8) {
          const long va8 = (long)((uint64_t)bf16x4_to_fp8x4(lo) | ((uint64_t)bf16x4_to_fp8x4(hi) << 32));
#pragma unroll
          for (int s = 0; s < QSUB; ++s) {
            const long pb8 = (long)((uint64_t)pk8[2 * t][s] | ((uint64_t)pk8[2 * t + 1][s] << 32));
            oacc[dd][s] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(va8, pb8, oacc[dd][s], 0, 0, 0);
          }
          continue;
        }
        Frag8<T> va;
        va.v = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
        for (int s = 0; s < QSUB; ++s) {
          Frag8<T> pb;
          pb.v = make_uint4(pk[2 * t][s].x, pk[2 * t][s].y, pk[2 * t + 1][s].x, pk[2 * t + 1][s].y);
#if ATTN_ABL == 3   // ablation: no P.V MFMA
          oacc[dd][s][t] += __uint_as_float(va.v.x ^ pb.v.y ^ va.v.z ^ pb.v.w);
#else
          mma_k32(oacc[dd][s], va, pb);
#endif
        }
      }
    }
  };

  // full tiles in the loop (one compute body: no per-tile copies of the accumulators between
  // a masked and an unmasked instance), the ragged last tile after it
  const int ntiles = t1;
  const int nfull = KVS ? min(p.nkv / KVT, t1) : p.nkv / KVT;
  issue_tile(t0 * KVT, t0 & 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = t0; t < nfull; ++t) {
    if (t + 1 < nfull) issue_full((t + 1) & 1);
    else if (t + 1 < ntiles) issue_tile((t + 1) * KVT, (t + 1) & 1);
    compute(t & 1, t * KVT, false, t == t0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int tr = KVS ? max(nfull, t0) : nfull;             // the ragged last tile
  if (tr < ntiles) compute(tr & 1, tr * KVT, true, tr == t0);

  T* op = reinterpret_cast<T*>(p.o) + (int64_t)b * p.nq * p.os + (int64_t)h * p.d;
#pragma unroll
  for (int s = 0; s < QSUB; ++s) {
    float lt;
    if constexpr (ONES) {
      lt = __shfl(oacc[ND - 1][s][0], 32 + lr, 64);
    } else {
      lt = lrun[s] + __shfl_xor(lrun[s], 16, 64);
      lt += __shfl_xor(lt, 32, 64);
    }
    const float inv = 1.0f / lt;
    const int qi = qbase + 16 * s + lr;
    if (qi >= p.nq) continue;
    if constexpr (KVS) {
      // this split's normalised output and log-sum-exp (fp32) for attn_kv_combine
      const int64_t row = ((int64_t)split * p.batch + b) * p.heads * p.nq + (int64_t)h * p.nq + qi;
      if (g == 0) p.lsepart[row] = mrun[s] + __log2f(lt);
      float* orow = p.opart + row * p.d;
#pragma unroll
      for (int dd = 0; dd < ND; ++dd) {
        const int d = 16 * dd + 4 * g;
        if (d >= p.d) continue;
        *reinterpret_cast<float4*>(orow + d) = make_float4(oacc[dd][s][0] * inv, oacc[dd][s][1] * inv,
                                                           oacc[dd][s][2] * inv, oacc[dd][s][3] * inv);
      }
      continue;
    }
    if (p.lse && g == 0) p.lse[((int64_t)b * p.heads + h) * p.nq + qi] = mrun[s] + __log2f(lt);
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
      const int d = 16 * dd + 4 * g;
      if (d >= p.d) continue;
      *reinterpret_cast<uint2*>(op + (int64_t)qi * p.os + d) =
          make_uint2(pack_bf16x2(oacc[dd][s][0] * inv, oacc[dd][s][1] * inv),
                     pack_bf16x2(oacc[dd][s][2] * inv, oacc[dd][s][3] * inv));
    }
  }
}

// ======================================================================================
// head_dim 40 (the UNet's 64x64 level: 4096 tokens, ~90 % of the attention time) on the
// 32x32x16 MFMA.  Per wave: 32 queries; per 64-key tile:
//   S^T[kv][q] = K Q^T   two 32-key blocks x three 16-wide head-dim chunks = 6 MFMAs (x16
//                        padding of d = 40 -> 48 instead of the x32 padding -> 64 of the
//                        16x16x32 form: 6 issues instead of 16);
//   O^T[d][q] += V^T P^T two 32-row head-dim blocks x four 16-key steps = 8 MFMAs; the B operand
//                        is the S^T accumulator converted in place (a 32x32 result has its column
//                        on the lane and its rows in registers; k order 16s + 8(j>>2) + 4h + (j&3)),
//                        the A operand two ds_read_b64_tr_b16 of the row-major V tile in that order.
// The row max is a tree over the lane's 32 scores plus one permlane32 swap.  Scale and running
// max ride in the head-dim padding (Q prescaled, Q[:, 40] = -m, K[:, 40] = 1), the softmax
// denominator in V's ones column (d = 40), as in attn32_kernel's MC / ONES forms.
// Templated on the head dim D (a multiple of 8): D = 40 (the 64x64 level) and D = 80 (the 32x32
// level).  Q.K^T runs over DQ = D + 1 (the max column) rounded up to 16 (48 / 96: 3 / 6 MFMAs per
// 32-key block), P.V over ND32 = ceil((D + 1) / 32) 32-row head-dim blocks (2 / 3, the ones column
// d = D carrying the denominator).
// SKEW: the block's waves in two phases one half-iteration apart, so the two waves of a block on a
// SIMD (waves w and w + 4) do not want the matrix pipe and the VALU at the same time: the upper half
// ("lagging" waves) run the softmax and P.V of tile t - 1 and then Q.K^T of tile t between the same
// barriers in which the lower half run Q.K^T, softmax and P.V of tile t.  Per wave the operations
// and their order are unchanged (bit-identical); V of tile t - 1 stays readable, so three K/V buffers.
// (__launch_bounds__' second argument is waves per SIMD: OCC blocks of NW waves need OCC * NW / 4; the
// default form meets it at 127 VGPRs unasked, the SKEW form is held to it)
// KVS: split-KV (config 2's single frame: 256 four-wave blocks left one wave per SIMD): block id =
// (query block, split); the split walks key tiles [t0, t1) and writes its normalised fp32 output and
// log-sum-exp, which attn_kv_combine merges
// PAIR: the tile loop unrolled by two, so each tile's K / V buffer is a compile-time constant (LDS
// fragment addresses as immediate offsets instead of a per-tile select + multiply-add) and the first
// tile of a pair issues its successor without the ragged-tile test
template <int V>
struct IntC {
  static constexpr int value = V;
};
// IL (QS = 2): the two query subtiles' phases interleaved inside each wave — S(1) = K Q1^T beside the
// exp / cvt of subtile 0, O(0) += V^T P0^T beside those of subtile 1 — so the wave's own VALU work
// fills the issue slots its MFMAs leave (the same-wave interleave overlaps where two waves on a SIMD
// do not: tools/mfma_valu_overlap.hip).  Each subtile keeps its own running-max decision, i.e. the
// QS = 1 kernel's per-wave arithmetic: bit-identical to it.
template <int NW, int OCC, int KT = 64, int D = 40, int QS = 1, bool SKEW = false, bool KVS = false,
          bool PAIR = false, bool IL = false>
__global__ __launch_bounds__(64 * NW, PAIR ? (OCC * NW + 3) / 4 : OCC) void attn_d40_kernel(const AttnArgs p) {
  typedef bf16_t T;
  typedef __attribute__((ext_vector_type(16))) float f32x16_t;
  static_assert(D % 8 == 0, "head dim");
  static_assert(QS == 1 || (QS == 2 && (KT == 64 || (IL && (KT == 128 || KT == 256)))), "query subtiles");
  constexpr int DQ = (D + 16) / 16 * 16, QC = DQ / 16, ND32 = (D + 32) / 32;
  constexpr int EPC = 8, CPR = (DQ > 32 * ND32 ? DQ : 32 * ND32) / 8, RCH = CPR + 1, ROW = RCH * EPC,
                TILE = KT * ROW, ES = 2;
  constexpr int NB = SKEW ? 3 : 2;                  // K/V tile buffers
  __shared__ uint4 smem[NB * 2 * TILE * ES / 16];
  T* const lds = reinterpret_cast<T*>(smem);
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5, i16 = lane & 15;
  int qb, h, b, split = 0;
  {
    const int nqb = (p.nq + 32 * QS * NW - 1) / (32 * QS * NW);
    const int bid = blockIdx.x, nblk = gridDim.x;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    int t = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
    if constexpr (KVS) {
      split = t % p.kvsplit;
      t /= p.kvsplit;
    }
    qb = t % nqb;
    const int hb = t / nqb;
    h = hb % p.heads;
    b = hb / p.heads;
  }
  static_assert(!(SKEW && KVS), "split-KV has one phase");
  const int ntiles_all = (p.nkv + KT - 1) / KT;
  const int t0 = KVS ? ntiles_all * split / p.kvsplit : 0;               // this block's key tiles
  const int t1 = KVS ? ntiles_all * (split + 1) / p.kvsplit : ntiles_all;
  // a wave owns QS subtiles of 32 queries: qbase + 32 s + r32
  const int qbase = qb * (32 * QS * NW) + wave * (32 * QS);
  const T* qp = reinterpret_cast<const T*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * p.d;
  const T* kp = reinterpret_cast<const T*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * p.d;
  const T* vp = reinterpret_cast<const T*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * p.d;
  constexpr int ONES_CHUNK = D / 8;                 // d = D: V ones column, K max column

  auto issue_tile = [&](int kv0, int buf) {
    const unsigned kb = lds0 + (unsigned)(buf * 2 * TILE * ES);
    const unsigned vb = kb + TILE * ES;
    for (int i = wave; i < RCH * (KT / 64); i += NW) {
      const int L = i * 64 + lane;
      const int row = L / RCH, c = L - row * RCH;
      const int kv = kv0 + row, d = c * EPC;
      const bool ok = kv < p.nkv && c < CPR && d < p.d;
      const bool kone = c == ONES_CHUNK && kv < p.nkv;
      const void* ks = ok ? (const void*)(kp + (int64_t)kv * p.ks + d)
                          : (kone ? (const void*)&kOnesBf16 : (const void*)&kZeros16);
      const void* vs = ok ? (const void*)(vp + (int64_t)kv * p.vs + d)
                          : (c == ONES_CHUNK ? (const void*)&kOnesBf16 : (const void*)&kZeros16);
      const unsigned off = __builtin_amdgcn_readfirstlane(i * 64 * 16);
      glds16(ks, kb + off);
      glds16(vs, vb + off);
    }
  };
  // full tiles: every lane's source is fixed but for the tile's key offset, so each of a wave's
  // (at most two) K/V chunk slots keeps a pointer that advances by one tile of rows per issue
  // (lanes of the constant columns 40..71 point at the ones / zeros rows and do not advance);
  // the general form above (bounds, selects, 64-bit multiplies per tile) serves the first and the
  // ragged last tile only
  constexpr int NSL = (RCH * (KT / 64) + NW - 1) / NW;   // chunk slots per wave
  const char* kq[NSL];
  const char* vq[NSL];
  int64_t kstep[NSL], vstep[NSL];
#pragma unroll
  for (int s2 = 0; s2 < NSL; ++s2) {
    const int i = wave + NW * s2;
    const int L = i * 64 + lane;
    const int row = L / RCH, c = L - row * RCH;
    const bool dat = i < RCH * (KT / 64) && c < CPR && c * EPC < p.d;
    const bool one = c == ONES_CHUNK;
    kq[s2] = dat ? reinterpret_cast<const char*>(kp + (int64_t)((t0 + 1) * KT + row) * p.ks + c * EPC)
                 : reinterpret_cast<const char*>(one ? (const void*)&kOnesBf16 : (const void*)&kZeros16);
    vq[s2] = dat ? reinterpret_cast<const char*>(vp + (int64_t)((t0 + 1) * KT + row) * p.vs + c * EPC)
                 : reinterpret_cast<const char*>(one ? (const void*)&kOnesBf16 : (const void*)&kZeros16);
    kstep[s2] = dat ? (int64_t)KT * p.ks * ES : 0;
    vstep[s2] = dat ? (int64_t)KT * p.vs * ES : 0;
  }
  unsigned soff[NSL];                // slot LDS offsets, wave-uniform (SGPRs, once)
#pragma unroll
  for (int s2 = 0; s2 < NSL; ++s2) soff[s2] = __builtin_amdgcn_readfirstlane((wave + NW * s2) * 64 * 16);
  auto issue_full = [&](int buf) {   // the next full tile (tile 1, 2, ... in order)
    const unsigned kb = lds0 + (unsigned)(buf * 2 * TILE * ES);
    const unsigned vb = kb + TILE * ES;
#pragma unroll
    for (int s2 = 0; s2 < NSL; ++s2) {
      const int i = wave + NW * s2;
      if (i >= RCH * (KT / 64)) break;
      const unsigned off = soff[s2];
      glds16(kq[s2], kb + off);
      glds16(vq[s2], vb + off);
      kq[s2] += kstep[s2];
      vq[s2] += vstep[s2];
    }
  };
  const float c2 = p.scale_log2;

  // Q^T (B operand) chunk c of subtile s: lane holds Q[q = qbase + 32 s + r32][d = 16c + 8hh .. +8]
  // * c2; the max column d = D is element 0 of chunk D / 16 in the hh = (D % 16) / 8 lanes
  // (initially -m = 0)
  uint4 qf[QS][QC];
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    const int qi = qbase + 32 * s + r32;
    const T* qrow = qp + (int64_t)qi * p.qs;
#pragma unroll
    for (int c = 0; c < QC; ++c) {
      const int dd = 16 * c + 8 * hh;
      if (qi < p.nq && dd < p.d) qf[s][c] = scale_bf16x8(*reinterpret_cast<const uint4*>(qrow + dd), c2);
      else qf[s][c] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  f32x16_t oacc[QS][ND32];
#pragma unroll
  for (int s = 0; s < QS; ++s)
#pragma unroll
    for (int db = 0; db < ND32; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[s][db][r] = 0.f;
  float mq[QS];
#pragma unroll
  for (int s = 0; s < QS; ++s) mq[s] = 0.f;

  typedef __attribute__((ext_vector_type(4))) short s4_t;
  typedef __attribute__((address_space(3))) s4_t lds_s4_t;
  // the lane's max over a subtile's 64 scores of this tile (a tree of max3, then the other half)
  auto tile_max = [&](const f32x16_t (&sa)[2]) {
    float t[11];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int a = 3 * k;
      t[k] = vmax3(a < 16 ? sa[0][a] : sa[1][a - 16], a + 1 < 16 ? sa[0][a + 1] : sa[1][a + 1 - 16],
                   a + 2 < 16 ? sa[0][a + 2] : sa[1][a + 2 - 16]);
    }
    t[10] = __builtin_elementwise_maximum(sa[1][14], sa[1][15]);
    const float u0 = vmax3(t[0], t[1], t[2]), u1 = vmax3(t[3], t[4], t[5]), u2 = vmax3(t[6], t[7], t[8]);
    float mx = vmax3(vmax3(u0, u1, u2), t[9], t[10]);
    unsigned w = __float_as_uint(mx);
    const auto sw = __builtin_amdgcn_permlane32_swap(w, w, false, false);
    return vmax3(__uint_as_float(sw[0]), __uint_as_float(sw[1]), mx);
  };
  auto to_p = [&](const f32x16_t (&sa)[2], uint4 (&pb)[2][2]) {   // bf16 P^T fragments of k-step (blk, st)
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) pv[j] = __builtin_amdgcn_exp2f(sa[blk][8 * st + j]);
        pb[blk][st] = make_uint4(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]), pack_bf16x2(pv[4], pv[5]),
                                 pack_bf16x2(pv[6], pv[7]));
      }
  };
  // S^T = K Q^T of one 64-key half of the tile in buffer buf: each K fragment read from LDS feeds the
  // MFMAs of every subtile
  auto qk = [&](int buf, int half, f32x16_t (&sacc)[QS][2]) {
    const T* Ks = lds + buf * 2 * TILE + half * 64 * ROW;
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
      for (int s = 0; s < QS; ++s)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[s][blk][r] = 0.f;
      const T* krow = Ks + (32 * blk + r32) * ROW + 8 * hh;
#pragma unroll
      for (int c = 0; c < QC; ++c) {
        const uint4 ka = *reinterpret_cast<const uint4*>(krow + 16 * c);
#pragma unroll
        for (int s = 0; s < QS; ++s)
          sacc[s][blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, ka),
                                                                 __builtin_bit_cast(bf16x8_t, qf[s][c]), sacc[s][blk], 0, 0, 0);
      }
    }
  };
  // the online softmax of S^T (running max, lazy rescale, P = exp2) and O^T += V^T P^T for the same
  // half of the tile in buffer buf
  auto smpv = [&](f32x16_t (&sacc)[QS][2], int buf, int half, bool first) {
    const T* Vs = lds + buf * 2 * TILE + TILE + half * 64 * ROW;
    float mx[QS];
    bool resc = first;
#pragma unroll
    for (int s = 0; s < QS; ++s) {
      mx[s] = tile_max(sacc[s]);
      resc = resc || mx[s] > kRescaleThr;
    }
    // accumulators are s * c2 - m already; the first tile always sets m (from m = 0).  One wave-
    // uniform branch for all subtiles (a subtile rescaled without need only moves m up to its max)
    if (first || __any(resc)) {
#pragma unroll
      for (int s = 0; s < QS; ++s) {
        const float tgt = mq[s] + mx[s];
        const float mn = bf16_rne(first ? tgt : fmaxf(mq[s], tgt));
        const float delta = mn - mq[s];
        const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-delta);   // (O = 0 on the first tile)
        mq[s] = mn;
#pragma unroll
        for (int db = 0; db < ND32; ++db) oacc[s][db] *= alpha;
        sacc[s][0] -= delta;
        sacc[s][1] -= delta;
        if (hh == (D % 16) / 8) qf[s][D / 16].x = (qf[s][D / 16].x & 0xffff0000u) | (__float_as_uint(-mn) >> 16);
      }
    }
    uint4 pb[QS][2][2];
#pragma unroll
    for (int s = 0; s < QS; ++s) to_p(sacc[s], pb[s]);
    // O^T += V^T P^T: A = V^T rows d (block db) for keys 16s' + {4hh..+3, 8 + 4hh..+3} of block blk;
    // each V fragment feeds every subtile
#pragma unroll
    for (int db = 0; db < ND32; ++db) {
      const int cb = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
#pragma unroll
      for (int blk = 0; blk < 2; ++blk)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const T* a0 = Vs + (32 * blk + 16 * st + 4 * hh + (i16 >> 2)) * ROW + cb;
          const uint2 lo = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0)));
          const uint2 hi = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0 + 8 * ROW)));
          const uint4 va = make_uint4(lo.x, lo.y, hi.x, hi.y);
#pragma unroll
          for (int s = 0; s < QS; ++s)
            oacc[s][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, va),
                                                                  __builtin_bit_cast(bf16x8_t, pb[s][blk][st]), oacc[s][db], 0, 0, 0);
        }
    }
  };
  static_assert(!IL || (QS == 2 && !SKEW && !KVS && !PAIR), "IL interleaves the two subtiles of the plain loop");
  auto compute_il = [&](int buf, int kv0, bool masked, bool first, int half) {
    first = first && half == 0;                      // (128-key tiles: the second half is never first)
    const T* Ks = lds + buf * 2 * TILE + half * 64 * ROW;
    const T* Vs = lds + buf * 2 * TILE + TILE + half * 64 * ROW;
    kv0 += 64 * half;
    f32x16_t sacc[2][2];
    uint4 ka[2][QC];                                 // K fragments, shared by both subtiles
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int c = 0; c < QC; ++c) ka[blk][c] = *reinterpret_cast<const uint4*>(Ks + (32 * blk + r32) * ROW + 8 * hh + 16 * c);
    auto qk1 = [&](int s) __attribute__((always_inline)) {
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[s][blk][r] = 0.f;
#pragma unroll
        for (int c = 0; c < QC; ++c)
          sacc[s][blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, ka[blk][c]),
                                                                 __builtin_bit_cast(bf16x8_t, qf[s][c]), sacc[s][blk], 0, 0, 0);
      }
    };
    auto mask1 = [&](int s) __attribute__((always_inline)) {
      if (masked) {
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kv0 + 32 * blk + 8 * (r >> 2) + 4 * hh + (r & 3) >= p.nkv) sacc[s][blk][r] = -INFINITY;
      }
    };
    auto resc1 = [&](int s) __attribute__((always_inline)) {   // attn_d40_kernel<QS = 1>'s decision, per subtile
      const float mx = tile_max(sacc[s]);
      if (first || __any(mx > kRescaleThr)) {
        const float tgt = mq[s] + mx;
        const float mn = bf16_rne(first ? tgt : fmaxf(mq[s], tgt));
        const float delta = mn - mq[s];
        const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-delta);
        mq[s] = mn;
#pragma unroll
        for (int db = 0; db < ND32; ++db) oacc[s][db] *= alpha;
        sacc[s][0] -= delta;
        sacc[s][1] -= delta;
        if (hh == (D % 16) / 8) qf[s][D / 16].x = (qf[s][D / 16].x & 0xffff0000u) | (__float_as_uint(-mn) >> 16);
      }
    };
    auto pv1 = [&](int s, const uint4 (&pb)[2][2]) __attribute__((always_inline)) {
#pragma unroll
      for (int db = 0; db < ND32; ++db) {
        const int cb = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const T* a0 = Vs + (32 * blk + 16 * st + 4 * hh + (i16 >> 2)) * ROW + cb;
            const uint2 lo = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0)));
            const uint2 hi = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0 + 8 * ROW)));
            const uint4 va = make_uint4(lo.x, lo.y, hi.x, hi.y);
            oacc[s][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, va),
                                                                  __builtin_bit_cast(bf16x8_t, pb[blk][st]), oacc[s][db], 0, 0, 0);
          }
      }
    };
    uint4 pb0[2][2], pb1[2][2];
    qk1(0);
    mask1(0);
    resc1(0);
    // S(1) beside P(0) (the compiler's interleave: pinning each MFMA to two exps and two other VALU
    // with sched_group_barrier measured slower, 212.6 -> 235 us at N = 4096)
    qk1(1);
    to_p(sacc[0], pb0);
    // P(0) is consumed here (an empty asm reading it), so the compiler cannot sink its exps below the
    // rescale branch into the P.V region
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int st = 0; st < 2; ++st)
        asm volatile("" ::"v"(pb0[blk][st].x), "v"(pb0[blk][st].y), "v"(pb0[blk][st].z), "v"(pb0[blk][st].w));
    mask1(1);
    resc1(1);
    // O(0) += V^T P0^T beside P(1) (subtile 1's row max moved beside it instead measured slower:
    // 214.4 -> 229.2 us)
    pv1(0, pb0);
    to_p(sacc[1], pb1);
    pv1(1, pb1);
  };
  auto compute = [&](int buf, int kv0, bool masked, bool first, int half) {
    if constexpr (IL) {
      compute_il(buf, kv0, masked, first, half);
      return;
    }
    f32x16_t sacc[QS][2];
    qk(buf, half, sacc);
    kv0 += 64 * half;
    if (masked) {
#pragma unroll
      for (int s = 0; s < QS; ++s)
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kv0 + 32 * blk + 8 * (r >> 2) + 4 * hh + (r & 3) >= p.nkv) sacc[s][blk][r] = -INFINITY;
    }
    smpv(sacc, buf, half, first && half == 0);
  };

  const int ntiles = t1;                                   // (tiles t0 .. t1 - 1 are this block's)
  const int nfull = KVS ? min(p.nkv / KT, t1) : p.nkv / KT;
  auto bufi = [](int t) { return NB == 3 ? t % 3 : t & 1; };
  auto issue_next = [&](int t) {   // tile t + 1 while tile t is multiplied
    if (t + 1 < nfull) issue_full(bufi(t + 1));
    else if (t + 1 < ntiles) issue_tile((t + 1) * KT, bufi(t + 1));
  };
  issue_tile(t0 * KT, bufi(t0));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#ifdef ATTN_PRIO   // ablation builds: static priority for the second-dispatched half of the waves
  if (__builtin_amdgcn_readfirstlane(wave) >= NW / 2) __builtin_amdgcn_s_setprio(1);
#endif
  if constexpr (!SKEW && PAIR) {
    // tile t in buffer BQ; SURE: tile t + 1 is known to be a full tile
    auto step = [&](int t, auto bq, auto sure) {
      constexpr int BQ = decltype(bq)::value;
      if (decltype(sure)::value || t + 1 < nfull) issue_full(BQ ^ 1);
      else if (t + 1 < ntiles) issue_tile((t + 1) * KT, BQ ^ 1);
#pragma unroll
      for (int hf = 0; hf < KT / 64; ++hf) compute(BQ, t * KT, false, t == t0, hf);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    };
    int t = t0;
    if ((t & 1) && t < nfull) step(t++, IntC<1>{}, IntC<0>{});
    for (; t + 1 < nfull; t += 2) {
      step(t, IntC<0>{}, IntC<1>{});
      step(t + 1, IntC<1>{}, IntC<0>{});
    }
    if (t < nfull) step(t, IntC<0>{}, IntC<0>{});
  } else if constexpr (!SKEW) {
    for (int t = t0; t < nfull; ++t) {
      issue_next(t);
#pragma unroll
      for (int hf = 0; hf < KT / 64; ++hf) compute(bufi(t), t * KT, false, t == t0, hf);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    const bool lag = __builtin_amdgcn_readfirstlane(wave) >= NW / 2;
    if (!lag) {
      for (int t = 0; t < nfull; ++t) {
        issue_next(t);
#pragma unroll
        for (int hf = 0; hf < KT / 64; ++hf) compute(bufi(t), t * KT, false, t == 0, hf);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    } else {
      // S^T of tile t - 1 stays in sp across the barrier
      f32x16_t sp[KT / 64][QS][2];
      for (int t = 0; t < nfull; ++t) {
        issue_next(t);
        if (t > 0) {
#pragma unroll
          for (int hf = 0; hf < KT / 64; ++hf) smpv(sp[hf], bufi(t - 1), hf, t == 1 && hf == 0);
        }
        __builtin_amdgcn_sched_barrier(0);   // tile t's S^T is not started under tile t - 1's P.V
#pragma unroll
        for (int hf = 0; hf < KT / 64; ++hf) qk(bufi(t), hf, sp[hf]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      if (nfull > 0) {
#pragma unroll
        for (int hf = 0; hf < KT / 64; ++hf) smpv(sp[hf], bufi(nfull - 1), hf, nfull == 1 && hf == 0);
      }
    }
  }
  const int tr = KVS ? max(nfull, t0) : nfull;             // the ragged last tile
  if (tr < ntiles) {
    for (int hf = 0; hf < KT / 64 && tr * KT + 64 * hf < p.nkv; ++hf)
      compute(bufi(tr), tr * KT, true, tr == t0, hf);
  }

  // denominator: O^T row d = D = block D / 32, register 4 ((D % 32) / 8) of the hh = 0 lane of this
  // column (a 32x32 result row 8 (r >> 2) + 4 hh + (r & 3) sits in register r of the hh half)
  static_assert(D % 8 == 0, "denominator row");
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    const float lt = __shfl(oacc[s][D / 32][4 * ((D % 32) / 8)], r32, 64);
    const float inv = 1.0f / lt;
    const int qi = qbase + 32 * s + r32;
    if (KVS && qi < p.nq) {
      // this split's normalised output and log-sum-exp (fp32) for attn_kv_combine
      const int64_t row = ((int64_t)split * p.batch + b) * p.heads * p.nq + (int64_t)h * p.nq + qi;
      if (hh == 0) p.lsepart[row] = mq[s] + __log2f(lt);
      float* orow = p.opart + row * D;
#pragma unroll
      for (int db = 0; db < ND32; ++db)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = 32 * db + 8 * g4 + 4 * hh;
          if (32 * db + 8 * g4 >= D) break;
          *reinterpret_cast<float4*>(orow + d) = make_float4(oacc[s][db][4 * g4] * inv, oacc[s][db][4 * g4 + 1] * inv,
                                                             oacc[s][db][4 * g4 + 2] * inv, oacc[s][db][4 * g4 + 3] * inv);
        }
    } else if (qi < p.nq) {
      if (p.lse && hh == 0) p.lse[((int64_t)b * p.heads + h) * p.nq + qi] = mq[s] + __log2f(lt);
      T* orow = reinterpret_cast<T*>(p.o) + (int64_t)b * p.nq * p.os + (int64_t)h * p.d + (int64_t)qi * p.os;
#pragma unroll
      for (int db = 0; db < ND32; ++db)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = 32 * db + 8 * g4 + 4 * hh;
          if (32 * db + 8 * g4 >= D) break;          // (compile-time: D % 8 == 0)
          *reinterpret_cast<uint2*>(orow + d) =
              make_uint2(pack_bf16x2(oacc[s][db][4 * g4] * inv, oacc[s][db][4 * g4 + 1] * inv),
                         pack_bf16x2(oacc[s][db][4 * g4 + 2] * inv, oacc[s][db][4 * g4 + 3] * inv));
        }
    }
  }
}

// buffer LDS-DMA of 16 bytes per lane (igemm_common.h's dma16s: per-lane offset in one VGPR, the
// wave-uniform part in soffset; out-of-range offsets read zeros)
__device__ __forceinline__ void attn_dma16s(__amdgpu_buffer_rsrc_t rsrc, int voff, int soff, unsigned lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds_addr)
      : "memory");
}

// head_dim 40 with the tile loop software-pipelined inside each wave: Q.K^T of tile t + 1 is issued
// beside the softmax exp / cvt of tile t, and P.V of tile t beside the rest of it, in one
// branch-free region whose interleave is fixed with sched_group_barrier (attn_d40_kernel's waves
// are phase-locked by the per-tile barrier: all of a block's waves issue Q.K^T, then all run the
// softmax VALU with the matrix pipe idle).  P.V(t) reads tile t's V while Q.K^T reads tile t + 1's
// K and tile t + 2 streams in: three LDS buffers.  The K / V tiles arrive by buffer LDS-DMA with
// one lane offset per slot (rows past n_kv read zeros); the max / ones columns (d = 40) are
// written once into every buffer and never DMA'd.  Same arithmetic per query as attn_d40_kernel
// (max column, ones column, bf16 P): bit-identical results.  8 waves x 32 queries per block.
template <int NW>
__global__ __launch_bounds__(64 * NW, 1) void attn_d40p_kernel(const AttnArgs p) {
  typedef bf16_t T;
  typedef __attribute__((ext_vector_type(16))) float f32x16_t;
  constexpr int D = 40, KT = 64, QC = 3, ND32 = 2;
  constexpr int EPC = 8, RCH = 9, ROW = RCH * EPC, TILE = KT * ROW, ES = 2, NBUF = 3;
  constexpr int DCH = D / EPC;                     // data chunks per row (5); chunk 5 = max / ones
  __shared__ uint4 smem[NBUF * 2 * TILE * ES / 16];
  T* const lds = reinterpret_cast<T*>(smem);
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5, i16 = lane & 15;
  int qb, h, b;
  {
    const int nqb = (p.nq + 32 * NW - 1) / (32 * NW);
    const int bid = blockIdx.x, nblk = gridDim.x;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    const int t = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
    qb = t % nqb;
    const int hb = t / nqb;
    h = hb % p.heads;
    b = hb / p.heads;
  }
  const int qbase = qb * (32 * NW) + wave * 32;
  const T* qp = reinterpret_cast<const T*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * D;
  const T* kp = reinterpret_cast<const T*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * D;
  const T* vp = reinterpret_cast<const T*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * D;
  const __amdgpu_buffer_rsrc_t rk =
      __builtin_amdgcn_make_buffer_rsrc((void*)kp, 0, (int)(((int64_t)(p.nkv - 1) * p.ks + D) * ES), 0x00020000);
  const __amdgpu_buffer_rsrc_t rv =
      __builtin_amdgcn_make_buffer_rsrc((void*)vp, 0, (int)(((int64_t)(p.nkv - 1) * p.vs + D) * ES), 0x00020000);

  // constant columns: chunk 5 of every row = (1.0, 0 ...) in K (max column) and V (ones column),
  // chunks 6..8 zero; the DMA below writes data chunks 0..4 only
  for (int i = tid; i < NBUF * 2 * KT * (RCH - DCH); i += 64 * NW) {
    const int c = DCH + i % (RCH - DCH), row = (i / (RCH - DCH)) % (NBUF * 2 * KT);
    smem[row * RCH + c] = c == DCH ? kOnesBf16 : kZeros16;
  }
  // DMA slots: instruction i (of RCH per tile and operand) covers 64 consecutive 16-byte chunks of
  // the [64 rows][9 chunks] tile; lanes of data chunks carry a fixed row offset, the rest are
  // masked off (exec) so the constant columns stay
  constexpr int NSL = (RCH + NW - 1) / NW;
  int koff[NSL], voff[NSL];
  bool dat[NSL];
#pragma unroll
  for (int s2 = 0; s2 < NSL; ++s2) {
    const int i = wave + NW * s2;
    const int L = i * 64 + lane;
    const int row = L / RCH, c = L - row * RCH;
    dat[s2] = i < RCH && c < DCH;
    koff[s2] = (row * p.ks + c * EPC) * ES;
    voff[s2] = (row * p.vs + c * EPC) * ES;
  }
  auto issue = [&](int t, int buf) __attribute__((always_inline)) {
    const unsigned kb = lds0 + (unsigned)(buf * 2 * TILE * ES);
    const unsigned vb = kb + TILE * ES;
    const int ktile = t * KT * p.ks * ES, vtile = t * KT * p.vs * ES;
#pragma unroll
    for (int s2 = 0; s2 < NSL; ++s2) {
      const int i = wave + NW * s2;
      if (i >= RCH) break;
      const unsigned off = __builtin_amdgcn_readfirstlane(i * 64 * 16);
      if (dat[s2]) {
        attn_dma16s(rk, koff[s2], __builtin_amdgcn_readfirstlane(ktile), __builtin_amdgcn_readfirstlane(kb + off));
        attn_dma16s(rv, voff[s2], __builtin_amdgcn_readfirstlane(vtile), __builtin_amdgcn_readfirstlane(vb + off));
      }
    }
  };
  const float c2 = p.scale_log2;
  uint4 qf[QC];
  {
    const int qi = qbase + r32;
    const T* qrow = qp + (int64_t)qi * p.qs;
#pragma unroll
    for (int c = 0; c < QC; ++c) {
      const int dd = 16 * c + 8 * hh;
      if (qi < p.nq && dd < D) qf[c] = scale_bf16x8(*reinterpret_cast<const uint4*>(qrow + dd), c2);
      else qf[c] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  f32x16_t oacc[ND32], sacc[2][2];   // sacc[c]: score slot c (tile being finished / next tile)
  float mq = 0.f;
#pragma unroll
  for (int db = 0; db < ND32; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[db][r] = 0.f;
  typedef __attribute__((ext_vector_type(4))) short s4_t;
  typedef __attribute__((address_space(3))) s4_t lds_s4_t;

  auto qk = [&](int s, int buf) __attribute__((always_inline)) {
    const T* Ks = lds + buf * 2 * TILE;
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[s][blk][r] = 0.f;
      const T* krow = Ks + (32 * blk + r32) * ROW + 8 * hh;
#pragma unroll
      for (int c = 0; c < QC; ++c) {
        const uint4 ka = *reinterpret_cast<const uint4*>(krow + 16 * c);
        sacc[s][blk] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, ka),
                                                               __builtin_bit_cast(bf16x8_t, qf[c]), sacc[s][blk], 0, 0, 0);
      }
    }
  };
  auto mask = [&](int s, int kv0) __attribute__((always_inline)) {
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kv0 + 32 * blk + 8 * (r >> 2) + 4 * hh + (r & 3) >= p.nkv) sacc[s][blk][r] = -INFINITY;
  };
  auto smax = [&](int s) __attribute__((always_inline)) {
    float t[11];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int a = 3 * k;
      t[k] = vmax3(a < 16 ? sacc[s][0][a] : sacc[s][1][a - 16], a + 1 < 16 ? sacc[s][0][a + 1] : sacc[s][1][a + 1 - 16],
                   a + 2 < 16 ? sacc[s][0][a + 2] : sacc[s][1][a + 2 - 16]);
    }
    t[10] = __builtin_elementwise_maximum(sacc[s][1][14], sacc[s][1][15]);
    const float u0 = vmax3(t[0], t[1], t[2]), u1 = vmax3(t[3], t[4], t[5]), u2 = vmax3(t[6], t[7], t[8]);
    float mx = vmax3(vmax3(u0, u1, u2), t[9], t[10]);
    unsigned w = __float_as_uint(mx);
    const auto sw = __builtin_amdgcn_permlane32_swap(w, w, false, false);
    return vmax3(__uint_as_float(sw[0]), __uint_as_float(sw[1]), mx);
  };
  auto rescale = [&](int s, float mx, bool first) __attribute__((always_inline)) {
    if (first || __any(mx > kRescaleThr)) {
      const float tgt = mq + mx;
      const float mn = bf16_rne(first ? tgt : fmaxf(mq, tgt));
      const float delta = mn - mq;
      const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-delta);
      mq = mn;
#pragma unroll
      for (int db = 0; db < ND32; ++db) oacc[db] *= alpha;
      sacc[s][0] -= delta;
      sacc[s][1] -= delta;
      if (hh == (D % 16) / 8) qf[D / 16].x = (qf[D / 16].x & 0xffff0000u) | (__float_as_uint(-mn) >> 16);
    }
  };
  // this tile's softmax + P.V (slot s, V of buffer buf) beside the next tile's Q.K^T (slot s ^ 1)
  auto body = [&](int s, int buf, int nbuf, bool next) __attribute__((always_inline)) {
    if (next) qk(s ^ 1, nbuf);
    uint4 pb[2][2];
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) pv[j] = __builtin_amdgcn_exp2f(sacc[s][blk][8 * st + j]);
        pb[blk][st] = make_uint4(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]), pack_bf16x2(pv[4], pv[5]),
                                 pack_bf16x2(pv[6], pv[7]));
      }
    const T* Vs = lds + buf * 2 * TILE + TILE;
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int db = 0; db < ND32; ++db) {
          const int cb = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
          const T* a0 = Vs + (32 * blk + 16 * st + 4 * hh + (i16 >> 2)) * ROW + cb;
          const uint2 lo = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0)));
          const uint2 hi = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0 + 8 * ROW)));
          const uint4 va = make_uint4(lo.x, lo.y, hi.x, hi.y);
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, va),
                                                             __builtin_bit_cast(bf16x8_t, pb[blk][st]), oacc[db], 0, 0, 0);
        }
    if (next) {
      // Q.K^T(next): 6 MFMAs, each beside one K read, four exp and two other VALU; then the P.V
      // MFMAs, each beside two V reads, one exp and two other VALU (masks: DS read 0x100, MFMA 0x8,
      // transcendental 0x400, VALU 0x2)
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        if (k + 1 < 6) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x400, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x400, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      }
    }
  };

  const int ntiles = (p.nkv + KT - 1) / KT;
  const int nfull = p.nkv / KT;
  issue(0, 0);
  if (1 < ntiles) issue(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  qk(0, 0);
  if (nfull == 0) mask(0, 0);
  rescale(0, smax(0), true);
  // tiles 0 .. ntiles - 2 have a next tile; the loop runs in pairs so score slots are compile-time
  auto step = [&](int s, int t) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // tile t + 1 landed for every wave; tile t - 1's buffer is free
    if (t + 2 < ntiles) issue(t + 2, (t + 2) % NBUF);
    body(s, t % NBUF, (t + 1) % NBUF, true);
    if (t + 1 >= nfull) mask(s ^ 1, (t + 1) * KT);
    rescale(s ^ 1, smax(s ^ 1), false);
  };
  int t = 0;
  for (; t + 2 < ntiles; t += 2) {
    step(0, t);
    step(1, t + 1);
  }
  if (t + 1 < ntiles) {
    step(0, t);
    ++t;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    body(1, t % NBUF, 0, false);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    body(0, t % NBUF, 0, false);
  }

  const float lt = __shfl(oacc[D / 32][4 * ((D % 32) / 8)], r32, 64);
  const float inv = 1.0f / lt;
  const int qi = qbase + r32;
  if (qi < p.nq) {
    if (p.lse && hh == 0) p.lse[((int64_t)b * p.heads + h) * p.nq + qi] = mq + __log2f(lt);
    T* orow = reinterpret_cast<T*>(p.o) + (int64_t)b * p.nq * p.os + (int64_t)h * D + (int64_t)qi * p.os;
#pragma unroll
    for (int db = 0; db < ND32; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * db + 8 * g4 + 4 * hh;
        if (32 * db + 8 * g4 >= D) break;
        *reinterpret_cast<uint2*>(orow + d) =
            make_uint2(pack_bf16x2(oacc[db][4 * g4] * inv, oacc[db][4 * g4 + 1] * inv),
                       pack_bf16x2(oacc[db][4 * g4 + 2] * inv, oacc[db][4 * g4 + 3] * inv));
      }
  }
}

int g_attn_waves = 0;   // 0: auto (8 when that still gives >= 256 blocks), 4 or 8: forced

template <int DP, int QSUB, bool ONES, bool F8 = false, bool MC = false>
int launch32_cfg(const AttnArgs& a, int batch, hipStream_t s) {
  const int blocks8 = (a.nq + 128 * QSUB - 1) / (128 * QSUB) * a.heads * batch;
  if (g_attn_waves == 8 || (g_attn_waves == 0 && blocks8 >= 256)) {
    // 8 waves share every K/V tile (one 512-thread block per CU): half the LDS-DMA bytes per FLOP
    const int nblk = (a.nq + 128 * QSUB - 1) / (128 * QSUB) * a.heads * batch;
    hipLaunchKernelGGL((attn32_kernel<DP, QSUB, ONES, 8, 1, F8, MC>), dim3(nblk), dim3(512), 0, s, a);
  } else {
    const int nblk = (a.nq + 64 * QSUB - 1) / (64 * QSUB) * a.heads * batch;
    hipLaunchKernelGGL((attn32_kernel<DP, QSUB, ONES, 4, 2, F8, MC>), dim3(nblk), dim3(256), 0, s, a);
  }
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

template <int DP, int QSUB, bool ONES, int NW, int OCC, bool F8 = false, bool MC = false>
int launch_occ(const AttnArgs& a, int batch, hipStream_t s) {
  const int nblk = (a.nq + 16 * QSUB * NW - 1) / (16 * QSUB * NW) * a.heads * batch;
  hipLaunchKernelGGL((attn32_kernel<DP, QSUB, ONES, NW, OCC, F8, MC>), dim3(nblk), dim3(64 * NW), 0, s, a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

int g_attn_maxcol = 1;   // tuning / A-B hook: 0 keeps the per-score FMA (no max column)
int g_attn_d40 = 1;      // tuning / A-B hook: 0 routes head_dim 40 to the 16x16x32 kernel

template <int DP, bool F8 = false, bool MC = false>
int launch32_dp_mc(const AttnArgs& a, int batch, hipStream_t s) {
  // query subtiles per wave: as many as stay spill-free (the ONES variant has no l registers)
  constexpr int QS1 = DP <= 48 ? 4 : (DP <= 96 ? 2 : 1);
  constexpr int QS0 = DP <= 96 ? 2 : 1;
  if constexpr (DP == 48) {
    // head_dim 40 (the 64x64 level): 8 waves x 2 query subtiles at 118 VGPRs -> two blocks per
    // CU whose phases drift apart, so one block's softmax VALU runs beside the other's MFMAs
    // (N=4096: 295 -> 265 us against one 8-wave block of 4 subtiles); needs >= 2 blocks per CU
    const int nblk2 = (a.nq + 255) / 256 * a.heads * batch;
    if (a.d == DP - 8 && g_attn_waves == 0 && nblk2 >= 512)
      return launch_occ<DP, 2, true, 8, 2, F8, MC>(a, batch, s);
  }
  if (a.d == DP - 8) return launch32_cfg<DP, QS1, true, F8, MC>(a, batch, s);
  return launch32_cfg<DP, QS0, false, F8, MC>(a, batch, s);
}

// split-KV merge: one thread per (row = (b, h, q), 4 head-dim columns); the splits' fp32 partials
// are weighted by 2^(lse_s - max lse) (log2 domain, like the kernels' lse) and summed in split order
template <int D>
__global__ __launch_bounds__(256) void attn_kv_combine(const AttnArgs p) {
  constexpr int NC = D / 4;
  const int64_t rows = (int64_t)p.batch * p.heads * p.nq;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= rows * NC) return;
  const int64_t row = gid / NC;
  const int c4 = (int)(gid - row * NC);
  float m = -INFINITY;
  for (int sp = 0; sp < p.kvsplit; ++sp) m = fmaxf(m, p.lsepart[sp * rows + row]);
  float den = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int sp = 0; sp < p.kvsplit; ++sp) {
    const float w = exp2f(p.lsepart[sp * rows + row] - m);
    const float4 o = *reinterpret_cast<const float4*>(p.opart + (sp * rows + row) * D + 4 * c4);
    den += w;
    acc.x += w * o.x; acc.y += w * o.y; acc.z += w * o.z; acc.w += w * o.w;
  }
  const float inv = 1.0f / den;
  const int qi = (int)(row % p.nq);
  const int64_t bh = row / p.nq;
  const int h = (int)(bh % p.heads), b = (int)(bh / p.heads);
  if (p.lse && c4 == 0) p.lse[row] = m + __log2f(den);
  bf16_t* orow = reinterpret_cast<bf16_t*>(p.o) + ((int64_t)b * p.nq + qi) * p.os + (int64_t)h * p.d + 4 * c4;
  *reinterpret_cast<uint2*>(orow) = make_uint2(pack_bf16x2(acc.x * inv, acc.y * inv), pack_bf16x2(acc.z * inv, acc.w * inv));
}

int g_attn_d80 = 1;      // tuning / A-B hook: 0 routes head_dim 80 to the 16x16x32 kernel
int g_attn_d160 = 0;     // tuning / A-B hook: 1 routes head_dim 160 to the 32x32x16 kernel (measured slower:
                         // B = 8 step 9.290 -> 9.373 ms, B = 1 4.180 -> 4.216, profiles/ab_r06/d160_*.json)
int g_attn_pair = 1;      // tuning / A-B hook (ldm_attention_set_pair): head_dim 80's two-tile unrolled loop
                         // (31.4 -> 30.5 us; at head_dim 40 it needed 5 spilled VGPRs to keep two blocks
                         // per CU: 222.0 -> 220.7 us, the step unchanged — not instantiated)
int g_attn_kvsplit = -1;   // tuning / A-B hook (ldm_attention_set_kvsplit): -1 planner, 0 off, k >= 2 forced

// split count: head_dim 40 — enough (query block, split) 8-wave blocks for two per CU, >= 4 key
// tiles per split; head_dim 80 (one 8-wave block per CU) — 128 blocks, >= 2 key tiles per split
// (config 2's 32x32 level: 4 splits of 4 tiles measured 9 us per step faster than 8 of 2, the merge
// traffic halved: profiles/ab_r06/kvsplit_counts_b1.json); 1 = no split
int kv_splits(const AttnArgs& a, int batch) {
  if (g_attn_kvsplit == 0 || !(a.d == 40 || (a.d == 80 && g_attn_d80) || a.d == 160)) return 1;
  // d = 160: the 32x32x16 route (hook) counts 128-query blocks, the default 16x16x32 kernel 64-query
  // four-wave blocks (its 8-wave form when that gives >= 256 blocks: never split)
  const int qpb = a.d == 160 ? (g_attn_d160 ? 128 : 64) : 256;
  const int nblk = (a.nq + qpb - 1) / qpb * a.heads * batch;
  if (a.d == 160 && !g_attn_d160 && (a.nq + 127) / 128 * a.heads * batch >= 256) return 1;
  const int target = a.d == 40 ? 512 : (a.d == 80 ? 128 : 256);
  const int ntiles = (a.nkv + 63) / 64;
  int sp = g_attn_kvsplit > 0 ? g_attn_kvsplit : (nblk >= target ? 1 : (target + nblk - 1) / nblk);
  // the planner keeps >= 4 key tiles per split at d = 40 (a short sequence is launch-bound: the
  // merge kernel would cost more than the occupancy buys), >= 2 at d = 80 and on the d = 160
  // 32x32x16 route; the 16x16x32 d = 160 kernel and forced splits go down to 1 / 2 tiles
  const int mint = a.d == 160 && !g_attn_d160 ? 1 : (g_attn_kvsplit > 0 || a.d != 40 ? 2 : 4);
  sp = min(sp, min(8, ntiles / mint));
  return sp >= 2 ? sp : 1;
}

size_t kv_workspace(const AttnArgs& a, int batch) {
  const int sp = kv_splits(a, batch);
  if (sp < 2) return 0;
  const size_t rows = (size_t)batch * a.heads * a.nq;
  return (size_t)sp * rows * (a.d * 4 + 4) + 256;
}

// split-KV launch: the partials kernel then the merge; a (with kvsplit, opart, lsepart) set by the caller
int launch_kv_split(const AttnArgs& a, int batch, hipStream_t s) {
  const int nblk = (a.nq + 255) / 256 * a.heads * batch * a.kvsplit;
  const int64_t n = (int64_t)batch * a.heads * a.nq * (a.d / 4);
  if (a.d == 40) {
    hipLaunchKernelGGL((attn_d40_kernel<8, 2, 64, 40, 1, false, true>), dim3(nblk), dim3(512), 0, s, a);
    LDM_CHECK_LAUNCH();
    hipLaunchKernelGGL((attn_kv_combine<40>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  } else if (a.d == 160 && !g_attn_d160) {
    const int nb4 = (a.nq + 63) / 64 * a.heads * batch * a.kvsplit;
    hipLaunchKernelGGL((attn32_kernel<160, 1, false, 4, 2, false, false, true>), dim3(nb4), dim3(256), 0, s, a);
    LDM_CHECK_LAUNCH();
    hipLaunchKernelGGL((attn_kv_combine<160>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  } else if (a.d == 160) {
    const int nb4 = (a.nq + 127) / 128 * a.heads * batch * a.kvsplit;
    hipLaunchKernelGGL((attn_d40_kernel<4, 1, 64, 160, 1, false, true>), dim3(nb4), dim3(256), 0, s, a);
    LDM_CHECK_LAUNCH();
    hipLaunchKernelGGL((attn_kv_combine<160>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((attn_d40_kernel<8, 1, 64, 80, 1, false, true>), dim3(nblk), dim3(512), 0, s, a);
    LDM_CHECK_LAUNCH();
    hipLaunchKernelGGL((attn_kv_combine<80>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
  }
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

int g_attn_skew = 0;     // tuning / A-B hook (ldm_attention_set_skew): 0 planner, 1 off, 2 on
int g_attn_il = 1;       // A/B hook (ldm_attention_set_il): head_dim 40 two-subtile interleave (IL) where >= 256 blocks
int g_attn_qs2 = 0;      // tuning / A-B hook: head_dim 40 as 64 queries per wave: 1 two subtiles in step,
                         // 2 the pipelined form (attn_d40p_kernel)

template <int DP, bool F8 = false>
int launch32_dp(const AttnArgs& a, int batch, hipStream_t s) {
  if constexpr (DP == 160) {
    if (!F8 && g_attn_d160 && a.d == 160) {
      // the 32x32x16 form at head_dim 160 (the 16x16 / 8x8 levels): 4 waves x 32 queries, one block
      // per CU (376 registers per lane, 100 KB of K / V tiles)
      hipLaunchKernelGGL((attn_d40_kernel<4, 1, 64, 160>), dim3((a.nq + 127) / 128 * a.heads * batch), dim3(256), 0, s,
                         a);
      LDM_CHECK_LAUNCH();
      return LDM_OK;
    }
  }
  if constexpr (DP == 80) {
    if (!F8 && g_attn_d80 && a.d == 80) {
      // the 32x32x16 form at head_dim 80 (the 32x32 level): 8 waves x 32 queries per block
      const int nb8 = (a.nq + 255) / 256 * a.heads * batch;
      if (nb8 >= 256 && g_attn_skew == 2)
        hipLaunchKernelGGL((attn_d40_kernel<8, 1, 64, 80, 1, true>), dim3(nb8), dim3(512), 0, s, a);
      else if (nb8 >= 256 && g_attn_pair == 2)   // A/B: 128-key tiles
        hipLaunchKernelGGL((attn_d40_kernel<8, 1, 128, 80, 1>), dim3(nb8), dim3(512), 0, s, a);
      else if (nb8 >= 256 && g_attn_pair == 3)   // A/B: 128-key tiles, two-tile unrolled loop
        hipLaunchKernelGGL((attn_d40_kernel<8, 1, 128, 80, 1, false, false, true>), dim3(nb8), dim3(512), 0, s, a);
      else if (nb8 >= 256 && g_attn_pair)
        hipLaunchKernelGGL((attn_d40_kernel<8, 1, 64, 80, 1, false, false, true>), dim3(nb8), dim3(512), 0, s, a);
      else if (nb8 >= 256) hipLaunchKernelGGL((attn_d40_kernel<8, 1, 64, 80>), dim3(nb8), dim3(512), 0, s, a);
      else hipLaunchKernelGGL((attn_d40_kernel<4, 2, 64, 80>), dim3((a.nq + 127) / 128 * a.heads * batch),
                              dim3(256), 0, s, a);
      LDM_CHECK_LAUNCH();
      return LDM_OK;
    }
  }
  // the max column pays at head_dim 40 (N=4096: 273 -> 252 us); at 80 it costs occupancy
  // (134 vs 122 VGPRs: 39.7 -> 41.0 us), so it is kept to DP = 48
  if constexpr (DP == 48) {
    if (!F8 && g_attn_d40 && a.d == 40) {
      // 32x32x16 kernel: 8 waves x 32 queries, two blocks per CU when there are >= 512 blocks
      const int nblk = (a.nq + 255) / 256 * a.heads * batch;
      // (measured at N=4096: 8 waves x 2 blocks per CU 241 us; 4 waves x 4 blocks 302 us — each K/V
      // tile then serves half the queries; 128-key tiles 249 us)
      const int nb2 = (a.nq + 511) / 512 * a.heads * batch;
      if (g_attn_qs2 == 2 && g_attn_waves == 0) {
        // 8 waves x 32 queries, the tile loop software-pipelined inside each wave
        hipLaunchKernelGGL((attn_d40p_kernel<8>), dim3(nblk), dim3(512), 0, s, a);
      } else if (g_attn_qs2 == 1 && g_attn_waves == 0 && nb2 >= 256) {
        // 8 waves x 64 queries (two subtiles sharing every K / V fragment read), one block per CU
        hipLaunchKernelGGL((attn_d40_kernel<8, 1, 64, 40, 2>), dim3(nb2), dim3(512), 0, s, a);
      } else if (g_attn_il && g_attn_waves == 0 && g_attn_skew < 2 && nb2 >= 256) {
        // 8 waves x 64 queries, the two subtiles' MFMA and softmax phases interleaved in each wave
        // (opbench, graph-replayed, N = 4096 B = 8: 226.0 -> 212.6 us; config 5's N = 2048 B = 16:
        // 118.4 -> 113.9; with sched_group_barrier-pinned interleaves slower: 235 / 128)
        // 128-key tiles (two 64-key halves per barrier, bit-identical to 64-key tiles): opbench 212.3 ->
        // 207.7 us, same-box step 9.123 -> 9.113 ms (another box: 219.3 -> 214.7, 9.420 -> 9.376);
        // 256-key tiles in between (profiles/r08m/attention_key_tiles.txt).  A/B: 2 = 64, 3 = 256
        if (g_attn_il == 2)
          hipLaunchKernelGGL((attn_d40_kernel<8, 1, 64, 40, 2, false, false, false, true>), dim3(nb2), dim3(512), 0, s, a);
        else if (g_attn_il == 3)
          hipLaunchKernelGGL((attn_d40_kernel<8, 1, 256, 40, 2, false, false, false, true>), dim3(nb2), dim3(512), 0, s, a);
        else
          hipLaunchKernelGGL((attn_d40_kernel<8, 1, 128, 40, 2, false, false, false, true>), dim3(nb2), dim3(512), 0, s, a);
      } else if (g_attn_waves == 4) {
        const int nb4 = (a.nq + 127) / 128 * a.heads * batch;
        hipLaunchKernelGGL((attn_d40_kernel<4, 4>), dim3(nb4), dim3(256), 0, s, a);
      } else if ((nblk >= 512 || g_attn_waves == 8) && g_attn_skew == 2) {
        hipLaunchKernelGGL((attn_d40_kernel<8, 2, 64, 40, 1, true>), dim3(nblk), dim3(512), 0, s, a);
      } else if ((nblk >= 512 || g_attn_waves == 8) && g_attn_skew == 3) {
        // A/B reference for the skewed form: the default kernel held to one block per CU (dynamic LDS pad)
        hipLaunchKernelGGL((attn_d40_kernel<8, 2>), dim3(nblk), dim3(512), 96 * 1024, s, a);
      } else if (nblk >= 512 || g_attn_waves == 8) hipLaunchKernelGGL((attn_d40_kernel<8, 2>), dim3(nblk), dim3(512), 0, s, a);
      else {
        const int nb4 = (a.nq + 127) / 128 * a.heads * batch;
        // (2-wave blocks of 64 queries for a single frame were measured slower: B = 1, N = 4096
        // 0.74 -> 1.07 ms for the step's five launches — each K/V tile then serves 64 queries)
        hipLaunchKernelGGL((attn_d40_kernel<4, 2>), dim3(nb4), dim3(256), 0, s, a);
      }
      LDM_CHECK_LAUNCH();
      return LDM_OK;
    }
    if (g_attn_maxcol && a.d % 8 == 0) return launch32_dp_mc<DP, F8, true>(a, batch, s);
  }
  return launch32_dp_mc<DP, F8, false>(a, batch, s);
}

// ======================================================================================
// fp8 attention at head_dim 40 (BASELINE config 5's 32x64 level, N = 2048) on the block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands: twice the bf16 MFMA rate per clock, and a
// 64-deep K per instruction, so per 64-key tile and wave
//   S^T = K Q^T + (-m)  2 MFMAs (one per 32-key block; d = 40 padded to 64; the running max
//                       enters as the C input, a splat of -m per query column)
//   O^T += V^T P^T      2 MFMAs (one per 32-row head-dim block, all 64 keys at once)
// against 6 + 8 x 32x32x16 bf16 issues (attn_d40_kernel).  Every 32-element operand block carries
// its own E8M0 scale (the instruction's per-lane scale operands, free): K per (key, d 0..31 /
// 32..63), V^T per (d, keys 0..31 / 32..63), Q per (query, d half), chosen so the block's max lands
// in [224, 448] — no clipping of large activations and no subnormal collapse of small ones
// (f8_block_exp).  A scale block is bytes 16b .. 16b + 15 of both lane halves, its scale in lane
// half b (tools/mfma_f8_scale_probe.hip), so K and Q give lane half hh d 16hh.. and 32 + 16hh..
// P keeps the unit scale (P' <= 2^8 under the lazy rescale).
// K and V are quantized once per call by attn_f8_prep into 4-KB LDS images per 64-key tile (K8:
// [key][64 B]; V8T: [d][64 keys in the P.V k order] with row 40 = 1.0, the softmax denominator)
// plus 256 scale bytes, 16-byte chunks XOR-swizzled so every ds_read_b128 is conflict-free; the
// attention kernel DMAs the images as they are (8 KB per tile, half the bf16 bytes).  Q is
// quantized in registers (prescaled by scale * log2(e)).
// ======================================================================================
constexpr int F8_IMG = 64 * 64;              // bytes per K8 / V8T tile image
constexpr float kF8Shift = 6.f;              // log2 of the P scale-up (see attn_f8_kernel)
constexpr float kF8Top = 8.f;                // rescale threshold on s c - m: P' <= 2^8

__device__ __forceinline__ int f8_swz(int row, int c) { return c ^ ((row >> 2) & 3); }
// P.V k order (the S^T accumulator registers as the B operand): byte j of lane half kb is key
// 32 (j >> 4) + 8 ((j >> 2) & 3) + 4 kb + (j & 3) of the tile
__device__ __forceinline__ int f8_pv_key(int kb, int j) { return 32 * (j >> 4) + 8 * ((j >> 2) & 3) + 4 * kb + (j & 3); }
__device__ __forceinline__ float bf16_bits_f(unsigned short u) { return __uint_as_float((unsigned)u << 16); }

// E8M0 exponent e (scale 2^e) for a 32-element block with max |x| = amax: the smallest e with
// amax 2^-e <= 448 (e4m3's max), so the block's largest value lands in [224, 448] and the rest keep
// e4m3's relative precision down to 2^-6 of it before going subnormal; clamped to [lo, hi]
__device__ __forceinline__ int f8_block_exp(float amax, int lo, int hi) {
  int e = 0;
  if (amax > 0.f) {
    int ex;
    const float m = frexpf(amax * (1.f / 448.f), &ex);
    e = m > 0.5f ? ex : ex - 1;
  }
  return min(max(e, lo), hi);
}

// grid (ceil(nkv / 64), heads, batch), 256 threads: one K8 and one V8T image per 64-key tile and
// the tile's 256 E8M0 scale bytes (sc: [lane][4]; byte i of lane (hh, r32) = scale block hh of
// K row 32 i + r32 for i < 2, of V^T row 32 (i - 2) + r32 for i >= 2)
__global__ __launch_bounds__(256) void attn_f8_prep(const AttnArgs p, uint8_t* __restrict__ k8,
                                                    uint8_t* __restrict__ v8t, uint8_t* __restrict__ sc) {
  __shared__ unsigned short vs[64][66];
  const int t = blockIdx.x, h = blockIdx.y, b = blockIdx.z, ntile = gridDim.x, tid = threadIdx.x;
  const int hd = p.d;
  const unsigned short* kp = reinterpret_cast<const unsigned short*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * hd;
  const unsigned short* vp = reinterpret_cast<const unsigned short*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * hd;
  const int64_t tile = ((int64_t)b * p.heads + h) * ntile + t;
  const int64_t img = tile * F8_IMG;
  uint8_t* const scale = sc + tile * 256;
  // V tile -> LDS (bf16 bits, zero past nkv / hd)
  for (int i = tid; i < 64 * 8; i += 256) {
    const int key = i >> 3, c = i & 7, k = t * 64 + key;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (k < p.nkv && 8 * c < hd) v = *reinterpret_cast<const uint4*>(vp + (int64_t)k * p.vs + 8 * c);
    const unsigned short* e = reinterpret_cast<const unsigned short*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) vs[key][8 * c + j] = e[j];
  }
  // K8: row r, chunk c = d 16c .. 16c + 15; the kernel gives lane half hh chunks hh and 2 + hh, so
  // the instruction's scale block b (bytes 16b .. of both halves) is d 32b .. 32b + 31 = chunks 2b,
  // 2b + 1 (threads c, c ^ 1), its scale in lane half b
  {
    const int r = tid >> 2, c = tid & 3, k = t * 64 + r;
    float f[16];
    float amax = 0.f;
#pragma unroll
    for (int hv = 0; hv < 2; ++hv) {
      const int d0 = 16 * c + 8 * hv;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (k < p.nkv && d0 < hd) v = *reinterpret_cast<const uint4*>(kp + (int64_t)k * p.ks + d0);
      const unsigned short* e = reinterpret_cast<const unsigned short*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[8 * hv + j] = bf16_bits_f(e[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) amax = fmaxf(amax, fabsf(f[j]));
    amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
    const int e = f8_block_exp(amax, -100, 100);
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = sat448(ldexpf(f[j], -e));
    const uint4 w = make_uint4(pack_fp8x4(f[0], f[1], f[2], f[3]), pack_fp8x4(f[4], f[5], f[6], f[7]),
                               pack_fp8x4(f[8], f[9], f[10], f[11]), pack_fp8x4(f[12], f[13], f[14], f[15]));
    *reinterpret_cast<uint4*>(k8 + img + r * 64 + f8_swz(r, c) * 16) = w;
    if ((c & 1) == 0) scale[((c >> 1) * 32 + (r & 31)) * 4 + (r >> 5)] = (uint8_t)(e + 127);
  }
  __syncthreads();
  // V8T: row dr (head-dim index), chunk c = k-order positions 16c .. 16c + 15 (lane half kb = c >> 1,
  // bytes 16 (c & 1) ..).  The instruction's scale block b is bytes 16b .. 16b + 15 of BOTH lane
  // halves (tools/mfma_f8_scale_probe.hip) = keys 32b .. 32b + 31: threads c, c ^ 2 form a block,
  // its scale in lane half b = c & 1
  {
    const int dr = tid >> 2, c = tid & 3, kb = c >> 1;
    float f[16];
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int key = f8_pv_key(kb, 16 * (c & 1) + j);
      float x = 0.f;
      if (dr < hd) x = bf16_bits_f(vs[key][dr]);
      else if (dr == hd) x = 1.f;
      f[j] = x;
      amax = fmaxf(amax, fabsf(x));
    }
    amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
    const int e = f8_block_exp(amax, -100, 100);   // the ones row: e = -8, 2^8 exact
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = sat448(ldexpf(f[j], -e));
    const uint4 w = make_uint4(pack_fp8x4(f[0], f[1], f[2], f[3]), pack_fp8x4(f[4], f[5], f[6], f[7]),
                               pack_fp8x4(f[8], f[9], f[10], f[11]), pack_fp8x4(f[12], f[13], f[14], f[15]));
    *reinterpret_cast<uint4*>(v8t + img + dr * 64 + f8_swz(dr, c) * 16) = w;
    if (kb == 0) scale[((c & 1) * 32 + (dr & 31)) * 4 + 2 + (dr >> 5)] = (uint8_t)(e + 127);
  }
}

typedef __attribute__((ext_vector_type(8))) int i32x8_t;

// E8M0 scales: byte OA of sa for the lane's A row block, byte OB of sb for its B column block (the
// instruction's op_sel).  The scale words stay live across the whole tile (the tile's four scale
// bytes in one dword): a scale extracted into its own register dies at the MFMA, and hipcc then
// lets the 16-pass instruction's destination overlap it — every output NaN (measured)
template <int OA, int OB>
__device__ __forceinline__ f32x16_t mma_f8(const i32x8_t a, const i32x8_t b, f32x16_t c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, OA, sa, OB, sb);
}

// a lane's 32 bytes (chunks 2 hh, 2 hh + 1) of row `row` of a swizzled 64-byte-row image
__device__ __forceinline__ i32x8_t f8_row32(const uint8_t* img, int row, int hh) {
  const uint4 lo = *reinterpret_cast<const uint4*>(img + row * 64 + f8_swz(row, 2 * hh) * 16);
  const uint4 hi = *reinterpret_cast<const uint4*>(img + row * 64 + f8_swz(row, 2 * hh + 1) * 16);
  i32x8_t v;
  v[0] = (int)lo.x; v[1] = (int)lo.y; v[2] = (int)lo.z; v[3] = (int)lo.w;
  v[4] = (int)hi.x; v[5] = (int)hi.y; v[6] = (int)hi.z; v[7] = (int)hi.w;
  return v;
}

// the K operand: chunks hh and 2 + hh of row `row` (d 16 hh .. +16 and 32 + 16 hh .. +16), so scale
// block b (bytes 16b .. 16b + 15 of both lane halves) is d 32b .. 32b + 31
__device__ __forceinline__ i32x8_t f8_row32k(const uint8_t* img, int row, int hh) {
  const uint4 lo = *reinterpret_cast<const uint4*>(img + row * 64 + f8_swz(row, hh) * 16);
  const uint4 hi = *reinterpret_cast<const uint4*>(img + row * 64 + f8_swz(row, 2 + hh) * 16);
  i32x8_t v;
  v[0] = (int)lo.x; v[1] = (int)lo.y; v[2] = (int)lo.z; v[3] = (int)lo.w;
  v[4] = (int)hi.x; v[5] = (int)hi.y; v[6] = (int)hi.z; v[7] = (int)hi.w;
  return v;
}

__device__ __forceinline__ float fp8_to_f(int byte) { return __builtin_amdgcn_cvt_f32_fp8(byte, 0); }

template <int NW, int OCC, int QS = 1>
__global__ __launch_bounds__(64 * NW, OCC) void attn_f8_kernel(const AttnArgs p, const uint8_t* __restrict__ k8,
                                                              const uint8_t* __restrict__ v8t,
                                                              const unsigned* __restrict__ sc, int e8_one) {
  constexpr int HD = 40;                       // head_dim (the max / ones column)
  __shared__ uint4 smem[2 * 2 * F8_IMG / 16];  // [buf][K8 | V8T]
  const uint8_t* const lds = reinterpret_cast<const uint8_t*>(smem);
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  int qb, h, b;
  {
    const int nqb = (p.nq + 32 * QS * NW - 1) / (32 * QS * NW);
    const int bid = blockIdx.x, nblk = gridDim.x;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    const int t = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
    qb = t % nqb;
    const int hb = t / nqb;
    h = hb % p.heads;
    b = hb / p.heads;
  }
  const int qbase = qb * (32 * QS * NW) + wave * (32 * QS);   // subtile s: queries qbase + 32 s + r32
  const int ntiles = (p.nkv + 63) / 64;
  const uint8_t* kimg = k8 + (((int64_t)b * p.heads + h) * ntiles) * F8_IMG;
  const uint8_t* vimg = v8t + (((int64_t)b * p.heads + h) * ntiles) * F8_IMG;
  const unsigned* scl = sc + (((int64_t)b * p.heads + h) * ntiles) * 64 + lane;   // [tile][lane] dwords

  auto issue_tile = [&](int t, int buf) {     // 8 x 1 KB: K8 then V8T
    for (int i = wave; i < 8; i += NW) {
      const uint8_t* src = (i < 4 ? kimg + (int64_t)t * F8_IMG + i * 1024 : vimg + (int64_t)t * F8_IMG + (i - 4) * 1024) +
                           lane * 16;
      glds16(src, __builtin_amdgcn_readfirstlane(lds0 + buf * 2 * F8_IMG + i * 1024));
    }
  };

  // Q (B operand, the K operand's layout): lane half hh holds Q[q = qbase + 32 s + r32] * scale *
  // log2(e) at d 16 hh + j (bytes j < 16, scale block 0 = d 0 .. 31) and d 32 + 16 hh + j - 16
  // (bytes 16 .. 31, block 1 = d 32 .. 63), each block / 2^e_b as e4m3; lane half b carries e_b + 127
  // in qsc
  const float c2 = p.scale_log2;
  i32x8_t qf[QS];
  int qsc[QS];
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    const int qi = qbase + 32 * s + r32;
    const bf16_t* qrow = reinterpret_cast<const bf16_t*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * HD +
                         (int64_t)qi * p.qs;
    float f[32];
#pragma unroll
    for (int c = 0; c < 4; ++c) {             // 8 d-values per 16-byte chunk
      const int d0 = (c < 2 ? 16 * hh : 32 + 16 * hh) + 8 * (c & 1);
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (qi < p.nq && d0 < HD) v = *reinterpret_cast<const uint4*>(qrow + d0);
      const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f[8 * c + 2 * j] = __uint_as_float(u[j] << 16) * c2;
        f[8 * c + 2 * j + 1] = __uint_as_float(u[j] & 0xffff0000u) * c2;
      }
    }
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      a0 = fmaxf(a0, fabsf(f[j]));
      a1 = fmaxf(a1, fabsf(f[16 + j]));
    }
    a0 = fmaxf(a0, __shfl_xor(a0, 32, 64));
    a1 = fmaxf(a1, __shfl_xor(a1, 32, 64));
    const int e0 = f8_block_exp(a0, -100, 100), e1 = f8_block_exp(a1, -100, 100);
    qsc[s] = (hh ? e1 : e0) + 127;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int e = c < 4 ? e0 : e1;
      qf[s][c] = (int)pack_fp8x4(sat448(ldexpf(f[4 * c], -e)), sat448(ldexpf(f[4 * c + 1], -e)),
                                 sat448(ldexpf(f[4 * c + 2], -e)), sat448(ldexpf(f[4 * c + 3], -e)));
    }
  }
  f32x16_t oacc[QS][2];
#pragma unroll
  for (int s = 0; s < QS; ++s)
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[s][db][r] = 0.f;
  // the running max enters S^T through the MFMA's C input: negm[s] = -m in every register (a
  // 32x32 result column is one query), so the accumulators come out as s c - m at no VALU cost and
  // the operands carry no max column (their scale blocks see only Q and K)
  float mq[QS];
  f32x16_t negm[QS];
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    mq[s] = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) negm[s][r] = 0.f;
  }

  auto tile_max = [&](const f32x16_t (&sa)[2]) {
    float t[11];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const int a = 3 * k;
      t[k] = vmax3(a < 16 ? sa[0][a] : sa[1][a - 16], a + 1 < 16 ? sa[0][a + 1] : sa[1][a + 1 - 16],
                   a + 2 < 16 ? sa[0][a + 2] : sa[1][a + 2 - 16]);
    }
    t[10] = __builtin_elementwise_maximum(sa[1][14], sa[1][15]);
    const float u0 = vmax3(t[0], t[1], t[2]), u1 = vmax3(t[3], t[4], t[5]), u2 = vmax3(t[6], t[7], t[8]);
    const float mx = vmax3(vmax3(u0, u1, u2), t[9], t[10]);
    unsigned w = __float_as_uint(mx);
    const auto sw = __builtin_amdgcn_permlane32_swap(w, w, false, false);
    return vmax3(__uint_as_float(sw[0]), __uint_as_float(sw[1]), mx);
  };

#ifdef LDM_F8_DEBUG
  float dbg[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  dbg[0] = (float)qsc[0];
#endif
  auto compute = [&](int buf, int kv0, bool masked, bool first, unsigned scw) {
    const uint8_t* Ks = lds + buf * 2 * F8_IMG;
    const uint8_t* Vs = Ks + F8_IMG;
    f32x16_t sacc[QS][2];
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      const i32x8_t ka = f8_row32k(Ks, 32 * blk + r32, hh);   // one K read for every subtile
#pragma unroll
      for (int s = 0; s < QS; ++s)
        sacc[s][blk] = blk == 0 ? mma_f8<0, 0>(ka, qf[s], negm[s], (int)scw, qsc[s])
                                : mma_f8<1, 0>(ka, qf[s], negm[s], (int)scw, qsc[s]);
    }
    if (masked) {
#pragma unroll
      for (int s = 0; s < QS; ++s)
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kv0 + 32 * blk + 8 * (r >> 2) + 4 * hh + (r & 3) >= p.nkv) sacc[s][blk][r] = -INFINITY;
    }
    float mx[QS];
    bool resc = first;
#pragma unroll
    for (int s = 0; s < QS; ++s) {
      mx[s] = tile_max(sacc[s]);
      resc = resc || mx[s] > kF8Top;
    }
#ifdef LDM_F8_DEBUG
    if (first) { dbg[2] = sacc[0][0][0]; dbg[3] = mx[0]; dbg[7] = (float)scw; }
#endif
    // accumulators are s c - m, m held ~6 below the running max: P' = 2^acc = 2^6 P lands the bulk of a flat softmax's probabilities (2^-9 .. 1)
    // in e4m3's normal range (2^-3 .. 2^6) instead of its 2^-9-step subnormals (rel-L2 at N=2048:
    // 9.2e-2 unshifted); the shift cancels in O / l (the ones row sums the same P').  Rescale when
    // a score would pass 2^8 (P' <= 256 < 448, e4m3's max); one wave-uniform branch for all
    // subtiles (a subtile rescaled without need only moves m up toward its max)
    if (first || __any(resc)) {
#pragma unroll
      for (int s = 0; s < QS; ++s) {
        const float want = mq[s] + mx[s] - kF8Shift;
        const float mn = first ? want : fmaxf(mq[s], want);
        const float delta = mn - mq[s];
        const float alpha = first ? 0.f : __builtin_amdgcn_exp2f(-delta);
        mq[s] = mn;
        oacc[s][0] *= alpha;
        oacc[s][1] *= alpha;
        sacc[s][0] -= delta;
        sacc[s][1] -= delta;
#pragma unroll
        for (int r = 0; r < 16; ++r) negm[s][r] = -mn;
      }
    }
    // P^T -> e4m3 B operand: byte j = 16 blk + r
    i32x8_t pb[QS];
#pragma unroll
    for (int s = 0; s < QS; ++s)
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        const int blk = w >> 2, r0 = 4 * (w & 3);
        pb[s][w] = (int)pack_fp8x4(__builtin_amdgcn_exp2f(sacc[s][blk][r0]), __builtin_amdgcn_exp2f(sacc[s][blk][r0 + 1]),
                                   __builtin_amdgcn_exp2f(sacc[s][blk][r0 + 2]), __builtin_amdgcn_exp2f(sacc[s][blk][r0 + 3]));
      }
#ifdef LDM_F8_DEBUG
    if (first) { dbg[4] = mq[0]; dbg[5] = __uint_as_float((unsigned)pb[0][0]); }
#endif
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const i32x8_t va = f8_row32(Vs, 32 * db + r32, hh);     // one V read for every subtile
#pragma unroll
      for (int s = 0; s < QS; ++s)
        oacc[s][db] = db == 0 ? mma_f8<2, 0>(va, pb[s], oacc[s][db], (int)scw, e8_one)
                              : mma_f8<3, 0>(va, pb[s], oacc[s][db], (int)scw, e8_one);
    }
  };

  const int nfull = p.nkv / 64;
  unsigned scn = scl[0];
  issue_tile(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // full tiles in the loop (no key mask: a runtime `masked` flag had the compiler if-convert the
  // mask into every tile, 96 VALU per tile and wave), the ragged last tile after it
  for (int t = 0; t < nfull; ++t) {
    const unsigned scw = scn;
    if (t + 1 < ntiles) {
      scn = scl[(int64_t)(t + 1) * 64];
      issue_tile(t + 1, (t + 1) & 1);
    }
    compute(t & 1, t * 64, false, t == 0, scw);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (nfull < ntiles) compute(nfull & 1, nfull * 64, true, nfull == 0, scn);

  // denominator: O^T row d = 40 = block 1 register 4 of the hh = 0 lane of this column
#ifdef LDM_F8_DEBUG
  dbg[6] = oacc[0][1][4];
  if (p.lse && blockIdx.x == 0)
    for (int i = 0; i < 8; ++i) p.lse[tid * 8 + i] = dbg[i];
#endif
#pragma unroll
  for (int s = 0; s < QS; ++s) {
    const float lt = __shfl(oacc[s][1][4], r32, 64);
    const float inv = 1.0f / lt;
    const int qi = qbase + 32 * s + r32;
    if (qi < p.nq) {
      bf16_t* orow = reinterpret_cast<bf16_t*>(p.o) + (int64_t)b * p.nq * p.os + (int64_t)h * HD + (int64_t)qi * p.os;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 8 * g4 + 4 * hh;
        *reinterpret_cast<uint2*>(orow + d) =
            make_uint2(pack_bf16x2(oacc[s][0][4 * g4] * inv, oacc[s][0][4 * g4 + 1] * inv),
                       pack_bf16x2(oacc[s][0][4 * g4 + 2] * inv, oacc[s][0][4 * g4 + 3] * inv));
      }
      *reinterpret_cast<uint2*>(orow + 32 + 4 * hh) =
          make_uint2(pack_bf16x2(oacc[s][1][0] * inv, oacc[s][1][1] * inv), pack_bf16x2(oacc[s][1][2] * inv, oacc[s][1][3] * inv));
    }
  }
}

// workspace: K8 images | V8T images | scale bytes (256 per tile)
size_t f8_workspace(const AttnArgs& a, int batch) {
  return (size_t)batch * a.heads * ((a.nkv + 63) / 64) * (2 * F8_IMG + 256);
}

#ifdef LDM_F8_DEBUG
float* g_f8_dbg = nullptr;
#endif
int launch_f8_d40(const AttnArgs& a0, int batch, void* ws, hipStream_t s) {
  AttnArgs a = a0;
#ifdef LDM_F8_DEBUG
  a.lse = g_f8_dbg;
#endif
  const int ntile = (a.nkv + 63) / 64;
  uint8_t* k8 = static_cast<uint8_t*>(ws);
  const size_t tiles = (size_t)batch * a.heads * ntile;
  uint8_t* v8t = k8 + tiles * F8_IMG;
  uint8_t* sc = v8t + tiles * F8_IMG;
  hipLaunchKernelGGL(attn_f8_prep, dim3(ntile, a.heads, batch), dim3(256), 0, s, a, k8, v8t, sc);
  LDM_CHECK_LAUNCH();
  const unsigned* scu = reinterpret_cast<const unsigned*>(sc);
  const int e8_one = 127 + (a.heads < 0);     // E8M0 2^0 for P (kept a run-time register value)
  const int nblk = (a.nq + 255) / 256 * a.heads * batch;
  const int nb2 = (a.nq + 511) / 512 * a.heads * batch;
  if (g_attn_qs2 == 1 && nb2 >= 256)   // 64 queries per wave (two subtiles), one 8-wave block per CU
    hipLaunchKernelGGL((attn_f8_kernel<8, 1, 2>), dim3(nb2), dim3(512), 0, s, a, k8, v8t, scu, e8_one);
  else if (nblk >= 512) hipLaunchKernelGGL((attn_f8_kernel<8, 2>), dim3(nblk), dim3(512), 0, s, a, k8, v8t, scu, e8_one);
  else {
    const int nb4 = (a.nq + 127) / 128 * a.heads * batch;
    hipLaunchKernelGGL((attn_f8_kernel<4, 2>), dim3(nb4), dim3(256), 0, s, a, k8, v8t, scu, e8_one);
  }
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

// fp8 P.V forward (bf16 inputs with 16-byte rows only)
int launch_fp8(const AttnArgs& a, int batch, hipStream_t s) {
  const int dp = (a.d + 15) / 16 * 16;
  if (a.qs % 8 || a.os % 4) return LDM_ERR_ALIGN;
  switch (dp) {
    case 48: return launch32_dp<48, true>(a, batch, s);
    case 64: return launch32_dp<64, true>(a, batch, s);
    case 80: return launch32_dp<80, true>(a, batch, s);
    case 96: return launch32_dp<96, true>(a, batch, s);
    case 128: return launch32_dp<128, true>(a, batch, s);
    case 160: return launch32_dp<160, true>(a, batch, s);
    default: return LDM_ERR_ARG;
  }
}

int g_attn_legacy = 0;   // tuning / A-B hook: 1 forces the 16x16x16 kernel

// bf16 with 16-byte Q rows: the x32 kernel; otherwise the generic one
int launch_bf16(const AttnArgs& a, int batch, hipStream_t s) {
  const int dp = (a.d + 15) / 16 * 16;
  if (!g_attn_legacy && a.qs % 8 == 0 && a.os % 4 == 0) {
    switch (dp) {
      case 48: return launch32_dp<48>(a, batch, s);
      case 64: return launch32_dp<64>(a, batch, s);
      case 80: return launch32_dp<80>(a, batch, s);
      case 96: return launch32_dp<96>(a, batch, s);
      case 128: return launch32_dp<128>(a, batch, s);
      case 160: return launch32_dp<160>(a, batch, s);
      default: break;
    }
  }
  return launch_t<bf16_t>(a, batch, s);
}

// ======================================================================================
// Backward (flash-attention-2 style, P recomputed from the saved log2-domain LSE):
//   D[q]   = sum_d dO[q][d] O[q][d]
//   P      = 2^(S c2 - lse2[q]),  dP = dO V^T,  dZ = P (dP - D[q])     (Z = scale Q K^T)
//   dV = P^T dO,  dK = scale dZ^T Q   (attn_bwd_kv: one block per 64 keys, loop over queries)
//   dQ = scale dZ K                   (attn_bwd_q : one block per 64 queries, loop over keys)
// Both loops stage the streamed operand pair (Q, dO) / (K, V) by LDS-DMA exactly like the
// forward's K/V tiles (double buffered, zero-filled past n and head_dim); the per-wave fixed
// operands live in registers.  Transposed fragments (dO^T, Q^T, K^T) come from the row-major
// LDS tiles via ds_read_b64_tr_b16 (bf16) or scalar reads (fp32).
// ======================================================================================
struct AttnBwdArgs {
  const char* q; const char* k; const char* v; const char* o; const char* dout;
  char* dq; char* dk; char* dv;
  int qs, ks, vs, os, dos, dqs, dkvs;
  int heads, d, nq, nkv;
  float scale, scale_log2;
  const float* lse;
  float* dvec;        // D [batch][heads][nq]
};

template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_dot(const AttnBwdArgs p, int batch) {
  // one 16-lane group per (b, h, q) row: D = sum_d dO * O
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
  const int l = threadIdx.x & 15;
  const int total = batch * p.heads * p.nq;
  float s = 0.f;
  int b = 0, h = 0, qi = 0;
  if (row < total) {
    qi = row % p.nq;
    const int bh = row / p.nq;
    h = bh % p.heads;
    b = bh / p.heads;
    const T* o = reinterpret_cast<const T*>(p.o) + ((int64_t)b * p.nq + qi) * p.os + (int64_t)h * p.d;
    const T* g = reinterpret_cast<const T*>(p.dout) + ((int64_t)b * p.nq + qi) * p.dos + (int64_t)h * p.d;
    for (int dd = l; dd < p.d; dd += 16) s += to_f(o[dd]) * to_f(g[dd]);
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) s += __shfl_xor(s, off, 16);
  if (row < total && l == 0) p.dvec[row] = s;
}

// A-operand fragment of a TRANSPOSED row-major LDS tile: lane (g, lr) gets tile[r0 + 4g + j][c0 + lr]
template <typename T, int ROW>
__device__ __forceinline__ Frag4<T> tr_frag(const T* tile, int r0, int c0, int g, int lr) {
  Frag4<T> f;
  if constexpr (sizeof(T) == 2) {
    typedef __attribute__((ext_vector_type(4))) short s4_t;
    typedef __attribute__((address_space(3))) s4_t lds_s4_t;
    const T* addr = tile + (r0 + 4 * g + (lr >> 2)) * ROW + c0 + 4 * (lr & 3);
    const s4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(addr));
    f.v = __builtin_bit_cast(uint2, x);
  } else {
    float* e = reinterpret_cast<float*>(&f.v);
#pragma unroll
    for (int j = 0; j < 4; ++j) e[j] = to_f(tile[(r0 + 4 * g + j) * ROW + c0 + lr]);
  }
  return f;
}

template <typename T>
__device__ __forceinline__ Frag4<T> pack4(const f32x4_t& v) {
  Frag4<T> f;
  if constexpr (sizeof(T) == 2) {
    bf16_t hb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) hb[r] = f2bf(v[r]);
    f.v = *reinterpret_cast<const uint2*>(hb);
  } else {
    float pv[4] = {v[0], v[1], v[2], v[3]};
    f.v = *reinterpret_cast<const uint4*>(pv);
  }
  return f;
}

// stage rows [r0, r0 + 64) of two [n][stride] operands (head h) into LDS tiles [64][ROW]
template <typename T, int DP>
__device__ __forceinline__ void stage_pair(const T* ap, int as, const T* bp, int bs, int n, int dh, int r0,
                                           unsigned abase, unsigned bbase, int wave, int lane) {
  constexpr int EPC = 16 / sizeof(T), CPR = DP / EPC, RCH = CPR + 1;
  for (int i = wave; i < RCH; i += 4) {
    const int L = i * 64 + lane;
    const int row = L / RCH, c = L - row * RCH;
    const int r = r0 + row, dd = c * EPC;
    const bool ok = r < n && c < CPR && dd < dh;
    const void* sa = ok ? (const void*)(ap + (int64_t)r * as + dd) : (const void*)&kZeros16;
    const void* sb = ok ? (const void*)(bp + (int64_t)r * bs + dd) : (const void*)&kZeros16;
    const unsigned off = __builtin_amdgcn_readfirstlane(i * 64 * 16);
    glds16(sa, abase + off);
    glds16(sb, bbase + off);
  }
}

template <typename T, int DP>
__global__ __launch_bounds__(256, (sizeof(T) == 2 && DP <= 80) ? 2 : 1) void attn_bwd_kv(const AttnBwdArgs p) {
  constexpr int ES = sizeof(T), EPC = 16 / ES, ND = DP / 16;
  constexpr int CPR = DP / EPC, RCH = CPR + 1, ROW = RCH * EPC, TILE = KVT * ROW;
  constexpr int NBUF = (2 * 2 * TILE * ES <= 96 * 1024) ? 2 : 1;   // fp32 at large d: single buffer
  __shared__ uint4 smem[NBUF * 2 * TILE * ES / 16];
  T* const lds = reinterpret_cast<T*>(smem);
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const int kv = blockIdx.x * 64 + wave * 16 + lr;       // this lane's key (B-operand column)
  const T* qp = reinterpret_cast<const T*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * p.d;
  const T* dop = reinterpret_cast<const T*>(p.dout) + (int64_t)b * p.nq * p.dos + (int64_t)h * p.d;
  const T* kp = reinterpret_cast<const T*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * p.d;
  const T* vp = reinterpret_cast<const T*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * p.d;
  const float* lse = p.lse + ((int64_t)b * p.heads + h) * p.nq;
  const float* dv = p.dvec + ((int64_t)b * p.heads + h) * p.nq;

  Frag4<T> kf[ND], vf[ND];                 // B operands: K^T / V^T columns = this lane's key
#pragma unroll
  for (int ds = 0; ds < ND; ++ds) {
    const int dd = 16 * ds + 4 * g;
    if (kv < p.nkv && dd < p.d) {
      kf[ds] = *reinterpret_cast<const Frag4<T>*>(kp + (int64_t)kv * p.ks + dd);
      vf[ds] = *reinterpret_cast<const Frag4<T>*>(vp + (int64_t)kv * p.vs + dd);
    } else {
      kf[ds] = Frag4<T>{};
      vf[ds] = Frag4<T>{};
    }
  }
  f32x4_t dkt[ND], dvt[ND];                // [d = 16 dd + 4g + r][key = lr]
#pragma unroll
  for (int i = 0; i < ND; ++i) { dkt[i] = f32x4_t{0.f, 0.f, 0.f, 0.f}; dvt[i] = f32x4_t{0.f, 0.f, 0.f, 0.f}; }
  const float c2 = p.scale_log2;

  auto compute = [&](int buf, int q0) {
    const T* Qs = lds + buf * 2 * TILE;
    const T* Ds = Qs + TILE;
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      // S[q][key] and dP[q][key]: rows q = qs*16 + 4g + r
      f32x4_t s = f32x4_t{0.f, 0.f, 0.f, 0.f}, dp = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < ND; ++ds) {
        const Frag4<T> qa = *reinterpret_cast<const Frag4<T>*>(Qs + (16 * qs + lr) * ROW + 16 * ds + 4 * g);
        const Frag4<T> da = *reinterpret_cast<const Frag4<T>*>(Ds + (16 * qs + lr) * ROW + 16 * ds + 4 * g);
        mma_k16(s, qa, kf[ds]);
        mma_k16(dp, da, vf[ds]);
      }
      f32x4_t pm, dz;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qi = q0 + 16 * qs + 4 * g + r;
        const bool ok = qi < p.nq && kv < p.nkv;
        const float pr = ok ? __builtin_amdgcn_exp2f(fmaf(s[r], c2, -lse[qi])) : 0.f;
        pm[r] = pr;
        dz[r] = ok ? pr * (dp[r] - dv[qi]) : 0.f;
      }
      const Frag4<T> pf = pack4<T>(pm), zf = pack4<T>(dz);
#pragma unroll
      for (int dd = 0; dd < ND; ++dd) {
        mma_k16(dvt[dd], tr_frag<T, ROW>(Ds, 16 * qs, 16 * dd, g, lr), pf);   // dV^T += dO^T P
        mma_k16(dkt[dd], tr_frag<T, ROW>(Qs, 16 * qs, 16 * dd, g, lr), zf);   // dK^T += Q^T dZ
      }
    }
  };

  const int ntiles = (p.nq + KVT - 1) / KVT;
  stage_pair<T, DP>(qp, p.qs, dop, p.dos, p.nq, p.d, 0, lds0, lds0 + TILE * ES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = NBUF == 2 ? (t & 1) : 0;
    if (NBUF == 2 && t + 1 < ntiles) {
      const unsigned nb = lds0 + (unsigned)((buf ^ 1) * 2 * TILE * ES);
      stage_pair<T, DP>(qp, p.qs, dop, p.dos, p.nq, p.d, (t + 1) * KVT, nb, nb + TILE * ES, wave, lane);
    }
    compute(buf, t * KVT);
    if (NBUF == 1 && t + 1 < ntiles) {
      __syncthreads();
      stage_pair<T, DP>(qp, p.qs, dop, p.dos, p.nq, p.d, (t + 1) * KVT, lds0, lds0 + TILE * ES, wave, lane);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (kv >= p.nkv) return;
  T* dkp = reinterpret_cast<T*>(p.dk) + ((int64_t)b * p.nkv + kv) * p.dkvs + (int64_t)h * p.d;
  T* dvp = reinterpret_cast<T*>(p.dv) + ((int64_t)b * p.nkv + kv) * p.dkvs + (int64_t)h * p.d;
#pragma unroll
  for (int dd = 0; dd < ND; ++dd) {
    const int d0 = 16 * dd + 4 * g;
    if (d0 >= p.d) continue;
    float kk[4], vv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { kk[r] = dkt[dd][r] * p.scale; vv[r] = dvt[dd][r]; }
    if constexpr (ES == 2) {
      bf16_t hk[4], hv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { hk[r] = f2bf(kk[r]); hv[r] = f2bf(vv[r]); }
      *reinterpret_cast<uint2*>(dkp + d0) = *reinterpret_cast<const uint2*>(hk);
      *reinterpret_cast<uint2*>(dvp + d0) = *reinterpret_cast<const uint2*>(hv);
    } else {
      *reinterpret_cast<float4*>(dkp + d0) = make_float4(kk[0], kk[1], kk[2], kk[3]);
      *reinterpret_cast<float4*>(dvp + d0) = make_float4(vv[0], vv[1], vv[2], vv[3]);
    }
  }
}

template <typename T, int DP>
__global__ __launch_bounds__(256, (sizeof(T) == 2 && DP <= 80) ? 2 : 1) void attn_bwd_q(const AttnBwdArgs p) {
  constexpr int ES = sizeof(T), EPC = 16 / ES, ND = DP / 16;
  constexpr int CPR = DP / EPC, RCH = CPR + 1, ROW = RCH * EPC, TILE = KVT * ROW;
  constexpr int NBUF = (2 * 2 * TILE * ES <= 96 * 1024) ? 2 : 1;   // fp32 at large d: single buffer
  __shared__ uint4 smem[NBUF * 2 * TILE * ES / 16];
  T* const lds = reinterpret_cast<T*>(smem);
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const int qi = blockIdx.x * 64 + wave * 16 + lr;       // this lane's query (B-operand column)
  const T* qp = reinterpret_cast<const T*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * p.d;
  const T* dop = reinterpret_cast<const T*>(p.dout) + (int64_t)b * p.nq * p.dos + (int64_t)h * p.d;
  const T* kp = reinterpret_cast<const T*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * p.d;
  const T* vp = reinterpret_cast<const T*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * p.d;
  const bool qok = qi < p.nq;
  const float lse_q = qok ? p.lse[((int64_t)b * p.heads + h) * p.nq + qi] : 0.f;
  const float d_q = qok ? p.dvec[((int64_t)b * p.heads + h) * p.nq + qi] : 0.f;

  Frag4<T> qf[ND], gf[ND];
#pragma unroll
  for (int ds = 0; ds < ND; ++ds) {
    const int dd = 16 * ds + 4 * g;
    if (qok && dd < p.d) {
      qf[ds] = *reinterpret_cast<const Frag4<T>*>(qp + (int64_t)qi * p.qs + dd);
      gf[ds] = *reinterpret_cast<const Frag4<T>*>(dop + (int64_t)qi * p.dos + dd);
    } else {
      qf[ds] = Frag4<T>{};
      gf[ds] = Frag4<T>{};
    }
  }
  f32x4_t dqt[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) dqt[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const float c2 = p.scale_log2;

  auto compute = [&](int buf, int k0) {
    const T* Ks = lds + buf * 2 * TILE;
    const T* Vs = Ks + TILE;
#pragma unroll
    for (int js = 0; js < 4; ++js) {
      // S^T[key][q], dP^T[key][q]: rows key = js*16 + 4g + r, column q = lr
      f32x4_t s = f32x4_t{0.f, 0.f, 0.f, 0.f}, dp = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < ND; ++ds) {
        const Frag4<T> ka = *reinterpret_cast<const Frag4<T>*>(Ks + (16 * js + lr) * ROW + 16 * ds + 4 * g);
        const Frag4<T> va = *reinterpret_cast<const Frag4<T>*>(Vs + (16 * js + lr) * ROW + 16 * ds + 4 * g);
        mma_k16(s, ka, qf[ds]);
        mma_k16(dp, va, gf[ds]);
      }
      f32x4_t dz;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kj = k0 + 16 * js + 4 * g + r;
        const bool ok = qok && kj < p.nkv;
        const float pr = ok ? __builtin_amdgcn_exp2f(fmaf(s[r], c2, -lse_q)) : 0.f;
        dz[r] = pr * (dp[r] - d_q);
      }
      const Frag4<T> zf = pack4<T>(dz);
#pragma unroll
      for (int dd = 0; dd < ND; ++dd) mma_k16(dqt[dd], tr_frag<T, ROW>(Ks, 16 * js, 16 * dd, g, lr), zf);  // dQ^T += K^T dZ^T
    }
  };

  const int ntiles = (p.nkv + KVT - 1) / KVT;
  stage_pair<T, DP>(kp, p.ks, vp, p.vs, p.nkv, p.d, 0, lds0, lds0 + TILE * ES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = NBUF == 2 ? (t & 1) : 0;
    if (NBUF == 2 && t + 1 < ntiles) {
      const unsigned nb = lds0 + (unsigned)((buf ^ 1) * 2 * TILE * ES);
      stage_pair<T, DP>(kp, p.ks, vp, p.vs, p.nkv, p.d, (t + 1) * KVT, nb, nb + TILE * ES, wave, lane);
    }
    compute(buf, t * KVT);
    if (NBUF == 1 && t + 1 < ntiles) {
      __syncthreads();
      stage_pair<T, DP>(kp, p.ks, vp, p.vs, p.nkv, p.d, (t + 1) * KVT, lds0, lds0 + TILE * ES, wave, lane);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (!qok) return;
  T* dqp = reinterpret_cast<T*>(p.dq) + ((int64_t)b * p.nq + qi) * p.dqs + (int64_t)h * p.d;
#pragma unroll
  for (int dd = 0; dd < ND; ++dd) {
    const int d0 = 16 * dd + 4 * g;
    if (d0 >= p.d) continue;
    float qq[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) qq[r] = dqt[dd][r] * p.scale;
    if constexpr (ES == 2) {
      bf16_t hq[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) hq[r] = f2bf(qq[r]);
      *reinterpret_cast<uint2*>(dqp + d0) = *reinterpret_cast<const uint2*>(hq);
    } else {
      *reinterpret_cast<float4*>(dqp + d0) = make_float4(qq[0], qq[1], qq[2], qq[3]);
    }
  }
}

// --------------------------------------------------------------------------------------
// bf16 backward on the full-rate 32x32x16 MFMA (head_dim <= 32 NDB; the 16x16x16 kernels above
// issue at half the FLOP rate on gfx950).  Layouts (32x32x16): A lane l = row l&31, k 8(l>>5)+j;
// B lane l = col l&31, k 8(l>>5)+j; C lane l col l&31, reg r row (r&3) + 8(r>>2) + 4(l>>5).
//   attn_bwd_kv32: a wave owns 32 keys (K, V rows as B operands in registers), loops over
//     64-query tiles of (Q, dO) staged by LDS-DMA (plus the tile's lse and D in LDS):
//       S = Q K^T, dP = dO V^T          (A = Q / dO rows; acc col = key, rows = queries)
//       P = 2^(S c2 - lse), dZ = P (dP - D)
//       dV^T += dO^T P, dK^T += Q^T dZ  (A = dO^T / Q^T by ds_read_b64_tr_b16 in the permuted
//                                        k order of the acc registers, B = the bf16 acc: as the
//                                        forward's P.V, attn_d40_kernel)
//   attn_bwd_q32: a wave owns 32 queries (Q, dO rows as B operands), loops over 64-key tiles of
//     (K, V):  S^T = K Q^T, dP^T = V dO^T, dZ^T = P^T (dP^T - D), dQ^T += K^T dZ^T.
// Per 64-row tile and wave: 28 (kv) / 20 (q) MFMAs of 32 cycles against 48 / 32 half-rate 16x16x16
// issues of 16 keys (or queries) per wave before.
// --------------------------------------------------------------------------------------
template <int NDB>
struct Bwd32 {
  static constexpr int CPR = NDB * 4;          // 16-byte chunks staged per row: NDB * 32 columns
  static constexpr int RCH = CPR + 1;          // + one pad chunk
  static constexpr int ROW = RCH * 8;          // bf16 elements per LDS row
  static constexpr int TILE = 64 * ROW;        // elements per staged operand tile
};

// rows [r0, r0 + 64) of two bf16 [n][stride] operands (head h) -> LDS tiles [64][ROW], zero past
// n and head_dim; RCH wave instructions of 1 KB each per operand
template <int NDB, int NW>
__device__ __forceinline__ void stage_pair32(const bf16_t* ap, int as, const bf16_t* bp, int bs, int n, int dh,
                                             int r0, unsigned abase, unsigned bbase, int wave, int lane) {
  constexpr int RCH = Bwd32<NDB>::RCH, CPR = Bwd32<NDB>::CPR;
  for (int i = wave; i < RCH; i += NW) {
    const int L = i * 64 + lane;
    const int row = L / RCH, c = L - row * RCH;
    const int r = r0 + row, dd = c * 8;
    const bool ok = r < n && c < CPR && dd < dh;
    const unsigned off = __builtin_amdgcn_readfirstlane(i * 64 * 16);
    glds16(ok ? (const void*)(ap + (int64_t)r * as + dd) : (const void*)&kZeros16, abase + off);
    glds16(ok ? (const void*)(bp + (int64_t)r * bs + dd) : (const void*)&kZeros16, bbase + off);
  }
}

// A operand X^T (rows d = 32 db + l&31, k = reduction rows of block blk, k-step st, in the acc's
// permuted order 16 st + 8 (j >> 2) + 4 hh + (j & 3)) from a row-major [64][ROW] tile
template <int ROW>
__device__ __forceinline__ bf16x8_t tr_a32(const bf16_t* tile, int blk, int st, int db, int lane) {
  typedef __attribute__((ext_vector_type(4))) short s4_t;
  typedef __attribute__((address_space(3))) s4_t lds_s4_t;
  const int i16 = lane & 15, hh = lane >> 5;
  const int cb = 32 * db + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
  const bf16_t* a0 = tile + (32 * blk + 16 * st + 4 * hh + (i16 >> 2)) * ROW + cb;
  const uint2 lo = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0)));
  const uint2 hi = __builtin_bit_cast(uint2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t*)(a0 + 8 * ROW)));
  return __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

__device__ __forceinline__ bf16x8_t pack8_bf16(const float* v) {
  return __builtin_bit_cast(bf16x8_t, make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                 pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])));
}

__device__ __forceinline__ f32x16_t mma32(const bf16x8_t a, const bf16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int NC, int NDB>
__global__ __launch_bounds__(256, 2) void attn_bwd_kv32(const AttnBwdArgs p) {
  using G = Bwd32<NDB>;
  constexpr int ROW = G::ROW, TILE = G::TILE;
  __shared__ uint4 smem[(2 * 2 * TILE * 2 + 2 * 128 * 4) / 16];
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);
  float* const vec = reinterpret_cast<float*>(lds + 2 * 2 * TILE);     // [buf][lse 64 | D 64]
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int h = blockIdx.y, b = blockIdx.z;
  const int key = blockIdx.x * 128 + wave * 32 + r32;
  const bf16_t* qp = reinterpret_cast<const bf16_t*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * p.d;
  const bf16_t* dop = reinterpret_cast<const bf16_t*>(p.dout) + (int64_t)b * p.nq * p.dos + (int64_t)h * p.d;
  const bf16_t* kp = reinterpret_cast<const bf16_t*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * p.d;
  const bf16_t* vp = reinterpret_cast<const bf16_t*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * p.d;
  const float* lse = p.lse + ((int64_t)b * p.heads + h) * p.nq;
  const float* dvec = p.dvec + ((int64_t)b * p.heads + h) * p.nq;

  bf16x8_t kf[NC], vf[NC];                 // B operands: K / V row of this lane's key, d 16c + 8hh ..
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int dd = 16 * c + 8 * hh;
    uint4 kk = make_uint4(0u, 0u, 0u, 0u), vv = kk;
    if (key < p.nkv && dd < p.d) {
      kk = *reinterpret_cast<const uint4*>(kp + (int64_t)key * p.ks + dd);
      vv = *reinterpret_cast<const uint4*>(vp + (int64_t)key * p.vs + dd);
    }
    kf[c] = __builtin_bit_cast(bf16x8_t, kk);
    vf[c] = __builtin_bit_cast(bf16x8_t, vv);
  }
  f32x16_t dkt[NDB], dvt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dkt[i][r] = 0.f; dvt[i][r] = 0.f; }
  const float c2 = p.scale_log2;

  auto stage = [&](int q0, int buf) {
    const unsigned qb = lds0 + (unsigned)(buf * 2 * TILE * 2);
    stage_pair32<NDB, 4>(qp, p.qs, dop, p.dos, p.nq, p.d, q0, qb, qb + TILE * 2, wave, lane);
  };
  // the tile's lse (+inf past nq: P = 0 there) and D, register-staged by the first two waves
  auto vec_load = [&](int q0) -> float {
    const int q = q0 + (tid & 63);
    if (tid < 64) return q < p.nq ? lse[q] : INFINITY;
    if (tid < 128) return q < p.nq ? dvec[q] : 0.f;
    return 0.f;
  };
  auto vec_store = [&](int buf, float v) {
    if (tid < 128) vec[buf * 128 + tid] = v;
  };

  auto compute = [&](int buf) {
    const bf16_t* Qs = lds + buf * 2 * TILE;
    const bf16_t* Ds = Qs + TILE;
    const float* lv = vec + buf * 128;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint4 qa = *reinterpret_cast<const uint4*>(Qs + (32 * qb + r32) * ROW + 16 * c + 8 * hh);
        const uint4 da = *reinterpret_cast<const uint4*>(Ds + (32 * qb + r32) * ROW + 16 * c + 8 * hh);
        s = mma32(__builtin_bit_cast(bf16x8_t, qa), kf[c], s);
        dp = mma32(__builtin_bit_cast(bf16x8_t, da), vf[c], dp);
      }
      // rows: query 32 qb + (r & 3) + 8 (r >> 2) + 4 hh
      bf16x8_t pb[2], zb[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float pv[8], zv[8];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int g4 = 2 * st + jj;
          const float4 l4 = *reinterpret_cast<const float4*>(lv + 32 * qb + 8 * g4 + 4 * hh);
          const float4 d4 = *reinterpret_cast<const float4*>(lv + 64 + 32 * qb + 8 * g4 + 4 * hh);
          const float lq[4] = {l4.x, l4.y, l4.z, l4.w}, dq[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * g4 + e;
            const float pr = __builtin_amdgcn_exp2f(fmaf(s[r], c2, -lq[e]));
            pv[4 * jj + e] = pr;
            zv[4 * jj + e] = pr * (dp[r] - dq[e]);
          }
        }
        pb[st] = pack8_bf16(pv);
        zb[st] = pack8_bf16(zv);
      }
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          dvt[db] = mma32(tr_a32<ROW>(Ds, qb, st, db, lane), pb[st], dvt[db]);   // dV^T += dO^T P
          dkt[db] = mma32(tr_a32<ROW>(Qs, qb, st, db, lane), zb[st], dkt[db]);   // dK^T += Q^T dZ
        }
      // one query block's S / dP live at a time (occupancy: kres.py)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const int ntiles = (p.nq + 63) / 64;
  stage(0, 0);
  vec_store(0, vec_load(0));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    float nv = 0.f;
    if (t + 1 < ntiles) {
      stage((t + 1) * 64, buf ^ 1);
      nv = vec_load((t + 1) * 64);
    }
    compute(buf);
    if (t + 1 < ntiles) vec_store(buf ^ 1, nv);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (key >= p.nkv) return;
  bf16_t* dkp = reinterpret_cast<bf16_t*>(p.dk) + ((int64_t)b * p.nkv + key) * p.dkvs + (int64_t)h * p.d;
  bf16_t* dvp = reinterpret_cast<bf16_t*>(p.dv) + ((int64_t)b * p.nkv + key) * p.dkvs + (int64_t)h * p.d;
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d0 = 32 * db + 8 * g4 + 4 * hh;
      if (d0 >= p.d) continue;
      const int r = 4 * g4;
      *reinterpret_cast<uint2*>(dkp + d0) =
          make_uint2(pack_bf16x2(dkt[db][r] * p.scale, dkt[db][r + 1] * p.scale),
                     pack_bf16x2(dkt[db][r + 2] * p.scale, dkt[db][r + 3] * p.scale));
      *reinterpret_cast<uint2*>(dvp + d0) =
          make_uint2(pack_bf16x2(dvt[db][r], dvt[db][r + 1]), pack_bf16x2(dvt[db][r + 2], dvt[db][r + 3]));
    }
}

template <int NC, int NDB>
__global__ __launch_bounds__(256, 2) void attn_bwd_q32(const AttnBwdArgs p) {
  using G = Bwd32<NDB>;
  constexpr int ROW = G::ROW, TILE = G::TILE;
  __shared__ uint4 smem[2 * 2 * TILE * 2 / 16];
  bf16_t* const lds = reinterpret_cast<bf16_t*>(smem);
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int h = blockIdx.y, b = blockIdx.z;
  const int qi = blockIdx.x * 128 + wave * 32 + r32;
  const bf16_t* qp = reinterpret_cast<const bf16_t*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * p.d;
  const bf16_t* dop = reinterpret_cast<const bf16_t*>(p.dout) + (int64_t)b * p.nq * p.dos + (int64_t)h * p.d;
  const bf16_t* kp = reinterpret_cast<const bf16_t*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * p.d;
  const bf16_t* vp = reinterpret_cast<const bf16_t*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * p.d;
  const bool qok = qi < p.nq;
  const float lse_q = qok ? p.lse[((int64_t)b * p.heads + h) * p.nq + qi] : 0.f;
  const float d_q = qok ? p.dvec[((int64_t)b * p.heads + h) * p.nq + qi] : 0.f;

  bf16x8_t qf[NC], gf[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int dd = 16 * c + 8 * hh;
    uint4 qq = make_uint4(0u, 0u, 0u, 0u), gg = qq;
    if (qok && dd < p.d) {
      qq = *reinterpret_cast<const uint4*>(qp + (int64_t)qi * p.qs + dd);
      gg = *reinterpret_cast<const uint4*>(dop + (int64_t)qi * p.dos + dd);
    }
    qf[c] = __builtin_bit_cast(bf16x8_t, qq);
    gf[c] = __builtin_bit_cast(bf16x8_t, gg);
  }
  f32x16_t dqt[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dqt[i][r] = 0.f;
  const float c2 = p.scale_log2;

  auto stage = [&](int k0, int buf) {
    const unsigned kb = lds0 + (unsigned)(buf * 2 * TILE * 2);
    stage_pair32<NDB, 4>(kp, p.ks, vp, p.vs, p.nkv, p.d, k0, kb, kb + TILE * 2, wave, lane);
  };
  auto compute = [&](int buf, int k0, bool masked) {
    const bf16_t* Ks = lds + buf * 2 * TILE;
    const bf16_t* Vs = Ks + TILE;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint4 ka = *reinterpret_cast<const uint4*>(Ks + (32 * kb + r32) * ROW + 16 * c + 8 * hh);
        const uint4 va = *reinterpret_cast<const uint4*>(Vs + (32 * kb + r32) * ROW + 16 * c + 8 * hh);
        s = mma32(__builtin_bit_cast(bf16x8_t, ka), qf[c], s);
        dp = mma32(__builtin_bit_cast(bf16x8_t, va), gf[c], dp);
      }
      // rows: key 32 kb + (r & 3) + 8 (r >> 2) + 4 hh; column: this lane's query
      bf16x8_t zb[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float zv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = 8 * st + j;
          const float pr = __builtin_amdgcn_exp2f(fmaf(s[r], c2, -lse_q));
          float z = pr * (dp[r] - d_q);
          if (masked && k0 + 32 * kb + (r & 3) + 8 * (r >> 2) + 4 * hh >= p.nkv) z = 0.f;
          zv[j] = z;
        }
        zb[st] = pack8_bf16(zv);
      }
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int st = 0; st < 2; ++st) dqt[db] = mma32(tr_a32<ROW>(Ks, kb, st, db, lane), zb[st], dqt[db]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const int ntiles = (p.nkv + 63) / 64;
  const int nfull = p.nkv / 64;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) stage((t + 1) * 64, buf ^ 1);
    if (t < nfull) compute(buf, t * 64, false);
    else compute(buf, t * 64, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (!qok) return;
  bf16_t* dqp = reinterpret_cast<bf16_t*>(p.dq) + ((int64_t)b * p.nq + qi) * p.dqs + (int64_t)h * p.d;
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d0 = 32 * db + 8 * g4 + 4 * hh;
      if (d0 >= p.d) continue;
      const int r = 4 * g4;
      *reinterpret_cast<uint2*>(dqp + d0) =
          make_uint2(pack_bf16x2(dqt[db][r] * p.scale, dqt[db][r + 1] * p.scale),
                     pack_bf16x2(dqt[db][r + 2] * p.scale, dqt[db][r + 3] * p.scale));
    }
}

int g_attn_bwd32 = 1;   // tuning / A-B hook (ldm_attention_set_bwd32): 0 routes bf16 to the 16x16x16 kernels

template <int NC, int NDB>
int launch_bwd32(const AttnBwdArgs& a, int batch, hipStream_t s) {
  hipLaunchKernelGGL((attn_bwd_kv32<NC, NDB>), dim3((a.nkv + 127) / 128, a.heads, batch), dim3(256), 0, s, a);
  LDM_CHECK_LAUNCH();
  hipLaunchKernelGGL((attn_bwd_q32<NC, NDB>), dim3((a.nq + 127) / 128, a.heads, batch), dim3(256), 0, s, a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

template <typename T, int DP>
int launch_bwd_dp(const AttnBwdArgs& a, int batch, hipStream_t s) {
  hipLaunchKernelGGL((attn_bwd_kv<T, DP>), dim3((a.nkv + 63) / 64, a.heads, batch), dim3(256), 0, s, a);
  LDM_CHECK_LAUNCH();
  hipLaunchKernelGGL((attn_bwd_q<T, DP>), dim3((a.nq + 63) / 64, a.heads, batch), dim3(256), 0, s, a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

template <typename T>
int launch_bwd(const AttnBwdArgs& a, int batch, hipStream_t s) {
  const int rows = batch * a.heads * a.nq;
  hipLaunchKernelGGL(attn_bwd_dot<T>, dim3((rows + 15) / 16), dim3(256), 0, s, a, batch);
  LDM_CHECK_LAUNCH();
  const int dp = (a.d + 15) / 16 * 16;
  if constexpr (sizeof(T) == 2) {
    // 32x32x16 forms: 16-byte-aligned row strides (the B-operand rows are 16-byte register loads)
    const bool al = a.qs % 8 == 0 && a.dos % 8 == 0 && a.ks % 8 == 0 && a.vs % 8 == 0;
    if (g_attn_bwd32 && al && a.d <= 64) {
      if (a.d <= 32) return launch_bwd32<2, 1>(a, batch, s);
      if (a.d <= 48) return launch_bwd32<3, 2>(a, batch, s);
      return launch_bwd32<4, 2>(a, batch, s);
    }
  }
  switch (dp) {
    case 16: return launch_bwd_dp<T, 16>(a, batch, s);
    case 32: return launch_bwd_dp<T, 32>(a, batch, s);
    case 48: return launch_bwd_dp<T, 48>(a, batch, s);
    case 64: return launch_bwd_dp<T, 64>(a, batch, s);
    case 80: return launch_bwd_dp<T, 80>(a, batch, s);
    case 96: return launch_bwd_dp<T, 96>(a, batch, s);
    case 128: return launch_bwd_dp<T, 128>(a, batch, s);
    case 160: return launch_bwd_dp<T, 160>(a, batch, s);
    default: return LDM_ERR_ARG;
  }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

namespace {
int attn_validate(const ldm_attn_params* q) {
  if (!q || !q->q || !q->k || !q->v || !q->o) return LDM_ERR_ARG;
  if (q->dtype != LDM_F32 && q->dtype != LDM_BF16) return LDM_ERR_ARG;
  if (q->batch <= 0 || q->heads <= 0 || q->n_q <= 0 || q->n_kv <= 0) return LDM_ERR_ARG;
  if (q->head_dim <= 0 || q->head_dim > 160 || q->head_dim % 8) return LDM_ERR_ALIGN;
  const int es = q->dtype == LDM_F32 ? 4 : 2;
  const int ce = 16 / es;
  if (q->k_stride % ce || q->v_stride % ce || q->q_stride % 4 || q->o_stride % 4) return LDM_ERR_ALIGN;
  if (!aligned16(q->k) || !aligned16(q->v) || !aligned16(q->q) || !aligned16(q->o)) return LDM_ERR_ALIGN;
  return LDM_OK;
}

AttnArgs attn_args(const ldm_attn_params* q) {
  AttnArgs a;
  a.q = static_cast<const char*>(q->q);
  a.k = static_cast<const char*>(q->k);
  a.v = static_cast<const char*>(q->v);
  a.o = static_cast<char*>(q->o);
  a.qs = q->q_stride; a.ks = q->k_stride; a.vs = q->v_stride; a.os = q->o_stride;
  a.heads = q->heads; a.d = q->head_dim; a.nq = q->n_q; a.nkv = q->n_kv;
  a.scale_log2 = q->scale * 1.4426950408889634f;
  a.lse = nullptr;
  a.kvsplit = 1; a.batch = q->batch;
  a.opart = nullptr; a.lsepart = nullptr;
  return a;
}
}  // namespace

extern "C" int ldm_attention(const ldm_attn_params* q, ldm_stream_t stream) {
  const int st = attn_validate(q);
  if (st != LDM_OK) return st;
  const AttnArgs a = attn_args(q);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return q->dtype == LDM_BF16 ? launch_bf16(a, q->batch, s) : launch_t<float>(a, q->batch, s);
}

namespace {
int g_fp8_scaled = 1;   // tuning / A-B hook (ldm_attention_set_fp8_scaled)
bool fp8_scaled_ok(const ldm_attn_params* q) {
  return g_fp8_scaled && q->head_dim == 40 && q->q_stride % 8 == 0 && q->k_stride % 8 == 0 && q->v_stride % 8 == 0 &&
         q->o_stride % 4 == 0;
}
}  // namespace

extern "C" size_t ldm_attention_workspace_bytes(const ldm_attn_params* q) {
  if (attn_validate(q) != LDM_OK || q->dtype != LDM_BF16 || g_attn_legacy || (q->head_dim == 40 && g_attn_d40 == 0) || g_attn_waves || g_attn_qs2 ||
      q->q_stride % 8 ||
      q->o_stride % 4)
    return 0;
  return kv_workspace(attn_args(q), q->batch);
}

extern "C" int ldm_attention_ws(const ldm_attn_params* q, void* workspace, int64_t workspace_bytes,
                                ldm_stream_t stream) {
  const int st = attn_validate(q);
  if (st != LDM_OK) return st;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t need = ldm_attention_workspace_bytes(q);
  if (need == 0) return ldm_attention(q, stream);
  if (!workspace || workspace_bytes < (int64_t)need || !aligned16(workspace)) return LDM_ERR_ARG;
  AttnArgs a = attn_args(q);
  a.kvsplit = kv_splits(a, q->batch);
  const size_t rows = (size_t)q->batch * q->heads * q->n_q;
  a.opart = static_cast<float*>(workspace);
  a.lsepart = a.opart + (size_t)a.kvsplit * rows * q->head_dim;
  return launch_kv_split(a, q->batch, s);
}

extern "C" void ldm_attention_set_pair(int enabled) { g_attn_pair = enabled < 0 ? 0 : enabled > 3 ? 3 : enabled; }

extern "C" void ldm_attention_set_kvsplit(int splits) { g_attn_kvsplit = splits < 0 ? -1 : (splits == 1 ? 0 : splits); }

extern "C" size_t ldm_attention_fp8_workspace_bytes(const ldm_attn_params* q) {
  if (attn_validate(q) != LDM_OK || q->dtype != LDM_BF16 || !fp8_scaled_ok(q)) return 0;
  return f8_workspace(attn_args(q), q->batch);
}

extern "C" int ldm_attention_fp8(const ldm_attn_params* q, void* workspace, int64_t workspace_bytes,
                                 ldm_stream_t stream) {
  const int st = attn_validate(q);
  if (st != LDM_OK) return st;
  if (q->dtype != LDM_BF16) return LDM_ERR_ARG;
  const AttnArgs a = attn_args(q);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (fp8_scaled_ok(q)) {
    if (!workspace || workspace_bytes < (int64_t)f8_workspace(a, q->batch) || !aligned16(workspace)) return LDM_ERR_ARG;
    return launch_f8_d40(a, q->batch, workspace, s);
  }
  return launch_fp8(a, q->batch, s);
}

extern "C" void ldm_attention_set_fp8_scaled(int enabled) { g_fp8_scaled = enabled ? 1 : 0; }
#ifdef LDM_F8_DEBUG
extern "C" void ldm_f8_debug_buffer(float* p) { g_f8_dbg = p; }
#endif

extern "C" void ldm_attention_set_waves(int waves) { g_attn_waves = (waves == 4 || waves == 8) ? waves : 0; }

extern "C" void ldm_attention_force_legacy(int legacy) { g_attn_legacy = legacy; }
extern "C" void ldm_attention_set_d80(int enabled) { g_attn_d80 = enabled ? 1 : 0; }
extern "C" void ldm_attention_set_d160(int enabled) { g_attn_d160 = enabled ? 1 : 0; }
extern "C" void ldm_attention_set_qs2(int mode) { g_attn_qs2 = mode == 1 || mode == 2 ? mode : 0; }
extern "C" void ldm_attention_set_il(int enabled) { g_attn_il = enabled < 0 ? 0 : enabled > 3 ? 3 : enabled; }
extern "C" void ldm_attention_set_skew(int mode) { g_attn_skew = mode >= 1 && mode <= 3 ? mode : 0; }
extern "C" void ldm_attention_set_bwd32(int enabled) { g_attn_bwd32 = enabled ? 1 : 0; }
extern "C" void ldm_attention_set_maxcol(int mode) {
  g_attn_maxcol = mode >= 1 ? 1 : 0;     // 0: per-score FMA, 16x16x32 kernel
  g_attn_d40 = mode >= 2 ? 1 : 0;        // 1: max column, 16x16x32 kernel; 2: 32x32x16 d = 40 kernel
}

extern "C" int ldm_attention_fwd_lse(const ldm_attn_params* q, float* lse, ldm_stream_t stream) {
  const int st = attn_validate(q);
  if (st != LDM_OK) return st;
  if (!lse) return LDM_ERR_ARG;
  AttnArgs a = attn_args(q);
  a.lse = lse;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return q->dtype == LDM_BF16 ? launch_bf16(a, q->batch, s) : launch_t<float>(a, q->batch, s);
}

extern "C" size_t ldm_attention_bwd_workspace_bytes(const ldm_attn_params* q) {
  if (!q || q->batch <= 0 || q->heads <= 0 || q->n_q <= 0) return 0;
  return ((size_t)q->batch * q->heads * q->n_q * sizeof(float) + 15) & ~(size_t)15;
}

extern "C" int ldm_attention_bwd(const ldm_attn_params* q, const void* o, const void* d_o, int do_stride,
                                 const float* lse, void* dq, void* dk, void* dv, int dq_stride, int dkv_stride,
                                 void* workspace, ldm_stream_t stream) {
  const int st = attn_validate(q);
  if (st != LDM_OK) return st;
  if (!o || !d_o || !lse || !dq || !dk || !dv || !workspace) return LDM_ERR_ARG;
  if (do_stride % 4 || dq_stride % 4 || dkv_stride % 4) return LDM_ERR_ALIGN;
  if (!aligned16(d_o) || !aligned16(workspace)) return LDM_ERR_ALIGN;
  const int es = q->dtype == LDM_F32 ? 4 : 2;
  const int ce = 16 / es;
  if (q->q_stride % ce || do_stride % ce) return LDM_ERR_ALIGN;   // Q / dO tiles are DMA-staged too
  AttnBwdArgs a;
  a.q = static_cast<const char*>(q->q);
  a.k = static_cast<const char*>(q->k);
  a.v = static_cast<const char*>(q->v);
  a.o = static_cast<const char*>(o);
  a.dout = static_cast<const char*>(d_o);
  a.dq = static_cast<char*>(dq);
  a.dk = static_cast<char*>(dk);
  a.dv = static_cast<char*>(dv);
  a.qs = q->q_stride; a.ks = q->k_stride; a.vs = q->v_stride; a.os = q->o_stride;
  a.dos = do_stride; a.dqs = dq_stride; a.dkvs = dkv_stride;
  a.heads = q->heads; a.d = q->head_dim; a.nq = q->n_q; a.nkv = q->n_kv;
  a.scale = q->scale;
  a.scale_log2 = q->scale * 1.4426950408889634f;
  a.lse = lse;
  a.dvec = static_cast<float*>(workspace);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return q->dtype == LDM_BF16 ? launch_bwd<bf16_t>(a, q->batch, s) : launch_bwd<float>(a, q->batch, s);
}
