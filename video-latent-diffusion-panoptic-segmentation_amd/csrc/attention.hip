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
};

__device__ const uint4 kZeros16 = {0u, 0u, 0u, 0u};
__device__ const uint4 kOnesBf16 = {0x3f80u, 0u, 0u, 0u};       // bf16 1.0 then zeros
__device__ const uint4 kOnesF32 = {0x3f800000u, 0u, 0u, 0u};    // fp32 1.0 then zeros

constexpr int KVT = 64;        // keys per tile
constexpr float kRescaleThr = 8.0f;

// 16 B per lane global -> LDS at M0 + 16 * lane (inline asm: see igemm.hip dma16; the
// consumer waits with an explicit vmcnt + barrier).  Per-lane 64-bit source address.
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
          pv[r] = __builtin_amdgcn_exp2f(fmaf(sacc[js][s][r], c2, mneg));
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

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int ldm_attention(const ldm_attn_params* q, ldm_stream_t stream) {
  if (!q || !q->q || !q->k || !q->v || !q->o) return LDM_ERR_ARG;
  if (q->dtype != LDM_F32 && q->dtype != LDM_BF16) return LDM_ERR_ARG;
  if (q->batch <= 0 || q->heads <= 0 || q->n_q <= 0 || q->n_kv <= 0) return LDM_ERR_ARG;
  if (q->head_dim <= 0 || q->head_dim > 160 || q->head_dim % 8) return LDM_ERR_ALIGN;
  const int es = q->dtype == LDM_F32 ? 4 : 2;
  const int ce = 16 / es;
  if (q->k_stride % ce || q->v_stride % ce || q->q_stride % 4 || q->o_stride % 4) return LDM_ERR_ALIGN;
  if (!aligned16(q->k) || !aligned16(q->v) || !aligned16(q->q) || !aligned16(q->o)) return LDM_ERR_ALIGN;
  AttnArgs a;
  a.q = static_cast<const char*>(q->q);
  a.k = static_cast<const char*>(q->k);
  a.v = static_cast<const char*>(q->v);
  a.o = static_cast<char*>(q->o);
  a.qs = q->q_stride; a.ks = q->k_stride; a.vs = q->v_stride; a.os = q->o_stride;
  a.heads = q->heads; a.d = q->head_dim; a.nq = q->n_q; a.nkv = q->n_kv;
  a.scale_log2 = q->scale * 1.4426950408889634f;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return q->dtype == LDM_BF16 ? launch_t<bf16_t>(a, q->batch, s) : launch_t<float>(a, q->batch, s);
}
