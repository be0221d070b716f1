// Fused multi-head attention forward (ldm_attention): softmax(Q K^T * scale) V, online softmax.
//
// Orientation ("swapped" products, so the softmax reduction axis stays inside one lane):
//   S^T[kv][q] = K[kv][:] . Q[q][:]      mfma A = K tile (LDS), B = Q (registers)
//   O^T[d][q] += V^T[d][kv] . P^T[kv][q]  mfma A = V^T tile (LDS), B = P (the S^T accumulator
//                                          registers, converted in place — no LDS round trip)
// With the 16x16x16 MFMA the accumulator of one 16-kv S^T fragment (lane holds kv = 4g+r for
// its q column) is exactly the B operand of the P.V product, and the row max needs only two
// cross-lane shuffles (lanes l, l^16, l^32, l^48 share a q column).
// Block = 4 waves x 32 query rows; K/V tiles of 64 keys staged through LDS (padded rows:
// conflict-free ds_read_b64 / b128).  head_dim is padded to DP (multiple of 16) with zeros.
// bf16: v_mfma_f32_16x16x16_bf16; fp32: v_mfma_f32_16x16x4_f32 (exact).
#include "common.h"

namespace {

struct AttnArgs {
  const char* q; const char* k; const char* v; char* o;
  int qs, ks, vs, os;
  int heads, d, nq, nkv;
  float scale_log2;
};

constexpr int QSUB = 2;   // 16-row q sub-tiles per wave
constexpr int KVT = 64;   // keys per tile

template <typename T, int DP>
__global__ __launch_bounds__(256) void attn_kernel(const AttnArgs p) {
  constexpr int ES = sizeof(T);
  constexpr int EPC = 16 / ES;          // elements per 16-B chunk
  constexpr int ND = DP / 16;
  constexpr int KROW = DP + EPC;        // row pitch (elements): 4*odd dwords -> conflict-free
  constexpr int VROW = KVT + EPC;
  constexpr int CPR = DP / EPC;         // 16-B chunks per K/V row
  __shared__ uint4 smem[(KVT * KROW + DP * VROW) * ES / 16];
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vt = Ks + KVT * KROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int h = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * (16 * QSUB * 4);  // 128 query rows per block
  const int qbase = q0 + wave * 16 * QSUB;

  const T* qp = reinterpret_cast<const T*>(p.q) + (int64_t)b * p.nq * p.qs + (int64_t)h * p.d;
  const T* kp = reinterpret_cast<const T*>(p.k) + (int64_t)b * p.nkv * p.ks + (int64_t)h * p.d;
  const T* vp = reinterpret_cast<const T*>(p.v) + (int64_t)b * p.nkv * p.vs + (int64_t)h * p.d;

  // Q fragments (B operand): lane holds Q[q = qbase + 16 qs + lr][d = 16 ds + 4g .. +3]
  Frag4<T> qf[QSUB][ND];
#pragma unroll
  for (int s = 0; s < QSUB; ++s) {
    const int qi = qbase + 16 * s + lr;
#pragma unroll
    for (int ds = 0; ds < ND; ++ds) {
      const int dd = 16 * ds + 4 * g;
      if (qi < p.nq && dd < p.d) {
        qf[s][ds] = *reinterpret_cast<const Frag4<T>*>(qp + (int64_t)qi * p.qs + dd);
      } else {
        qf[s][ds] = Frag4<T>{};
      }
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

  for (int kv0 = 0; kv0 < p.nkv; kv0 += KVT) {
    __syncthreads();
    // ---- stage K tile [kv][d] and V^T tile [d][kv]
    for (int idx = tid; idx < KVT * CPR; idx += 256) {
      const int row = idx / CPR, c = idx - row * CPR;
      const int kv = kv0 + row, d = c * EPC;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (kv < p.nkv && d < p.d) val = *reinterpret_cast<const uint4*>(kp + (int64_t)kv * p.ks + d);
      *reinterpret_cast<uint4*>(Ks + row * KROW + d) = val;
    }
    for (int idx = tid; idx < KVT * CPR; idx += 256) {
      const int row = idx & (KVT - 1), c = idx / KVT;
      const int kv = kv0 + row, d = c * EPC;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (kv < p.nkv && d < p.d) val = *reinterpret_cast<const uint4*>(vp + (int64_t)kv * p.vs + d);
      const T* e = reinterpret_cast<const T*>(&val);
#pragma unroll
      for (int j = 0; j < EPC; ++j) Vt[(d + j) * VROW + row] = e[j];
    }
    __syncthreads();

    // ---- S^T = K Q^T  (4 kv sub-tiles x QSUB q sub-tiles)
    f32x4_t sacc[4][QSUB];
#pragma unroll
    for (int js = 0; js < 4; ++js)
#pragma unroll
      for (int s = 0; s < QSUB; ++s) sacc[js][s] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < ND; ++ds) {
#pragma unroll
      for (int js = 0; js < 4; ++js) {
        const Frag4<T> ka = *reinterpret_cast<const Frag4<T>*>(Ks + (16 * js + lr) * KROW + 16 * ds + 4 * g);
#pragma unroll
        for (int s = 0; s < QSUB; ++s) mma_k16(sacc[js][s], ka, qf[s][ds]);
      }
    }

    // ---- online softmax (log2 domain); P packed into the PV B operand
    Frag4<T> pf[4][QSUB];
#pragma unroll
    for (int s = 0; s < QSUB; ++s) {
      float mx = -INFINITY;
#pragma unroll
      for (int js = 0; js < 4; ++js)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kv = kv0 + 16 * js + 4 * g + r;
          float v = sacc[js][s][r] * p.scale_log2;
          if (kv >= p.nkv) v = -INFINITY;
          sacc[js][s][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(mrun[s], mx);
      const float alpha = __builtin_amdgcn_exp2f(mrun[s] - mnew);
      mrun[s] = mnew;
      float lsum = 0.f;
#pragma unroll
      for (int js = 0; js < 4; ++js) {
        float pv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pv[r] = __builtin_amdgcn_exp2f(sacc[js][s][r] - mnew);
          lsum += pv[r];
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
      lrun[s] = lrun[s] * alpha + lsum;
#pragma unroll
      for (int i = 0; i < ND; ++i) oacc[i][s] *= alpha;
    }

    // ---- O^T += V^T P^T
#pragma unroll
    for (int dd = 0; dd < ND; ++dd) {
#pragma unroll
      for (int js = 0; js < 4; ++js) {
        const Frag4<T> va = *reinterpret_cast<const Frag4<T>*>(Vt + (16 * dd + lr) * VROW + 16 * js + 4 * g);
#pragma unroll
        for (int s = 0; s < QSUB; ++s) mma_k16(oacc[dd][s], va, pf[js][s]);
      }
    }
  }

  // ---- normalise and store O[q][h*d + d]
  T* op = reinterpret_cast<T*>(p.o) + (int64_t)b * p.nq * p.os + (int64_t)h * p.d;
#pragma unroll
  for (int s = 0; s < QSUB; ++s) {
    float lt = lrun[s] + __shfl_xor(lrun[s], 16, 64);
    lt += __shfl_xor(lt, 32, 64);
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

template <typename T, int DP>
int launch_dp(const AttnArgs& a, int batch, hipStream_t s) {
  dim3 grid((a.nq + 127) / 128, a.heads, batch);
  hipLaunchKernelGGL((attn_kernel<T, DP>), grid, dim3(256), 0, s, a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
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
