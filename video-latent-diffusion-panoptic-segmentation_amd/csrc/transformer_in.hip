// Fused Transformer2DModel input half at the 64x64 UNet level (ldm_transformer_in):
//   norm (GroupNorm, producer statistics) -> proj_in (+ bias) -> h      (stored: to_out's residual)
//   -> norm1 (LayerNorm) folded into the fused to_q/k/v GEMM -> qkv     (stored: the attention input)
// for diffusers Transformer2DModel / BasicTransformerBlock.attn1, reached via
// /root/reference/ldmseg/models/unet.py:361-425 — in ONE launch instead of gn_apply + two
// ldm_conv2d calls (profiles/r04*: 12 + 24 + 52 us per block at B = 8, M = 32768, C = 320).
//
// One 8-wave block per CU owns a 128-row tile; wave w owns rows 16 w .. 16 w + 15 for BOTH GEMMs
// (8 (M) x 1 (N), as ldm_feedforward's GEGLU phase), so every A operand lives in VGPRs as MFMA
// fragments and only the weights go through LDS:
//   - x rows (10 k32 fragments per lane) are loaded once and GroupNorm'd in registers with the
//     per-(batch, channel) scale / shift finalised from the producer's unit accumulators (the same
//     fp64 reduction and fmaf as gn_apply, so the A operand equals gn_apply's output bit for bit);
//   - proj_in: 10 weight stages ([160 rows][64 K], 20 KB each) into 2 x 10 accumulators;
//   - its output tile h = bf16(acc + b) becomes the QKV A operand without leaving the registers:
//     a v_permlane32_swap + v_permlane16_swap pair per two D fragments turns "4 channels of a row per
//     lane" (the 16x16 accumulator layout) into "8 consecutive channels of a row per lane" — exactly
//     the k32 A fragment, and a 16-byte store of h;
//   - the LayerNorm row statistics are summed in the order ldm_conv2d's row writer uses (fp32 8-
//     channel partials, fp32 over each 160-column tile, fp64 over the two tiles), gathered across the
//     row's four lanes by shuffles, so the fold's (rstd, -rstd mean) are those of the unfused path;
//   - QKV: three 320-column chunks of 10 weight stages each, epilogue rstd (acc - mean c1) + bias
//     (the ln_rows form of ldm_conv2d) -> bf16 -> the same permlane pair -> 16-byte stores.
// The weights stream by LDS-DMA through 7 stage slots (6 stages in flight, counted vmcnt, one raw
// barrier per stage, as ldm_feedforward); the MFMA sequence per output element and every rounding
// point are those of the three unfused launches, so h and qkv agree with them bit for bit.
// Per tile: 26.8 MFLOP x 4 ... 105 MFLOP of MFMA work against 800 KB of weight stages.
#include "igemm_common.h"

namespace {
namespace tik {
constexpr int NT = 512;
constexpr int BM = 128;                    // rows per tile
constexpr int C = 320;                     // model width: proj_in K / N, QKV K
constexpr int NQ = 3 * C;                  // QKV N
constexpr int KC = C / 32;                 // k32 fragments of a row (10)
constexpr int SN = 160;                    // weight rows per stage (half of a 320-column chunk)
constexpr int FN = SN / 16;                // fragments per wave per stage (10)
constexpr int STAGE_B = SN * 128;          // one [160][64] bf16 weight stage (20 KB)
constexpr int INS = 3;                     // DMA instructions per wave per stage (20 + 4 dummies)
constexpr int NSLOT = 7;                   // stage slots: 6 stages in flight while one is multiplied
constexpr int S_IN = 10;                   // proj_in stages (5 K x 2 N halves)
constexpr int S_Q = 10;                    // stages per QKV chunk
constexpr int NCH = NQ / C;                // QKV chunks (3)
constexpr int NST = S_IN + NCH * S_Q;      // stages per tile (40)
constexpr int EPI_ST = KC;                 // 16-byte stores per wave instruction stream per epilogue
constexpr int CONST_OFF = NSLOT * STAGE_B;
// constants in LDS (fp32 unless noted): QKV c1 [960], QKV bias [960], proj_in bias [320],
// GroupNorm scale [320] / shift [320], group (mean, rstd) [64] float2, unit accumulators
// [<= 512] double2 (slots x units of one batch)
constexpr int OFF_C1 = 0, OFF_BQ = NQ, OFF_BIN = 2 * NQ, OFF_SC = OFF_BIN + C, OFF_SH = OFF_SC + C,
              OFF_GST = OFF_SH + C, OFF_URED = OFF_GST + 128;
constexpr int MAX_URED = 256;            // slots (<= 8) x units (C / 10 = 32)
constexpr int CONST_FLOATS = OFF_URED + 4 * MAX_URED;
constexpr int DUMMY_OFF = CONST_OFF + CONST_FLOATS * 4;   // 1 KB target of the dummy DMA instructions
constexpr int LDS_B = DUMMY_OFF + 1024;
static_assert(LDS_B <= 160 * 1024, "LDS");
static_assert(C % SN == 0 && SN % 32 == 0 && (SN / 8) <= 8 * INS, "stage geometry");
}  // namespace tik

// s_waitcnt vmcnt(n) for the constants of the unrolled stage loop
__device__ __forceinline__ void tin_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
// DMA instructions this wave may leave in flight when it waits for stage u of a 10-stage run:
// the younger stages (min(5, stages left)) x 3, plus the 10 epilogue stores issued after the
// previous run's last stage, which are younger than the six stages following it
__host__ __device__ constexpr int tin_younger(int u, bool last, int ins = tik::INS) {
  const int left = last ? tik::S_Q - 1 - u : tik::NSLOT - 2;
  const int ahead = left < tik::NSLOT - 2 ? left : tik::NSLOT - 2;
  return ins * ahead + (u <= tik::NSLOT - 2 ? tik::EPI_ST : 0);
}
static_assert(tin_younger(0, false) == 25 && tin_younger(6, false) == 15 && tin_younger(5, true) == 22 &&
              tin_younger(6, true) == 9 && tin_younger(7, true) == 6 && tin_younger(8, true) == 3 &&
              tin_younger(9, true) == 0 && tin_younger(4, true) == 25, "tin_wait cases");

// Two 16x16 D fragments of one row block (a: columns 32p + 0..15, b: 32p + 16..31; lane (g, lr) holds
// columns 4g..4g+3 of its fragment, packed bf16 x 2 per dword) -> per lane 8 CONSECUTIVE columns
// 32p + 8g .. + 7 of row lr: permlane32 swaps the upper half of a with the lower half of b, then
// permlane16 swaps rows 1 / 3 of a with rows 0 / 2 of b (rows = 16-lane groups).
__device__ __forceinline__ uint4 d_pair_to_row8(uint2 a, uint2 b) {
  auto r0 = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
  auto r1 = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
  auto s0 = __builtin_amdgcn_permlane16_swap(r0[0], r0[1], false, false);
  auto s1 = __builtin_amdgcn_permlane16_swap(r1[0], r1[1], false, false);
  return make_uint4(s0[0], s1[0], s0[1], s1[1]);
}
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// MODE (tuning / A-B; the default is 1): bit 0 issues a stage's DMA between its two k32 halves
// (beside the first half's MFMAs) instead of before them (50.7 -> 48.6 us, tools/opbench.py tin_l0);
// bit 1 drops the dummy DMA instructions (waves 4-7 issue two per stage, counted per wave: 62.7 us,
// the per-wave counts spill 64 VGPRs); bit 2 gives waves 4-7 static priority 1 (no gain); ablations:
// bit 3 no weight stream (43.4 us), bit 4 no MFMA (fragments kept live: slower, the reads serialise).
// What bounds it: the 8 (M) x 1 (N) form reads one 1-KB W fragment per 16x16x32 MFMA, i.e. the LDS
// array's 256 B/clk exactly when the MFMA pipes are full, so neither runs near its peak.
template <int MODE>
__global__ __launch_bounds__(512, 1) void transformer_in_kernel(const ConvArgs pi, const ConvArgs pq,
                                                                const double* __restrict__ gacc, int gunit,
                                                                int gslots, int groups, float geps,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta) {
  using namespace tik;
  __shared__ uint4 smem[LDS_B / 16];
  const int M = pi.M, hw = pi.hw_out;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ (((8 * wv + drow) >> 1) & 7);   // source-side swizzle (igemm)

  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  float* const cst = reinterpret_cast<float*>(reinterpret_cast<char*>(smem) + CONST_OFF);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)pi.a0, 0, pi.a0_bytes, kBufFlags);
  const __amdgpu_buffer_rsrc_t rwi = __builtin_amdgcn_make_buffer_rsrc((void*)pi.w, 0, pi.w_bytes, kBufFlags);
  const __amdgpu_buffer_rsrc_t rwq = __builtin_amdgcn_make_buffer_rsrc((void*)pq.w, 0, pq.w_bytes, kBufFlags);

  // per-kernel column constants
  for (int i = tid; i < NQ; i += NT) {
    cst[OFF_C1 + i] = pq.ln_c1[i];
    cst[OFF_BQ + i] = pq.bias ? pq.bias[i] : 0.f;
  }
  for (int i = tid; i < C; i += NT) cst[OFF_BIN + i] = pi.bias ? pi.bias[i] : 0.f;

  const int vo = (drow * C + 8 * dchunk) * 2;   // lane part of a weight row's source offset (kpad = C)
  // stage s of the tile (0..39): proj_in (s < 10) or QKV chunk (s - 10) / 10; K block kb, N half nh
  auto issue = [&](int s) {
    if (MODE & 8) return;                          // ablation: no weight stream
    const bool is_in = s < S_IN;
    const int t = is_in ? s : s - S_IN;
    const int u = is_in ? t : t % S_Q;
    const int row0 = (is_in ? 0 : (t / S_Q) * C) + SN * (u & 1);
    const int kb = u >> 1;
    const unsigned base = lds0 + (unsigned)((s % NSLOT) * STAGE_B);
#pragma unroll
    for (int i = 0; i < INS; ++i) {
      const int ii = wv + 8 * i;                 // DMA instruction of the stage: rows 8 ii .. 8 ii + 7
      const bool real = ii < SN / 8;
      if ((MODE & 2) && !real) break;
      const int soff = __builtin_amdgcn_readfirstlane(real ? ((row0 + 8 * ii) * C + 64 * kb) * 2 : kOOB);
      const unsigned dst = __builtin_amdgcn_readfirstlane(real ? base + ii * 1024 : lds0 + DUMMY_OFF);
      if (is_in) dma16s(rwi, vo, soff, dst);
      else dma16s(rwq, vo, soff, dst);
    }
  };

  f32x4_t acc[2][FN];
  auto zero_acc = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[h][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  };
  // one stage: acc[nh] += W_stage (160 x 64) . A[:, 64 kb .. +64); `mid` runs between the halves
  auto mma_stage = [&](int slot, const uint4* af, int nh, auto mid) {
    const uint4* Ws = smem + slot * (STAGE_B / 16);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 1) {
        mid();
        __builtin_amdgcn_sched_barrier(0);
      }
      Frag8<bf16_t> wf[FN], xa;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = 16 * j + lr;
        wf[j].v = Ws[r * 8 + swz(r, 4 * ks + g)];
      }
      xa.v = af[ks];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if (MODE & 16) {                               // ablation: fragments read, no MFMA
          asm volatile("" ::"v"(wf[j].v.x), "v"(wf[j].v.w), "v"(xa.v.x));
          continue;
        }
        if (nh == 0) mma_k32(acc[0][j], wf[j], xa);
        else mma_k32(acc[1][j], wf[j], xa);
      }
      // LDS reads two fragments ahead of the MFMAs (ldm_feedforward's window)
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
      for (int j = 0; j < FN - 2; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if ((MODE & 4) && wv >= 4) __builtin_amdgcn_s_setprio(1);
  const int tiles = M / BM;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int m0 = tile * BM;
    const int bat = m0 / hw;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // previous tile done with LDS
#pragma unroll
    for (int s = 0; s < NSLOT - 1; ++s) issue(s);
    // ---- x rows of this wave (lane (g, lr): row 16 w + lr, channels 32 kc + 8 g .. + 7)
    const int mg = m0 + 16 * wave + lr;
    uint4 xf[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) xf[kc] = bload(rx, (mg * C + 32 * kc + 8 * g) * 2);
    // ---- GroupNorm (mean, rstd) of this batch from the producer's unit accumulators (gn_apply's
    //      reduction order), then per-channel scale / shift
    const int units = C / gunit, upg = (C / groups) / gunit;
    double2* ured = reinterpret_cast<double2*>(cst + OFF_URED);
    for (int i = tid; i < gslots * units; i += NT) {
      const int sl = i / units, uu = i - sl * units;
      ured[i] = *reinterpret_cast<const double2*>(gacc + (((int64_t)bat * gslots + sl) * units + uu) * 2);
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);       // x and the accumulators (compiler-visible vmcnt(0))
    __syncthreads();
    float2* gst = reinterpret_cast<float2*>(cst + OFF_GST);
    for (int gi = tid; gi < groups; gi += NT) {
      double sa = 0.0, sq = 0.0;
      for (int sl = 0; sl < gslots; ++sl)
        for (int k = 0; k < upg; ++k) {
          const double2 v = ured[sl * units + gi * upg + k];
          sa += v.x;
          sq += v.y;
        }
      const double cnt = (double)hw * (C / groups);
      const double mean = sa / cnt;
      double var = sq / cnt - mean * mean;
      if (var < 0.0) var = 0.0;
      gst[gi] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)geps)));
    }
    __syncthreads();
    for (int c = tid; c < C; c += NT) {
      const float2 ms = gst[c / (C / groups)];
      const float sc = ms.y * gamma[c];
      cst[OFF_SC + c] = sc;
      cst[OFF_SH + c] = fmaf(-ms.x, sc, beta[c]);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int c = 32 * kc + 8 * g;
      float v[8];
      unpack8(xf[kc], v);
      const float4 s0 = *reinterpret_cast<const float4*>(cst + OFF_SC + c);
      const float4 s1 = *reinterpret_cast<const float4*>(cst + OFF_SC + c + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(cst + OFF_SH + c);
      const float4 h1 = *reinterpret_cast<const float4*>(cst + OFF_SH + c + 4);
      v[0] = fmaf(v[0], s0.x, h0.x); v[1] = fmaf(v[1], s0.y, h0.y);
      v[2] = fmaf(v[2], s0.z, h0.z); v[3] = fmaf(v[3], s0.w, h0.w);
      v[4] = fmaf(v[4], s1.x, h1.x); v[5] = fmaf(v[5], s1.y, h1.y);
      v[6] = fmaf(v[6], s1.z, h1.z); v[7] = fmaf(v[7], s1.w, h1.w);
      xf[kc] = pack8(v);
    }

    // ---- proj_in: 10 stages
    zero_acc();
    const int ins = (MODE & 2) && wv >= 4 ? INS - 1 : INS;
#pragma unroll
    for (int s = 0; s < S_IN; ++s) {
      tin_wait(ins * (NSLOT - 2));
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (!(MODE & 1)) issue(s + NSLOT - 1);
      mma_stage(s % NSLOT, &xf[2 * (s >> 1)], s & 1, [&]() {
        if (MODE & 1) issue(s + NSLOT - 1);
      });
    }
    // ---- h = bf16(acc + b_in): to HBM (16-byte stores) and into the QKV A fragments; the
    //      LayerNorm row statistics in the row writer's order
    uint4 hf[KC];
    float ps[KC], pq2[KC];
    bf16_t* hout = reinterpret_cast<bf16_t*>(pi.out);
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
        const int n = SN * nh + 16 * j + 4 * g;
        const float4 ba = *reinterpret_cast<const float4*>(cst + OFF_BIN + n);
        const float4 bb = *reinterpret_cast<const float4*>(cst + OFF_BIN + n + 16);
        const uint2 a = make_uint2(pk2(acc[nh][j][0] + ba.x, acc[nh][j][1] + ba.y),
                                   pk2(acc[nh][j][2] + ba.z, acc[nh][j][3] + ba.w));
        const uint2 b = make_uint2(pk2(acc[nh][j + 1][0] + bb.x, acc[nh][j + 1][1] + bb.y),
                                   pk2(acc[nh][j + 1][2] + bb.z, acc[nh][j + 1][3] + bb.w));
        const int p = 5 * nh + j / 2;            // 32-column group
        hf[p] = d_pair_to_row8(a, b);
        *reinterpret_cast<uint4*>(hout + (int64_t)mg * C + 32 * p + 8 * g) = hf[p];
        float st[8];
        unpack8(hf[p], st);
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          s += st[k];
          q = fmaf(st[k], st[k], q);
        }
        ps[p] = s;
        pq2[p] = q;
      }
    // 8-channel chunk c of the row = group p = c / 4 of lane g = c % 4; per 160-column tile the
    // chunks are summed in order (fp32), the two tiles in fp64 (exact)
    double rsum = 0.0, rsq = 0.0;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int c = 20 * t; c < 20 * t + 20; ++c) {
        a += __shfl(ps[c >> 2], (c & 3) * 16 + lr, 64);
        b += __shfl(pq2[c >> 2], (c & 3) * 16 + lr, 64);
      }
      rsum += (double)a;
      rsq += (double)b;
    }
    const float2 rs = ln_row_from(rsum, rsq, pq.ln_inv_k, pq.ln_eps);

    // ---- QKV: three 320-column chunks
    bf16_t* qout = reinterpret_cast<bf16_t*>(pq.out);
    for (int q = 0; q < NCH; ++q) {
      const bool last = q + 1 == NCH;
      zero_acc();
#pragma unroll
      for (int u = 0; u < S_Q; ++u) {
        const int s = S_IN + S_Q * q + u;
        if (ins == INS) tin_wait(last ? tin_younger(u, true) : tin_younger(u, false));
        else tin_wait(last ? tin_younger(u, true, INS - 1) : tin_younger(u, false, INS - 1));
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (!(MODE & 1) && s + NSLOT - 1 < NST) issue(s + NSLOT - 1);
        mma_stage(s % NSLOT, &hf[2 * (u >> 1)], u & 1, [&]() {
          if ((MODE & 1) && s + NSLOT - 1 < NST) issue(s + NSLOT - 1);
        });
      }
      // rstd (acc - mean c1) + bias -> bf16 -> 16-byte row stores
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int j = 0; j < FN; j += 2) {
          const int n = C * q + SN * nh + 16 * j + 4 * g;
          const float4 ca = *reinterpret_cast<const float4*>(cst + OFF_C1 + n);
          const float4 cb = *reinterpret_cast<const float4*>(cst + OFF_C1 + n + 16);
          const float4 ba = *reinterpret_cast<const float4*>(cst + OFF_BQ + n);
          const float4 bb = *reinterpret_cast<const float4*>(cst + OFF_BQ + n + 16);
          const f32x4_t& x = acc[nh][j];
          const f32x4_t& y = acc[nh][j + 1];
          const uint2 a = make_uint2(pk2(fmaf(rs.y, ca.x, fmaf(rs.x, x[0], ba.x)), fmaf(rs.y, ca.y, fmaf(rs.x, x[1], ba.y))),
                                     pk2(fmaf(rs.y, ca.z, fmaf(rs.x, x[2], ba.z)), fmaf(rs.y, ca.w, fmaf(rs.x, x[3], ba.w))));
          const uint2 b = make_uint2(pk2(fmaf(rs.y, cb.x, fmaf(rs.x, y[0], bb.x)), fmaf(rs.y, cb.y, fmaf(rs.x, y[1], bb.y))),
                                     pk2(fmaf(rs.y, cb.z, fmaf(rs.x, y[2], bb.z)), fmaf(rs.y, cb.w, fmaf(rs.x, y[3], bb.w))));
          const int p = 5 * nh + j / 2;
          *reinterpret_cast<uint4*>(qout + (int64_t)mg * NQ + C * q + 32 * p + 8 * g) = d_pair_to_row8(a, b);
        }
    }
  }
}
}  // namespace

// ---------------------------------------------------------------------------------------
// host side
namespace {
int g_tin_mode = 1;   // tuning / A-B hook (ldm_transformer_in_set_mode)
}
extern "C" void ldm_transformer_in_set_mode(int mode) { g_tin_mode = mode; }

extern "C" int ldm_transformer_in(const ldm_gn_fold* gn, const ldm_conv_params* pin, const ldm_conv_params* qkv,
                                  ldm_stream_t stream) {
  using namespace tik;
  if (!gn || !pin || !qkv) return LDM_ERR_ARG;
  const auto a16 = [](const void* x) { return (reinterpret_cast<uintptr_t>(x) & 15) == 0; };
  const int64_t hw = (int64_t)pin->h_out * pin->w_out;
  const int64_t M = (int64_t)pin->batch * hw;
  if (pin->dtype != LDM_BF16 || qkv->dtype != LDM_BF16 || pin->ksize != 1 || qkv->ksize != 1 || pin->stride != 1 ||
      pin->upsample || pin->a1 || pin->c1 || pin->h_in != pin->h_out || pin->w_in != pin->w_out)
    return LDM_ERR_ARG;
  if (pin->c0 != C || pin->n != C || pin->kpad != C || qkv->n != NQ || qkv->kpad != C || qkv->c0 != C)
    return LDM_ERR_ARG;
  if (pin->out_layout != LDM_OUT_NHWC || qkv->out_layout != LDM_OUT_NHWC || pin->act != LDM_ACT_NONE ||
      qkv->act != LDM_ACT_NONE || pin->temb || qkv->temb || pin->residual || qkv->residual || pin->gn_partial ||
      qkv->gn_partial || pin->out_f32 || qkv->out_f32 || pin->ln_rows || !qkv->ln_c1 || qkv->ln_inv_k <= 0.f)
    return LDM_ERR_ARG;
  if ((int64_t)qkv->batch * qkv->h_out * qkv->w_out != M || hw % BM || M <= 0) return LDM_ERR_ARG;
  if (!gn->acc || !gn->gamma || !gn->beta || gn->groups <= 0 || gn->groups > 64 || C % gn->groups ||
      gn->unit <= 0 || (C / gn->groups) % gn->unit || gn->slots <= 0 || gn->slots * (C / gn->unit) > MAX_URED)
    return LDM_ERR_ARG;
  if (!pin->a0 || !pin->w || !qkv->w || !pin->out || !qkv->out) return LDM_ERR_ARG;
  if (!a16(pin->a0) || !a16(pin->w) || !a16(qkv->w) || !a16(pin->out) || !a16(qkv->out) || !a16(pin->bias) ||
      !a16(qkv->bias) || !a16(qkv->ln_c1) || !a16(gn->acc))
    return LDM_ERR_ALIGN;
  if (M * NQ * 2 >= (1LL << 31) - 64) return LDM_ERR_ARG;

  ConvArgs ai{}, aq{};
  ai.a0 = (const char*)pin->a0;
  ai.a0_bytes = (int)(M * C * 2);
  ai.w = (const char*)pin->w;
  ai.w_bytes = C * C * 2;
  ai.bias = pin->bias;
  ai.out = (char*)pin->out;
  ai.M = (int)M;
  ai.hw_out = (int)hw;
  aq.w = (const char*)qkv->w;
  aq.w_bytes = NQ * C * 2;
  aq.bias = qkv->bias;
  aq.ln_c1 = qkv->ln_c1;
  aq.ln_inv_k = qkv->ln_inv_k;
  aq.ln_eps = qkv->ln_eps;
  aq.out = (char*)qkv->out;
  const int tiles = (int)(M / BM);
  const int grid = tiles < 256 ? tiles : 256;
#define TIN_LAUNCH(m)                                                                                     \
  hipLaunchKernelGGL(transformer_in_kernel<m>, dim3(grid), dim3(NT), 0, (hipStream_t)stream, ai, aq, gn->acc, \
                     gn->unit, gn->slots, gn->groups, gn->eps, gn->gamma, gn->beta)
  switch (g_tin_mode) {
    case 0: TIN_LAUNCH(0); break;
    case 2: TIN_LAUNCH(2); break;
    case 9: TIN_LAUNCH(9); break;
    case 17: TIN_LAUNCH(17); break;
    default: TIN_LAUNCH(1); break;
  }
#undef TIN_LAUNCH
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
