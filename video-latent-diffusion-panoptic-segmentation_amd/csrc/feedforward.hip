// Fused transformer feed-forward: diffusers FeedForward(GEGLU) of the 64x64 UNet level
// (BasicTransformerBlock ff: ff.net.0 = GEGLU(C -> 2F), ff.net.2 = Linear(F -> C), + residual;
// reached via /root/reference/ldmseg/models/unet.py:361-425) in ONE kernel whose GEGLU
// intermediate never leaves the CU.
//
// Why: at C = 320, F = 1280, M = 32768 rows the unfused pair writes and re-reads an 84 MB
// [M][F] intermediate and runs as two launches (the A-register-stationary GEGLU ~95 us, the
// K = 1280 FF2 ~50 us; profiles/r03a_shape_breakdown.txt).  Here one 8-wave block per CU owns a
// 128-row tile for both GEMMs:
//   - the tile's rows x (the residual stream, LayerNorm norm3 folded as in ldm_conv2d's ln_rows
//     form) sit in VGPRs as MFMA fragments for the whole tile (16 rows x 320 K per wave);
//   - the hidden dimension is walked in 64-wide chunks: per chunk the 128 packed GEGLU columns
//     (64 hidden + 64 gate, 16-column interleave) are computed from 5 LDS stages of W1 (128 x 64),
//     h * gelu(g) is rounded to bf16 into a 16 KB LDS tile, and the FF2 accumulators (128 x 320
//     fp32 in VGPRs) take that tile times one 320 x 64 stage of W2;
//   - the weights stream by LDS-DMA through one chunk's worth of fixed stage regions (120 KB): a
//     stage is re-filled for the next chunk as soon as it is consumed, so five stages are in
//     flight (counted vmcnt, one raw barrier per stage); every CU streams the same weights, so
//     they come from its XCD's L2.
// Per chunk and tile: 15.7 MFLOP against 120 KB of weight stages (131 FLOP/B).
// Measured (tools/opbench.py ff_l0, M = 32768): 110 us against 136-140 us for the two launches;
// ablations: no weight loads 87 us, no GELU math 91 us — the GELU VALU (16 values per lane and
// chunk, all waves in the same phase) and the weight stream each still cost ~20 us over the
// ~32 us of MFMA work.  What it took (each step measured): the x rows' compiler-visible wait
// before the stage loop (without it hipcc put vmcnt(n) waits for them inside the loop, draining
// the weight stream every stage), DMA source offsets split into one lane VGPR + soffset, an
// opaque thread index for the row writer (its hoisted address arithmetic held ~100 VGPRs through
// the loop), and sched_group_barrier windows that keep LDS reads two fragments ahead of the
// MFMAs (the default schedule reused one register quad).  Packed-f32 GELU (v_pk_fma) and a
// 4-wave / 512-register form were measured slower (114, 160 us).
// Epilogue: bf16(acc + b2) staged once, then ldm_conv2d's PRE row writer (residual, row
// statistics) — the same rounding points and K order as the unfused ars GEGLU + tile FF2 pair
// (per output element the same MFMA instruction sequence), so the results agree bit for bit.
// Geometry: 512 threads = 8 waves.  GEGLU: 8 (M) x 1 (N), wave tile 16 rows x 128 packed columns
// (8 fragments; each wave holds only its own rows of x); FF2: 4 (M) x 2 (N), wave tile 32 rows x
// 160 columns (2 x 10 fragments: each W2 fragment read from LDS feeds two MFMAs); all
// v_mfma_f32_16x16x32_bf16 with D[n][m] = W . X^T (lane (g, lr): channels 4g..4g+3 of row lr).
#include "igemm_common.h"

namespace {
namespace ffk {
constexpr int NT = 512;
constexpr int BM = 128;                 // rows per tile
constexpr int C = 320;                  // model width: GEGLU K and FF2 N
constexpr int KC = C / 32;              // k32 fragments of a row of x (10)
constexpr int CH = 64;                  // hidden channels per chunk
constexpr int PW1 = 2 * CH;             // packed GEGLU columns per chunk (128)
constexpr int KS1 = C / 64;             // W1 stages per chunk (5)
constexpr int SPC = KS1 + 1;            // stages per chunk (5 x W1, 1 x W2)
constexpr int FM = 2;                   // FF2: 16-row fragments per wave (32 rows)
constexpr int FN1 = PW1 / 16;           // GEGLU: fragments per wave (all 128 packed columns: 8)
constexpr int FN2 = C / 2 / 16;         // FF2 fragments per wave (160 columns: 10)
constexpr int W1_B = PW1 * 128;         // a W1 stage: 128 packed rows x 64 K (16 KB)
constexpr int W2_B = C * 128;           // the W2 stage: 320 rows x 64 K (40 KB)
constexpr int W1_INS = PW1 / 8 / 8;     // DMA instructions per wave for a W1 stage (2)
constexpr int W2_INS = C / 8 / 8;       // ... for the W2 stage (5)
constexpr int CHUNK_INS = KS1 * W1_INS + W2_INS;
// a chunk's six stages have fixed LDS regions (the ring holds exactly one chunk): W1 stage st at
// st x 16 KB, W2 at 80 KB.  Stage (c + 1, st) is issued as soon as (c, st) is consumed, so five
// stages (~100 KB) are in flight while one is multiplied.
constexpr int H_OFF = KS1 * W1_B + W2_B;   // bf16 [128][64] GEGLU output tile (16 KB)
__host__ __device__ constexpr int stage_ins(int st) { return st < KS1 ? W1_INS : W2_INS; }
// DMA instructions a wave may leave in flight when it waits for stage st: every other stage of the
// stream except st - 1 (just consumed, re-issued after the barrier); in the last chunk only the
// stages after st (and (c, 5) is issued after the st = 0 wait)
__host__ __device__ constexpr int younger_steady(int st) {
  return CHUNK_INS - stage_ins(st) - stage_ins((st + SPC - 1) % SPC);
}
__host__ __device__ constexpr int younger_last(int st) {
  int n = 0;
  for (int s = st + 1; s < SPC; ++s) n += (st == 0 && s == SPC - 1) ? 0 : stage_ins(s);
  return n;
}
constexpr int COL_OFF = H_OFF + BM * 128;
constexpr int MAXF = 1280;              // hidden width bound: b1 and c1 ([2F] fp32 each) in LDS
constexpr int COL_END = COL_OFF + 2 * (2 * MAXF) * 4 + C * 4;   // + b2
// proj_out behind the feed-forward reuses all of it: five [128][64] h images (80 KB) + two
// 320 x 64 weight slots (80 KB)
constexpr int LDS_B = 160 * 1024;
static_assert(COL_END <= LDS_B && KS1 * BM * 128 + 2 * C * 128 <= LDS_B, "LDS");
constexpr int HP = C + 8;               // epilogue staging pitch (bf16)
static_assert(BM * HP * 2 + BM * (C / 8) * 2 * 4 <= COL_OFF, "epilogue staging exceeds the ring + H");
static_assert(BM * HP * 2 + gn_red_floats<NT, C, BM, 8>() * 4 <= LDS_B, "proj_out GroupNorm scratch exceeds LDS");
static_assert(LDS_B <= 160 * 1024, "LDS");
}  // namespace ffk

// s_waitcnt vmcnt(n) for the constant n of an unrolled stage (immediate operand)
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
static_assert(ffk::younger_steady(0) == 8 && ffk::younger_steady(1) == 11 && ffk::younger_steady(5) == 8 &&
              ffk::younger_last(0) == 8 && ffk::younger_last(2) == 9 && ffk::younger_last(4) == 5 &&
              ffk::younger_last(5) == 0, "vm_wait cases");

// Transformer2DModel.proj_out fused behind the feed-forward (ldm_feedforward with a third
// parameter block): the feed-forward's output rows h = bf16(bf16(acc + b2) + h_old) go straight
// into LDS as the A operand of proj_out (5 x [128 rows][64 K] swizzled images, 80 KB) instead of
// to HBM, then out = proj_out(h) + x_in over five 320 x 64 weight stages (two 40 KB slots), with
// ldm_conv2d's PRE row writer (residual, GroupNorm partials) — the same values and rounding
// points as the separate proj_out call on the stored h.
__device__ __forceinline__ void proj_out_tile(const ConvArgs& p2, const ConvArgs& p3, __amdgpu_buffer_rsrc_t rw3,
                                              int m0, f32x4_t (&acc)[ffk::FM][ffk::FN2], uint4* smem,
                                              unsigned lds0, int tid, int wv, int lane) {
  using namespace ffk;
  const int wave = tid >> 6, wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, g = lane >> 4;
  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ (((8 * wv + drow) >> 1) & 7);
  constexpr int HA_B = BM * 128;          // one [128][64] K image of h
  constexpr int SL0 = 0;                  // the two weight slots, then the five h images
  constexpr int HA0 = 2 * W2_B;
  const int vo3 = (drow * C + 8 * dchunk) * 2;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // every wave left the ring / H / columns
  // h = bf16(bf16(acc + b2) + h_old) into the A images (lane: channels n..n+3 of row ml)
  bf16_t* ha = reinterpret_cast<bf16_t*>(reinterpret_cast<char*>(smem) + HA0);
  const bf16_t* hold = reinterpret_cast<const bf16_t*>(p2.residual);
#pragma unroll
  for (int j = 0; j < FN2; ++j) {
    const int n = 160 * wn + 16 * j + 4 * g;
    const float4 b4 = p2.bias ? *reinterpret_cast<const float4*>(p2.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = 32 * wm + 16 * i + lr;
      const int m = m0 + ml;
      float r[4] = {0.f, 0.f, 0.f, 0.f};
      if (hold && m < p3.M) {
        const uint2 u = *reinterpret_cast<const uint2*>(hold + (int64_t)m * C + n);
        r[0] = __uint_as_float(u.x << 16); r[1] = __uint_as_float(u.x & 0xffff0000u);
        r[2] = __uint_as_float(u.y << 16); r[3] = __uint_as_float(u.y & 0xffff0000u);
      }
      bf16_t h[4];
      h[0] = f2bf(bf2f(f2bf(acc[i][j][0] + b4.x)) + r[0]);
      h[1] = f2bf(bf2f(f2bf(acc[i][j][1] + b4.y)) + r[1]);
      h[2] = f2bf(bf2f(f2bf(acc[i][j][2] + b4.z)) + r[2]);
      h[3] = f2bf(bf2f(f2bf(acc[i][j][3] + b4.w)) + r[3]);
      const int kst = n >> 6, ch = (n & 63) >> 3;
      *reinterpret_cast<uint2*>(ha + kst * (HA_B / 2) + ml * 64 + swz(ml, ch) * 8 + (n & 7)) =
          *reinterpret_cast<const uint2*>(h);
    }
  }
  auto issue = [&](int st) {   // proj_out weight stage st (K [64 st, +64)) into slot st & 1
    const unsigned base = lds0 + (unsigned)(SL0 + (st & 1) * W2_B);
#pragma unroll
    for (int i = 0; i < W2_INS; ++i) {
      const int qq = wv + 8 * i;
      dma16s(rw3, vo3, __builtin_amdgcn_readfirstlane((8 * qq * C + 64 * st) * 2),
             __builtin_amdgcn_readfirstlane(base + qq * 1024));
    }
  };
  issue(0);
  issue(1);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < KS1; ++st) {
    if (st + 1 < KS1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W2_INS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // stage st and every h image landed
    const uint4* Ws = smem + (SL0 + (st & 1) * W2_B) / 16;
    const uint4* Hs = smem + (HA0 + st * HA_B) / 16;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      Frag8<bf16_t> hf[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ml = 32 * wm + 16 * i + lr;
        hf[i].v = Hs[ml * 8 + swz(ml, 4 * ks + g)];
      }
#pragma unroll
      for (int j = 0; j < FN2; ++j) {
        const int r = 160 * wn + 16 * j + lr;
        Frag8<bf16_t> wf;
        wf.v = Ws[r * 8 + swz(r, 4 * ks + g)];
#pragma unroll
        for (int i = 0; i < FM; ++i) mma_k32(acc[i][j], wf, hf[i]);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
      for (int j = 0; j < FN2 - 1; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (st + 2 < KS1) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // every wave is done with slot st & 1
      issue(st + 2);
    }
  }
  // out = bf16(acc + b_po) staged over the h images, then the PRE row writer (residual x_in,
  // GroupNorm partials, 16-B row stores)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  bf16_t* stg = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
  for (int j = 0; j < FN2; ++j) {
    const int n = 160 * wn + 16 * j + 4 * g;
    const float4 b4 = p3.bias ? *reinterpret_cast<const float4*>(p3.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = 32 * wm + 16 * i + lr;
      bf16_t h[4] = {f2bf(acc[i][j][0] + b4.x), f2bf(acc[i][j][1] + b4.y), f2bf(acc[i][j][2] + b4.z),
                     f2bf(acc[i][j][3] + b4.w)};
      *reinterpret_cast<uint2*>(stg + ml * HP + n) = *reinterpret_cast<const uint2*>(h);
    }
  }
  __syncthreads();
  int tid_late = tid;
  asm volatile("" : "+v"(tid_late));
  epilogue_fast<BM, C, NT, true, false>(p3, m0, 0, stg, HP, reinterpret_cast<float*>(smem) + BM * HP / 2, tid_late);
  __syncthreads();
}

__global__ __launch_bounds__(512, 1) void feedforward_kernel(const ConvArgs g1, const ConvArgs p2, const ConvArgs p3) {
  using namespace ffk;
  __shared__ uint4 smem[LDS_B / 16];
  const int F = p2.kpad;                  // hidden width (FF2 K)
  const int NC = F / CH;                  // chunks
  const int M = g1.M;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ (((8 * wv + drow) >> 1) & 7);   // source-side swizzle (igemm)

  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)g1.a0, 0, g1.a0_bytes, kBufFlags);
  const __amdgpu_buffer_rsrc_t rw1 = __builtin_amdgcn_make_buffer_rsrc((void*)g1.w, 0, g1.w_bytes, kBufFlags);
  const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc((void*)p2.w, 0, p2.w_bytes, kBufFlags);
  bf16_t* const hs = reinterpret_cast<bf16_t*>(reinterpret_cast<char*>(smem) + H_OFF);
  float* const sb1 = reinterpret_cast<float*>(reinterpret_cast<char*>(smem) + COL_OFF);
  float* const sc1 = sb1 + 2 * MAXF;
  float* const sb2 = sc1 + 2 * MAXF;

  // the GEGLU column constants (packed bias, LayerNorm-fold column sums) in LDS: a global load
  // inside the stage loop would make hipcc drain the weight stream (vmcnt(0)) before its use.
  // Staged per tile when the proj_out stages overwrite them after the chunk loop.
  auto stage_cols = [&]() {
    for (int i = tid; i < g1.n; i += NT) {
      sb1[i] = g1.bias ? g1.bias[i] : 0.f;
      sc1[i] = g1.ln_rows ? g1.ln_c1[i] : 0.f;
    }
    for (int i = tid; i < C; i += NT) sb2[i] = p2.bias ? p2.bias[i] : 0.f;
  };
  const bool po = p3.w != nullptr;
  const __amdgpu_buffer_rsrc_t rw3 = __builtin_amdgcn_make_buffer_rsrc((void*)(po ? p3.w : p2.w), 0, po ? p3.w_bytes : 0, kBufFlags);
  if (!po) stage_cols();

  const int vo1 = (drow * g1.kpad + 8 * dchunk) * 2, vo2 = (drow * F + 8 * dchunk) * 2;
  // stage st of chunk c: W1 K stage st (< 5) or the W2 stage (5), into its fixed LDS region
  auto issue = [&](int c, int st) {
#ifdef LDM_ABL_NO_LOADS   // ablation build: weights never fetched (LDS holds stale data)
    return;
#endif
    const unsigned base = lds0 + (unsigned)(st * W1_B);
    // lane part of the source offset (row drow of a DMA instruction's 8, swizzled chunk) in one
    // loop-invariant VGPR, the instruction's rows / K stage / chunk in soffset
    if (st < KS1) {
#pragma unroll
      for (int i = 0; i < W1_INS; ++i) {
        const int qq = wv + 8 * i;
        dma16s(rw1, vo1, __builtin_amdgcn_readfirstlane(((PW1 * c + 8 * qq) * g1.kpad + 64 * st) * 2),
               __builtin_amdgcn_readfirstlane(base + qq * 1024));
      }
    } else {
#pragma unroll
      for (int i = 0; i < W2_INS; ++i) {
        const int qq = wv + 8 * i;
        dma16s(rw2, vo2, __builtin_amdgcn_readfirstlane((8 * qq * F + CH * c) * 2),
               __builtin_amdgcn_readfirstlane(base + qq * 1024));
      }
    }
  };

  const int tiles = (M + BM - 1) / BM;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int m0 = tile * BM;
    if (po) stage_cols();   // (ordered before its first use by the stage loop's barriers)
    // the first chunk's W1 stages fly while x and the LayerNorm rows load
#pragma unroll
    for (int st = 0; st < KS1; ++st) issue(0, st);
    // ---- GEGLU rows of this wave: 16 wave + lr; x fragments: lane (g, lr) holds
    //      x[row][32 kc + 8 g, +8) (40 VGPRs: the GEGLU runs 8 (M) x 1 (N) so no row is held twice)
    const int mg = m0 + 16 * wave + lr;
    uint4 xf[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) xf[kc] = bload(rx, mg < M ? (mg * C + 32 * kc + 8 * g) * 2 : kOOB);
    const float2 lnr = (g1.ln_rows && mg < M) ? ln_row(g1, mg) : make_float2(1.f, 0.f);
    f32x4_t acc2[FM][FN2];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN2; ++j) acc2[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    f32x4_t acc1[FN1];
    // a wait hipcc can see: its waitcnt model does not count the asm LDS-DMA, so with x still
    // "pending" it would put vmcnt(n) waits before the x fragments' uses inside the stage loop —
    // draining the weight stream every stage.  One full wait per tile instead (vmcnt(0)).
    __builtin_amdgcn_s_waitcnt(0x0f70);
    for (int c = 0; c < NC; ++c) {
      const bool last = c + 1 == NC;
#pragma unroll
      for (int st = 0; st < SPC; ++st) {          // compile-time stage: x fragments by constant index
        // stage (c, st) landed for this wave, then every wave's part (and (c, st - 1) is consumed)
        vm_wait(last ? younger_last(st) : younger_steady(st));
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (st == 0) issue(c, SPC - 1);
        else if (!last) issue(c + 1, st - 1);
        const uint4* Ws = smem + st * (W1_B / 16);
        if (st < KS1) {
          if (st == 0) {
#pragma unroll
            for (int j = 0; j < FN1; ++j) acc1[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            Frag8<bf16_t> wf[FN1], xa;        // all of the step's W fragments in flight at once
#pragma unroll
            for (int j = 0; j < FN1; ++j) {
              const int r = 16 * j + lr;
              wf[j].v = Ws[r * 8 + swz(r, 4 * ks + g)];
            }
            xa.v = xf[2 * st + ks];
#pragma unroll
            for (int j = 0; j < FN1; ++j) {
#ifdef LDM_ABL_NO_MFMA   // ablation build: fragments read, no MFMA issued
              asm volatile("" ::"v"(wf[j].v.x), "v"(wf[j].v.w), "v"(xa.v.x));
              continue;
#endif
              mma_k32(acc1[j], wf[j], xa);
            }
            // a sliding window of LDS reads two fragments ahead of the MFMAs (the default schedule
            // reuses one register quad: every MFMA then waits out its ds_read)
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
            for (int j = 0; j < FN1 - 2; ++j) {
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
          if (st == KS1 - 1) {
            // h * gelu(g) (LayerNorm fold: rstd (acc - mean c1) + bias) -> bf16 H tile; fragments j
            // (hidden) and j + 1 (gate) hold the same 4 channels of the same row in one lane
#pragma unroll
            for (int j = 0; j < FN1; j += 2) {
              const int pc = PW1 * c + 16 * j + 4 * g;   // packed column
              const int hl = 8 * j + 4 * g;              // hidden column in the chunk
              const float4 bh = *reinterpret_cast<const float4*>(sb1 + pc);
              const float4 bg = *reinterpret_cast<const float4*>(sb1 + pc + 16);
              const float4 ch = *reinterpret_cast<const float4*>(sc1 + pc);
              const float4 cg = *reinterpret_cast<const float4*>(sc1 + pc + 16);
              const float bhv[4] = {bh.x, bh.y, bh.z, bh.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
              const float chv[4] = {ch.x, ch.y, ch.z, ch.w}, cgv[4] = {cg.x, cg.y, cg.z, cg.w};
              const int ml = 16 * wave + lr;
              bf16_t h[4];
#pragma unroll
              for (int k = 0; k < 4; ++k) {
#ifdef LDM_ABL_NO_GELU   // ablation build: the GEGLU epilogue's math replaced by one multiply-add
                h[k] = f2bf(acc1[j][k] * acc1[j + 1][k] + bhv[k] + cgv[k]);
#else
                h[k] = f2bf(fmaf(lnr.y, chv[k], fmaf(lnr.x, acc1[j][k], bhv[k])) *
                            gelu_f(fmaf(lnr.y, cgv[k], fmaf(lnr.x, acc1[j + 1][k], bgv[k]))));
#endif
              }
              *reinterpret_cast<uint2*>(hs + ml * 64 + swz(ml, hl >> 3) * 8 + (hl & 7)) =
                  *reinterpret_cast<const uint2*>(h);
            }
          }
        } else {
          // FF2: acc2 += H (128 x 64) . W2[:, 64 c, +64)^T
          const uint4* Hs = reinterpret_cast<const uint4*>(hs);
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            Frag8<bf16_t> ha[FM];
#pragma unroll
            for (int i = 0; i < FM; ++i) {
              const int ml = 32 * wm + 16 * i + lr;
              ha[i].v = Hs[ml * 8 + swz(ml, 4 * ks + g)];
            }
#pragma unroll
            for (int j = 0; j < FN2; ++j) {
              const int r = 160 * wn + 16 * j + lr;
              Frag8<bf16_t> wf;
              wf.v = Ws[r * 8 + swz(r, 4 * ks + g)];
#ifdef LDM_ABL_NO_MFMA
              asm volatile("" ::"v"(wf.v.x), "v"(wf.v.w), "v"(ha[0].v.x), "v"(ha[1].v.y));
              continue;
#endif
#pragma unroll
              for (int i = 0; i < FM; ++i) mma_k32(acc2[i][j], wf, ha[i]);
            }
            // H fragments and one W fragment ahead, then one W read per MFMA pair
            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
            for (int j = 0; j < FN2 - 1; ++j) {
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            // keep the next k32 step's fragment reads from being hoisted beside this step's
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    }

    if (po) {
      proj_out_tile(p2, p3, rw3, m0, acc2, smem, lds0, tid, wv, lane);
      continue;
    }
    // ---- epilogue: bf16(acc + b2) staged over the ring, then the PRE row writer (residual, row
    //      statistics, 16-B row stores)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // every wave left the ring / H
    bf16_t* stg = reinterpret_cast<bf16_t*>(smem);
#pragma unroll
    for (int j = 0; j < FN2; ++j) {
      const int n = 160 * wn + 16 * j + 4 * g;
      const float4 b4 = *reinterpret_cast<const float4*>(sb2 + n);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ml = 32 * wm + 16 * i + lr;
        bf16_t h[4] = {f2bf(acc2[i][j][0] + b4.x), f2bf(acc2[i][j][1] + b4.y), f2bf(acc2[i][j][2] + b4.z),
                       f2bf(acc2[i][j][3] + b4.w)};
        *reinterpret_cast<uint2*>(stg + ml * HP + n) = *reinterpret_cast<const uint2*>(h);
      }
    }
    __syncthreads();
    // the row writer sees an opaque copy of the thread index: otherwise its per-thread address
    // arithmetic is hoisted above the stage loop and held in VGPRs through it, leaving no room to
    // keep a step's W fragments in flight
    int tid_late = tid;
    asm volatile("" : "+v"(tid_late));
    epilogue_fast<BM, C, NT, true, false>(p2, m0, 0, stg, HP, reinterpret_cast<float*>(smem) + BM * HP / 2, tid_late);
    __syncthreads();   // the next tile's x loads / stages reuse LDS
  }
}
}  // namespace

// ---------------------------------------------------------------------------------------
// host side
extern "C" int ldm_feedforward(const ldm_conv_params* g, const ldm_conv_params* f, const ldm_conv_params* po,
                               ldm_stream_t stream) {
  using namespace ffk;
  if (!g || !f) return LDM_ERR_ARG;
  const auto a16 = [](const void* x) { return (reinterpret_cast<uintptr_t>(x) & 15) == 0; };
  const int64_t M = (int64_t)g->batch * g->h_out * g->w_out;
  const int F = f->kpad;
  if (g->dtype != LDM_BF16 || f->dtype != LDM_BF16 || g->ksize != 1 || f->ksize != 1 || g->stride != 1 ||
      f->stride != 1 || g->upsample || f->upsample || g->a1 || g->c1 || f->c1)
    return LDM_ERR_ARG;
  if (g->c0 != C || g->kpad != C || f->n != C || g->out_layout != LDM_OUT_GEGLU || f->out_layout != LDM_OUT_NHWC)
    return LDM_ERR_ARG;
  if (F % CH || F > MAXF || g->n != 2 * F || f->c0 != F) return LDM_ERR_ARG;
  if ((int64_t)f->batch * f->h_out * f->w_out != M || g->h_out != g->h_in || g->w_out != g->w_in) return LDM_ERR_ARG;
  if (g->act != LDM_ACT_NONE || f->act != LDM_ACT_NONE || g->temb || f->temb || g->residual || g->row_stats ||
      g->gn_partial || f->gn_partial || f->ln_rows || g->out_f32 || f->out_f32)
    return LDM_ERR_ARG;
  if (g->ln_rows && !g->ln_c1) return LDM_ERR_ARG;
  if (!g->a0 || !g->w || !f->w || (!f->out && !po)) return LDM_ERR_ARG;
  if (po) {   // proj_out behind the feed-forward: h is not stored
    if (po->dtype != LDM_BF16 || po->ksize != 1 || po->stride != 1 || po->upsample || po->a1 || po->c1 ||
        po->c0 != C || po->n != C || po->kpad != C || po->out_layout != LDM_OUT_NHWC || po->act != LDM_ACT_NONE ||
        po->temb || po->row_stats || po->ln_rows || po->out_f32 || !po->w || !po->out || f->row_stats ||
        (int64_t)po->batch * po->h_out * po->w_out != M)
      return LDM_ERR_ARG;
    if (po->gn_partial && ((po->h_out * po->w_out) % 64 || C % (po->gn_unit > 0 ? po->gn_unit : 1)))
      return LDM_ERR_ARG;
    if (!a16(po->w) || !a16(po->out) || !a16(po->residual) || !a16(po->bias)) return LDM_ERR_ALIGN;
  }
  if (!a16(g->a0) || !a16(g->w) || !a16(f->w) || !a16(f->out) || !a16(f->residual) || !a16(f->bias) ||
      !a16(f->row_stats) || (g->ln_rows && !a16(g->ln_rows)))
    return LDM_ERR_ALIGN;
  if (M <= 0) return LDM_OK;
  if (M * C * 2 >= (1LL << 31) - 64 || M * 16 >= (1LL << 31)) return LDM_ERR_ARG;

  ConvArgs a1{}, a2{};
  a1.a0 = (const char*)g->a0;
  a1.a0_bytes = (int)(M * C * 2);
  a1.c0 = C;
  a1.w = (const char*)g->w;
  a1.w_bytes = (int)((int64_t)g->n * g->kpad * 2);
  a1.n = g->n;
  a1.kpad = g->kpad;
  a1.bias = g->bias;
  a1.ln_rows = g->ln_rows;
  a1.ln_c1 = g->ln_c1;
  a1.ln_inv_k = g->ln_inv_k;
  a1.ln_eps = g->ln_eps;
  a1.M = (int)M;
  a2.w = (const char*)f->w;
  a2.w_bytes = (int)((int64_t)C * F * 2);
  a2.n = C;
  a2.kpad = F;
  a2.bias = f->bias;
  a2.residual = (const char*)f->residual;
  a2.out = (char*)f->out;
  a2.out_layout = LDM_OUT_NHWC;
  a2.act = LDM_ACT_NONE;
  a2.row_stats = f->row_stats;
  a2.M = (int)M;
  a2.hw_out = (int)M;
  a2.ksplit = 1;
  const int tiles = (int)((M + BM - 1) / BM);
  const int grid = tiles < 256 ? tiles : 256;
  ConvArgs a3{};
  if (po) {
    a3.w = (const char*)po->w;
    a3.w_bytes = C * C * 2;
    a3.n = C;
    a3.kpad = C;
    a3.bias = po->bias;
    a3.residual = (const char*)po->residual;
    a3.out = (char*)po->out;
    a3.out_layout = LDM_OUT_NHWC;
    a3.act = LDM_ACT_NONE;
    a3.M = (int)M;
    a3.hw_out = po->h_out * po->w_out;
    a3.ksplit = 1;
    a3.gn_part = po->gn_partial;
    a3.gn_unit = po->gn_unit > 0 ? po->gn_unit : 1;
    a3.gn_slots = po->gn_slots > 0 ? po->gn_slots : 1;
  }
  hipLaunchKernelGGL(feedforward_kernel, dim3(grid), dim3(NT), 0, (hipStream_t)stream, a1, a2, a3);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
