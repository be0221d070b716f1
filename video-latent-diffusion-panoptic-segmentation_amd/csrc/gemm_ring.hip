// Deep-ring 1x1 GEMM for the UNet's 16x16 / 8x8 / mid levels (M = 2048 / 512 rows at B = 8):
// Transformer2DModel proj_in / to_out / proj_out, the norm1-folded QKV, ff.net.2, the up-block
// 1x1 shortcuts (/root/reference/ldmseg/models/unet.py:361-425 down_blocks[2..3], mid, up_blocks[0..1]).
// Its own translation unit on the shared igemm helpers (igemm_common.h); ldm_conv2d (igemm.hip)
// dispatches to it through ldm_igemm::ring_cfg / launch_ring.
//
// Why: at these levels a GEMM has 160-640 tiles of the two-blocks-per-CU kernels, walks K = 1280-5120
// serially and keeps ONE K tile in flight per block, so every K step waits out the LDS-DMA latency
// (~1 us under load: proj 1280 at 16x16 25 us for 20 K steps; hipBLASLt takes 21 us on the same
// shape).  Here a block owns one tile of a grid sized to the 256 CUs (128x80 at M = 2048, 32x80 at
// M = 512, ...), walks all of K (no split-K slab) and keeps AHEAD + 1 K steps of operands in flight
// in an NSLOT-deep LDS ring (MI355X_MICROARCH.md "ring-gemm": ~68 GB/s per CU with three K steps in
// flight).
//
// Roles (one block per CU): NL = 4 loader waves issue the LDS-DMA of every K step (A rows then B rows,
// 128 B per operand row, the igemm XOR swizzle applied on the source side) and publish a slot with a
// per-wave FULL word in LDS behind a counted vmcnt that leaves AHEAD younger steps in flight; NC
// consumer waves (CWM x CWN wave tiles of 16x16x32 bf16 MFMA fragments, D[n][m] = W . A^T as in
// igemm) wait for the four FULL words, read both k32 halves of their fragments, release the slot with
// a per-wave FREE word and multiply.  No block barrier inside the K loop.
// Epilogue (all waves): the accumulators pass through the igemm bf16 pre-activation staging (bias,
// LayerNorm fold, activation) into the freed ring and leave through epilogue_fast (residual, 16-B row
// stores, GroupNorm partials, LayerNorm row statistics); GEGLU stores h * gelu(g) straight from the
// accumulator pairs (the 16-column hidden / gate interleave of the packed weight).
#include "igemm_common.h"

namespace {
namespace ring {
constexpr int NL = 4;          // loader waves
constexpr int KS = 64;         // K per step (128 B per operand row)
constexpr int FLAG_INTS = 128; // FULL [NSLOT][8] at 0 and FREE [NSLOT][8] at 64 (NSLOT, NL, NC <= 8)
}  // namespace ring

// vmcnt(n * PER) for a runtime n in [0, N]: one compile-time immediate per case
template <int PER, int N>
__device__ __forceinline__ void wait_steps(int n) {
  static_assert(N * PER <= 63, "vmcnt range");
  if constexpr (N == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (n >= N) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N * PER) : "memory");
    else wait_steps<PER, N - 1>(n);
  }
}

// ring flag words (LDS byte address): one ds_read_b128 of four consecutive words with its own
// lgkmcnt wait, a single ds_write_b32 without one
__device__ __forceinline__ int4 lds_flag_ld4(unsigned addr) {
  int4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
__device__ __forceinline__ bool all_at_least(int4 v, int n, int need) {
  return v.x >= need && (n < 2 || v.y >= need) && (n < 3 || v.z >= need) && (n < 4 || v.w >= need);
}
__device__ __forceinline__ void lds_flag_st(unsigned addr, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

template <int BM, int BN, int CWM, int CWN, int NSLOT, int AHEAD, bool GEGLU>
__global__ __launch_bounds__(64 * (ring::NL + CWM * CWN), 1) void gemm_ring_kernel(const ConvArgs p) {
  using namespace ring;
  constexpr int NC = CWM * CWN;
  constexpr int NT = 64 * (NL + NC);
  constexpr int WM = BM / CWM, WN = BN / CWN;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && BM % 8 == 0 && BN % 8 == 0, "tile");
  static_assert(NSLOT <= 8 && NC <= 8 && AHEAD + 2 <= NSLOT, "ring");
  constexpr int SLOT_U4 = (BM + BN) * 8;                 // uint4 per slot
  constexpr int NI = (BM + BN) / 8;                      // 1-KB DMA instructions per step
  constexpr int PER = (NI + NL - 1) / NL;                // per loader wave (padded with dummies)
  constexpr int HP = BN + 8;                             // bf16 staging pitch
  constexpr int RING_U4 = NSLOT * SLOT_U4;
  constexpr int STAGE_U4 = (BM * HP * 2 + 15) / 16;
  constexpr int RED_U4 = (gn_red_floats<NT, BN, BM, 8>() * 4 + 15) / 16;
  constexpr int MAIN_U4 = RING_U4 > STAGE_U4 ? (RING_U4 > RED_U4 ? RING_U4 : RED_U4) : (STAGE_U4 > RED_U4 ? STAGE_U4 : RED_U4);
  __shared__ uint4 smem[MAIN_U4 + FLAG_INTS / 4 + 64];   // + flags + 1 KB dummy DMA target
  int* flags = reinterpret_cast<int*>(smem + MAIN_U4);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, g = lane >> 4;

  // tile: XCD-contiguous ids (blocks b and b + 8 share an XCD), grouped raster over M panels; with
  // split K (ksplit > 1) a tile's splits are adjacent ids and each walks its own range of K steps
  int tm, tn, split;
  {
    const int nblk = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    int tile = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
    split = tile % p.ksplit;
    tile /= p.ksplit;
    grouped_tile(tile, (p.M + BM - 1) / BM, p.tiles_n, p.group_m, tm, tn);
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nsteps_all = p.kpad / KS;
  const int s0 = nsteps_all * split / p.ksplit;
  const int nsteps = nsteps_all * (split + 1) / p.ksplit - s0;   // this block's K steps

  if (tid < FLAG_INTS) flags[tid] = 0;
  __syncthreads();

  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  // FULL [NSLOT][8] / FREE [NSLOT][8] words, accessed by ds_read_b32 / ds_write_b32 in inline asm: a
  // volatile generic pointer compiles to flat loads, which count on vmcnt and made every poll drain
  // the loader's DMA stream
  const unsigned full0 = lds0 + (unsigned)(MAIN_U4 * 16), free0 = full0 + 64 * 4;
  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (wave < NL) {
    // ------------------------------------------------------------------ loader waves
    const int lw = wave;
    const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)p.a0, 0, p.a0_bytes, kBufFlags);
    const __amdgpu_buffer_rsrc_t ra1 =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.a1 ? p.a1 : p.a0), 0, p.a1 ? p.a1_bytes : 0, kBufFlags);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, p.w_bytes, kBufFlags);
    const unsigned dummy = lds0 + (unsigned)((MAIN_U4 + FLAG_INTS / 4) * 16);
    // lane geometry of one 8-row x 128-B instruction: row 8q + drow, LDS chunk position lane & 7
    // holding logical chunk (lane & 7) ^ ((row >> 1) & 7); q = lw + NL i has the parity of lw, so
    // the swizzle term (4q + (drow >> 1)) & 7 is fixed per wave
    const int drow = lane >> 3;
    const int dchunk = (lane & 7) ^ ((4 * lw + (drow >> 1)) & 7);
    // this lane's A rows (instruction i: row 8 q + drow, q = lw + NL i < BM / 8): the input pixel of
    // tap (0, 0) (negative in the padding is fine: only in-image taps are fetched) and a bit per
    // in-image tap; a 1x1 GEMM has the row itself and one tap
    const bool conv = p.ksize > 1;
    int apix[PER];
    unsigned amsk[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int q = lw + NL * i;
      const int m = m0 + 8 * q + drow;
      apix[i] = 0;
      amsk[i] = 0u;
      if (8 * q < BM && m < p.M) {
        if (conv) {
          const int b = m / p.hw_out, pix = m - b * p.hw_out;
          const int oy = pix / p.w_out, ox = pix - oy * p.w_out;
          const int iy0 = oy * p.stride - p.pad, ix0 = ox * p.stride - p.pad;
          apix[i] = (b * p.h_in + iy0) * p.w_in + ix0;
          unsigned msk = 0u;
          for (int ky = 0; ky < p.ksize; ++ky)
            for (int kx = 0; kx < p.ksize; ++kx)
              if ((unsigned)(iy0 + ky) < (unsigned)p.h_in && (unsigned)(ix0 + kx) < (unsigned)p.w_in)
                msk |= 1u << (ky * p.ksize + kx);
          amsk[i] = msk;
        } else {
          apix[i] = m;
          amsk[i] = 1u;
        }
      }
    }
    // wave-uniform K position of step s0 + s: K is tap-major and a 64-deep step lies in one tap
    int ch = (s0 * KS) % p.cin, tap = (s0 * KS) / p.cin;
    int ky = tap / p.ksize, kx = tap - ky * p.ksize;
    for (int s = 0; s < nsteps + AHEAD; ++s) {
      if (s < nsteps) {
        const int slot = s % NSLOT;
        if (s >= NSLOT) {            // the consumers released step s - NSLOT from this slot
          const int need = s - NSLOT + 1;
          while (!all_at_least(lds_flag_ld4(free0 + slot * 32), NC, need) ||
                 (NC > 4 && !all_at_least(lds_flag_ld4(free0 + slot * 32 + 16), NC - 4, need)))
            __builtin_amdgcn_s_sleep(1);
        }
        const unsigned sbase = lds0 + (unsigned)(slot * SLOT_U4 * 16);
        const int k0 = (s0 + s) * KS;
        const int sel = __builtin_amdgcn_readfirstlane((p.c1 > 0 && ch >= p.c0) ? 1 : 0);   // step-aligned concat
        const int cs = sel ? p.c1 : p.c0;
        const int choff = (sel ? ch - p.c0 : ch) + dchunk * 8;
        const int tapoff = ky * p.w_in + kx;
        const unsigned tbit = 1u << tap;
        const __amdgpu_buffer_rsrc_t ra = sel ? ra1 : ra0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
          if (p.abl == 2) break;                               // ablation: no operand DMA
          const int q = lw + NL * i;
          if (q < NI) {
            const unsigned dst = __builtin_amdgcn_readfirstlane(sbase + (unsigned)(q * 1024));
            const int r = 8 * q + drow;
            if (8 * q < BM) {
              const int off = (amsk[i] & tbit) ? ((apix[i] + tapoff) * cs + choff) * 2 : kOOB;
              dma16(ra, off, dst);
            } else {
              const int n = n0 + r - BM;
              const int off = n < p.n ? (n * p.kpad + k0 + dchunk * 8) * 2 : kOOB;
              dma16(rw, off, dst);
            }
          } else {
            dma16(rw, kOOB, __builtin_amdgcn_readfirstlane(dummy));   // keeps PER instructions per step
          }
        }
        ch += KS;
        if (ch == p.cin) {
          ch = 0;
          ++tap;
          if (++kx == p.ksize) { kx = 0; ++ky; }
        }
      }
      const int t = s - AHEAD;
      if (t >= 0) {
        const int younger = min(AHEAD, nsteps - 1 - t);       // steps issued after t
        wait_steps<PER, AHEAD>(younger);
        lds_flag_st(full0 + ((t % NSLOT) * 8 + lw) * 4, t + 1);   // this wave's share of step t landed
      }
    }
  } else {
    // ------------------------------------------------------------------ consumer waves
    // Software-pipelined: step t + 1's FULL poll and fragment reads are issued between the two k32
    // halves of step t's MFMAs (sched_barrier-pinned), so the LDS round trips hide under the matrix
    // pipe instead of idling it (one consumer wave per SIMD has no partner wave to overlap with).
    const int cw = wave - NL;
    const int cwm = cw / CWN, cwn = cw - cwm * CWN;
    const int sl = (lr >> 1) & 7;
    Frag8<bf16_t> af[2][2][FM], bfr[2][2][FN];               // [buffer][k32 half][fragment]
    auto fetch = [&](int t, int b) {
      const int slot = t % NSLOT;
      if (p.abl != 2)
        while (!all_at_least(lds_flag_ld4(full0 + slot * 32), NL, t + 1)) __builtin_amdgcn_s_sleep(0);
      asm volatile("" ::: "memory");
      // row r = base + 16 f + lr: swz(r, c) = c ^ ((lr >> 1) & 7) for every fragment
      const uint4* As = smem + slot * SLOT_U4 + (cwm * WM + lr) * 8;
      const uint4* Bs = smem + slot * SLOT_U4 + BM * 8 + (cwn * WN + lr) * 8;
      if (p.abl == 1) return;                                  // ablation: no fragment reads / MFMA
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cch = (ks * 4 + g) ^ sl;
#pragma unroll
        for (int i = 0; i < FM; ++i) af[b][ks][i].v = As[i * 128 + cch];
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[b][ks][j].v = Bs[j * 128 + cch];
      }
    };
    auto release = [&](int t) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lds_flag_st(free0 + ((t % NSLOT) * 8 + cw) * 4, t + 1); // fragments in registers: slot free
    };
    auto mma_half = [&](int b, int ks) {
      if (p.abl == 1) return;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i) mma_k32(acc[i][j], bfr[b][ks][j], af[b][ks][i]);
    };
    fetch(0, 0);
    release(0);
    for (int t = 0; t < nsteps; t += 2) {
      // buffer 0 holds step t; buffer 1 receives step t + 1 (and the reverse for the odd half)
      mma_half(0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < nsteps) fetch(t + 1, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma_half(0, 1);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 >= nsteps) break;
      release(t + 1);
      mma_half(1, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < nsteps) fetch(t + 2, 0);
      __builtin_amdgcn_sched_barrier(0);
      mma_half(1, 1);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < nsteps) release(t + 2);
    }
  }
  __syncthreads();                                             // ring drained: LDS is the staging area

  if (p.ksplit > 1) {
    // split K: the raw fp32 tile -> LDS [BM][BN + 4] -> this split's slab as full rows (the
    // reduction kernel applies bias, time embedding, activation, residual and statistics)
    constexpr int PITCH = BN + 4;
    static_assert(BM * PITCH <= MAIN_U4 * 4, "fp32 stage exceeds the ring");
    float* stage = reinterpret_cast<float*>(smem);
    if (wave >= NL) {
      const int cw = wave - NL;
      const int cwm = cw / CWN, cwn = cw - cwm * CWN;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          *reinterpret_cast<float4*>(stage + (cwm * WM + i * 16 + lr) * PITCH + cwn * WN + j * 16 + 4 * g) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
    __syncthreads();
    write_partial_rows<BM, BN, NT>(p, p.partial + (int64_t)split * p.M * p.n, m0, n0, stage, PITCH);
    return;
  }

  if constexpr (GEGLU) {
    // h * gelu(g) from the accumulators: fragments j (hidden) and j + 1 (gate) hold the two halves of
    // the same 4 output channels of the same pixel in one lane (16-column interleave, WN % 32 == 0)
    static_assert(FN % 2 == 0 && WN % 32 == 0, "GEGLU pairs");
    if (wave < NL) return;
    const int cw = wave - NL;
    const int cwm = cw / CWN, cwn = cw - cwm * CWN;
    const int NO = p.n >> 1;
    float2 lnr[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + cwm * WM + i * 16 + lr;
      lnr[i] = (p.ln_rows && m < p.M) ? ln_row(p, m) : make_float2(1.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < FN; j += 2) {
      const int pc = n0 + cwn * WN + j * 16 + 4 * g;            // packed column of the hidden values
      if (pc >= p.n) continue;
      const int oc = (pc >> 5) * 16 + (pc & 15);                // output channel
      float bh[4], bg[4], ch[4], cg[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bh[r] = p.bias ? p.bias[pc + r] : 0.f;
        bg[r] = p.bias ? p.bias[pc + 16 + r] : 0.f;
        ch[r] = p.ln_rows ? p.ln_c1[pc + r] : 0.f;
        cg[r] = p.ln_rows ? p.ln_c1[pc + 16 + r] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + cwm * WM + i * 16 + lr;
        if (m >= p.M) continue;
        float v[4];
        const float2 rs = lnr[i];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          v[r] = fmaf(rs.y, ch[r], fmaf(rs.x, acc[i][j][r], bh[r])) *
                 gelu_f(fmaf(rs.y, cg[r], fmaf(rs.x, acc[i][j + 1][r], bg[r])));
        store4<bf16_t>(p.out, (int64_t)m * NO + oc, v, false);
      }
    }
  } else {
    // bias, LayerNorm fold and activation from the accumulators, staged once as bf16 [BM][HP]
    bf16_t* hs = reinterpret_cast<bf16_t*>(smem);
    if (wave >= NL) {
      const int cw = wave - NL;
      const int cwm = cw / CWN, cwn = cw - cwm * CWN;
      float2 lnr[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + cwm * WM + i * 16 + lr;
        lnr[i] = (p.ln_rows && m < p.M) ? ln_row(p, m) : make_float2(1.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int nl = cwn * WN + j * 16 + 4 * g;
        const int n = n0 + nl;
        float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f), c4 = b4;
        if (p.bias && n < p.n) b4 = *reinterpret_cast<const float4*>(p.bias + n);
        if (p.ln_rows && n < p.n) c4 = *reinterpret_cast<const float4*>(p.ln_c1 + n);
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int ml = cwm * WM + i * 16 + lr;
          const int m = m0 + ml;
          float v[4] = {acc[i][j][0] + b4.x, acc[i][j][1] + b4.y, acc[i][j][2] + b4.z, acc[i][j][3] + b4.w};
          if (p.ln_rows && m < p.M) {                 // rstd (acc - mean c1) + bias
            const float2 rs = lnr[i];
            v[0] = fmaf(rs.y, c4.x, fmaf(rs.x, acc[i][j][0], b4.x));
            v[1] = fmaf(rs.y, c4.y, fmaf(rs.x, acc[i][j][1], b4.y));
            v[2] = fmaf(rs.y, c4.z, fmaf(rs.x, acc[i][j][2], b4.z));
            v[3] = fmaf(rs.y, c4.w, fmaf(rs.x, acc[i][j][3], b4.w));
          }
          if (p.act != LDM_ACT_NONE) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = act_f(v[r], p.act);
          }
          bf16_t h[4] = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
          *reinterpret_cast<uint2*>(hs + ml * HP + nl) = *reinterpret_cast<const uint2*>(h);
        }
      }
    }
    __syncthreads();
    epilogue_fast<BM, BN, NT, true, false>(p, m0, n0, hs, HP, reinterpret_cast<float*>(smem));
  }
}
}  // namespace

namespace ldm_igemm {

// Ring configurations (RingCfg, igemm_common.h): (BM, BN) gives ~256 tiles at the deep levels' M,
// so every CU owns one tile
static int g_ring_mode = 0;   // tuning hook (ldm_conv2d_set_ring): 0 planner, 1 never, 2 whenever legal,
                              // 3 / 4: whenever legal in ablation mode 1 (no MFMA) / 2 (no operand DMA)
static int g_ring_split = 0;  // tuning hook (ldm_conv2d_set_ring_split): 0 planner, > 0 forced K splits
int ring_abl() { return g_ring_mode >= 3 ? g_ring_mode - 2 : 0; }

bool ring_legal(const ldm_conv_params* q, int es, bool mixed) {
  const auto a16 = [](const void* x) { return (reinterpret_cast<uintptr_t>(x) & 15) == 0; };
  // 1x1 GEMMs, and 3x3 convs (stride 1 / 2, zero padding 1) as implicit GEMMs over tap-major K whose
  // 64-deep steps each lie in one tap of one source
  if (es != 2 || mixed || q->upsample || q->pad_mode != 0) return false;
  if (!((q->ksize == 1 && q->stride == 1) || (q->ksize == 3 && (q->stride == 1 || q->stride == 2)))) return false;
  if (q->c0 % ring::KS || q->c1 % ring::KS || q->kpad % ring::KS) return false;
  if (q->kpad != q->ksize * q->ksize * (q->c0 + q->c1)) return false;
  if (q->out_layout != LDM_OUT_NHWC && q->out_layout != LDM_OUT_GEGLU) return false;
  if (q->out_f32) return false;
  if (q->out_layout == LDM_OUT_GEGLU && (q->act != LDM_ACT_NONE || q->residual || q->row_stats || q->gn_partial))
    return false;
  if (!a16(q->out) || !a16(q->bias) || !a16(q->residual) || !a16(q->ln_c1) || (q->n & 7)) return false;
  if (q->ln_rows && (reinterpret_cast<uintptr_t>(q->ln_rows) & 15)) return false;
  const int64_t M = (int64_t)q->batch * q->h_out * q->w_out;
  // GroupNorm partials: a 32- or 128-row tile lies in one batch (hw % 64 == 0 is validated)
  if (M * q->n * 2 >= (1LL << 31) - 64 || M * (q->c0 + q->c1) * 2 >= (1LL << 31) - 64) return false;
  return true;
}

// config id for this call (0 = not the ring kernel)
int ring_cfg(const ldm_conv_params* q, int es, bool mixed, int M, bool plan_forced, RingCfg* out) {
  if (g_ring_mode == 1 || plan_forced || !ring_legal(q, es, mixed)) return 0;
  const bool geglu = q->out_layout == LDM_OUT_GEGLU;
  const int K = q->c0 + q->c1;
  const int nsteps = q->kpad / ring::KS;
  if (q->ksize == 3 || g_ring_split > 0) {
    // 3x3 convs (and forced splits): 128x80 tiles, K split toward one block per CU (>= 16 steps
    // each); the fp32 slabs go through the split-K reduction kernel, which also applies the time
    // embedding, residual and GroupNorm partials.  Not planned: at the 8x8 level (B = 8) it ran
    // 41.9 us against the split 64x160 tiles' 34.2 (3x3 1280, graph-timed; the weight stream of a
    // 3x3 conv, 29.5 MB read by 4 M tiles, misses L2 where the 1x1 GEMMs' 3.3 MB hits)
    if (geglu || q->row_stats || q->ln_rows || q->out_layout != LDM_OUT_NHWC || q->n % 80) return 0;
    const bool want = g_ring_mode >= 2 || g_ring_split > 0;
    if (!want) return 0;
    const int tiles = ((M + 127) / 128) * (q->n / 80);
    int ks = g_ring_split > 0 ? g_ring_split : std::max(1, std::min(16, (256 + tiles / 2) / tiles));
    ks = std::max(1, std::min(ks, nsteps / 16));
    if (ks == 1 && q->temb) return 0;                    // (the unsplit ring epilogue has no time embedding)
    if (out) *out = RingCfg{3, 128, 80, ks};
    return 3;
  }
  if (q->temb) return 0;
  RingCfg c{0, 0, 0, 1};
  // planner: the B = 8 deep levels (16x16: M = 2048, 8x8: M = 512) and their B = 1..16 neighbours
  // with >= 128 tiles; mode 2 takes any legal M
  const bool any = g_ring_mode >= 2;
  if (geglu) {
    return 0;                       // (the GEGLU form is written but not instantiated: 128x160 consumer tiles
                                    // spill with the double-buffered fragments)
  } else if (q->n % 80 == 0) {
    // planner range from the graph-timed opbench A/B (profiles/r05d_ring_ops.txt): the ring wins on
    // K <= 2560 at M = 2048 and K <= 1280 at M = 512; the deeper-K ff.net.2 (K = 5120) and the 8x8
    // concat shortcut stay on the split-K tiles, whose partial sums run on more CUs at once
    if (M >= 1024 && (any || (M <= 2048 && q->n <= 1280 && K <= 2560))) c = {1, 128, 80, 1};
    else if (M < 1024 && (any || (M >= 256 && q->n <= 1280 && K <= 1280))) c = {2, 32, 80, 1};
  }
  if (!c.id) return 0;
  if (!any) {
    const int tiles = ((M + c.bm - 1) / c.bm) * (q->n / c.bn);
    if (tiles < 128) return 0;
  }
  if (out) *out = c;
  return c.id;
}

int launch_ring(ConvArgs a, hipStream_t s, const RingCfg& c) {
  a.tiles_n = a.n / c.bn;
  const int ntiles = ((a.M + c.bm - 1) / c.bm) * a.tiles_n;
  a.nblk = ntiles * a.ksplit;
  if (c.id == 1 || c.id == 3)
    hipLaunchKernelGGL((gemm_ring_kernel<128, 80, 4, 1, 5, 3, false>), dim3(a.nblk), dim3(64 * 8), 0, s, a);
  else if (c.id == 2)
    hipLaunchKernelGGL((gemm_ring_kernel<32, 80, 2, 1, 8, 5, false>), dim3(a.nblk), dim3(64 * 6), 0, s, a);
  else
    return LDM_ERR_ARG;
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

}  // namespace ldm_igemm

extern "C" void ldm_conv2d_set_ring(int mode) { ldm_igemm::g_ring_mode = (mode >= 1 && mode <= 4) ? mode : 0; }
extern "C" void ldm_conv2d_set_ring_split(int ks) { ldm_igemm::g_ring_split = ks > 0 ? std::min(ks, 16) : 0; }
