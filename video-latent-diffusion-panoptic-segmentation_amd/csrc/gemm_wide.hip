// Wide-tile persistent 1x1 GEMM for the large-N transformer projections: the LayerNorm-folded
// QKV (to_q/k/v of diffusers Attention) and GEGLU ff.net.0 of every BasicTransformerBlock that
// the reference UNet runs through Transformer2DModel (/root/reference/ldmseg/models/unet.py:361-425).
// Its own translation unit on the shared igemm helpers (igemm_common.h); ldm_conv2d (igemm.hip)
// dispatches to it through ldm_igemm::wide_bm / launch_wide.
//
// Why: the 128x160 two-blocks-per-CU tiles receive 36 KB of operands per 64-deep K tile for
// 2.6 MFLOP (71 FLOP/B) and their main loops are bound by operand delivery into LDS.
// A 256x320 tile receives 72 KB per 64 of K for 10.5 MFLOP (146 FLOP/B).  Such a tile needs all of
// a CU (8 waves of 64x160 fp32 accumulators, a 144 KB two-slot LDS ring), so the launch is
// persistent: one block per CU walks its tiles (XCD-contiguous ids, grouped raster) and the LDS-DMA
// stream never stops at a tile boundary — the next tile's first K tile is in flight while the
// current tile's epilogue runs.  Tuning log: a four-slot ring of 32-deep slices
// (64-B operand rows) kept more bytes in flight but ran 10-30 % slower: every wave instruction then
// fetches 16 half cache lines.
//
// The epilogue runs from registers and never touches the ring.  Per-tile column constants (bias,
// LayerNorm-fold column sums) and row constants (LayerNorm-fold row statistics) arrive with the
// tile's first K tile by LDS-DMA into a small double-buffered scratch, so no compiler-visible global
// load is left in the kernel (hipcc would wait vmcnt(0) for it and drain the prefetch).  The only
// wait that must not drain is the one after an epilogue: its stores are raw buffer stores (rows
// past M dropped by the range check), so their count per lane is fixed and the wait is counted.
//   NHWC (QKV): act(acc + bias) with the LayerNorm fold, packed to bf16; lanes (g, lr) and
//     (g ^ 1, lr) exchange one fragment's halves so every lane stores 16 B (8 channels).
//   GEGLU: h * gelu(g) from the hidden / gate fragment pair that shares a lane, 8-B stores.
// Geometry: 512 threads = 8 waves as 4 (M) x 2 (N); wave tile 64 x 160 = 4 x 10 fragments of
// v_mfma_f32_16x16x32_bf16 (D[n][m] = W . A^T: lane (g, lr) holds channels 4g..4g+3 of pixel lr).
#include "igemm_common.h"

namespace {
namespace wide {
constexpr int NT = 512;
constexpr int BM = 256;
constexpr int BN = 320;
constexpr int WM = 64, WN = 160;    // wave tile: 4 waves along M, 2 along N
constexpr int FM = WM / 16;         // 4 fragments along M
constexpr int FN = WN / 16;         // 10 along N
constexpr int KS = 64;              // K per ring slot (128 B per operand row)
constexpr int NSLOT = 2;
constexpr int SLOT_U4 = (BM + BN) * 8;      // uint4 per slot (72 KB)
constexpr int A_INS = BM / 8 / 8;           // A DMA instructions per wave and K tile (8 rows each): 4
constexpr int B_INS = BN / 8 / 8;           // 5
// scratch floats per tile: bias [320] at 0, c1 [320] at 512, fp64 rows [256][2] at 1024 — eight
// wave DMA instructions of 1 KB (one per wave), each from one source (the buffer descriptor is
// wave-uniform).  Issued with a tile's SECOND K tile (after every wave left the previous tile's
// epilogue), so one buffer suffices.
constexpr int SCR_F = 2048;
// L2 prefetch: the 576 operand lines of K tile s + 2 are touched by 1-byte LDS-DMA loads (64 per
// instruction, into a dummy LDS row per wave) while K tile s + 1 streams, so the DMA of every K tile
// finds its lines in the XCD's L2 instead of waiting on Infinity-Cache / HBM latency
constexpr int PF_INS = 2;                   // per wave: 72 of the 576 lines
#ifndef WIDE_PFD
#define WIDE_PFD 2
#endif
constexpr int PFD = WIDE_PFD;               // K tiles ahead of the one being multiplied that are touched
constexpr int PF_BYTES = 64 * 8;            // dummy LDS: 64 B per wave
constexpr int SCR_C1 = 512, SCR_ROW = 1024;
constexpr int NST = FM * FN / 2;            // epilogue store instructions per lane (20)
}  // namespace wide

// GEGLU: the epilogue form (one instantiation per form)
template <bool GEGLU>
__global__ __launch_bounds__(512, 2) void gemm_wide_kernel(const ConvArgs p) {
  using namespace wide;
  __shared__ uint4 smem[NSLOT * SLOT_U4 + SCR_F / 4 + PF_BYTES / 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 15, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  // DMA lane geometry: one wave instruction = 8 rows x 128 B; wave wv's instruction i covers rows
  // 8 (wv + 8 i) + (lane >> 3); the lane at chunk position lane & 7 fetches logical chunk
  // (lane & 7) ^ ((row >> 1) & 7) (source-side swizzle; (row >> 1) & 7 does not depend on i)
  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ (((8 * wv + drow) >> 1) & 7);
  // scratch DMA on a tile's first K tile: one instruction per wave

  const int tiles_m = (p.M + BM - 1) / BM;
  const int ntiles = tiles_m * p.tiles_n;
  const int G = gridDim.x;
  int vb;
  {
    const int bid = blockIdx.x, xcd = bid & 7, qq = G >> 3, rem = G & 7;
    vb = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
  }
  const int my_tiles = vb < ntiles ? (ntiles - 1 - vb) / G + 1 : 0;
  const int nks = p.kpad / KS;
  const int total = my_tiles * nks;

  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const unsigned scr0 = lds0 + NSLOT * SLOT_U4 * 16;
  float* scr = reinterpret_cast<float*>(smem + NSLOT * SLOT_U4);
  const unsigned pf0 = scr0 + SCR_F * 4 + wv * 64;
  const __amdgpu_buffer_rsrc_t ra0 = __builtin_amdgcn_make_buffer_rsrc((void*)p.a0, 0, p.a0_bytes, kBufFlags);
  const __amdgpu_buffer_rsrc_t ra1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.a1 ? p.a1 : p.a0), 0, p.a1 ? p.a1_bytes : 0, kBufFlags);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, p.w_bytes, kBufFlags);
#ifdef LDM_ABL_NO_PREFETCH
  const __amdgpu_buffer_rsrc_t rnone = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, 0, kBufFlags);
#endif
  const __amdgpu_buffer_rsrc_t rbias =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.bias, 0, p.bias ? p.n * 4 : 0, kBufFlags);
  const __amdgpu_buffer_rsrc_t rc1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.ln_c1, 0, p.ln_rows ? p.n * 4 : 0, kBufFlags);
  const __amdgpu_buffer_rsrc_t rrow =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.ln_rows, 0, p.ln_rows ? p.M * 16 : 0, kBufFlags);
  const int n_out = GEGLU ? (p.n >> 1) : p.n;
  const __amdgpu_buffer_rsrc_t rout =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.out, 0, (int)((int64_t)p.M * n_out * 2), kBufFlags);

  auto coords = [&](int r, int& m0, int& n0) {
    int tm, tn;
    grouped_tile(r * G + vb, tiles_m, p.tiles_n, p.group_m, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  const int vob = (drow * p.kpad + dchunk * 8) * 2;
  // step s of this block's stream = K tile (s mod nks) of its tile s / nks
  auto issue = [&](int s) {
#ifdef LDM_ABL_NO_LOADS
    return;
#endif
    const int r = s / nks, kt = s - r * nks;
    int m0, n0;
    coords(r, m0, n0);
    const unsigned abase = lds0 + (unsigned)((s & 1) * SLOT_U4 * 16);
    const unsigned bbase = abase + BM * 128;
    const int k0 = kt * KS;
    const int sel = (p.c1 > 0 && k0 >= p.c0) ? 1 : 0;   // concat boundary is slice aligned (host)
    const int cs = sel ? p.c1 : p.c0;
    const int choff = (sel ? k0 - p.c0 : k0) + dchunk * 8;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      const int q = wv + 8 * i;                         // instruction index: rows 8q .. 8q + 7
      const int m = m0 + 8 * q + drow;
      const int off = m < p.M ? (m * cs + choff) * 2 : kOOB;
      const unsigned dst = __builtin_amdgcn_readfirstlane(abase + q * 8 * 128);
      if (sel) dma16(ra1, off, dst);
      else dma16(ra0, off, dst);
    }
    // B rows are always in range (N is a multiple of the tile): the lane part of the offset stays
    // one loop-invariant VGPR and the rows / K tile go in soffset (per-instruction offsets held in
    // VGPRs spilled, and hipcc's waits for the reloads drained the DMA stream)
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int q = wv + 8 * i;
      dma16s(rw, vob, __builtin_amdgcn_readfirstlane(((n0 + 8 * q) * p.kpad + k0) * 2),
             __builtin_amdgcn_readfirstlane(bbase + q * 8 * 128));
    }
    if (kt == 1) {
      // instruction wv: 0, 1 bias [256 wv, +256); 2, 3 c1; 4..7 fp64 rows [m0 + 64 (wv - 4), +64)
      const unsigned sb = scr0 + wv * 1024;
      const int e = (wv & 1) * 256 + lane * 4;          // first float of this lane's 16 B (bias / c1)
      const int off = wv < 4 ? (e < BN ? (n0 + e) * 4 : kOOB) : (m0 * 16 + (wv - 4) * 1024 + lane * 16);
      const unsigned dst = __builtin_amdgcn_readfirstlane(sb);
      if (wv < 2) dma16(rbias, off, dst);
      else if (wv < 4) dma16(rc1, off, dst);
      else dma16(rrow, off, dst);
    }
  };

  // touch (L2 prefetch) the operand lines of K tile s: line L = 72 wv + 64 i + lane < 72 (wv + 1);
  // L < 256: A row m0 + L, else B row n0 + L - 256 (one 128-B line each)
  auto prefetch = [&](int s) {
    const int r = s / nks, kt = s - r * nks;
    int m0, n0;
    coords(r, m0, n0);
    const int k0 = kt * KS;
    const int sel = (p.c1 > 0 && k0 >= p.c0) ? 1 : 0;
    const int cs = sel ? p.c1 : p.c0;
    const int kk = sel ? k0 - p.c0 : k0;
#pragma unroll
    for (int i = 0; i < PF_INS; ++i) {
      const int j = 64 * i + lane;
      const int L = 72 * wv + j;
      int off_a = kOOB, off_b = kOOB;
      if (j < 72) {
        if (L < BM) {
          const int m = m0 + L;
          if (m < p.M) off_a = (m * cs + kk) * 2;
        } else {
          const int n = n0 + L - BM;
          if (n < p.n) off_b = (n * p.kpad + k0) * 2;
        }
      }
      // the A and B lines of one instruction may both occur: two loads, each with the other's lanes
      // out of range (no memory access)
#ifdef LDM_ABL_NO_PREFETCH   // ablation build: the same counted instructions on empty descriptors
      touch1(rnone, off_a, pf0);
      touch1(rnone, off_b, pf0);
#else
      touch1(sel ? ra1 : ra0, off_a, pf0);
      touch1(rw, off_b, pf0);
#endif
    }
  };

  f32x4_t acc[FM][FN];
  auto compute = [&](int slot) {
    // row r = base + 16 f + lr: swz(r, c) = c ^ ((lr >> 1) & 7) for every fragment f, so each
    // operand needs one lane address per k32 step and the fragments are immediate offsets (the
    // per-fragment addresses otherwise occupied ~10 VGPRs that spilled)
    const uint4* As = smem + slot * SLOT_U4 + (wm * WM + lr) * 8;
    const uint4* Bs = smem + slot * SLOT_U4 + BM * 8 + (wn * WN + lr) * 8;
    const int sl = (lr >> 1) & 7;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int cch = (ks * 4 + g) ^ sl;
      Frag8<bf16_t> af[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i].v = As[i * 128 + cch];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        Frag8<bf16_t> bf;
        bf.v = Bs[j * 128 + cch];
#ifdef LDM_ABL_NO_MFMA   // ablation build: fragments read from LDS, no MFMA issued
        asm volatile("" ::"v"(bf.v.x), "v"(bf.v.w));
        if (j == 0) {
#pragma unroll
          for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(af[i].v.x), "v"(af[i].v.w));
        }
        continue;
#endif
#pragma unroll
        for (int i = 0; i < FM; ++i) mma_k32(acc[i][j], bf, af[i]);
      }
      // keep the second k32 step's fragment reads from being hoisted beside the first step's
      // (160 accumulator registers leave no room for two steps' fragments)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if (total > 0) issue(0);
#pragma unroll
  for (int q = 1; q < PFD; ++q)
    if (total > q) prefetch(q);
  int s = 0;
  for (int r = 0; r < my_tiles; ++r) {
    int m0, n0;
    coords(r, m0, n0);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nks; ++kt, ++s) {
      // K tile s landed for this wave; younger and allowed to stay in flight: the prefetch of K tile
      // s + 1 (issued right after this tile's DMA) and, after an epilogue, its NST stores
      const bool pf = s + PFD - 1 < total, epi = kt == 0 && r > 0;
      if (pf && epi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PF_INS + NST) : "memory");
      else if (epi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
      else if (pf) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PF_INS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // every wave's part of tile s is in LDS, and every wave is done with slot (s + 1) & 1
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (s + 1 < total) issue(s + 1);
      if (s + PFD < total) prefetch(s + PFD);
      compute(s & 1);
    }
    // ---- epilogue from registers; this tile's scratch landed with its second K tile
    const float* sbias = scr;
    const float* sc1 = sbias + SCR_C1;
    const double2* srow = reinterpret_cast<const double2*>(sbias + SCR_ROW);
    float2 lnr[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (p.ln_rows) {
        const double2 st = srow[wm * WM + i * 16 + lr];
        lnr[i] = ln_row_from(st.x, st.y, p.ln_inv_k, p.ln_eps);
      } else {
        lnr[i] = make_float2(1.f, 0.f);
      }
    }
    if constexpr (GEGLU) {
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
        const int cl = wn * WN + j * 16 + 4 * g;                 // tile column of the hidden values
        const int oc = ((n0 + cl) >> 5) * 16 + ((n0 + cl) & 15); // output channel
        const float4 bh = *reinterpret_cast<const float4*>(sbias + cl);
        const float4 bg = *reinterpret_cast<const float4*>(sbias + cl + 16);
        const float4 ch = *reinterpret_cast<const float4*>(sc1 + cl);
        const float4 cg = *reinterpret_cast<const float4*>(sc1 + cl + 16);
        const float bhv[4] = {bh.x, bh.y, bh.z, bh.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
        const float chv[4] = {ch.x, ch.y, ch.z, ch.w}, cgv[4] = {cg.x, cg.y, cg.z, cg.w};
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = m0 + wm * WM + i * 16 + lr;
          const float2 rs = lnr[i];
          bf16_t h[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            h[k] = f2bf(fmaf(rs.y, chv[k], fmaf(rs.x, acc[i][j][k], bhv[k])) *
                        gelu_f(fmaf(rs.y, cgv[k], fmaf(rs.x, acc[i][j + 1][k], bgv[k]))));
          const uint2 u = *reinterpret_cast<const uint2*>(h);
          const int off = (m < p.M && n0 + cl < p.n) ? (int)(((int64_t)m * n_out + oc) * 2) : kOOB;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, u),
                                                rout, off, 0, 0);
        }
      }
    } else {
      // act(acc + bias), LayerNorm fold; lanes g and g ^ 1 trade halves of a fragment pair so each
      // stores 8 consecutive channels: even g -> fragment j channels 4g..4g+7, odd g -> fragment
      // j + 1 channels 4(g-1)..4(g-1)+7 (16 + ... of the pair)
      const bool odd = g & 1;
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
        const int c0 = wn * WN + j * 16 + 4 * g;                 // this lane's columns in fragment j
        const float4 b0 = *reinterpret_cast<const float4*>(sbias + c0);
        const float4 b1 = *reinterpret_cast<const float4*>(sbias + c0 + 16);
        const float4 k0 = *reinterpret_cast<const float4*>(sc1 + c0);
        const float4 k1 = *reinterpret_cast<const float4*>(sc1 + c0 + 16);
        const float bv0[4] = {b0.x, b0.y, b0.z, b0.w}, bv1[4] = {b1.x, b1.y, b1.z, b1.w};
        const float kv0[4] = {k0.x, k0.y, k0.z, k0.w}, kv1[4] = {k1.x, k1.y, k1.z, k1.w};
        // the stored 8 columns: even g: c0 .. c0 + 7 of fragment j; odd g: c0 + 12 .. c0 + 19
        const int cst = odd ? c0 + 12 : c0;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int m = m0 + wm * WM + i * 16 + lr;
          const float2 rs = lnr[i];
          float v0[4], v1[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v0[k] = act_f(fmaf(rs.y, kv0[k], fmaf(rs.x, acc[i][j][k], bv0[k])), p.act);
            v1[k] = act_f(fmaf(rs.y, kv1[k], fmaf(rs.x, acc[i][j + 1][k], bv1[k])), p.act);
          }
          bf16_t h0[4] = {f2bf(v0[0]), f2bf(v0[1]), f2bf(v0[2]), f2bf(v0[3])};
          bf16_t h1[4] = {f2bf(v1[0]), f2bf(v1[1]), f2bf(v1[2]), f2bf(v1[3])};
          const uint2 u0 = *reinterpret_cast<const uint2*>(h0), u1 = *reinterpret_cast<const uint2*>(h1);
          // send the half the partner stores: even sends fragment j + 1, odd sends fragment j
          const uint2 snd = odd ? u0 : u1;
          uint2 rcv;
          rcv.x = __shfl_xor((int)snd.x, 16, 64);
          rcv.y = __shfl_xor((int)snd.y, 16, 64);
          const uint4 out = odd ? make_uint4(rcv.x, rcv.y, u1.x, u1.y) : make_uint4(u0.x, u0.y, rcv.x, rcv.y);
          const int off = (m < p.M && n0 + cst < p.n) ? (int)(((int64_t)m * p.n + n0 + cst) * 2) : kOOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, out),
                                                 rout, off, 0, 0);
        }
      }
    }
  }
}
}  // namespace

namespace ldm_igemm {

// legal: bf16 1x1 GEMM (one source, or a concat whose boundary is 64-channel aligned), N a
// multiple of 320, NHWC (bias / activation / LayerNorm fold) or GEGLU (bias / LayerNorm fold); no
// residual, row or GroupNorm statistics, time embedding, split-K or fp32 output
static int g_wide_mode = 0;   // tuning hook: 0 planner, 1 never, 2 whenever legal
bool wide_legal(const ldm_conv_params* q, int es, bool mixed) {
  const auto a16 = [](const void* x) { return (reinterpret_cast<uintptr_t>(x) & 15) == 0; };
  if (es != 2 || mixed || q->ksize != 1 || q->stride != 1 || q->upsample || q->pad_mode != 0) return false;
  // >= 2 K tiles per tile: the scratch arrives with a tile's second K tile
  if (q->c0 % wide::KS || q->c1 % wide::KS || q->kpad % wide::KS || q->kpad < 2 * wide::KS || q->n % wide::BN)
    return false;
  if (q->out_layout != LDM_OUT_NHWC && q->out_layout != LDM_OUT_GEGLU) return false;
  if (q->out_f32 || q->temb || q->residual || q->row_stats || q->gn_partial) return false;
  if (q->out_layout == LDM_OUT_GEGLU && q->act != LDM_ACT_NONE) return false;
  if (!a16(q->out) || !a16(q->bias) || !a16(q->ln_c1)) return false;
  if (q->ln_rows && (reinterpret_cast<uintptr_t>(q->ln_rows) & 15)) return false;
  const int64_t M = (int64_t)q->batch * q->h_out * q->w_out;
  if (M * q->n * 2 >= (1LL << 31) - 64 || M * 16 >= (1LL << 31)) return false;
  return true;
}

// rows per tile for this call, 0 = not the wide kernel
int wide_bm(const ldm_conv_params* q, int es, bool mixed, int M, bool plan_forced) {
  if (g_wide_mode == 1 || plan_forced || !wide_legal(q, es, mixed)) return 0;
  if (g_wide_mode == 2) return wide::BM;
  const int tiles = ((M + wide::BM - 1) / wide::BM) * (q->n / wide::BN);
  // enough tiles to give every CU one, K deep enough to amortise the per-tile epilogue: K = 320 (five
  // K tiles) stays on the two-blocks-per-CU tiles / gemm_ars (r03a graph-step breakdown: QKV 320 ->
  // 960 57 -> 73 us and the GEGLU 320 -> 2560 100 -> 106 us on this kernel)
  if (tiles >= 256 && q->kpad >= 384) return wide::BM;
  return 0;
}

int launch_wide(ConvArgs a, hipStream_t s, int bm) {
  if (bm != wide::BM) return LDM_ERR_ARG;
  a.tiles_n = a.n / wide::BN;
  const int ntiles = ((a.M + wide::BM - 1) / wide::BM) * a.tiles_n;
  const int grid = std::min(ntiles, 256);
  a.nblk = grid;
  if (a.out_layout == LDM_OUT_GEGLU) hipLaunchKernelGGL((gemm_wide_kernel<true>), dim3(grid), dim3(wide::NT), 0, s, a);
  else hipLaunchKernelGGL((gemm_wide_kernel<false>), dim3(grid), dim3(wide::NT), 0, s, a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

}  // namespace ldm_igemm

extern "C" void ldm_conv2d_set_wide(int mode) { ldm_igemm::g_wide_mode = (mode >= 1 && mode <= 2) ? mode : 0; }
