// A-register-stationary 1x1 GEMM for the short-K projections of the 64x64 UNet level
// (K = 320: proj_in, the LayerNorm-folded QKV, to_out, the LayerNorm-folded GEGLU ff.net.0).
// Included by igemm.hip inside its anonymous namespace (uses ConvArgs and its helpers).
//
// Why a separate kernel: a 128x128 tile of a K = 320 GEMM receives 164 KB of operands for
// 10.5 MFLOP (64 FLOP/B).  At the ~65 GB/s per CU an XCD's L2 delivers into LDS
// (MI355X_MICROARCH.md "Indexed rows") that is 2.5 us of operand delivery against 1.1 us of MFMA
// work, and every tile restarts its pipeline (5 K tiles, prologue latency, staged epilogue).
// Here one 4-wave block (one wave per SIMD: 512 registers per lane, the accumulators in AGPRs)
// owns a 256-row panel of A for the whole launch and keeps it in VGPRs as MFMA fragments (64 rows
// x K per wave: 4 x 10 x 16 B per lane at K = 320), so only the weight
// streams: 160-column B tiles in 64-wide K stages through a 3-slot LDS-DMA ring that runs
// continuously across the block's N tiles (the next tile's stages are in flight while the
// current tile's epilogue runs).  Per 160-column tile the CU receives 100 KB of B for 26 MFLOP
// (262 FLOP/B): MFMA-bound.  The epilogue is wave-private: the accumulators (bias, LayerNorm
// fold, activation / GEGLU applied) go to the wave's own LDS staging rows as bf16, then leave
// as 16-B row-contiguous stores with the residual and the per-row (sum, sumsq) — no block barrier.
namespace ars {
constexpr int NW = 4, NT = 256;         // waves, threads
constexpr int RPP = NT / 8;             // B rows per DMA pass (8 lanes x 16 B per 128-B row)
constexpr int BN = 160, NF = BN / 16;   // N tile, 16-wide fragments per N tile
constexpr int NS = 3;                   // LDS ring slots (two stages in flight)
constexpr int STAGE_U4 = BN * 8;        // one 160 x 64 bf16 stage = 160 rows x 128 B
constexpr int HP = BN + 8;              // NHWC staging pitch (bf16)
constexpr int HPG = BN / 2 + 8;         // GEGLU staging pitch (bf16)
constexpr int MAXT = 8;                 // N tiles per block at most (bias / c1 columns kept in LDS)
constexpr int COL_U4 = MAXT * BN / 4;   // uint4 per column array (bias, LayerNorm c1)
}  // namespace ars

// The block's bias and LayerNorm-fold column sums, staged in LDS once: epilogue loads from global
// memory would each wait (vmcnt, issue order) behind the B stages in flight — ten serial L2 round
// trips per tile (the epilogue ablation: 35 of 61 us of a K=320 QKV launch).
__device__ __forceinline__ void ars_stage_cols(const ConvArgs& p, float* cb, float* c1, int col0, int ncols) {
  for (int c = threadIdx.x; c < ncols / 4; c += blockDim.x) {
    const int n = col0 + 4 * c;
    reinterpret_cast<float4*>(cb)[c] = p.bias ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    reinterpret_cast<float4*>(c1)[c] = p.ln_rows ? *reinterpret_cast<const float4*>(p.ln_c1 + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int KC, int RF>
__global__ __launch_bounds__(256, 1) void gemm_ars_kernel(const ConvArgs p, int nsplit) {
  using namespace ars;
  constexpr int WROWS = RF * 16;                    // rows per wave
  constexpr int BM = NW * WROWS;                    // rows per block
  constexpr int KS = KC / 2;                        // 64-wide K stages per N tile
  constexpr int STG_U4 = (WROWS * HP * 2 + 15) / 16;
  constexpr int PASSES = BN / RPP;                  // LDS-DMA instructions per wave and stage
  static_assert(KC % 2 == 0, "K must be a multiple of 64");
  static_assert(BN % RPP == 0 && PASSES == 5, "vmcnt counts below assume 5 DMAs per wave and stage");
  __shared__ uint4 smem[NS * STAGE_U4 + NW * STG_U4 + 2 * COL_U4];

  // ---- block -> (panel, N range); XCD-aware: each XCD gets a contiguous run of ids, so the
  //      nsplit blocks of one A panel run on one XCD and share its L2
  int tile;
  {
    const int bid = blockIdx.x, nblk = p.nblk;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    tile = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
  }
  const int panel = tile / nsplit, part = tile - panel * nsplit;
  const int tiles_total = p.n / BN;
  const int tb0 = tiles_total * part / nsplit, tb1 = tiles_total * (part + 1) / nsplit;
  const int ntile = tb1 - tb0;
  const int nst = ntile * KS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int lr = lane & 15, g = lane >> 4;
  const int cc = tid & 7, rr = tid >> 3;            // DMA: row rr (+RPP i), 16-B chunk position cc
  const int mw0 = panel * BM + wv * WROWS;          // first row of this wave

  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a0, 0, p.a0_bytes, kBufFlags);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, p.w_bytes, kBufFlags);
  // source-side XOR swizzle (LDS-DMA writes lane-linearly): the lane at chunk position cc of
  // row r fetches logical chunk cc ^ ((r >> 1) & 7); (rr + 32 i) >> 1 & 7 == rr >> 1 & 7
  const int cl = cc ^ ((rr >> 1) & 7);

  auto issue = [&](int q) {
    const int t = tb0 + q / KS, ks = q - (q / KS) * KS;
    const unsigned base = lds0 + (unsigned)((q % NS) * STAGE_U4 * 16);
    const int kb = (ks * 64 + cl * 8) * 2;
#pragma unroll
    for (int i = 0; i < PASSES; ++i) {
      const int n = t * BN + rr + RPP * i;
      dma16(rw, n * p.kpad * 2 + kb, __builtin_amdgcn_readfirstlane(base + (RPP * i + 8 * wv) * 128));
    }
  };

  // ---- prologue: the first two B stages, then this wave's A rows as MFMA fragments
  //      (lane (g, lr) holds K values [32 c + 8 g, +8) of row 16 f + lr)
  if (nst > 0) issue(0);
  if (nst > 1) issue(1);
  uint4 af[RF][KC];
#pragma unroll
  for (int f = 0; f < RF; ++f) {
    const int m = mw0 + 16 * f + lr;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      af[f][c] = bload(ra, m < p.M ? (m * p.c0 + 32 * c + 8 * g) * 2 : kOOB);
  }
  // LayerNorm fold: (rstd, -rstd * mean) of this lane's rows
  float2 lnr[RF];
#pragma unroll
  for (int f = 0; f < RF; ++f) {
    const int m = mw0 + 16 * f + lr;
    lnr[f] = (p.ln_rows && m < p.M) ? ln_row(p, m) : make_float2(1.f, 0.f);
  }

  f32x4_t acc[RF][NF];
#pragma unroll
  for (int f = 0; f < RF; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16_t* stg = reinterpret_cast<bf16_t*>(smem + NS * STAGE_U4 + wv * STG_U4);
  const bool geglu = p.out_layout == LDM_OUT_GEGLU;
  const bool has_act = p.act != LDM_ACT_NONE;
  float* colb = reinterpret_cast<float*>(smem + NS * STAGE_U4 + NW * STG_U4);
  float* colc = colb + 4 * COL_U4;
  ars_stage_cols(p, colb, colc, tb0 * BN, ntile * BN);   // visible after the first stage barrier

  for (int tl = 0; tl < ntile; ++tl) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int q = tl * KS + ks;
      // stage q landed (this wave's part): the younger stage q + 1 may stay in flight, except
      // after an epilogue (its stores count on vmcnt too) or at the end of the stream
      if (q == 0 || ks == 0 || q + 1 >= nst) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      }
      // raw barrier: every wave's part of stage q is in LDS, and every wave is done with slot
      // (q + 2) % 3 (stage q - 1), which the next DMA overwrites
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (q + 2 < nst) issue(q + 2);
      const uint4* Bs = smem + (q % NS) * STAGE_U4;
      Frag8<bf16_t> bfr[2][NF];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const int r = j * 16 + lr;
          bfr[kk][j].v = Bs[r * 8 + swz(r, kk * 4 + g)];
        }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
          for (int f = 0; f < RF; ++f) {
            Frag8<bf16_t> a;
            a.v = af[f][ks * 2 + kk];
            mma_k32(acc[f][j], bfr[kk][j], a);
          }
      // schedule: the first K step's NF LDS reads, then one read of the second K step behind every
      // RF MFMAs of the first, then the second step's MFMAs (one wave per SIMD: the reads' latency
      // has to hide under this wave's own MFMAs)
      __builtin_amdgcn_sched_group_barrier(0x100, NF, 0);
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, RF, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NF * RF, 0);
    }

    // ---- epilogue of N tile tb0 + tl (wave-private; the next tile's stages are in flight)
    const int nt0 = (tb0 + tl) * BN;
#ifdef LDM_ABL_ARS_NOEPI   // ablation build: accumulators kept alive, no epilogue
    {
      float t = 0.f;
#pragma unroll
      for (int f = 0; f < RF; ++f)
#pragma unroll
        for (int j = 0; j < NF; ++j) t += acc[f][j][0];
      if (t == 12345.f) reinterpret_cast<float*>(p.out)[tid] = t;
      continue;
    }
#endif
    // per-row addresses are recomputed here from opaque copies: hoisted out of the tile loop they
    // would be dozens of live 64-bit values, spilled next to the A fragments
    int mwe = mw0, ne = p.n, le = lane;
    asm volatile("" : "+s"(mwe), "+s"(ne), "+v"(le));
    if (geglu) {
      // fragments j (hidden) and j + 1 (gate) hold the same 4 output channels of the same row
#pragma unroll
      for (int j = 0; j < NF; j += 2) {
        const int pc = nt0 + 16 * j + 4 * g;
        float4 bh = make_float4(0.f, 0.f, 0.f, 0.f), bg = bh, ch = bh, cg = bh;
        {
          const int lc = pc - tb0 * BN;
          bh = *reinterpret_cast<const float4*>(colb + lc); bg = *reinterpret_cast<const float4*>(colb + lc + 16);
          ch = *reinterpret_cast<const float4*>(colc + lc); cg = *reinterpret_cast<const float4*>(colc + lc + 16);
        }
        const float bhv[4] = {bh.x, bh.y, bh.z, bh.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
        const float chv[4] = {ch.x, ch.y, ch.z, ch.w}, cgv[4] = {cg.x, cg.y, cg.z, cg.w};
#pragma unroll
        for (int f = 0; f < RF; ++f) {
          bf16_t h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float hv = fmaf(lnr[f].y, chv[r], fmaf(lnr[f].x, acc[f][j][r], bhv[r]));
            const float gv = fmaf(lnr[f].y, cgv[r], fmaf(lnr[f].x, acc[f][j + 1][r], bgv[r]));
            h[r] = f2bf(hv * gelu_f(gv));
          }
          *reinterpret_cast<uint2*>(stg + (16 * f + lr) * HPG + 8 * j + 4 * g) = *reinterpret_cast<const uint2*>(h);
        }
      }
      asm volatile("" ::: "memory");   // one wave's LDS writes and reads stay in order
      const int NO = ne >> 1;
      bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
#pragma unroll
      for (int i = 0; i < WROWS * 10 / 64 + 1; ++i) {
        const int idx = le + 64 * i;
        if (idx >= WROWS * 10) break;
        const int r = idx / 10, c = idx - (idx / 10) * 10;
        const int m = mwe + r;
        const uint4 x = *reinterpret_cast<const uint4*>(stg + r * HPG + 8 * c);
#ifdef LDM_ABL_ARS_NOSTORE
        if (x.x == 0x12345678u && m < p.M)
#else
        if (m < p.M)
#endif
          *reinterpret_cast<uint4*>(out + (int64_t)m * NO + (nt0 >> 1) + 8 * c) = x;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int n = nt0 + 16 * j + 4 * g;
        float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f), c4 = b4;
        b4 = *reinterpret_cast<const float4*>(colb + n - tb0 * BN);
        c4 = *reinterpret_cast<const float4*>(colc + n - tb0 * BN);
        const float bv[4] = {b4.x, b4.y, b4.z, b4.w}, cv[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
        for (int f = 0; f < RF; ++f) {
          bf16_t h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = fmaf(lnr[f].y, cv[r], fmaf(lnr[f].x, acc[f][j][r], bv[r]));
            h[r] = f2bf(has_act ? act_f(v, p.act) : v);
          }
          *reinterpret_cast<uint2*>(stg + (16 * f + lr) * HP + 16 * j + 4 * g) = *reinterpret_cast<const uint2*>(h);
        }
      }
      asm volatile("" ::: "memory");
      // 16 les per row: chunk c16 (columns 8 c16 ..) and, for c16 < 4, chunk 16 + c16
      const int rg = le >> 4, c16 = le & 15;
      const bool two = c16 < 4;
      const bf16_t* res = reinterpret_cast<const bf16_t*>(p.residual);
      bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
      const int N = ne;
      constexpr int IT = WROWS / 4, GP = 4;            // rows per le; residual rows in flight
#pragma unroll
      for (int i0 = 0; i0 < IT; i0 += GP) {
      uint4 rv0[GP], rv1[GP];
      if (res) {
#pragma unroll
        for (int u = 0; u < GP; ++u) {
          const int m = mwe + (i0 + u) * 4 + rg;
          const int64_t o = (int64_t)min(m, p.M - 1) * N + nt0 + 8 * c16;
          rv0[u] = *reinterpret_cast<const uint4*>(res + o);
          rv1[u] = *reinterpret_cast<const uint4*>(res + o + (two ? 128 : 0));   // unconditional: no branch + vmcnt(0)
        }
      }
#pragma unroll
      for (int u = 0; u < GP; ++u) {
        const int it = i0 + u;
        const int r = it * 4 + rg, m = mwe + r;
        float v0[8], v1[8];
        unpack8(*reinterpret_cast<const uint4*>(stg + r * HP + 8 * c16), v0);
        unpack8(*reinterpret_cast<const uint4*>(stg + r * HP + (two ? 128 : 0) + 8 * c16), v1);
        if (res) {
          float r0[8], r1[8];
          unpack8(rv0[u], r0);
          unpack8(rv1[u], r1);
#pragma unroll
          for (int k = 0; k < 8; ++k) { v0[k] += r0[k]; v1[k] += r1[k]; }
        }
        const uint4 p0 = pack8(v0), p1 = pack8(v1);
        const int64_t o = (int64_t)m * N + nt0 + 8 * c16;
#ifdef LDM_ABL_ARS_NOSTORE
        if (p0.x == 0x12345678u && m < p.M) {
#else
        if (m < p.M) {
#endif
          *reinterpret_cast<uint4*>(out + o) = p0;
          if (two) *reinterpret_cast<uint4*>(out + o + 128) = p1;
        }
        if (p.row_stats) {
          float s0[8], s1[8], a = 0.f, b = 0.f;
          unpack8(p0, s0);
          unpack8(p1, s1);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            a += s0[k];
            b += s0[k] * s0[k];
            if (two) { a += s1[k]; b += s1[k] * s1[k]; }
          }
#pragma unroll
          for (int o2 = 8; o2 > 0; o2 >>= 1) { a += __shfl_xor(a, o2, 64); b += __shfl_xor(b, o2, 64); }
          if (c16 == 0 && m < p.M) {
            unsafeAtomicAdd(p.row_stats + 2 * (int64_t)m, (double)a);
            unsafeAtomicAdd(p.row_stats + 2 * (int64_t)m + 1, (double)b);
          }
        }
      }
      }
    }
#pragma unroll
    for (int f = 0; f < RF; ++f)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
}

// Two-blocks-per-CU form (the default): 4 waves x 32 rows (128-row panels, A 80 + accumulators
// 80 registers per lane), the 3-slot B ring is the only LDS (60 KB), and the epilogue stages each
// wave's 16-row slices in its quarter of the ring slot the tile's last stage was just read from
// (one block barrier; the slot is refilled only after the next stage's barrier).  One block's
// epilogue (GELU math, stores draining) runs beside the other block's MFMAs.
namespace ars2 {
constexpr int NW = 4, NT = 256, RF = 2, WROWS = RF * 16, BM = NW * WROWS;
constexpr int BN = 160, NF = BN / 16, NS = 3;
constexpr int STAGE_U4 = BN * 8;             // 160 rows x 128 B
constexpr int PASSES = BN / (NT / 8);        // LDS-DMA instructions per thread and stage (5)
constexpr int WSTG = STAGE_U4 * 16 / NW;     // staging bytes per wave (5120: 16 rows x 320 B)
// staging chunk position: 16-B chunk c of row r, rotated inside its group of 4 (bank spread)
__device__ __forceinline__ int sc(int r, int c) { return (c & ~3) | ((c ^ r) & 3); }
}  // namespace ars2

template <int KC>
__global__ __launch_bounds__(256, 2) void gemm_ars2_kernel(const ConvArgs p, int nsplit) {
  using namespace ars2;
  constexpr int KS = KC / 2;
  static_assert(KC % 2 == 0 && PASSES == 5, "vmcnt counts below assume 5 DMAs per thread and stage");
  __shared__ uint4 smem[NS * STAGE_U4 + 2 * ars::COL_U4];

  int tile;
  {
    const int bid = blockIdx.x, nblk = p.nblk;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    tile = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
  }
  const int panel = tile / nsplit, part = tile - panel * nsplit;
  const int tiles_total = p.n / BN;
  const int tb0 = tiles_total * part / nsplit, tb1 = tiles_total * (part + 1) / nsplit;
  const int ntile = tb1 - tb0;
  const int nst = ntile * KS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int lr = lane & 15, g = lane >> 4;
  const int cc = tid & 7, rr = tid >> 3;
  const int mw0 = panel * BM + wv * WROWS;

  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.a0, 0, p.a0_bytes, kBufFlags);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, p.w_bytes, kBufFlags);
  const int cl = cc ^ ((rr >> 1) & 7);
  // per-lane part of every B source offset (row rr, swizzled chunk); the rest is wave-uniform
  const int vb = rr * p.kpad * 2 + cl * 16;

  auto issue = [&](int q) {
    const int t = tb0 + q / KS, ks = q - (q / KS) * KS;
    const unsigned base = lds0 + (unsigned)((q % NS) * STAGE_U4 * 16);
    const int sb = __builtin_amdgcn_readfirstlane(t * BN * p.kpad * 2 + ks * 128);
    const int srow = __builtin_amdgcn_readfirstlane(32 * p.kpad * 2);
#pragma unroll
    for (int i = 0; i < PASSES; ++i)
      dma16(rw, vb + sb + i * srow, __builtin_amdgcn_readfirstlane(base + (32 * i + 8 * wv) * 128));
  };

  if (nst > 0) issue(0);
  if (nst > 1) issue(1);
  uint4 af[RF][KC];
#pragma unroll
  for (int f = 0; f < RF; ++f) {
    const int m = mw0 + 16 * f + lr;
#pragma unroll
    for (int c = 0; c < KC; ++c)
      af[f][c] = bload(ra, m < p.M ? (m * p.c0 + 32 * c + 8 * g) * 2 : kOOB);
  }
  float2 lnr[RF];
#pragma unroll
  for (int f = 0; f < RF; ++f) {
    const int m = mw0 + 16 * f + lr;
    lnr[f] = (p.ln_rows && m < p.M) ? ln_row(p, m) : make_float2(1.f, 0.f);
  }
  f32x4_t acc[RF][NF];
#pragma unroll
  for (int f = 0; f < RF; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const bool geglu = p.out_layout == LDM_OUT_GEGLU;
  const bool has_act = p.act != LDM_ACT_NONE;
  float* colb = reinterpret_cast<float*>(smem + NS * STAGE_U4);
  float* colc = colb + 4 * ars::COL_U4;
  ars_stage_cols(p, colb, colc, tb0 * BN, ntile * BN);

  for (int tl = 0; tl < ntile; ++tl) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int q = tl * KS + ks;
      if (q == 0 || ks == 0 || q + 1 >= nst) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (q + 2 < nst) issue(q + 2);
      const uint4* Bs = smem + (q % NS) * STAGE_U4;
      Frag8<bf16_t> bfr[2][NF];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const int r = j * 16 + lr;
          bfr[kk][j].v = Bs[r * 8 + swz(r, kk * 4 + g)];
        }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
          for (int f = 0; f < RF; ++f) {
            Frag8<bf16_t> a;
            a.v = af[f][ks * 2 + kk];
            mma_k32(acc[f][j], bfr[kk][j], a);
          }
      __builtin_amdgcn_sched_group_barrier(0x100, NF, 0);
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, RF, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NF * RF, 0);
    }

    // ---- epilogue: every wave is done reading the slot of stage (tl + 1) * KS - 1
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int nt0 = (tb0 + tl) * BN;
    int mwe = mw0, ne = p.n, le = lane;
    asm volatile("" : "+s"(mwe), "+s"(ne), "+v"(le));
    char* stg = reinterpret_cast<char*>(smem + (((tl + 1) * KS - 1) % NS) * STAGE_U4) + wv * WSTG;
#pragma unroll
    for (int f = 0; f < RF; ++f) {
      const int mf = mwe + 16 * f;                     // first row of this 16-row slice
      if (geglu) {
        // pitch 192 B (12 chunks): 80 output columns = 10 chunks per row
#pragma unroll
        for (int j = 0; j < NF; j += 2) {
          const int pc = nt0 + 16 * j + 4 * g;
          float4 bh = make_float4(0.f, 0.f, 0.f, 0.f), bg = bh, ch = bh, cg = bh;
          {
            const int lc = pc - tb0 * BN;
            bh = *reinterpret_cast<const float4*>(colb + lc); bg = *reinterpret_cast<const float4*>(colb + lc + 16);
            ch = *reinterpret_cast<const float4*>(colc + lc); cg = *reinterpret_cast<const float4*>(colc + lc + 16);
          }
          const float bhv[4] = {bh.x, bh.y, bh.z, bh.w}, bgv[4] = {bg.x, bg.y, bg.z, bg.w};
          const float chv[4] = {ch.x, ch.y, ch.z, ch.w}, cgv[4] = {cg.x, cg.y, cg.z, cg.w};
          bf16_t h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float hv = fmaf(lnr[f].y, chv[r], fmaf(lnr[f].x, acc[f][j][r], bhv[r]));
            const float gv = fmaf(lnr[f].y, cgv[r], fmaf(lnr[f].x, acc[f][j + 1][r], bgv[r]));
            h[r] = f2bf(hv * gelu_f(gv));
          }
          const int c = j + (g >> 1);                  // output column 8 j + 4 g -> chunk j + g / 2
          *reinterpret_cast<uint2*>(stg + lr * 192 + sc(lr, c) * 16 + (g & 1) * 8) = *reinterpret_cast<const uint2*>(h);
        }
        asm volatile("" ::: "memory");
        const int NO = ne >> 1;
        bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int idx = le + 64 * i;
          if (idx >= 160) break;
          const int r = idx / 10, c = idx - (idx / 10) * 10;
          const uint4 x = *reinterpret_cast<const uint4*>(stg + r * 192 + sc(r, c) * 16);
          const int m = mf + r;
          if (m < p.M) *reinterpret_cast<uint4*>(out + (int64_t)m * NO + (nt0 >> 1) + 8 * c) = x;
        }
      } else {
        // pitch 320 B (20 chunks)
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const int n = nt0 + 16 * j + 4 * g;
          float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f), c4 = b4;
          b4 = *reinterpret_cast<const float4*>(colb + n - tb0 * BN);
          c4 = *reinterpret_cast<const float4*>(colc + n - tb0 * BN);
          const float bv[4] = {b4.x, b4.y, b4.z, b4.w}, cv[4] = {c4.x, c4.y, c4.z, c4.w};
          bf16_t h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = fmaf(lnr[f].y, cv[r], fmaf(lnr[f].x, acc[f][j][r], bv[r]));
            h[r] = f2bf(has_act ? act_f(v, p.act) : v);
          }
          const int c = 2 * j + (g >> 1);
          *reinterpret_cast<uint2*>(stg + lr * 320 + sc(lr, c) * 16 + (g & 1) * 8) = *reinterpret_cast<const uint2*>(h);
        }
        asm volatile("" ::: "memory");
        // 16 lanes per row: chunk c16 and, for c16 < 4, chunk 16 + c16; 4 rows per pass
        const int rg = le >> 4, c16 = le & 15;
        const bool two = c16 < 4;
        const bf16_t* res = reinterpret_cast<const bf16_t*>(p.residual);
        bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
        const int N = ne;
#pragma unroll
        for (int i0 = 0; i0 < 4; i0 += 2) {
        uint4 rv0[2], rv1[2];
        if (res) {
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int m = mf + (i0 + u) * 4 + rg;
            const int64_t o = (int64_t)min(m, p.M - 1) * N + nt0 + 8 * c16;
            rv0[u] = *reinterpret_cast<const uint4*>(res + o);
            rv1[u] = *reinterpret_cast<const uint4*>(res + o + (two ? 128 : 0));   // unconditional: no branch + vmcnt(0)
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int it = i0 + u;
          const int r = it * 4 + rg, m = mf + r;
          float v0[8], v1[8];
          unpack8(*reinterpret_cast<const uint4*>(stg + r * 320 + sc(r, c16) * 16), v0);
          unpack8(*reinterpret_cast<const uint4*>(stg + r * 320 + sc(r, (two ? 16 : 0) + c16) * 16), v1);
          if (res) {
            float r0[8], r1[8];
            unpack8(rv0[u], r0);
            unpack8(rv1[u], r1);
#pragma unroll
            for (int k = 0; k < 8; ++k) { v0[k] += r0[k]; v1[k] += r1[k]; }
          }
          const uint4 p0 = pack8(v0), p1 = pack8(v1);
          const int64_t o = (int64_t)m * N + nt0 + 8 * c16;
          if (m < p.M) {
            *reinterpret_cast<uint4*>(out + o) = p0;
            if (two) *reinterpret_cast<uint4*>(out + o + 128) = p1;
          }
          if (p.row_stats) {
            float s0[8], s1[8], a = 0.f, b = 0.f;
            unpack8(p0, s0);
            unpack8(p1, s1);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              a += s0[k];
              b += s0[k] * s0[k];
              if (two) { a += s1[k]; b += s1[k] * s1[k]; }
            }
#pragma unroll
            for (int o2 = 8; o2 > 0; o2 >>= 1) { a += __shfl_xor(a, o2, 64); b += __shfl_xor(b, o2, 64); }
            if (c16 == 0 && m < p.M) {
              unsafeAtomicAdd(p.row_stats + 2 * (int64_t)m, (double)a);
              unsafeAtomicAdd(p.row_stats + 2 * (int64_t)m + 1, (double)b);
            }
          }
        }
        }
      }
      asm volatile("" ::: "memory");   // this slice's staging reads precede the next slice's writes
    }
#pragma unroll
    for (int f = 0; f < RF; ++f)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
}

// legal: bf16 1x1 single-source GEMM, K = 320 exactly (no K padding), N a multiple of 160, NHWC
// (bias / activation / residual / row statistics / LayerNorm fold) or GEGLU (bias / LayerNorm
// fold); no time embedding, GroupNorm partials or split-K
int g_ars_mode = 0;   // tuning hook: 0 planner, 1 never, 2 whenever legal, 3 the one-block-per-CU form
bool ars_legal(const ldm_conv_params* q, int es, bool mixed) {
  const auto a16 = [](const void* x) { return (reinterpret_cast<uintptr_t>(x) & 15) == 0; };
  if (es != 2 || mixed || q->ksize != 1 || q->stride != 1 || q->upsample || q->c1 != 0 || q->pad_mode != 0) return false;
  if (q->c0 != 320 || q->kpad != 320 || q->n % ars::BN) return false;
  if (q->out_layout != LDM_OUT_NHWC && q->out_layout != LDM_OUT_GEGLU) return false;
  if (q->out_f32 || q->temb || q->gn_partial) return false;
  if (q->out_layout == LDM_OUT_GEGLU && (q->residual || q->row_stats || q->act != LDM_ACT_NONE)) return false;
  if (!a16(q->out) || !a16(q->residual) || !a16(q->bias) || !a16(q->ln_c1) || !a16(q->row_stats)) return false;
  if (q->ln_rows && (reinterpret_cast<uintptr_t>(q->ln_rows) & 15)) return false;
  return true;
}
// planner: 64x64-level shapes (>= 64 panels of 256 rows)
bool use_ars(const ldm_conv_params* q, int es, bool mixed, int M) {
  if (g_ars_mode == 1 || g_force_bm || !ars_legal(q, es, mixed)) return false;
  return g_ars_mode >= 2 || (M >= 64 * 256 && q->out_layout == LDM_OUT_GEGLU);
}

int launch_ars(ConvArgs a, hipStream_t s) {
  if (g_ars_mode != 3) {
    const int panels = (a.M + ars2::BM - 1) / ars2::BM;
    const int T = a.n / ars2::BN;
    const int nsplit = std::max((T + ars::MAXT - 1) / ars::MAXT, std::min(T, (512 + panels / 2) / panels));
    a.nblk = panels * nsplit;
    hipLaunchKernelGGL((gemm_ars2_kernel<10>), dim3(a.nblk), dim3(ars2::NT), 0, s, a, nsplit);
    LDM_CHECK_LAUNCH();
    return LDM_OK;
  }
  const int panels = (a.M + 255) / 256;
  const int T = a.n / ars::BN;
  const int nsplit = std::max((T + ars::MAXT - 1) / ars::MAXT, std::min(T, (256 + panels / 2) / panels));
  a.nblk = panels * nsplit;
  hipLaunchKernelGGL((gemm_ars_kernel<10, 4>), dim3(a.nblk), dim3(ars::NT), 0, s, a, nsplit);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
