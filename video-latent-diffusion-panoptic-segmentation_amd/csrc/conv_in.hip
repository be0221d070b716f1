// The UNet's conv_in in one launch (ldm_conv_in): /root/reference/ldmseg/models/unet.py:357 on the
// 8 / 12-channel conv modify_encoder builds (:178-233), read straight from the sampler's NCHW sources
// [x_t || rgb (|| cond)] (trainers_ldm_cond.py:1134-1141).  Unfused it is ldm_nchw_to_nhwc (the concat,
// fp32 -> bf16, 8 / 12 -> 16 channels) plus a K = 144 implicit GEMM on 128 x 160 tiles whose time goes
// to its epilogue (7.4 + 24.4 us at B = 8, profiles/r08_step_trace.txt) for 1.5 GFLOP and a 21 MB
// output.
//
// A block (4 waves) owns one output row of one image (W <= 64 pixels x N <= 320 channels; the packed
// weight is re-read per block, so the row, not a slice of it, is the unit — a (row, channel quarter)
// grid read the weight fragments 4x as often and ran slower than the two launches):
//   1. the three source rows (all 16 padded channels, every load in flight) staged in LDS as bf16 — the
//      values ldm_nchw_to_nhwc stores — channel-fastest, so each 8-channel half of a tap of a pixel is one
//      16-B LDS read: the MFMA A fragments (k = (ky, kx, c) tap-major) come straight from the staged rows,
//      no im2col copy (an im2col pass cost ~8 of 22 us);
//   2. wave w: channels N / 4 w .. + N / 4 over all pixels; its packed-weight fragments straight
//      from global (L2-resident: the whole [N][kpad] weight is 120 KB) into registers, 16x16x32 MFMAs
//      D[n][px] = W . A^T over the K steps that hold real taps (144 -> 5 x 32) — the same k32 chunks in
//      the same order as ldm_conv2d's tap-major K tiles, so the result is the two launches' bit for bit;
//   3. + bias, bf16, staged in LDS, stored as 16-B runs of the NHWC rows, and the GroupNorm unit
//      statistics of the stored values (fp32 per block, one fp64 atomic pair per unit) into slot
//      (row % slots) of the caller's zeroed accumulators — what the next GroupNorm consumes.
#include "common.h"

namespace {
namespace cin {
constexpr int NT = 256;
constexpr int MAXW = 64;
constexpr int MAXN = 320;
constexpr int CP = 16;                 // padded input channels
constexpr int KS = 5;                  // k32 steps: 9 taps x 16 = 144 <= 160
constexpr int NW = NT / 64;
}  // namespace cin

struct ConvInArgs {
  const void* src[3];
  int c[3], dt[3];
  int batch, H, W;
  const bf16_t* w;
  int n, kpad;
  const float* bias;
  bf16_t* out;
  double* gn;
  int unit, slots;
};

__device__ __forceinline__ float ld_src(const void* p, int64_t i, int dt) {
  return dt == LDM_BF16 ? bf2f(reinterpret_cast<const bf16_t*>(p)[i]) : reinterpret_cast<const float*>(p)[i];
}

template <int NPW>   // n-fragments of a wave's channel quarter (N / 64)
__global__ __launch_bounds__(256) void conv_in_kernel(const ConvInArgs a) {
  using namespace cin;
  constexpr int CG = 16 * NPW;                                // channels per wave (a quarter of N)
  constexpr int RW = MAXW + 2;                                // staged input row (x = -1 .. W)
  __shared__ __attribute__((aligned(16))) bf16_t R[3 * RW * CP];   // the three input rows [r][x + 1][c], bf16
  __shared__ uint4 Ts[MAXW * 4 * CG / 8];                     // the bf16 output row [px][N]
  __shared__ float red[NT * 2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int b = blockIdx.x / a.H, y = blockIdx.x - b * a.H;
  const int W = a.W, HW = a.H * a.W;
  const int n0 = wave * CG;

  // weight fragments first (their loads overlap the staging): lane (g, lr) of n-fragment j, step s
  // holds W[n0 + 16 j + lr][32 s + 8 g .. + 8]
  uint4 wf[NPW][KS];
#pragma unroll
  for (int j = 0; j < NPW; ++j)
#pragma unroll
    for (int s = 0; s < KS; ++s)
#ifndef CIN_ABL_NO_W
      wf[j][s] = *reinterpret_cast<const uint4*>(a.w + (int64_t)(n0 + 16 * j + lr) * a.kpad + 32 * s + 8 * g);
#else
      wf[j][s] = make_uint4(j + lr, s, g, 0u);
#endif

  // 1. the three source rows y - 1 .. y + 1 of all 16 (padded) channels, as bf16, channel-fastest:
  //    R[r][x + 1][c] (32 B per pixel), every global load in flight
  constexpr int NR = (3 * CP * RW + NT - 1) / NT;
  float rv[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int e = tid + NT * i;                               // e = (r, c, x + 1): x fastest (coalesced)
    const int r = e / (CP * RW), rem = e - r * (CP * RW), c = rem / RW, xx = rem - c * RW - 1;
    const int yy = y + r - 1;
    rv[i] = 0.f;
    if (e < 3 * CP * RW && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)W) {
      int cc = c, s = 0;
      while (s < 2 && cc >= a.c[s]) { cc -= a.c[s]; ++s; }
      if (cc < a.c[s]) rv[i] = ld_src(a.src[s], ((int64_t)b * a.c[s] + cc) * HW + (int64_t)yy * W + xx, a.dt[s]);
    }
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int e = tid + NT * i;
    const int r = e / (CP * RW), rem = e - r * (CP * RW), c = rem / RW, x1 = rem - c * RW;
    if (e < 3 * CP * RW) R[(r * RW + x1) * CP + c] = f2bf(rv[i]);
  }
  __syncthreads();

  // 2. D[n][px]: wave w takes its CG channels over all W / 16 pixel fragments.  The A fragment of
  //    pixel px, k chunk kc = 4 s + g (k = 16 tap + 8 h .. + 8: tap kc / 2, channel half kc % 2) is one
  //    16-B read of R at (ky, px + kx) — no im2col copy; chunks past tap 8 are zero
  const int nmf = W / 16;
  const uint4* R4 = reinterpret_cast<const uint4*>(R);
  f32x4_t acc[4][NPW];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < NPW; ++j) acc[m][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    if (m >= nmf) break;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int kc = 4 * s + g, tap = kc >> 1, h = kc & 1;
      const int ky = tap / 3, kx = tap - 3 * ky;
      Frag8<bf16_t> af;
      af.v = tap < 9 ? R4[(ky * RW + 16 * m + lr + kx) * 2 + h] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int j = 0; j < NPW; ++j) {
        Frag8<bf16_t> w8;
        w8.v = wf[j][s];
#ifndef CIN_ABL_NO_MFMA
        mma_k32(acc[m][j], w8, af);
#else
        acc[m][j][0] += __uint_as_float(w8.v.x ^ af.v.x);
#endif
      }
    }
  }
  // 3. + bias -> bf16 row [px][N] in LDS (lane: channels n0 + 16 j + 4 g .. + 3 of pixel 16 m + lr)
  const int N = a.n;
  bf16_t* T = reinterpret_cast<bf16_t*>(Ts);
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int n = n0 + 16 * j + 4 * g;
    const float4 b4 = *reinterpret_cast<const float4*>(a.bias + n);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if (m >= nmf) break;
      bf16_t h[4] = {f2bf(acc[m][j][0] + b4.x), f2bf(acc[m][j][1] + b4.y), f2bf(acc[m][j][2] + b4.z),
                     f2bf(acc[m][j][3] + b4.w)};
      *reinterpret_cast<uint2*>(T + (16 * m + lr) * N + n) = *reinterpret_cast<const uint2*>(h);
    }
  }
  __syncthreads();
  // the output row is one contiguous W x N run of the NHWC tensor: 16-B stores
  uint4* orow = reinterpret_cast<uint4*>(a.out + ((int64_t)b * HW + (int64_t)y * W) * N);
#ifndef CIN_ABL_NO_STORE   // (ablation builds)
  for (int i = tid; i < W * N / 8; i += NT) orow[i] = Ts[i];
#else
  if (Ts[tid].x == 0x12345u) orow[tid] = Ts[tid];
#endif
  if (!a.gn) return;
  // GroupNorm unit statistics of the stored values: thread (unit u, pixel part q)
  const int nu = N / a.unit, parts = NT / nu;
  const int u = tid % nu, q = tid / nu;
  float s1 = 0.f, s2 = 0.f;
  if (q < parts)
    for (int px = q; px < W; px += parts)
      for (int k = 0; k < a.unit; ++k) {
        const float v = bf2f(T[px * N + u * a.unit + k]);
        s1 += v;
        s2 = fmaf(v, v, s2);
      }
  red[2 * tid] = s1;
  red[2 * tid + 1] = s2;
  __syncthreads();
  if (tid < nu) {
    float t1 = 0.f, t2 = 0.f;
    for (int p = 0; p < parts; ++p) { t1 += red[2 * (p * nu + tid)]; t2 += red[2 * (p * nu + tid) + 1]; }
    double* d = a.gn + (((int64_t)b * a.slots + y % a.slots) * nu + tid) * 2;
    unsafeAtomicAdd(d, (double)t1);
    unsafeAtomicAdd(d + 1, (double)t2);
  }
}
}  // namespace

extern "C" int ldm_conv_in(const ldm_conv_in_params* p, ldm_stream_t stream) {
  using namespace cin;
  if (!p || !p->src[0] || !p->w || !p->bias || !p->out) return LDM_ERR_ARG;
  if (p->dtype != LDM_BF16 || p->batch <= 0 || p->height <= 0 || p->width <= 0 || p->width > MAXW || p->width % 16)
    return LDM_ERR_ARG;
  int ctot = 0;
  for (int i = 0; i < 3; ++i) {
    if (p->c[i] < 0 || (p->c[i] > 0 && !p->src[i]) || (p->c[i] > 0 && p->src_dtype[i] != LDM_F32 &&
                                                        p->src_dtype[i] != LDM_BF16))
      return LDM_ERR_ARG;
    ctot += p->c[i];
  }
  if (ctot <= 0 || ctot > CP || p->kpad < 9 * CP || p->kpad < 32 * KS || p->kpad % 8) return LDM_ERR_ARG;
  if (p->n % 64 || p->n > MAXN) return LDM_ERR_ARG;                       // 4 waves x 16k channels
  if (p->gn_partial && (p->gn_unit <= 0 || p->n % p->gn_unit || p->gn_slots <= 0 || p->n / p->gn_unit > NT))
    return LDM_ERR_ARG;
  const auto a16 = [](const void* x) { return (reinterpret_cast<uintptr_t>(x) & 15) == 0; };
  if (!a16(p->w) || !a16(p->out) || !a16(p->bias)) return LDM_ERR_ALIGN;
  ConvInArgs a{};
  for (int i = 0; i < 3; ++i) { a.src[i] = p->src[i]; a.c[i] = p->c[i]; a.dt[i] = p->src_dtype[i]; }
  a.batch = p->batch; a.H = p->height; a.W = p->width;
  a.w = static_cast<const bf16_t*>(p->w); a.n = p->n; a.kpad = p->kpad; a.bias = p->bias;
  a.out = static_cast<bf16_t*>(p->out);
  a.gn = p->gn_partial; a.unit = p->gn_unit; a.slots = p->gn_slots;
  const dim3 grid(p->batch * p->height);                                // one output row per block
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int npw = p->n / 64;
  if (npw == 5) hipLaunchKernelGGL(conv_in_kernel<5>, grid, dim3(NT), 0, s, a);
  else if (npw == 4) hipLaunchKernelGGL(conv_in_kernel<4>, grid, dim3(NT), 0, s, a);
  else if (npw == 2) hipLaunchKernelGGL(conv_in_kernel<2>, grid, dim3(NT), 0, s, a);
  else if (npw == 1) hipLaunchKernelGGL(conv_in_kernel<1>, grid, dim3(NT), 0, s, a);
  else return LDM_ERR_ARG;
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
