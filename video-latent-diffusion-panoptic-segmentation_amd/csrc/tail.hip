// The UNet tail in one launch (ldm_unet_tail): conv_norm_out (GroupNorm) -> SiLU -> conv_out
// (3x3, C -> cout = 4) -> optionally the DDIM step of the sampler
// (/root/reference/ldmseg/models/unet.py:428-431, ldmseg/schedulers/ddim_scheduler.py:218-269,
// trainers_ldm_cond.py:1144-1162).  Unfused it is three launches that re-read the 21 MB activation
// (GroupNorm apply 12.5 us, conv_out on 32-column MFMA tiles padded from 4 outputs 41 us, DDIM 4 us).
//
// A block (8 waves) owns R = 2 output rows of one image (all W <= 64 pixels, all cout channels); blocks are
// numbered XCD-contiguously so one image's row pairs share an XCD and its L2 serves the halo rows a
// neighbour also reads.  Per 64-channel block the (R + 2) x (W + 2) input halo is loaded once (the
// next block's loads in flight during this block's MFMAs), normalised with the producer's GroupNorm
// accumulators (the gn_apply arithmetic: y = silu(x * scale + shift) rounded to bf16), zero outside
// the image (conv padding after the activation), and stored in LDS with the 16-B chunk swizzle
// c ^ (pixel & 7).  The conv is 16x16x32 bf16 MFMA on D[n][m] = W . A^T with the weight rows
// (n = output channel) padded from cout to 16 by zero lanes: the MFMA work (0.75 GFLOP padded) is
// ~1 us of the chip; the launch is bound by one read of the activation.  Epilogue: bias, the model
// output rounded to its dtype (bf16 on the bf16 path, as the unfused conv stores it), NCHW stores,
// and with the DDIM step fused the (prev, x0) pair from the same device arithmetic as ldm_ddim_step.
#include "common.h"

namespace {
namespace tail {
constexpr int NT = 512;
constexpr int R = 2;           // output rows per block
constexpr int CB = 64;         // channels per halo block
constexpr int MAXW = 64;
constexpr int MAXC = 640;
constexpr int HP = MAXW + 2;   // halo pixels per row
constexpr int HALO_U4 = (R + 2) * HP * (CB / 8);     // 16-B chunks per halo buffer (2112)
constexpr int PER = (HALO_U4 + NT - 1) / NT;         // chunks per thread (5)
constexpr int HALO_PAD = PER * NT;                   // every thread's PER slots exist (no branch)
}  // namespace tail

struct TailArgs {
  const bf16_t* h;
  int batch, H, W, C;
  const double* acc;
  int unit, slots, groups;
  float eps;
  const float* gamma;
  const float* beta;
  const bf16_t* w;
  int kpad, cout;
  const float* bias;
  void* eps_out;
  int eps_dt;
  const void* sample;
  int sample_dt;
  const int64_t* t;
  const float* ac;
  float final_ac;
  int step_ratio, pred, clip;
  float clip_range;
  int use_clipped, ntrain;
  void* prev;
  void* x0;
  int out_dt;
};

__device__ __forceinline__ float ld_any(const void* p, int64_t i, int dt) {
  return dt == LDM_BF16 ? bf2f(reinterpret_cast<const bf16_t*>(p)[i]) : reinterpret_cast<const float*>(p)[i];
}
__device__ __forceinline__ void st_any(void* p, int64_t i, float v, int dt) {
  if (dt == LDM_BF16) reinterpret_cast<bf16_t*>(p)[i] = f2bf(v);
  else reinterpret_cast<float*>(p)[i] = v;
}

__global__ __launch_bounds__(512) void unet_tail_kernel(const TailArgs a) {
  using namespace tail;
  __shared__ uint4 halo[2][HALO_PAD];
  __shared__ __attribute__((aligned(16))) float2 ss[MAXC];   // per-channel (scale, shift) of this image
  __shared__ float2 gst[64];
  __shared__ double2 ured[2 * 64 * 8];             // slots x units accumulators (<= 1024 entries)
  __shared__ uint4 wl[4 * 9 * MAXC / 8];           // conv_out weight rows [cout][9 C] bf16

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;
  const int H = a.H, W = a.W, C = a.C, HPw = W + 2;
  const int rpi = H / R;                            // row tiles per image
  int tile;
  {
    const int nblk = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, qq = nblk >> 3, rem = nblk & 7;
    tile = (xcd < rem ? xcd * (qq + 1) : rem * (qq + 1) + (xcd - rem) * qq) + (bid >> 3);
  }
  const int b = tile / rpi, y0 = (tile - b * rpi) * R;
  const int ncb = C / CB;
  const int nhalo = (R + 2) * HPw * (CB / 8);       // chunks of this width's halo

  // this thread's halo chunks (the same pixels for every channel block): global element offset of the
  // chunk at channel block 0 (-1 outside the image or past the halo) and its swizzled LDS slot
  int gofs[PER], lslot[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int q = tid + NT * i;
    const int hp = q >> 3, ch = q & 7;
    const int hr = hp / HPw, hc = hp - hr * HPw;
    const int y = y0 - 1 + hr, x = hc - 1;
    lslot[i] = q < nhalo ? hp * 8 + (ch ^ (hc & 7)) : q;     // past the halo: a padding slot
    gofs[i] = (q < nhalo && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W)
                  ? (int)((((int64_t)b * H + y) * W + x) * C + ch * 8) : -1;
  }
  // two channel blocks of loads in flight (80 KB per CU): the block before last's MFMAs and this
  // block's transform hide them
  // raw buffer loads: an offset past the buffer (outside the image) reads zeros, no branch
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.h, 0, (int)((int64_t)a.batch * H * W * C * 2), 0x00020000);
  int boff[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) boff[i] = gofs[i] >= 0 ? gofs[i] * 2 : 0x7ffff000;
  uint4 raw[2][PER];
  auto load = [&](int cb, uint4 (&r)[PER]) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
#ifdef TAIL_ABL_NO_LOAD
      r[i] = make_uint4(0u, 0u, 0u, 0u);
#else
      r[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rh, boff[i] + cb * CB * 2, 0, 0));
#endif
    }
  };
  load(0, raw[0]);
  if (ncb > 1) load(1, raw[1]);

  // GroupNorm (mean, rstd) per group of image b from the producer's unit accumulators (gn_apply's
  // arithmetic), then per-channel (scale, shift); the conv_out weight rows into LDS
  const int un = C / a.unit, upg = C / a.groups / a.unit, cpg = C / a.groups;
  for (int i = tid; i < a.slots * un; i += NT) {
    const int sl = i / un, u = i - sl * un;
    ured[i] = *reinterpret_cast<const double2*>(a.acc + (((int64_t)b * a.slots + sl) * un + u) * 2);
  }
  const int kw = 9 * C / 8;                         // 16-B chunks per weight row
  for (int i = tid; i < a.cout * kw; i += NT) {
    const int n = i / kw, k = i - n * kw;
    wl[i] = *reinterpret_cast<const uint4*>(a.w + (int64_t)n * a.kpad + k * 8);
  }
  __syncthreads();
  for (int gi = tid; gi < a.groups; gi += NT) {
    double sa = 0.0, sq = 0.0;
    for (int sl = 0; sl < a.slots; ++sl)
      for (int k = 0; k < upg; ++k) {
        const double2 v = ured[sl * un + gi * upg + k];
        sa += v.x;
        sq += v.y;
      }
    const double cnt = (double)H * W * cpg;
    const double mean = sa / cnt;
    double var = sq / cnt - mean * mean;
    if (var < 0.0) var = 0.0;
    gst[gi] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)a.eps)));
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    const float2 ms = gst[c / cpg];
    const float sc = ms.y * a.gamma[c];
    ss[c] = make_float2(sc, fmaf(-ms.x, sc, a.beta[c]));
  }
  __syncthreads();

  // output fragments: 16 consecutive pixels of one output row; wave w takes fragments w, w + 8
  const int fpr = W / 16;                           // fragments per row
  const int nfrag = R * fpr;                        // <= 8
  f32x4_t acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const bool wok = lr < a.cout;
  const int wrow = wok ? lr : 0;
  auto stage = [&](int cb, uint4 (&rw)[PER]) {
    uint4* hb = halo[cb & 1];
    // normalise + SiLU the loaded chunks into LDS (zeros stay zero: padding after the activation)
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const bf16_t* e = reinterpret_cast<const bf16_t*>(&rw[i]);
      const float4* s4 = reinterpret_cast<const float4*>(ss + cb * CB + ((tid + NT * i) & 7) * 8);
      bf16_t o[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 q = s4[j];                    // (scale, shift) of channels 2j, 2j + 1
#ifdef TAIL_ABL_NO_XFORM
        o[2 * j] = e[2 * j];
        o[2 * j + 1] = e[2 * j + 1] ^ (bf16_t)(q.x == 12345.f);
#else
        o[2 * j] = f2bf(silu_f(fmaf(bf2f(e[2 * j]), q.x, q.y)));
        o[2 * j + 1] = f2bf(silu_f(fmaf(bf2f(e[2 * j + 1]), q.z, q.w)));
#endif
      }
      const uint4 v = *reinterpret_cast<const uint4*>(o);
      const bool in = gofs[i] >= 0;                  // outside the image: zero (padding after SiLU)
      hb[lslot[i]] = make_uint4(in ? v.x : 0u, in ? v.y : 0u, in ? v.z : 0u, in ? v.w : 0u);
    }
    if (cb + 2 < ncb) load(cb + 2, rw);              // two blocks ahead, into the buffer just consumed
  };
  // the channel-block loop unrolled by two: raw[0] / raw[1] keep fixed registers (a runtime-selected
  // buffer made hipcc copy them at the back edge and wait for the prefetch loads it had just issued)
  auto mfma_block = [&](int cb) {
    uint4* hb = halo[cb & 1];
#pragma unroll
    for (int fi = 0; fi < 2; ++fi) {
      const int f = wave + 8 * fi;
      if (f >= nfrag) break;
      const int ry = f / fpr, x0 = (f - ry * fpr) * 16;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
        const int hc = x0 + lr + kx;
        const int hp = (ry + ky) * HPw + hc;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          Frag8<bf16_t> wf, af;
          const uint4 wv = wl[wrow * kw + (tap * C + cb * CB + ks * 32) / 8 + g];   // branch-free zero rows
          wf.v = make_uint4(wok ? wv.x : 0u, wok ? wv.y : 0u, wok ? wv.z : 0u, wok ? wv.w : 0u);
          af.v = hb[hp * 8 + ((ks * 4 + g) ^ (hc & 7))];
#ifdef TAIL_ABL_NO_MFMA
          asm volatile("" ::"v"(wf.v.x), "v"(af.v.x));
#else
          mma_k32(acc[fi], wf, af);                  // D[n][m]: lane (g, lr) channels 4g.., pixel lr
#endif
        }
      }
    }
    // the next iteration writes the other buffer; the one after rewrites this one behind its barrier
  };
#ifndef TAIL_ABL_NO_LOOP
  for (int cb = 0; cb < ncb; cb += 2) {
    stage(cb, raw[0]);
    __syncthreads();
    mfma_block(cb);
    if (cb + 1 >= ncb) break;
    stage(cb + 1, raw[1]);
    __syncthreads();
    mfma_block(cb + 1);
  }
#else
  if (raw[0][0].x == 12345u && raw[1][0].x == 777u) acc[0][0] = 1.f;
#endif

  // epilogue: lanes g = 0 hold channels 0..3 of pixel lr (cout <= 4 real rows of the 16)
  if (g != 0) return;
  DdimCoef dc{};
  const bool ddim = a.prev || a.x0;
  if (ddim) dc = ddim_coef(a.ac, *a.t, a.step_ratio, a.final_ac, a.ntrain);
#pragma unroll
  for (int fi = 0; fi < 2; ++fi) {
    const int f = wave + 8 * fi;
    if (f >= nfrag) break;
    const int ry = f / fpr, x = (f - ry * fpr) * 16 + lr;
    const int y = y0 + ry;
    float smp[4] = {0.f, 0.f, 0.f, 0.f};
    if (ddim) {                                      // every sample load in flight before any math
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r < a.cout) smp[r] = ld_any(a.sample, (((int64_t)b * a.cout + r) * H + y) * W + x, a.sample_dt);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r >= a.cout) break;
      float m = acc[fi][r] + a.bias[r];
      if (a.eps_dt == LDM_BF16) m = bf2f(f2bf(m));    // the model output as the unfused conv stores it
      const int64_t idx = (((int64_t)b * a.cout + r) * H + y) * W + x;
      if (a.eps_out) st_any(a.eps_out, idx, m, a.eps_dt);
      if (ddim) {
        const float2 pr = ddim_apply(dc, m, smp[r], a.pred, a.clip, a.clip_range, a.use_clipped);
        if (a.prev) st_any(a.prev, idx, pr.x, a.out_dt);
        if (a.x0) st_any(a.x0, idx, pr.y, a.out_dt);
      }
    }
  }
}
}  // namespace

extern "C" int ldm_unet_tail(const ldm_unet_tail_params* p, ldm_stream_t stream) {
  using namespace tail;
  if (!p || !p->h || !p->gn_acc || !p->gamma || !p->beta || !p->w || !p->bias) return LDM_ERR_ARG;
  if (p->batch <= 0 || p->height <= 0 || p->height % R || p->width <= 0 || p->width > MAXW || p->width % 16)
    return LDM_ERR_ARG;
  if (p->c <= 0 || p->c % CB || p->c > MAXC || p->cout <= 0 || p->cout > 4 || p->kpad < 9 * p->c || p->kpad % 8)
    return LDM_ERR_ARG;
  if (p->groups <= 0 || p->groups > 64 || p->c % p->groups || p->gn_unit <= 0 || (p->c / p->groups) % p->gn_unit ||
      p->gn_slots <= 0 || p->gn_slots * (p->c / p->gn_unit) > 1024)
    return LDM_ERR_ARG;
  const bool ddim = p->prev || p->x0;
  if (!p->eps_out && !ddim) return LDM_ERR_ARG;
  if (p->eps_dtype != LDM_F32 && p->eps_dtype != LDM_BF16) return LDM_ERR_ARG;
  if (ddim && (!p->sample || !p->t || !p->alphas_cumprod || p->step_ratio <= 0 || p->num_train_timesteps <= 0 ||
               p->prediction_type < 0 || p->prediction_type > 2 ||
               (p->out_dtype != LDM_F32 && p->out_dtype != LDM_BF16) ||
               (p->sample_dtype != LDM_F32 && p->sample_dtype != LDM_BF16)))
    return LDM_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(p->h) & 15) || (reinterpret_cast<uintptr_t>(p->w) & 15)) return LDM_ERR_ALIGN;
  // the kernel works in int BYTE offsets with 0x7ffff000 as the zero-padding sentinel: the tensor's
  // byte size must stay below the sentinel so offsets never wrap and the sentinel is always out of range
  if ((int64_t)p->batch * p->height * p->width * p->c * 2 >= (1LL << 31) - 4096) return LDM_ERR_ARG;
  TailArgs a;
  a.h = static_cast<const bf16_t*>(p->h);
  a.batch = p->batch; a.H = p->height; a.W = p->width; a.C = p->c;
  a.acc = p->gn_acc; a.unit = p->gn_unit; a.slots = p->gn_slots; a.groups = p->groups; a.eps = p->eps;
  a.gamma = p->gamma; a.beta = p->beta;
  a.w = static_cast<const bf16_t*>(p->w); a.kpad = p->kpad; a.cout = p->cout; a.bias = p->bias;
  a.eps_out = p->eps_out; a.eps_dt = p->eps_dtype;
  a.sample = p->sample; a.sample_dt = p->sample_dtype; a.t = p->t; a.ac = p->alphas_cumprod;
  a.final_ac = p->final_alpha_cumprod; a.step_ratio = p->step_ratio; a.pred = p->prediction_type;
  a.clip = p->clip_sample; a.clip_range = p->clip_range; a.use_clipped = p->use_clipped_model_output;
  a.ntrain = p->num_train_timesteps; a.prev = p->prev; a.x0 = p->x0; a.out_dt = p->out_dtype;
  const int blocks = p->batch * (p->height / R);
  hipLaunchKernelGGL(unet_tail_kernel, dim3(blocks), dim3(NT), 0, reinterpret_cast<hipStream_t>(stream), a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
