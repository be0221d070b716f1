// Implicit-GEMM convolution / GEMM on CDNA4 MFMA (ldm_conv2d).
//
// One kernel covers every matmul-shaped op of the denoising path: 3x3 convs (stride 1/2,
// optional nearest-2x upsampled input, optional two-source channel concat), 1x1 convs /
// linears, and the ConvTranspose k2s2 of the seg-VAE decoder (pixel-shuffle epilogue).
//   rows m   = output pixels (b, oy, ox)              [NHWC activations]
//   cols n   = output channels                         [weights packed n-major, K contiguous]
//   k        = (ky, kx, c) tap-major                    [K tiles of 128 bytes]
// Tile BM x BN x (128 B of K); 256 threads = 2x2 waves, each wave (BM/2) x (BN/2) built from
// 16x16 MFMA fragments.  Operands are staged global -> registers -> LDS (XOR-swizzled 16-B
// chunks, conflict-free ds_read_b128), double-buffered with one barrier per K tile; the
// register stage is where conv zero-padding, upsample and concat addressing happen.
// The same code runs bf16 (v_mfma_f32_16x16x32_bf16) and exact fp32 (v_mfma_f32_16x16x4_f32).
#include "common.h"

namespace {

struct ConvArgs {
  const char* a0;
  const char* a1;
  int c0, c1, cin;
  int batch, h_in, w_in, h_out, w_out, hw_out;
  int ksize, stride, upsample, pad;
  const char* w;
  int n, kpad, K;
  const float* bias;
  const float* temb;
  int temb_stride;
  const char* residual;
  char* out;
  int out_layout, act, out_f32;
  int M;
};

__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void igemm_kernel(const ConvArgs p) {
  constexpr int ES = sizeof(T);
  constexpr int BK = 128 / ES;  // elements per K tile
  constexpr int CE = 16 / ES;   // elements per 16-byte chunk
  constexpr int AI = BM / 32;   // A chunks per thread per K tile
  constexpr int BI = BN / 32;
  constexpr int FM = BM / 32;   // 16x16 fragments per wave along M (wave tile = BM/2)
  constexpr int FN = BN / 32;
  __shared__ uint4 smem[2 * (BM + BN) * 8];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int cc = tid & 7, rr = tid >> 3;

  int a_b[AI], a_y[AI], a_x[AI];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + rr + 32 * i;
    a_ok[i] = m < p.M;
    const int b = m / p.hw_out;
    const int pix = m - b * p.hw_out;
    a_b[i] = b;
    a_y[i] = pix / p.w_out;
    a_x[i] = pix - a_y[i] * p.w_out;
  }

  uint4 ra[AI], rb[BI];
  const uint4 zero4 = make_uint4(0, 0, 0, 0);

  auto load_tile = [&](int kt) {
    const int k = kt * BK + cc * CE;
    const bool kval = k < p.K;
    const int tap = k / p.cin;
    const int ch = k - tap * p.cin;
    const int ky = tap / p.ksize;
    const int kx = tap - ky * p.ksize;
    const char* src;
    int cs, choff;
    if (ch < p.c0) { src = p.a0; cs = p.c0; choff = ch; }
    else { src = p.a1; cs = p.c1; choff = ch - p.c0; }
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      bool ok = a_ok[i] && kval;
      int iy, ix;
      if (p.upsample) {
        const int uy = a_y[i] + ky - p.pad, ux = a_x[i] + kx - p.pad;
        ok = ok && uy >= 0 && uy < 2 * p.h_in && ux >= 0 && ux < 2 * p.w_in;
        iy = uy >> 1;
        ix = ux >> 1;
      } else {
        iy = a_y[i] * p.stride + ky - p.pad;
        ix = a_x[i] * p.stride + kx - p.pad;
        ok = ok && iy >= 0 && iy < p.h_in && ix >= 0 && ix < p.w_in;
      }
      const int64_t off = ((((int64_t)a_b[i] * p.h_in + iy) * p.w_in + ix) * cs + choff) * ES;
      ra[i] = ok ? *reinterpret_cast<const uint4*>(src + off) : zero4;
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int n = n0 + rr + 32 * i;
      const int64_t off = ((int64_t)n * p.kpad + kt * BK + cc * CE) * ES;
      rb[i] = (n < p.n) ? *reinterpret_cast<const uint4*>(p.w + off) : zero4;
    }
  };

  auto store_tile = [&](int buf) {
    uint4* As = smem + buf * (BM + BN) * 8;
    uint4* Bs = As + BM * 8;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int r = rr + 32 * i;
      As[r * 8 + swz(r, cc)] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int r = rr + 32 * i;
      Bs[r * 8 + swz(r, cc)] = rb[i];
    }
  };

  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, g = lane >> 4;
  auto compute = [&](int buf) {
    const uint4* As = smem + buf * (BM + BN) * 8;
    const uint4* Bs = As + BM * 8;
    constexpr int KSTEPS = (ES == 2) ? 2 : 1;  // 32-wide k steps per tile
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      Frag8<T> af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * (BM / 2) + i * 16 + lr;
        if constexpr (ES == 2) {
          af[i].v = As[r * 8 + swz(r, ks * 4 + g)];
        } else {
          reinterpret_cast<Frag8<float>&>(af[i]).v[0] = As[r * 8 + swz(r, 2 * g)];
          reinterpret_cast<Frag8<float>&>(af[i]).v[1] = As[r * 8 + swz(r, 2 * g + 1)];
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * (BN / 2) + j * 16 + lr;
        if constexpr (ES == 2) {
          bfr[j].v = Bs[r * 8 + swz(r, ks * 4 + g)];
        } else {
          reinterpret_cast<Frag8<float>&>(bfr[j]).v[0] = Bs[r * 8 + swz(r, 2 * g)];
          reinterpret_cast<Frag8<float>&>(bfr[j]).v[1] = Bs[r * 8 + swz(r, 2 * g + 1)];
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) mma_k32(acc[i][j], af[i], bfr[j]);
    }
  };

  const int nk = p.kpad / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load_tile(kt + 1);
    compute(kt & 1);
    if (more) store_tile((kt + 1) & 1);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  const int N = p.n;
  if (p.out_layout == LDM_OUT_GEGLU) {
    // columns are packed in 16-wide (hidden, gate) pairs: fragment j even = hidden, j+1 = gate
    const int nout = N >> 1;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
        const int np = n0 + wn * (BN / 2) + j * 16;  // packed column of this pair (multiple of 32)
        const int nh = np + lr, ng = np + 16 + lr;
        const int nc = (np >> 1) + lr;
        if (nh >= N) continue;
        const float bh = p.bias ? p.bias[nh] : 0.f;
        const float bg = p.bias ? p.bias[ng] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * (BM / 2) + i * 16 + g * 4 + r;
          if (m >= p.M) continue;
          const float h = acc[i][j][r] + bh;
          const float gt = acc[i][j + 1][r] + bg;
          const float v = h * gelu_f(gt);
          const int64_t idx = (int64_t)m * nout + nc;
          if (p.out_f32) reinterpret_cast<float*>(p.out)[idx] = v;
          else Elem<T>::store(reinterpret_cast<T*>(p.out) + idx, v);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + lr;
      if (n >= N) continue;
      const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + g * 4 + r;
        if (m >= p.M) continue;
        const int b = m / p.hw_out;
        float v = acc[i][j][r] + bn;
        if (p.temb) v += p.temb[(int64_t)b * p.temb_stride + n];
        if (p.act == LDM_ACT_SILU) v = silu_f(v);
        int64_t idx;
        if (p.out_layout == LDM_OUT_NHWC) {
          idx = (int64_t)m * N + n;
        } else if (p.out_layout == LDM_OUT_NCHW) {
          const int pix = m - b * p.hw_out;
          idx = ((int64_t)b * N + n) * p.hw_out + pix;
        } else {  // LDM_OUT_SHUFFLE2: n = (dy*2+dx)*Cout + co -> pixel (2y+dy, 2x+dx)
          const int cout = N >> 2;
          const int q = n / cout, co = n - q * cout;
          const int dy = q >> 1, dx = q & 1;
          const int pix = m - b * p.hw_out;
          const int y = pix / p.w_out, x = pix - y * p.w_out;
          idx = (((int64_t)b * 2 * p.h_out + 2 * y + dy) * 2 * p.w_out + 2 * x + dx) * cout + co;
        }
        if (p.residual) v += to_f(reinterpret_cast<const T*>(p.residual)[idx]);
        if (p.out_f32) reinterpret_cast<float*>(p.out)[idx] = v;
        else Elem<T>::store(reinterpret_cast<T*>(p.out) + idx, v);
      }
    }
  }
}

template <typename T, int BM, int BN>
int launch_bm_bn(const ConvArgs& a, hipStream_t s) {
  dim3 grid((a.n + BN - 1) / BN, (a.M + BM - 1) / BM);
  hipLaunchKernelGGL((igemm_kernel<T, BM, BN>), grid, dim3(256), 0, s, a);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

template <typename T, int BM>
int launch_bm(const ConvArgs& a, hipStream_t s, int bn) {
  if (bn == 32) return launch_bm_bn<T, BM, 32>(a, s);
  if (bn == 64) return launch_bm_bn<T, BM, 64>(a, s);
  return launch_bm_bn<T, BM, 128>(a, s);
}

template <typename T>
int launch_t(const ConvArgs& a, hipStream_t s, int bm, int bn) {
  if (bm == 32) return launch_bm<T, 32>(a, s, bn);
  if (bm == 64) return launch_bm<T, 64>(a, s, bn);
  return launch_bm<T, 128>(a, s, bn);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int ldm_conv2d(const ldm_conv_params* q, ldm_stream_t stream) {
  if (!q) return LDM_ERR_ARG;
  if (q->dtype != LDM_F32 && q->dtype != LDM_BF16) return LDM_ERR_ARG;
  const int es = q->dtype == LDM_F32 ? 4 : 2;
  const int ce = 16 / es;
  if (q->ksize != 1 && q->ksize != 3) return LDM_ERR_ARG;
  if (q->stride != 1 && q->stride != 2) return LDM_ERR_ARG;
  if (q->upsample && (q->stride != 1)) return LDM_ERR_ARG;
  if (q->batch <= 0 || q->h_in <= 0 || q->w_in <= 0 || q->h_out <= 0 || q->w_out <= 0) return LDM_ERR_ARG;
  if (q->c0 <= 0 || q->c1 < 0 || (q->c1 > 0 && !q->a1)) return LDM_ERR_ARG;
  if (q->c0 % ce || q->c1 % ce) return LDM_ERR_ALIGN;
  if (q->kpad % 64) return LDM_ERR_ALIGN;
  const int cin = q->c0 + q->c1;
  const int K = q->ksize * q->ksize * cin;
  if (K > q->kpad || q->n <= 0) return LDM_ERR_ARG;
  if (!aligned16(q->a0) || (q->a1 && !aligned16(q->a1)) || !aligned16(q->w)) return LDM_ERR_ALIGN;
  const int pad = q->ksize / 2;
  const int hin_eff = q->upsample ? 2 * q->h_in : q->h_in;
  const int win_eff = q->upsample ? 2 * q->w_in : q->w_in;
  if (q->h_out != (hin_eff + 2 * pad - q->ksize) / q->stride + 1) return LDM_ERR_ARG;
  if (q->w_out != (win_eff + 2 * pad - q->ksize) / q->stride + 1) return LDM_ERR_ARG;
  if (q->out_layout == LDM_OUT_GEGLU && (q->n % 32 || q->residual || q->temb)) return LDM_ERR_ARG;
  if (q->out_layout == LDM_OUT_SHUFFLE2 && (q->n % 4 || q->temb || q->upsample)) return LDM_ERR_ARG;
  const int64_t M64 = (int64_t)q->batch * q->h_out * q->w_out;
  if (M64 >= (1LL << 31)) return LDM_ERR_ARG;

  ConvArgs a;
  a.a0 = static_cast<const char*>(q->a0);
  a.a1 = static_cast<const char*>(q->a1);
  a.c0 = q->c0; a.c1 = q->c1; a.cin = cin;
  a.batch = q->batch; a.h_in = q->h_in; a.w_in = q->w_in;
  a.h_out = q->h_out; a.w_out = q->w_out; a.hw_out = q->h_out * q->w_out;
  a.ksize = q->ksize; a.stride = q->stride; a.upsample = q->upsample; a.pad = pad;
  a.w = static_cast<const char*>(q->w);
  a.n = q->n; a.kpad = q->kpad; a.K = K;
  a.bias = q->bias; a.temb = q->temb; a.temb_stride = q->temb_stride;
  a.residual = static_cast<const char*>(q->residual);
  a.out = static_cast<char*>(q->out);
  a.out_layout = q->out_layout; a.act = q->act; a.out_f32 = q->out_f32;
  a.M = (int)M64;

  const int bm = a.M <= 32 ? 32 : (a.M <= 64 ? 64 : 128);
  int bn = a.n <= 32 ? 32 : (a.n <= 64 ? 64 : 128);
  if (q->out_layout == LDM_OUT_GEGLU && bn < 64) bn = 64;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  return q->dtype == LDM_BF16 ? launch_t<bf16_t>(a, s, bm, bn) : launch_t<float>(a, s, bm, bn);
}
