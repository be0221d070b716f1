// Microbenchmark: do MFMA and VALU instructions of DIFFERENT waves on one SIMD overlap on gfx950?
// 512-thread blocks (8 waves = 2 per SIMD), one block per CU.  Waves 0-3 run a stream of
// v_mfma_f32_32x32x16_bf16 (four independent accumulators), waves 4-7 a stream of VALU work
// (mode 1: v_exp_f32, mode 2: v_fma_f32, mode 3: v_pk_fma_f32), each on independent registers.
// Timed alone (the other half of the waves exits at once) and together.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_valu_overlap.hip -o /tmp/ovl && /tmp/ovl
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(16))) float f16x_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf8_t;
typedef __attribute__((ext_vector_type(2))) float f2_t;

template <int VMODE>
__global__ __launch_bounds__(512, 1) void ovl(float* out, int n_mfma, int n_valu, int run_mfma, int run_valu) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float sink = 0.f;
  if (wave < 4) {
    if (!run_mfma) return;
    f16x_t a0 = {}, a1 = {}, a2 = {}, a3 = {};
    bf8_t x, y;
    for (int i = 0; i < 8; ++i) { x[i] = (__bf16)(0.001f * (lane + i)); y[i] = (__bf16)(0.002f * (lane - i)); }
    for (int i = 0; i < n_mfma; ++i) {
      a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, a3, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) sink += a0[r] + a1[r] + a2[r] + a3[r];
  } else {
    if (!run_valu) return;
    float v[16];
    for (int k = 0; k < 16; ++k) v[k] = 0.001f * (lane + k);
    for (int i = 0; i < n_valu; ++i) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if constexpr (VMODE == 1) v[k] = __builtin_amdgcn_exp2f(v[k]) * -0.5f;
        else if constexpr (VMODE == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[k]) : "v"(0.999f), "v"(0.001f));
      }
      if constexpr (VMODE == 3) {
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
          f2_t p = {v[k], v[k + 1]};
          const f2_t m = {0.999f, 0.999f}, c = {0.001f, 0.001f};
          p = __builtin_elementwise_fma(p, m, c);
          v[k] = p[0];
          v[k + 1] = p[1];
        }
      }
    }
    for (int k = 0; k < 16; ++k) sink += v[k];
  }
  if (sink == 12345.f) out[blockIdx.x * 512 + threadIdx.x] = sink;
}

// same-wave interleave: every wave issues one MFMA then F independent VALU ops (v_exp_f32 when
// EXP, else v_fma_f32), in one instruction stream; 1 or 2 waves per SIMD (NW = 4 / 8)
template <bool EXP, int F>
__global__ __launch_bounds__(512, 1) void same_wave(float* out, int n, int do_mfma, int do_valu) {
  const int lane = threadIdx.x & 63;
  f16x_t a[4] = {};
  bf8_t x, y;
  for (int i = 0; i < 8; ++i) { x[i] = (__bf16)(0.001f * (lane + i)); y[i] = (__bf16)(0.002f * (lane - i)); }
  float v[16];
  for (int k = 0; k < 16; ++k) v[k] = 0.001f * (lane + k);
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (do_mfma) a[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, a[j], 0, 0, 0);
      if (do_valu) {
#pragma unroll
        for (int k = 0; k < F; ++k) {
          if constexpr (EXP) asm volatile("v_exp_f32 %0, %0" : "+v"(v[(4 * j + k) & 15]));
          else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[(4 * j + k) & 15]) : "v"(0.999f), "v"(0.001f));
        }
      }
    }
  }
  float sink = 0.f;
  for (int r = 0; r < 16; ++r) sink += a[0][r] + a[1][r] + a[2][r] + a[3][r] + v[r];
  if (sink == 12345.f) out[blockIdx.x * 512 + threadIdx.x] = sink;
}

template <bool EXP, int F>
float run_sw(float* d, int n, int nthreads, int m, int v) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((same_wave<EXP, F>), dim3(256), dim3(nthreads), 0, 0, d, n, m, v);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((same_wave<EXP, F>), dim3(256), dim3(nthreads), 0, 0, d, n, m, v);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5 * 1e3f;
}

template <bool EXP, int F>
void sw(float* d, const char* name, int nthreads) {
  const int n = 4000;
  const float tm = run_sw<EXP, F>(d, n, nthreads, 1, 0), tv = run_sw<EXP, F>(d, n, nthreads, 0, 1),
              tb = run_sw<EXP, F>(d, n, nthreads, 1, 1);
  printf("same-wave %-10s x%d, %d waves/SIMD: mfma %7.1f  valu %7.1f  both %7.1f us (sum %7.1f)\n", name, F,
         nthreads / 256, tm, tv, tb, tm + tv);
}

template <int VMODE>
float run(float* d, int nm, int nv, int rm, int rv) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(ovl<VMODE>, dim3(256), dim3(512), 0, 0, d, nm, nv, rm, rv);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(ovl<VMODE>, dim3(256), dim3(512), 0, 0, d, nm, nv, rm, rv);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5 * 1e3f;
}

template <int VMODE>
void mode(float* d, const char* name, int nm, int nv) {
  const float tm = run<VMODE>(d, nm, nv, 1, 0), tv = run<VMODE>(d, nm, nv, 0, 1), tb = run<VMODE>(d, nm, nv, 1, 1);
  printf("%-14s mfma alone %8.1f us   valu alone %8.1f us   both %8.1f us   (sum %8.1f, overlap %5.1f %%)\n", name, tm,
         tv, tb, tm + tv, 100.f * (tm + tv - tb) / (tm < tv ? tm : tv));
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 512 * sizeof(float));
  // per wave: 4 n_mfma MFMAs x 32 cycles; VALU: 16 n_valu instructions (exp 8 cyc, fma 4 cyc issue)
  mode<1>(d, "v_exp_f32", 4000, 4000);
  mode<2>(d, "v_fma_f32", 4000, 8000);
  mode<3>(d, "v_pk_fma_f32", 4000, 8000);
  sw<true, 1>(d, "v_exp_f32", 256);
  sw<true, 2>(d, "v_exp_f32", 256);
  sw<true, 4>(d, "v_exp_f32", 256);
  sw<false, 4>(d, "v_fma_f32", 256);
  sw<false, 6>(d, "v_fma_f32", 256);
  sw<true, 2>(d, "v_exp_f32", 512);
  sw<false, 4>(d, "v_fma_f32", 512);
  hipFree(d);
  return 0;
}
