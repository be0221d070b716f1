// Layout probe for v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands (gfx950), unit scales:
// A lane l holds A[row = l & 31][k = 32 (l >> 5) + j], j = 0..31 (byte j of its 8 dwords);
// B lane l holds B[k = 32 (l >> 5) + j][col = l & 31]; C lane l reg r = D[row (r&3) + 8 (r>>2) + 4 (l>>5)][col l&31].
// Prints the max |error| against a host product of the same e4m3 values (0 = layout confirmed).
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_f8_probe.hip -o tools/mfma_f8_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
typedef __attribute__((ext_vector_type(8))) int i32x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

__global__ void probe(const uint8_t* A, const uint8_t* B, float* D, int scale) {
  const int l = threadIdx.x;
  i32x8_t a, b;
  for (int w = 0; w < 8; ++w) {
    uint32_t va = 0, vb = 0;
    for (int e = 0; e < 4; ++e) {
      const int k = 32 * (l >> 5) + 4 * w + e;
      va |= (uint32_t)A[(l & 31) * 64 + k] << (8 * e);
      vb |= (uint32_t)B[k * 32 + (l & 31)] << (8 * e);
    }
    a[w] = (int)va;
    b[w] = (int)vb;
  }
  f32x16_t c;
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, scale, 0, scale);
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

static float e4m3(uint8_t v) {   // OCP e4m3fn decode
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float x = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + m / 8.f, e - 7);
  if (e == 15 && m == 7) x = NAN;
  return s ? -x : x;
}

int main() {
  uint8_t hA[32 * 64], hB[64 * 32];
  unsigned seed = 12345;
  auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return seed >> 24; };
  for (auto& v : hA) { v = rnd() & 0x7f; if (((v >> 3) & 15) == 15) v &= 0x77; if (rnd() & 1) v |= 0x80; }
  for (auto& v : hB) { v = rnd() & 0x7f; if (((v >> 3) & 15) == 15) v &= 0x77; if (rnd() & 1) v |= 0x80; }
  uint8_t *dA, *dB; float* dD;
  hipMalloc(&dA, sizeof(hA)); hipMalloc(&dB, sizeof(hB)); hipMalloc(&dD, 32 * 32 * 4);
  hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  float hD[32 * 32];
  volatile int scale = 127;     // E8M0 2^0, passed at run time
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, (int)scale);
  hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
  double maxerr = 0, maxref = 0;
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double ref = 0;
      for (int k = 0; k < 64; ++k) ref += (double)e4m3(hA[i * 64 + k]) * e4m3(hB[k * 32 + j]);
      maxerr = fmax(maxerr, fabs(ref - hD[i * 32 + j]));
      maxref = fmax(maxref, fabs(ref));
    }
  printf("mfma_scale_f32_32x32x64 e4m3 layout probe: max|err| %.3g (max|ref| %.3g) -> %s\n", maxerr, maxref,
         maxerr <= 1e-3 * maxref ? "LAYOUT OK" : "LAYOUT MISMATCH");
  return maxerr <= 1e-3 * maxref ? 0 : 1;
}
