// Scale-block probe for v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3, gfx950): which lane's E8M0 scale
// multiplies byte j of lane half hh of an A row (B column).  mfma_f8_probe.hip pins the byte layout
// only up to a k permutation shared by A and B (any such permutation gives the same product with unit
// scales); the 32-element scale blocks depend on the hardware k order.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_f8_scale_probe.hip -o tools/mfma_f8_scale_probe
// Trial (side, hh, j): one operand holds a single 1.0 at row / column 0, lane half hh, byte j, the
// other all 1.0; lane 0's scale for that operand is 2^1, lane 32's 2^2 (all others 2^0), so D[0][*]
// (A side) or D[*][0] (B side) reads 2 or 4: the scale of lane 0 or lane 32 applies to that byte.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((ext_vector_type(8))) int i32x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

__global__ void probe(int side, int hh, int j, float* D) {
  const int l = threadIdx.x;
  i32x8_t a, b;
  const uint32_t ones = 0x38383838u;   // e4m3 1.0 = 0x38
  for (int w = 0; w < 8; ++w) {
    uint32_t one_byte = 0;
    if ((l & 31) == 0 && (l >> 5) == hh && (j >> 2) == w) one_byte = 0x38u << (8 * (j & 3));
    a[w] = (int)(side == 0 ? one_byte : ones);
    b[w] = (int)(side == 0 ? ones : one_byte);
  }
  const int sc = l == 0 ? 128 : (l == 32 ? 129 : 127);
  f32x16_t c;
  for (int r = 0; r < 16; ++r) c[r] = 0.f;
  if (side == 0) c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sc, 0, 127);
  else c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, 127, 0, sc);
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

int main() {
  float* dD;
  hipMalloc(&dD, 32 * 32 * 4);
  float hD[32 * 32];
  for (int side = 0; side < 2; ++side) {
    std::printf("%s operand: byte j of lane half hh -> value (2: lane 0's scale, 4: lane 32's)\n", side ? "B" : "A");
    for (int hh = 0; hh < 2; ++hh) {
      std::printf("  hh=%d:", hh);
      for (int j = 0; j < 32; ++j) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, side, hh, j, dD);
        hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
        std::printf(" %g", side == 0 ? hD[0 * 32 + 5] : hD[5 * 32 + 0]);
      }
      std::printf("\n");
    }
  }
  hipFree(dD);
  return 0;
}
