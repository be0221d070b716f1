// WRITE_SIZE calibration for the store shapes of this library's epilogues (MI355X_MICROARCH.md
// "HBM": rocprofv3's WRITE_SIZE is calibrated only for 16-B-per-lane streaming stores).
//
//   hipcc --offload-arch=gfx950 -O3 tools/write_calib.hip -o tools/write_calib
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d OUT -o w -- tools/write_calib
//
// Every kernel writes exactly BYTES (64 MiB) of a [rows][640 B] bf16 matrix (320 channels per row,
// the 64x64-level activation width), one launch each:
//   st16_rows   16 B per lane, consecutive lanes consecutive 16 B (the staged row writer);
//   st8_rows    8 B per lane, consecutive lanes consecutive 8 B;
//   st8_dfrag   8 B per lane in the 16x16 MFMA accumulator layout (lane (g, lr): row lr, channels
//               4g..4g+3 of a 16-channel fragment; a wave instruction covers 16 rows x 32 B), the
//               fragments of a row written by consecutive instructions — the register GEGLU /
//               feed-forward epilogue shape;
//   st16_dpair  16 B per lane after the permlane pair (lane (g, lr): row lr, channels 8g..8g+7 of a
//               32-channel group; 16 rows x 64 B per instruction) — ldm_transformer_in's stores.
// The launch prints nothing; the counter values are read from the rocprofv3 CSV.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t BYTES = 64ull << 20;
constexpr int ROWB = 640;                      // bytes per row
constexpr int ROWS = (int)(BYTES / ROWB);       // 104857 rows
constexpr int NT = 256;

__global__ __launch_bounds__(NT) void st16_rows(uint4* out) {
  const size_t n = BYTES / 16;
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < n; i += (size_t)gridDim.x * NT)
    out[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}
__global__ __launch_bounds__(NT) void st8_rows(uint2* out) {
  const size_t n = BYTES / 8;
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < n; i += (size_t)gridDim.x * NT)
    out[i] = make_uint2((unsigned)i, 1u);
}
// one wave per 16-row block: 20 fragments of 16 channels x 16 rows, 8 B per lane each
__global__ __launch_bounds__(NT) void st8_dfrag(char* out) {
  const int lane = threadIdx.x & 63, g = lane >> 4, lr = lane & 15;
  const int wave = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int nblk = (ROWS + 15) / 16;
  for (int rb = wave; rb < nblk; rb += gridDim.x * (NT / 64)) {
    const int row = rb * 16 + lr;
    if (row >= ROWS) continue;
#pragma unroll
    for (int j = 0; j < 20; ++j)
      *reinterpret_cast<uint2*>(out + (size_t)row * ROWB + (16 * j + 4 * g) * 2) = make_uint2(row, j);
  }
}
__global__ __launch_bounds__(NT) void st16_dpair(char* out) {
  const int lane = threadIdx.x & 63, g = lane >> 4, lr = lane & 15;
  const int wave = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int nblk = (ROWS + 15) / 16;
  for (int rb = wave; rb < nblk; rb += gridDim.x * (NT / 64)) {
    const int row = rb * 16 + lr;
    if (row >= ROWS) continue;
#pragma unroll
    for (int p = 0; p < 10; ++p)
      *reinterpret_cast<uint4*>(out + (size_t)row * ROWB + (32 * p + 8 * g) * 2) = make_uint4(row, p, 0, 0);
  }
}

int main() {
  char* buf = nullptr;
  if (hipMalloc(&buf, BYTES + 4096) != hipSuccess) return 1;
  const int grid = 2048;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(st16_rows, dim3(grid), dim3(NT), 0, 0, reinterpret_cast<uint4*>(buf));
    hipLaunchKernelGGL(st8_rows, dim3(grid), dim3(NT), 0, 0, reinterpret_cast<uint2*>(buf));
    hipLaunchKernelGGL(st8_dfrag, dim3(grid), dim3(NT), 0, 0, buf);
    hipLaunchKernelGGL(st16_dpair, dim3(grid), dim3(NT), 0, 0, buf);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  hipFree(buf);
  std::printf("write_calib: 4 kernels x %zu bytes x 2\n", BYTES);
  return 0;
}
