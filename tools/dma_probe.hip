// Probe: per-CU LDS-DMA (buffer_load_dwordx4 ... lds) delivery rate for the operand pattern of the
// GEMM kernels (8 rows x 128 B per wave instruction, 72 KB per K tile per CU, 512 threads).
//   ./dma_probe            prints GB/s per CU for each variant
// Variants: src = one 72 KB region shared by every block (L2-resident) / a private region per
// block walked through a 256 MB buffer (HBM / Infinity Cache); in-flight = one or two K tiles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kBufFlags = 0x00020000;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, int voff, unsigned lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds_addr)
      : "memory");
}

// one K tile = 576 rows x 128 B (256 A rows + 320 B rows), 9 instructions per wave
template <int INFLIGHT>
__global__ __launch_bounds__(512, 1) void probe(const char* src, int src_bytes, int shared, int iters, int row_stride,
                                                float* sink) {
  __shared__ uint4 smem[2 * 576 * 8];
  typedef __attribute__((address_space(3))) uint4 lds_u4_t;
  const unsigned lds0 = (unsigned)(uintptr_t)(lds_u4_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, src_bytes, kBufFlags);
  const int dr = lane >> 3, ch = lane & 7;
  auto issue = [&](int it) {
    const unsigned base = lds0 + (unsigned)((it & 1) * 576 * 128);
    // block-private: walk a window of the buffer; shared: the same 72 KB for every block
    const long long blk_off = shared ? 0 : ((long long)blockIdx.x * iters + it) * 576LL * row_stride;
    const int boff = (int)(blk_off % ((long long)src_bytes - 576LL * row_stride));
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int q = wv + 8 * i;
      const int row = 8 * q + dr;
      dma16(r, boff + row * row_stride + ch * 16, __builtin_amdgcn_readfirstlane(base + q * 1024));
    }
  };
  issue(0);
  for (int it = 0; it < iters; ++it) {
    if (INFLIGHT == 2) {
      if (it + 1 < iters) issue(it + 1);
      if (it + 1 < iters) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (it + 1 < iters) issue(it + 1);
    }
  }
  __syncthreads();
  if (tid == 0) sink[blockIdx.x] = reinterpret_cast<float*>(smem)[lane];
}

int main() {
  const int bytes = 256 << 20;
  char* src;
  float* sink;
  hipMalloc(&src, bytes);
  hipMemset(src, 1, bytes);
  hipMalloc(&sink, 4096 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 200, blocks = 256;
  for (int stride : {128, 640, 2560}) {
    for (int shared : {1, 0}) {
      for (int infl : {1, 2}) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
          hipEventRecord(e0);
          if (infl == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(512), 0, 0, src, bytes, shared, iters, stride, sink);
          else hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(512), 0, 0, src, bytes, shared, iters, stride, sink);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms;
          hipEventElapsedTime(&ms, e0, e1);
          if (ms < best) best = ms;
        }
        const double per_cu = 576.0 * 128 * iters / (best * 1e-3) / 1e9;
        printf("row_stride %5d  src %-8s  k-tiles in flight %d : %7.3f ms  %6.1f GB/s per CU  %6.2f TB/s chip\n",
               stride, shared ? "shared" : "private", infl, best, per_cu, per_cu * blocks / 1e3);
      }
    }
  }
  return 0;
}
