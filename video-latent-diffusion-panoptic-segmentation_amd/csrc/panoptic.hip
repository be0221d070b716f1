// Panoptic head of the sampling path (ldm_panoptic_pixels / ldm_panoptic_finalize).
//
// Replaces the per-image CPU loop of TrainerDiffusion.compute_pq (trainers_ldm_cond.py:1287-1330)
// and the argmax / confidence threshold of decode_latents (:426-435):
//   pred  = argmax_k logits[k]                       (first maximal index, torch.argmax)
//   conf  = max_k softmax(logits)_k                  ('max')   or   top1 - top2   ('topk_diff')
//   pred  = ignore_label where conf < mask_th        (threshold_output)
//   label k survives iff k != ignore_label, count(pred == k) >= count_th and
//            count(pred == k) / count(sigmoid(logits[k]) >= mask_th) >= overlap_th
//            (a zero denominator is numpy's inf: the label survives)
//   out   = pred + 1 where pred survives, else 0     (cleaned_pred + 1)
// Logits are NCHW fp32, one image = K planes of hw pixels; consecutive threads take
// consecutive pixels, so every plane read is a coalesced row.  HBM-bound: two passes over
// the K planes (max, then the softmax sum and the sigmoid counts, as torch's two-pass
// softmax does), one int32 write per pixel; the per-label histograms are reduced per wave
// (ballot + popcount for the K mask counts) and per block in LDS before one global atomic
// per (block, label).
#include "common.h"

#include <algorithm>
#include <math.h>

namespace {

constexpr int PAN_MAX_K = 1024;

__global__ __launch_bounds__(256) void panoptic_pixels_kernel(const float* __restrict__ logits, int K, int hw,
                                                              int conf_mode, float mask_th, int ignore_label,
                                                              int32_t* __restrict__ pred, int32_t* __restrict__ counts,
                                                              int32_t* __restrict__ mask_counts) {
  __shared__ int cnt_s[PAN_MAX_K], msk_s[PAN_MAX_K];
  const int b = blockIdx.y;
  for (int k = threadIdx.x; k < K; k += 256) { cnt_s[k] = 0; msk_s[k] = 0; }
  __syncthreads();
  const float* img = logits + (int64_t)b * K * hw;
  const int lane = threadIdx.x & 63;
  const int stride = gridDim.x * 256;
  for (int p0 = blockIdx.x * 256; p0 < hw; p0 += stride) {   // block-uniform trip count
    const int p = p0 + threadIdx.x;
    const bool ok = p < hw;
    // pass 1: max, its first index, and the runner-up value
    float m1 = -INFINITY, m2 = -INFINITY;
    int am = 0;
    for (int k = 0; k < K; ++k) {
      const float v = ok ? img[(int64_t)k * hw + p] : 0.f;
      if (v > m1) { m2 = m1; m1 = v; am = k; }
      else if (v > m2) m2 = v;
    }
    // pass 2: softmax denominator and the per-label sigmoid counts
    float s = 0.f;
    for (int k = 0; k < K; ++k) {
      const float v = ok ? img[(int64_t)k * hw + p] : 0.f;
      s += expf(v - m1);
      const float sg = 1.0f / (1.0f + expf(-v));
      const unsigned long long bal = __ballot(ok && sg >= mask_th);
      if (lane == 0 && bal) atomicAdd(&msk_s[k], __popcll(bal));
    }
    int lab = am;
    if (conf_mode != 0) {
      const float p1 = 1.0f / s;
      const float conf = conf_mode == 2 ? p1 - expf(m2 - m1) / s : p1;
      if (conf < mask_th) lab = ignore_label;
    }
    if (ok) {
      pred[(int64_t)b * hw + p] = lab;
      if (lab >= 0 && lab < K) atomicAdd(&cnt_s[lab], 1);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += 256) {
    if (cnt_s[k]) atomicAdd(&counts[(int64_t)b * K + k], cnt_s[k]);
    if (msk_s[k]) atomicAdd(&mask_counts[(int64_t)b * K + k], msk_s[k]);
  }
}

__global__ __launch_bounds__(256) void panoptic_finalize_kernel(const int32_t* __restrict__ pred,
                                                                const int32_t* __restrict__ counts,
                                                                const int32_t* __restrict__ mask_counts, int K,
                                                                int hw, int count_th, double overlap_th,
                                                                int ignore_label, int32_t* __restrict__ keep,
                                                                int32_t* __restrict__ out) {
  __shared__ int keep_s[PAN_MAX_K];
  const int b = blockIdx.y;
  for (int k = threadIdx.x; k < K; k += 256) {
    const int c = counts[(int64_t)b * K + k];
    const int mc = mask_counts[(int64_t)b * K + k];
    // trainers_ldm_cond.py:1309-1315: count_i < count_th or the ignore label -> dropped;
    // count / mask_count < overlap_th -> dropped (float64 division; mc == 0 gives inf: kept)
    bool kp = c > 0 && c >= count_th && k != ignore_label;
    if (kp && mc > 0 && (double)c / (double)mc < overlap_th) kp = false;
    keep_s[k] = kp ? 1 : 0;
    if (blockIdx.x == 0) keep[(int64_t)b * K + k] = kp ? 1 : 0;
  }
  __syncthreads();
  const int stride = gridDim.x * 256;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < hw; p += stride) {
    const int lab = pred[(int64_t)b * hw + p];
    out[(int64_t)b * hw + p] = (lab >= 0 && lab < K && keep_s[lab]) ? lab + 1 : 0;
  }
}

int grid_x(int hw, int batch) {
  // ~4 resident blocks per CU over the whole batch, each block sweeping a pixel range
  const int want = std::max(1, (256 * 4 + batch - 1) / batch);
  return std::max(1, std::min((hw + 255) / 256, want));
}

}  // namespace

extern "C" int ldm_panoptic_pixels(const float* logits, int batch, int k, int hw, int conf_mode, float mask_th,
                                   int ignore_label, int32_t* pred, int32_t* counts, int32_t* mask_counts,
                                   ldm_stream_t stream) {
  if (!logits || !pred || !counts || !mask_counts) return LDM_ERR_ARG;
  if (batch <= 0 || k <= 0 || k > PAN_MAX_K || hw <= 0 || conf_mode < 0 || conf_mode > 2) return LDM_ERR_ARG;
  if ((int64_t)batch * k * hw >= (1LL << 40)) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(counts, 0, sizeof(int32_t) * batch * k, s) != hipSuccess) return LDM_ERR_LAUNCH;
  if (hipMemsetAsync(mask_counts, 0, sizeof(int32_t) * batch * k, s) != hipSuccess) return LDM_ERR_LAUNCH;
  hipLaunchKernelGGL(panoptic_pixels_kernel, dim3(grid_x(hw, batch), batch), dim3(256), 0, s, logits, k, hw,
                     conf_mode, mask_th, ignore_label, pred, counts, mask_counts);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}

extern "C" int ldm_panoptic_finalize(const int32_t* pred, const int32_t* counts, const int32_t* mask_counts,
                                     int batch, int k, int hw, int count_th, double overlap_th, int ignore_label,
                                     int32_t* keep, int32_t* out, ldm_stream_t stream) {
  if (!pred || !counts || !mask_counts || !keep || !out) return LDM_ERR_ARG;
  if (batch <= 0 || k <= 0 || k > PAN_MAX_K || hw <= 0) return LDM_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(panoptic_finalize_kernel, dim3(grid_x(hw, batch), batch), dim3(256), 0, s, pred, counts,
                     mask_counts, k, hw, count_th, overlap_th, ignore_label, keep, out);
  LDM_CHECK_LAUNCH();
  return LDM_OK;
}
