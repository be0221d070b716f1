#!/bin/bash
# Round-5 deep-level GEMM experiment: planner vs forced plans (ring depth 4 at one block per CU)
# and the hipBLASLt reference point at the 16x16 / 8x8 UNet shapes.
set -e
mkdir -p gpurun_out/r5
timeout -k 10 300 python tools/opbench.py --iters 30 --only gemm_proj_1280_l2 gemm_qkv_1280 gemm_ff2_5120 \
  gemm_geglu_1280_l2 gemm_proj_1280_l3 gemm_qkv_1280_l3 gemm_geglu_1280_l3 gemm_ff2_5120_l3 conv3_l3_1280 \
  --plans auto 128,160,1,4 128,160,2,4 128,160,4,4 128,160,8,4 128,160,2 64,160,2 64,64,1 \
  > gpurun_out/r5/deep_plans.txt 2>&1
timeout -k 10 200 python tools/opbench.py --iters 30 --only mm_proj_1280 mm_qkv_1280 mm_ff2_5120 mm_geglu_1280 \
  mm_proj_1280_l3 mm_qkv_1280_l3 mm_geglu_1280_l3 mm_conv_l3_1280 mm_conv_l2_1280 > gpurun_out/r5/deep_mm.txt 2>&1
