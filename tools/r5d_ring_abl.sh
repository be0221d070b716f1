#!/bin/bash
# ring GEMM ablations: 0 planner, 1 igemm, 2 ring, 3 ring without MFMA / fragment reads, 4 ring without operand DMA
set -e
mkdir -p gpurun_out/r5d
timeout -k 10 300 python tools/opbench.py --graph --iters 30 --only gemm_proj_1280_l2 gemm_ff2_5120 gemm_proj_1280_l3 gemm_ff2_5120_l3 gemm_short_l2_2560 gemm_short_l3_2560 \
  --ring 1 2 3 4 > gpurun_out/r5d/ring_abl.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -q --timeout 120 --timeout-method thread > gpurun_out/r5d/ring_tests.txt 2>&1
timeout -k 10 300 python tools/opbench.py --graph --iters 30 --only gemm_geglu_1280_l3 gemm_qkv_1280_l3 gemm_qkv_1280 gemm_geglu_1280_l2 \
  --plans auto 64,160,1 128,128,1 64,64,1 > gpurun_out/r5d/geglu_plans.txt 2>&1
