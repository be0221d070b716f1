#!/bin/bash
mkdir -p gpurun_out/r5n
timeout -k 10 300 python tools/opbench.py --graph --iters 20 --only gemm_proj_640 gemm_qkv_640 gemm_ff2_2560 gemm_proj_320 gemm_qkv_1280 gemm_qkv_1280_l3 --ring 0 2 > gpurun_out/r5n/ring32.txt 2>&1
cat gpurun_out/r5n/ring32.txt
