#!/bin/bash
mkdir -p gpurun_out/r5j
CASES="conv3_l0_320 conv3_up_l0_960 conv3_l1_640 conv3_l1_in_320 conv3_up_l1_1920 conv3_up_l1_1280 conv3_up_l1_960 conv3_l2_1280 conv3_l2_up_2560"
timeout -k 10 300 python -u -m pytest tests/test_gpu_igemm_plans.py tests/test_gpu_ops.py -q -x --timeout 120 --timeout-method thread -k "halo or conv or plan" > gpurun_out/r5j/halo_tests.txt 2>&1; tail -3 gpurun_out/r5j/halo_tests.txt
timeout -k 10 300 python tools/opbench.py --graph --iters 20 --only $CASES > gpurun_out/r5j/halo_new.txt 2>&1 || exit 1
timeout -k 10 300 python tools/opbench.py --graph --iters 20 --lib ablx/libhalo_prev.so --only $CASES > gpurun_out/r5j/halo_old.txt 2>&1 || exit 1
paste gpurun_out/r5j/halo_old.txt gpurun_out/r5j/halo_new.txt
