set -e
mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -v --timeout 120 --timeout-method thread > gpurun_out/r5c/ring_tests.txt 2>&1
timeout -k 10 300 python tools/opbench.py --iters 30 --only gemm_proj_1280_l2 gemm_ff2_5120 gemm_proj_1280_l3 gemm_ff2_5120_l3 gemm_geglu_1280_l3 gemm_short_l2_2560 gemm_short_l3_2560 gemm_short_l2_1920 --ring 0 1 > gpurun_out/r5c/ring_ops.txt 2>&1
