set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wide_tests.log 2>&1
rc=$?
tail -5 gpurun_out/wide_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/opbench.py --iters 20 --wide 1 2 --only gemm_qkv_320 gemm_geglu_320 gemm_proj_320 gemm_ff2_1280 gemm_geglu_640 gemm_qkv_640 gemm_proj_640 gemm_ff2_2560 gemm_geglu_1280 gemm_qkv_1280 gemm_proj_1280_l2 gemm_ff2_5120 gemm_short_l2_2560 mm_geglu_320 mm_geglu_640 mm_geglu_1280 > gpurun_out/wide_opbench.txt 2>&1
rc=$?
cat gpurun_out/wide_opbench.txt
exit $rc
