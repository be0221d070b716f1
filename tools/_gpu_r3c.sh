set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r3c_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/opbench.py --iters 20 --wide 1 2 --only gemm_qkv_320 gemm_geglu_320 gemm_geglu_640 gemm_qkv_640 gemm_geglu_1280 gemm_plain_2560_320 > gpurun_out/wide_opbench.txt 2>&1
rc=$?
cat gpurun_out/wide_opbench.txt
exit $rc
