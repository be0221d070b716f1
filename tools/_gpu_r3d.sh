set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3d_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
C="gemm_qkv_320 gemm_geglu_320 gemm_geglu_640 gemm_qkv_640 gemm_geglu_1280 gemm_plain_2560_320"
timeout -k 10 300 python -u tools/opbench.py --iters 20 --wide 1 2 --only $C > gpurun_out/wide_opbench.txt 2>&1 || exit 1
echo "== no prefetch" >> gpurun_out/wide_opbench.txt
timeout -k 10 300 python -u tools/opbench.py --iters 20 --wide 2 --lib exp/libnopf.so --only $C >> gpurun_out/wide_opbench.txt 2>&1 || exit 1
cat gpurun_out/wide_opbench.txt
