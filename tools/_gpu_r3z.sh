# wide kernel: explicit lane-base LDS addressing + soffset B loads vs the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3z_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r3z_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
W="gemm_geglu_640 gemm_geglu_1280 gemm_qkv_640 gemm_qkv_1280"
: > gpurun_out/r3z_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 20 --only $W >> gpurun_out/r3z_ops.txt 2>&1 || exit 1
echo "== old" >> gpurun_out/r3z_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 20 --lib exp/libwideold.so --only $W >> gpurun_out/r3z_ops.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3z_ops.txt
