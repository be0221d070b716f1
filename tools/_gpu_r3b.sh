set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_repack.py tests/test_gpu_train_step.py tests/test_gpu_train_full.py tests/test_gpu_train_unet.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r3b_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/opbench.py --iters 20 --wide 1 2 --only gemm_qkv_320 gemm_geglu_320 gemm_geglu_640 gemm_qkv_640 gemm_geglu_1280 gemm_qkv_1280 > gpurun_out/wide_opbench.txt 2>&1
rc=$?
cat gpurun_out/wide_opbench.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 > gpurun_out/r3b_train.json 2> gpurun_out/r3b_train.err
rc=$?
cat gpurun_out/r3b_train.json
exit $rc
