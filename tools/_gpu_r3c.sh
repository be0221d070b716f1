set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/dma_probe > gpurun_out/dma_probe.txt 2>&1; cat gpurun_out/dma_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_fullsize.py tests/test_gpu_ars.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1
rc=$?
tail -25 gpurun_out/r3c_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/opbench.py --iters 20 --wide 1 2 --only gemm_qkv_320 gemm_geglu_320 gemm_geglu_640 gemm_qkv_640 gemm_geglu_1280 gemm_plain_2560_320 > gpurun_out/wide_opbench.txt 2>&1
rc=$?
cat gpurun_out/wide_opbench.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3c_bench.json 2>gpurun_out/r3c_bench.err
rc=$?
cat gpurun_out/r3c_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['windows_ms_per_step'], d['roofline']['frac'], {k:(v.get('ms'),v.get('frac_mfma')) for k,v in d['roofline']['kernels_per_step'].items()})"
exit $rc
