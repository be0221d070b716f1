# fused feed-forward: parity (two-launch form, torch fp32, whole UNet), op timing, headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_feedforward.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r3w_tests.log | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/opbench.py --iters 20 --only ff_l0 ff_l0_unfused gemm_geglu_320 gemm_ff2_1280 > gpurun_out/r3w_ops.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3w_ops.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3w_bench.json 2> gpurun_out/r3w_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3w_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
