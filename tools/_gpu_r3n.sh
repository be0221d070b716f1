# fp8 attention on the block-scaled MFMA (config 5): parity, op timing, config-5 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_config5.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1
rc=$?
grep -E "rel-L2|rel err|passed|failed|Error|error" gpurun_out/r3n_tests.log | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/opbench.py --iters 20 --only attn_c5_2048_d40 attn_c5_2048_d40_fp8 attn_c5_2048_d40_fp8pv attn_4096_d40 attn_4096_d40_fp8 > gpurun_out/r3n_ops.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3n_ops.txt
timeout -k 10 300 python -u bench.py --frames 16 --latent 32x64 --fp8 --no-cpu-baseline > gpurun_out/r3n_c5fp8.json 2> gpurun_out/r3n_c5fp8.err || exit 1
timeout -k 10 300 python -u bench.py --frames 16 --latent 32x64 --no-cpu-baseline > gpurun_out/r3n_c5.json 2> gpurun_out/r3n_c5.err || exit 1
for f in r3n_c5fp8 r3n_c5; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernels_per_step']['attention'])"; done
