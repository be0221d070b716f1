# small-image GroupNorm (gn_small) parity + config 5 line; wgrad per-shape timing and ablations
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "group_norm" --timeout 200 --timeout-method thread > gpurun_out/r3j_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3j_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
W="wgrad_l0_320 wgrad_l1_640 wgrad_l2_1280 wgrad_l3_1280 wgrad_up_960 wgrad_geglu_320 wgrad_ff2_1280 wgrad_proj_320 wgrad_qkv_320"
timeout -k 10 200 python -u tools/opbench.py --iters 10 --only $W > gpurun_out/r3j_wgrad.txt 2>&1 || exit 1
echo "== no loads" >> gpurun_out/r3j_wgrad.txt
timeout -k 10 200 python -u tools/opbench.py --iters 10 --lib exp/libnoloads.so --only $W >> gpurun_out/r3j_wgrad.txt 2>&1 || exit 1
echo "== no mfma" >> gpurun_out/r3j_wgrad.txt
timeout -k 10 200 python -u tools/opbench.py --iters 10 --lib exp/libnomfma.so --only $W >> gpurun_out/r3j_wgrad.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3j_wgrad.txt
LDM_BENCH_DETAIL=1 timeout -k 10 300 python -u bench.py --frames 16 --latent 32x64 --no-cpu-baseline > gpurun_out/r3j_c5.json 2> gpurun_out/r3j_c5.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3j_c5.json')); print('c5', d['value'], d['ms_per_step'])"
grep -v amdgpu.ids gpurun_out/r3j_c5.err | head -12
