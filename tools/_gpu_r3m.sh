# wgrad reciprocal pixel decode A/B; wide GEMM touch-prefetch A/B; train + headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3m_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
W="wgrad_l0_320 wgrad_l1_640 wgrad_l2_1280 wgrad_l3_1280 wgrad_up_960 wgrad_geglu_320 wgrad_ff2_1280 wgrad_proj_320 wgrad_qkv_320"
G="gemm_geglu_640 gemm_geglu_1280 gemm_qkv_640 gemm_qkv_1280"
timeout -k 10 200 python -u tools/opbench.py --iters 10 --only $W $G > gpurun_out/r3m_ops.txt 2>&1 || exit 1
echo "== intdiv wgrad" >> gpurun_out/r3m_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 10 --lib exp/libintdiv.so --only $W >> gpurun_out/r3m_ops.txt 2>&1 || exit 1
echo "== wide no prefetch" >> gpurun_out/r3m_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 10 --lib exp/libwidenopf.so --only $G >> gpurun_out/r3m_ops.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3m_ops.txt
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3m_train.json 2> gpurun_out/r3m_train.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3m_train.json')); print('train', d['value'], d['ms_per_step'])"
timeout -k 10 200 python -u bench.py --no-cpu-baseline --profile-steps 1 > gpurun_out/r3m_bench.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3m_bench.json')); print('bench', d['value'], d['windows_ms_per_step'])"
