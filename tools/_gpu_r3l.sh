# igemm 2-stage tiles with L2 touches two K tiles ahead: parity, A/B op timing, headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_igemm_plans.py tests/test_gpu_ops.py tests/test_gpu_modules.py tests/test_gpu_ars.py tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3l_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
C="conv3_l2_1280 conv3_l3_1280 gemm_proj_320 gemm_qkv_320 gemm_ff2_1280 gemm_proj_640 gemm_ff2_2560 gemm_ff2_5120 gemm_proj_1280_l2 gemm_qkv_1280 conv3_l2_up_2560 conv3_upsample_640"
timeout -k 10 200 python -u tools/opbench.py --iters 20 --only $C > gpurun_out/r3l_ops.txt 2>&1 || exit 1
echo "== no prefetch" >> gpurun_out/r3l_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 20 --lib exp/libnopf.so --only $C >> gpurun_out/r3l_ops.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3l_ops.txt
for i in 1 2; do
LDMSEG_HIP_LIB=exp/libnopf.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --profile-steps 1 > gpurun_out/r3l_old$i.json 2>/dev/null || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --profile-steps 1 > gpurun_out/r3l_new$i.json 2>/dev/null || exit 1
done
for f in r3l_old1 r3l_new1 r3l_old2 r3l_new2; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['windows_ms_per_step'])"; done
W="wgrad_l0_320 wgrad_l2_1280 wgrad_up_960 wgrad_geglu_320 wgrad_qkv_320"
for v in wgold wgA wgB wgC; do echo "== $v" >> gpurun_out/r3l_wgrad.txt; timeout -k 10 200 python -u tools/opbench.py --iters 10 --lib exp/lib$v.so --only $W >> gpurun_out/r3l_wgrad.txt 2>&1 || exit 1; done
echo "== current" >> gpurun_out/r3l_wgrad.txt; timeout -k 10 200 python -u tools/opbench.py --iters 10 --only $W >> gpurun_out/r3l_wgrad.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3l_wgrad.txt
