# wgrad row walker: parity + A/B vs the decode-per-row build, train
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_train_full.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3t_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3t_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
W="wgrad_l0_320 wgrad_l1_640 wgrad_l2_1280 wgrad_l3_1280 wgrad_up_960 wgrad_geglu_320 wgrad_ff2_1280 wgrad_proj_320 wgrad_qkv_320"
timeout -k 10 200 python -u tools/opbench.py --iters 10 --only $W > gpurun_out/r3t_ops.txt 2>&1 || exit 1
echo "== decode per row" >> gpurun_out/r3t_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 10 --lib exp/libwgdec.so --only $W >> gpurun_out/r3t_ops.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3t_ops.txt
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3t_train.json 2> gpurun_out/r3t_train.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3t_train.json')); print('train', d['value'], d['ms_per_step'])"
