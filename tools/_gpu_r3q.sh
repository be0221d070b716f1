# small-batch attention blocks + in-place QKV weight gradient: parity, B=1 line, train profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train_full.py tests/test_gpu_train_step.py tests/test_gpu_train_unet.py tests/test_gpu_loops_golden.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3q_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3q_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --frames 1 --no-cpu-baseline > gpurun_out/r3q_b1.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3q_b1.json')); print('b1', d['value'], d['ms_per_step'])"
bash tools/_gpu_r3p.sh
