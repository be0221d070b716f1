# training reductions: parts-parallel slab reduction + wgrad_reduce loads in flight; parity + train bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_train_full.py tests/test_gpu_train_step.py tests/test_gpu_train_unet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ae_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3ae_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3ae_train.json 2> gpurun_out/r3ae_train.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3ae_train.json')); print('train', d['value'], d['ms_per_step'])"
