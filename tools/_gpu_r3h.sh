# planner B=1 rules + tiled repack: parity, then bench lines (headline, B=1, train)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_repack.py tests/test_gpu_modules.py tests/test_gpu_ops.py tests/test_gpu_igemm_plans.py tests/test_gpu_train_full.py tests/test_gpu_train_step.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3h_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r3h_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3h_bench.json 2> gpurun_out/r3h_bench.err || exit 1
timeout -k 10 300 python -u bench.py --frames 1 --no-cpu-baseline > gpurun_out/r3h_b1.json 2> gpurun_out/r3h_b1.err || exit 1
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3h_train.json 2> gpurun_out/r3h_train.err || exit 1
for f in r3h_bench r3h_b1 r3h_train; do python -c "import json,sys; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'])"; done
