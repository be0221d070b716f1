set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3e_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r3e_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
LDM_BENCH_DETAIL=1 timeout -k 10 400 python -u bench.py > gpurun_out/r3e_bench.json 2>gpurun_out/r3e_bench.err || exit 1
cat gpurun_out/r3e_bench.json
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3e_train.json 2> gpurun_out/r3e_train.err || exit 1
cat gpurun_out/r3e_train.json
bash tools/profile_bench.sh r03a
