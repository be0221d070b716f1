#!/bin/bash
# full GPU suite + default bench line (TAG names the gpurun_out subdirectory)
TAG=${1:-r5}
mkdir -p gpurun_out/$TAG
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/$TAG/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
