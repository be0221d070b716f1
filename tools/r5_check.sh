#!/bin/bash
# quick GPU check: selected tests, B=1 and B=8 bench lines (no CPU leg), optional extra command
TAG=${1:-r5}; TESTS=${2:-tests/test_gpu_igemm_plans.py}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/$TAG/tests.txt 2>&1 || { tail -30 gpurun_out/$TAG/tests.txt; exit 1; }
tail -3 gpurun_out/$TAG/tests.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --frames 1 > gpurun_out/$TAG/bench_b1.json 2> gpurun_out/$TAG/bench_b1.err || exit 2
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 3
python3 -c "
import json
for f in ['bench_b1','bench']:
    d=json.loads(open('gpurun_out/$TAG/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d.get('windows_ms_per_step'))"
