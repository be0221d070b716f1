#!/bin/bash
TAG=${1:-r5}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/stats_b1 -o bench \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --frames 1 > gpurun_out/$TAG/bench_b1.log 2> gpurun_out/$TAG/bench_b1.err || exit $?
python3 tools/step_trace.py "$(ls gpurun_out/$TAG/stats_b1/*kernel_trace.csv | head -1)" --top 40 > gpurun_out/$TAG/step_trace_b1.txt
head -24 gpurun_out/$TAG/step_trace_b1.txt
