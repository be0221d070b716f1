#!/bin/bash
# kernel trace of the default bench (graph-replayed steps) -> per-launch step breakdown
TAG=${1:-r5}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/stats -o bench \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench_stats.log 2> gpurun_out/$TAG/bench_stats.err || exit $?
python3 tools/step_trace.py "$(ls gpurun_out/$TAG/stats/*kernel_trace.csv | head -1)" --top 40 > gpurun_out/$TAG/step_trace.txt
head -30 gpurun_out/$TAG/step_trace.txt
