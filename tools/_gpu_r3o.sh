# config 2 (B=1) kernel profile of the graph-replayed step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03b1 -o b1 \
  -- python3 bench.py --frames 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3o_b1.log 2>&1 || exit 1
grep '"metric"' gpurun_out/r3o_b1.log | cut -c1-300
