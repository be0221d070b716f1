# training iteration (config 3) kernel profile of the current tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03train2 -o train \
  -- python3 bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3p_train.log 2>&1 || exit 1
grep '"metric"' gpurun_out/r3p_train.log | cut -c1-300
