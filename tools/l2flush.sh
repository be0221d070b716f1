#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of an op with and without a preceding L2 flush or its step producer, each
# counter in its own --pmc pass (run from the repo root ON the GPU box).
#   tools/l2flush.sh TAG CASE KERNEL_REGEX [CASE KERNEL_REGEX ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
while [ $# -ge 2 ]; do
  CASE=$1; KRX=$2; shift 2
  for PREV in none flush producer; do
    for C in FETCH_SIZE WRITE_SIZE; do
      lc=$( [ $C = FETCH_SIZE ] && echo fetch || echo write )
      timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/${CASE}_${PREV}_$lc" -o pmc \
        -- python3 tools/l2flush.py --case "$CASE" --prev $PREV --iters 20 >> "$OUT/run.log" 2>&1 || exit $?
    done
  done
  python3 tools/l2flush_summary.py "$OUT" "$KRX" | tee -a "$OUT/summary.txt"
  mkdir -p "$OUT/done_$CASE"
  for d in "$OUT"/${CASE}_*; do [ -d "$d" ] && mv "$d" "$OUT/done_$CASE/"; done
done
