#!/bin/bash
# Profile `python3 bench.py` on the GPU box and write the committed summaries under profiles/.
#   tools/profile_bench.sh TAG            (run from the repo root, on the GPU box)
# Pass 1: kernel trace + stats of the default bench command (its JSON line is kept).
# Pass 2/3: FETCH_SIZE and WRITE_SIZE, each in its own --pmc run (no other trace domains),
#           over eager (non-graph) steps of the same workload.
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o bench \
  -- python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_stats.log" 2> "$OUT/bench_stats.err"
LDM_OPLOG="$OUT/oplog_fetch.json" timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
  -d "$OUT/fetch" -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --profile-steps 1 \
  > "$OUT/fetch.log" 2>&1
LDM_OPLOG="$OUT/oplog_write.json" timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
  -d "$OUT/write" -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --profile-steps 1 \
  > "$OUT/write.log" 2>&1
# per-op traffic table (the op log of the FETCH pass; both passes run the same launches)
python3 tools/traffic_table.py --fetch "$OUT/fetch" --write "$OUT/write" --oplog "$OUT/oplog_fetch.json" \
  --md "profiles/${TAG}_traffic_per_op.md" --json "$OUT/traffic.json" > /dev/null
# per-step launch breakdown of the graph-replayed step (kernel trace of pass 1)
python3 tools/step_trace.py "$(ls "$OUT"/stats/*kernel_trace.csv | head -1)" --top 40 > "profiles/${TAG}_step_trace.txt"
python3 tools/rocprof_summary.py --stats "$OUT/stats" --fetch "$OUT/fetch" --write "$OUT/write" --tag "$TAG" \
  --bench "$OUT/bench_stats.log"
mkdir -p gpurun_out/profiles && cp profiles/${TAG}_*.* gpurun_out/profiles/
