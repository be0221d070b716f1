#!/bin/bash
# The GPU-box steps of a round, one subcommand per gpurun call (run from the repo root ON the box;
# everything lands under gpurun_out/$TAG, which gpurun copies back; nothing here retries a GPU step).
#
#   tools/gpu_round.sh suite  TAG [PYTEST_ARGS...]  full `pytest -m gpu` (or the given tests) + smoke
#   tools/gpu_round.sh bench  TAG                   default bench line (no CPU leg) and the B=1 line
#   tools/gpu_round.sh modes  TAG                   every bench mode once -> modes.jsonl
#   tools/gpu_round.sh trace  TAG [BENCH_ARGS...]   rocprofv3 kernel trace of the graph-replayed step
#                                                    -> step_trace.txt (tools/step_trace.py)
#   tools/gpu_round.sh ab     TAG ARGS...           same-box A/B of captured step graphs (tools/ab_step.py)
#
# The rocprofv3 profile set committed under profiles/ (stats, families, per-op traffic, step trace)
# is tools/profile_bench.sh TAG.
set -o pipefail
CMD=$1; TAG=${2:-rX}; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
case "$CMD" in
  suite)
    ARGS=${*:-tests -m gpu}
    timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread $ARGS \
      > "$OUT/gpu_tests.txt" 2>&1
    rc=$?
    tail -5 "$OUT/gpu_tests.txt"
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit $?
    tail -3 "$OUT/smoke.txt"
    ;;
  bench)
    timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --frames 1 > "$OUT/bench_b1.json" 2> "$OUT/bench_b1.err" || exit $?
    python3 - "$OUT" <<'EOF'
import json, sys
for f in ("bench", "bench_b1"):
    d = json.loads(open(f"{sys.argv[1]}/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("windows_ms_per_step"))
EOF
    ;;
  modes)
    run() { echo "== $*" >&2; timeout -k 10 400 python3 bench.py "$@" 2>> "$OUT/modes.err" | tail -1 >> "$OUT/modes.jsonl"; }
    run --no-cpu-baseline --frames 1 && run --no-cpu-baseline --frames 16 --latent 32x64 && \
      run --no-cpu-baseline --frames 16 --latent 32x64 --fp8 && run --mode train --no-cpu-baseline && \
      run --mode ae --no-cpu-baseline && run --mode sample --no-cpu-baseline || exit 1
    python3 - "$OUT" <<'EOF'
import json, sys
for l in open(f"{sys.argv[1]}/modes.jsonl"):
    d = json.loads(l)
    print(d["metric"][:60], d["value"], d.get("ms_per_step"), d.get("dtype"), json.dumps(d.get("config"))[:100])
EOF
    ;;
  trace)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o bench \
      -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/bench_stats.log" 2> "$OUT/bench_stats.err" \
      || exit $?
    python3 tools/step_trace.py "$(ls "$OUT"/stats/*kernel_trace.csv | head -1)" --top 40 > "$OUT/step_trace.txt"
    head -24 "$OUT/step_trace.txt"
    ;;
  ab)
    timeout -k 10 600 python3 tools/ab_step.py "$@" > "$OUT/ab.txt" 2> "$OUT/ab.err" || exit $?
    tail -20 "$OUT/ab.txt"
    ;;
  *)
    echo "usage: tools/gpu_round.sh suite|bench|modes|trace|ab TAG [ARGS...]" >&2; exit 2 ;;
esac
