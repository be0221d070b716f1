#!/bin/bash
# every bench mode once (JSON lines appended to gpurun_out/$TAG/modes.jsonl)
TAG=${1:-r5}
mkdir -p gpurun_out/$TAG
run() { echo "== $*" >&2; timeout -k 10 400 python bench.py "$@" 2>>gpurun_out/$TAG/modes.err | tail -1 >> gpurun_out/$TAG/modes.jsonl; }
run --no-cpu-baseline --frames 1 || exit 1
run --no-cpu-baseline --frames 16 --latent 32x64 || exit 1
run --no-cpu-baseline --frames 16 --latent 32x64 --fp8 || exit 1
run --mode train --no-cpu-baseline || exit 1
run --mode ae --no-cpu-baseline || exit 1
run --mode sample --no-cpu-baseline || exit 1
python3 -c "
import json
for l in open('gpurun_out/$TAG/modes.jsonl'):
    d=json.loads(l); print(d['metric'][:60], d['value'], d.get('ms_per_step'), d.get('dtype'), json.dumps(d.get('config'))[:120])"
