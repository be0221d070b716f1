# round-3 final tree: full GPU suite, smoke, default bench, headline rocprof + PMC (r03c), train + B=1 kernel profiles, bench lines of every mode
# train + B=1 kernel profiles, bench lines of every mode
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1
rc=$?
tail -4 gpurun_out/r3d_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3d_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r3d_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err || exit 1
cat gpurun_out/r3d_bench.json
M=gpurun_out/r3d_modes.jsonl; : > $M
timeout -k 10 300 python -u bench.py --frames 1 --no-cpu-baseline >> $M 2>> gpurun_out/r3d_modes.err || exit 1
timeout -k 10 300 python -u bench.py --frames 16 --latent 32x64 --no-cpu-baseline >> $M 2>> gpurun_out/r3d_modes.err || exit 1
timeout -k 10 300 python -u bench.py --frames 16 --latent 32x64 --fp8 --no-cpu-baseline >> $M 2>> gpurun_out/r3d_modes.err || exit 1
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline >> $M 2>> gpurun_out/r3d_modes.err || exit 1
timeout -k 10 300 python -u bench.py --mode sample --steps 3 --warmup 1 --no-cpu-baseline >> $M 2>> gpurun_out/r3d_modes.err || exit 1
timeout -k 10 300 python -u bench.py --mode ae --steps 5 --warmup 2 --no-cpu-baseline >> $M 2>> gpurun_out/r3d_modes.err || exit 1
python -c "
import json
for l in open('$M'):
    d=json.loads(l); print(d['metric'][:70], d['value'], d['ms_per_step'])"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03dtrain -o train \
  -- python3 bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3d_train.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03db1 -o b1 \
  -- python3 bench.py --frames 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3d_b1.log 2>&1 || exit 1
bash tools/profile_bench.sh r03d
