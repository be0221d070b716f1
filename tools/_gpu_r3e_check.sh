# final-tree check: full GPU suite, smoke, default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3e_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r3e_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3e_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r3e_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3e_bench.json 2> gpurun_out/r3e_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3e_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
