set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/_dbg_po.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r3ac.log 2>&1
rc=$?
grep -E "eye|perm|row0|passed|failed|Error" gpurun_out/r3ac.log | head -20
exit $rc
