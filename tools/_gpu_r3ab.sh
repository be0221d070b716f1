# proj_out fusion: op-level parity first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_feedforward.py -x -q -k proj_out --timeout 200 --timeout-method thread > gpurun_out/r3ab_tests.log 2>&1
rc=$?
grep -E "max \||passed|failed|Error" gpurun_out/r3ab_tests.log | head -10
exit $rc
