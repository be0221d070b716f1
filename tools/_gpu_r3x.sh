# fused feed-forward: parity + op timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_feedforward.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3x_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/opbench.py --iters 20 --only ff_l0 ff_l0_unfused ff_po_l0 ff_po_l0_separate > gpurun_out/r3x_ops.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3x_ops.txt
