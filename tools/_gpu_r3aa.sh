# d40 attention: incremental K/V tile pointers vs the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q -k "attention or attn" --timeout 200 --timeout-method thread > gpurun_out/r3aa_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r3aa_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
W="attn_4096_d40 attn_c5_2048_d40 attn_1024_d80 attn_256_d160"
: > gpurun_out/r3aa_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 20 --only $W >> gpurun_out/r3aa_ops.txt 2>&1 || exit 1
echo "== old" >> gpurun_out/r3aa_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 20 --lib exp/libattnold.so --only $W >> gpurun_out/r3aa_ops.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3aa_ops.txt
