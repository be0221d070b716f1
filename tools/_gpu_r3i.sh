# attention backward on 32x32x16 (parity + timing) ; planner A/B (old vs new igemm) on the headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_ops.py -x -q -k attention --timeout 200 --timeout-method thread > gpurun_out/r3i_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r3i_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/opbench.py --iters 10 --only attn_bwd_4096_d40 attn_bwd_4096_d40_old attn_bwd_1024_d80 > gpurun_out/r3i_opbench.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3i_opbench.txt
for i in 1 2; do
LDMSEG_HIP_LIB=exp/libold.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --profile-steps 1 > gpurun_out/r3i_old$i.json 2>/dev/null || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --profile-steps 1 > gpurun_out/r3i_new$i.json 2>/dev/null || exit 1
done
for f in r3i_old1 r3i_new1 r3i_old2 r3i_new2; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['windows_ms_per_step'])"; done
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3i_train.json 2> gpurun_out/r3i_train.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3i_train.json')); print('train', d['value'], d['ms_per_step'])"
