# wgrad L2 behaviour (PMC passes over opbench), ring A/B, vectorized repack parity + train
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_repack.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3s_tests.log 2>&1
rc=$?
tail -2 gpurun_out/r3s_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_wg_hit -o p -- python3 tools/opbench.py --iters 2 --only wgrad_l0_320 wgrad_l0_320_old wgrad_qkv_320 > gpurun_out/r3s_pmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_wg_fetch -o p -- python3 tools/opbench.py --iters 2 --only wgrad_l0_320 wgrad_l0_320_old wgrad_qkv_320 > gpurun_out/r3s_pmc2.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3s_train.json 2> gpurun_out/r3s_train.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r3s_train.json')); print('train', d['value'], d['ms_per_step'])"
