# config 2 (B=1) per-shape breakdown + config 5 (T=16 32x64, fp8 attention) lines + train-mode kernel profile
set -o pipefail
mkdir -p gpurun_out
LDM_BENCH_DETAIL=1 timeout -k 10 300 python -u bench.py --frames 1 --no-cpu-baseline > gpurun_out/r3f_b1.json 2> gpurun_out/r3f_b1.err || exit 1
cat gpurun_out/r3f_b1.json; grep -v amdgpu.ids gpurun_out/r3f_b1.err | head -45
LDM_BENCH_DETAIL=1 timeout -k 10 300 python -u bench.py --frames 16 --latent 32x64 --fp8 --no-cpu-baseline > gpurun_out/r3f_c5.json 2> gpurun_out/r3f_c5.err || exit 1
cat gpurun_out/r3f_c5.json; grep -v amdgpu.ids gpurun_out/r3f_c5.err | head -12
timeout -k 10 300 python -u bench.py --frames 16 --latent 32x64 --no-cpu-baseline > gpurun_out/r3f_c5bf.json 2> gpurun_out/r3f_c5bf.err || exit 1
cat gpurun_out/r3f_c5bf.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03train -o train \
  -- python3 bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r3f_train.log 2>&1 || exit 1
tail -2 gpurun_out/r3f_train.log
LDM_BENCH_DETAIL=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3f_bench.json 2> gpurun_out/r3f_bench.err || exit 1
cat gpurun_out/r3f_bench.json
bash tools/profile_bench.sh r03a
