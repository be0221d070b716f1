# fused feed-forward ablations (no weight loads / no MFMA / no GELU math)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r3y_ops.txt
timeout -k 10 200 python -u tools/opbench.py --iters 20 --only ff_l0 ff_l0_unfused >> gpurun_out/r3y_ops.txt 2>&1 || exit 1
for v in noload nomfma nogelu; do
  echo "== $v" >> gpurun_out/r3y_ops.txt
  timeout -k 10 200 python -u tools/opbench.py --iters 20 --lib exp/libff$v.so --only ff_l0 >> gpurun_out/r3y_ops.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r3y_ops.txt
