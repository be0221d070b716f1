set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/wide_abl.txt
: > $OUT
C="gemm_geglu_1280 gemm_geglu_640 gemm_geglu_320 gemm_qkv_640"
for L in base exp/libvnoload.so exp/libvnomfma.so exp/libvvm0.so; do
  echo "== $L" >> $OUT
  if [ $L = base ]; then A=""; else A="--lib $L"; fi
  timeout -k 10 120 python -u tools/opbench.py --iters 20 --wide 2 $A --only $C >> $OUT 2>&1 || exit 1
done
cat $OUT
