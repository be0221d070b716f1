#!/bin/bash
mkdir -p gpurun_out/r5m
for lib in "" ablx/libwide_pfd3.so ablx/libwide_pfd4.so ablx/libwide_pfd6.so "" ; do
  echo "== ${lib:-product}" >> gpurun_out/r5m/pfd.txt
  LDMSEG_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> gpurun_out/r5m/pfd.txt || exit 1
  LDMSEG_HIP_LIB=$lib timeout -k 10 200 python tools/opbench.py --graph --iters 20 --only gemm_geglu_1280_l2 gemm_geglu_640 gemm_qkv_640 >> gpurun_out/r5m/pfd.txt 2>&1 || exit 1
done
cat gpurun_out/r5m/pfd.txt
