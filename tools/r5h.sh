#!/bin/bash
mkdir -p gpurun_out/r5h
rm -f gpurun_out/r5h/tail_abl.txt
for lib in "" ablx/libtail_NO_LOOP.so ablx/libtail_NO_XFORM.so ablx/libtail_NO_LOAD.so ablx/libtail_NO_MFMA.so ablx/libtail_NL_NX.so; do
  echo "== lib ${lib:-product}" >> gpurun_out/r5h/tail_abl.txt
  timeout -k 10 200 python tools/opbench.py --graph --iters 20 ${lib:+--lib $lib} --only tail_l0 tail_l0_eps >> gpurun_out/r5h/tail_abl.txt 2>&1 || exit 1
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_tail.py -q --timeout 120 --timeout-method thread > gpurun_out/r5h/tail_tests.txt 2>&1; tail -2 gpurun_out/r5h/tail_tests.txt
