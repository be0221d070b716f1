#!/bin/bash
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u -m pytest tests/test_gpu_tail.py -v --timeout 120 --timeout-method thread > gpurun_out/r5f/tail_tests.txt 2>&1
tail -12 gpurun_out/r5f/tail_tests.txt
