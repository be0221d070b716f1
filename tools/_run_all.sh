timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest.log 2>&1; tail -3 gpurun_out/pytest.log
LDM_BENCH_DETAIL=1 timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err; cat gpurun_out/bench.log; grep -v amdgpu.ids gpurun_out/bench.err | head -30
