source scripts/r4_call.sh
step r4tests 900 gpurun_out/r4_tests.log python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_r4.py tests/test_gpu_r4_procs.py
step gpusuite 900 gpurun_out/gpu_suite.log python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/
step bench 600 gpurun_out/bench_default.json python bench.py --no-cpu-baseline
