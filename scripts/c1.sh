source scripts/r4_call.sh
step mfma 60 ./scripts/mfma_probe > gpurun_out/mfma_probe.txt 2>&1
step r4tests 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_r4.py tests/test_gpu_r4_procs.py > gpurun_out/r4_tests.log 2>&1
step bench3 300 python bench.py --workload cfg3 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err
