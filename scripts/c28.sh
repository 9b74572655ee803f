source scripts/r4_call.sh
step oopw 600 gpurun_out/t28_oopw.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_r4.py -k "out_of_place"
step toop 1200 gpurun_out/t28_oop.log env LPGPU_SWEEP_OOP=1 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_r4.py tests/test_gpu_parity.py tests/test_gpu_xs.py tests/test_gpu_r3.py tests/test_gpu_r2.py
step ab4 900 gpurun_out/ab28_4.log bash scripts/ab_env.sh cfg4 3 - LPGPU_SWEEP_OOP=1
step ab3 900 gpurun_out/ab28_3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_SWEEP_OOP=1
