source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step t 900 gpurun_out/t21.log python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_r4.py tests/test_gpu_parity.py tests/test_gpu_xs.py tests/test_gpu_r3.py tests/test_gpu_r2.py
step ab4 900 gpurun_out/ab21_4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_LIB=$VD/cap.so
step ab3 900 gpurun_out/ab21_3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_LIB=$VD/cap.so
