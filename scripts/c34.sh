source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step t 900 gpurun_out/t34.log python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_r4.py tests/test_gpu_r3.py tests/test_gpu_parity.py tests/test_gpu_xs.py
step ab3 900 gpurun_out/ab34_3.log bash scripts/ab_env.sh cfg3 3 - LPGPU_LIB=$VD/r4e.so
step ab4 900 gpurun_out/ab34_4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_LIB=$VD/r4e.so
