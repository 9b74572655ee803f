source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step t 900 gpurun_out/t12.log python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_r4.py tests/test_gpu_r3.py tests/test_gpu_parity.py tests/test_gpu_xs.py
step ab3 900 gpurun_out/ab3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_LIB=$VD/prev.so LPGPU_LIB=$VD/notail.so LPGPU_LIB=$VD/noepi.so
step ab4 900 gpurun_out/ab4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_LIB=$VD/prev.so LPGPU_LIB=$VD/head.so
