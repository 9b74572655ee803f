source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step t 900 gpurun_out/t11.log python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_r4.py tests/test_gpu_r3.py -k "partial or recovery or cfg3 or shapes or explicit or misplacement"
step ab3 900 gpurun_out/ab3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_LIB=$VD/inloop.so LPGPU_LIB=$VD/head.so LPGPU_LIB=$VD/noepi.so
step ab4 900 gpurun_out/ab4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_LIB=$VD/inloop.so LPGPU_LIB=$VD/head.so LPGPU_LIB=$VD/noepi.so
