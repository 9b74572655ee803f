source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step t 900 gpurun_out/t31.log python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_r3.py tests/test_gpu_r4.py tests/test_gpu_r4_procs.py
step ab4 900 gpurun_out/ab31_4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_LIB=$VD/r4d.so
