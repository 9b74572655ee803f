source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step t 900 gpurun_out/t22.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_r4.py -k "tail"
step ab4 900 gpurun_out/ab22_4.log bash scripts/ab_env.sh cfg4 3 - LPGPU_LIB=$VD/cap.so
