source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step ab4 900 gpurun_out/ab30_4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_LIB=$VD/sa2.so LPGPU_LIB=$VD/sa18.so LPGPU_LIB=$VD/la2.so
step ab3 900 gpurun_out/ab30_3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_LIB=$VD/sa2.so LPGPU_LIB=$VD/sa18.so LPGPU_LIB=$VD/la2.so
