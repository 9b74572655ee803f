source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step ab4 900 gpurun_out/ab27_4.log bash scripts/ab_env.sh cfg4 3 - LPGPU_LIB=$VD/oop.so
step ab3 900 gpurun_out/ab27_3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_LIB=$VD/oop.so
