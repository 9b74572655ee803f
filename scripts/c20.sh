source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step ab4 900 gpurun_out/ab20_4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_SWEEP_D=3 LPGPU_SWEEP_TAIL=0 LPGPU_LIB=$VD/noepi.so LPGPU_LIB=$VD/notail.so
step ab3 900 gpurun_out/ab20_3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_SWEEP_TAIL=0 LPGPU_LIB=$VD/noepi.so LPGPU_LIB=$VD/notail.so
