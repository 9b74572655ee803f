source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step ab4 900 gpurun_out/ab4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_LIB=$VD/qp0.so LPGPU_LIB=$VD/head.so
step ab3 600 gpurun_out/ab3.log bash scripts/ab_env.sh cfg3 1 - LPGPU_LIB=$VD/qp0.so LPGPU_LIB=$VD/head.so
step ab3e 300 gpurun_out/ab3e.log bash scripts/ab_env.sh cfg3 1 LPGPU_LIB=$VD/noepi.so
step ab4e 300 gpurun_out/ab4e.log bash scripts/ab_env.sh cfg4 1 LPGPU_LIB=$VD/noepi.so
