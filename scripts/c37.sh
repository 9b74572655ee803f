source scripts/r4_call.sh
step ab4 900 gpurun_out/ab37_4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_SWEEP_D=3 LPGPU_SWEEP_D=2
