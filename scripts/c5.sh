source scripts/r4_call.sh
step ab3 600 gpurun_out/ab3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_SWEEP_D4=3 LPGPU_SWEEP_D4=4 LPGPU_SWEEP_W8=1
step ab4 600 gpurun_out/ab4.log bash scripts/ab_env.sh cfg4 1 - LPGPU_SWEEP_D=3
