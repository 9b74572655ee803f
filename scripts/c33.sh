source scripts/r4_call.sh
step ab3 900 gpurun_out/ab33_3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_SWEEP_W8=1 LPGPU_SWEEP_D4=3
