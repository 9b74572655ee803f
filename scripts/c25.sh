source scripts/r4_call.sh
L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/stamps.so
step clk3 300 gpurun_out/clk_r04_cfg3_b64.txt env LPGPU_LIB=$L python scripts/sel_clocks.py mixed 4096 4096 64
step clk3e 300 gpurun_out/clk_r04_cfg3_b64_events.txt env LPGPU_LIB=$L python scripts/sel_clocks.py mixed 4096 4096 64 --events
