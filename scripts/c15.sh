source scripts/r4_call.sh
step ramp2 600 gpurun_out/ramp2.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ramp2 -o run -- python3 scripts/ramp_probe2.py cfg3 cfg4
python3 scripts/ramp_summary.py gpurun_out/ramp2/run_kernel_trace.csv > gpurun_out/ramp2_summary.txt 2>&1
