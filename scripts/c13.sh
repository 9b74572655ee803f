source scripts/r4_call.sh
step ramp 600 gpurun_out/ramp.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ramp -o run -- python3 scripts/ramp_probe.py cfg3 cfg4
python3 scripts/ramp_summary.py $(ls gpurun_out/ramp/*/run_kernel_trace.csv gpurun_out/ramp/run_kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/ramp_summary.txt 2>&1
