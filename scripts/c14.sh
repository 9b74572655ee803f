source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
for v in head noepi notail; do
step ramp_$v 600 gpurun_out/ramp_$v.log env LPGPU_LIB=$VD/$v.so rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ramp_$v -o run -- python3 scripts/ramp_probe.py cfg3 cfg4
python3 scripts/ramp_summary.py gpurun_out/ramp_$v/run_kernel_trace.csv > gpurun_out/ramp_summary_$v.txt 2>&1
done
