# the PMC traffic stamp of the final sources (they differ from 123a49ea by a comment)
source scripts/r4_call.sh
step pmc 1200 gpurun_out/final5_pmc.log bash scripts/gpu_run.sh pmc
step bench 900 gpurun_out/final5_bench.log python bench.py --traffic-json gpurun_out/hbm_traffic.json --no-cpu-baseline
