# closing measurements of a build (round 4, second pass): suite, smoke, PMC
# traffic stamped with these sources, bench lines, rocprof summary, rehearsals
source scripts/r4_call.sh
step suite 1200 gpurun_out/final4_suite.log python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread
step smoke 300 gpurun_out/final4_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step pmc 1200 gpurun_out/final4_pmc.log bash scripts/gpu_run.sh pmc
step bench 900 gpurun_out/final4_bench.log python bench.py --traffic-json gpurun_out/hbm_traffic.json
step drv 600 gpurun_out/final4_drv.log python bench.py --steps 20 --warmup 5 --traffic-json gpurun_out/hbm_traffic.json
step prof 900 gpurun_out/final4_prof.log bash scripts/gpu_run.sh proffinal
step dist2 300 gpurun_out/final4_dist2.log env LPGPU_XR_XCD=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload cfg4r8 --steps 128 --warmup 8 --no-rccl
step heat2 300 gpurun_out/final4_heat2.log env LPGPU_XR_XCD=1 LPGPU_BENCH_FORCE_HEAT=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --workload cfg3 --steps 64 --warmup 5 --no-rccl
step configs 600 gpurun_out/final4_configs.log python bench.py --configs
