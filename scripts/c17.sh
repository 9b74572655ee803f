source scripts/r4_call.sh
VD=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants
step t 900 gpurun_out/t17.log python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_r4.py tests/test_gpu_parity.py tests/test_gpu_xs.py
step ab3 900 gpurun_out/ab17_3.log bash scripts/ab_env.sh cfg3 2 - LPGPU_LIB=$VD/r4c.so
step ab4 900 gpurun_out/ab17_4.log bash scripts/ab_env.sh cfg4 2 - LPGPU_LIB=$VD/r4c.so
for i in 1 2; do
step drv_heat$i 600 gpurun_out/drv_heat$i.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step drv_cold$i 600 gpurun_out/drv_cold$i.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline --device-warmup-ms 0
done
step dist2_heat 300 gpurun_out/dist2_heat.log env LPGPU_XR_XCD=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload cfg4r8 --steps 128 --warmup 8 --no-rccl
