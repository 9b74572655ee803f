# device warm-up A/B at the driver's bench command, then default and the rehearsal
source scripts/r4_call.sh
for i in 1 2; do
step drv_heat$i 600 gpurun_out/drv_heat$i.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step drv_cold$i 600 gpurun_out/drv_cold$i.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline --device-warmup-ms 0
done
step def_heat 900 gpurun_out/def_heat.log python bench.py --no-cpu-baseline
step dist2_heat 300 gpurun_out/dist2_heat.log env LPGPU_XR_XCD=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload cfg4r8 --steps 128 --warmup 8 --no-rccl
