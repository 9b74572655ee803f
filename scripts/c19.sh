source scripts/r4_call.sh
step dist2_heat 300 gpurun_out/dist2_heat.log env LPGPU_XR_XCD=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload cfg4r8 --steps 128 --warmup 8 --no-rccl
step drv 600 gpurun_out/drv19.log python bench.py --steps 20 --warmup 5
step def 600 gpurun_out/def19.log python bench.py --no-cpu-baseline
