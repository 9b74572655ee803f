source scripts/r4_call.sh
step heat2 300 gpurun_out/heat2.log env LPGPU_XR_XCD=1 LPGPU_BENCH_FORCE_HEAT=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload cfg3 --steps 64 --warmup 5 --no-rccl
