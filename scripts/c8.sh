
# the 8-GPU rank kernel (k_sel<XR>, 4096 rows, G = 64) as two ranks on the one GPU
step dist2 300 gpurun_out/bench_dist2_cfg4r8.json env LPGPU_XR_XCD=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload cfg4r8 --steps 128 --warmup 8 --no-rccl
# and as one process (the same rows and kernel shapes without the cross-rank hop)
step one8 300 gpurun_out/bench_cfg4r8_1gpu.json python bench.py --workload cfg4r8 --no-cpu-baseline --steps 128
