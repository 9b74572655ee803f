source scripts/r4_call.sh
step smoke 300 gpurun_out/final6_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step drv 600 gpurun_out/final6_drv.log python bench.py --gpus 1 --steps 20 --warmup 5
step bench 900 gpurun_out/final6_bench.log python bench.py
