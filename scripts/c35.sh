source scripts/r4_call.sh
for i in 1 2 3; do
for E in 1 8; do
step pe${E}_$i 300 gpurun_out/pe${E}_$i.log python bench.py --workload cfg3 --no-cfg3 --steps 20 --warmup 5 --no-cpu-baseline --profile-every $E
done
done
