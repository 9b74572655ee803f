source scripts/r4_call.sh
for i in 1 2 3; do
for H in 150 400; do
step drv_h${H}_$i 600 gpurun_out/drv_h${H}_$i.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline --device-warmup-ms $H
done
done
