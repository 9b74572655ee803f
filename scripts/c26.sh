source scripts/r4_call.sh
step geo 600 gpurun_out/geo_probe.txt python scripts/geo_probe.py
