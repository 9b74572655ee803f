source scripts/r4_call.sh
step oopw 600 gpurun_out/t29_oopw.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_r4.py -k "out_of_place"
