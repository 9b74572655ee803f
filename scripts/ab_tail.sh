#!/bin/bash
# same-box A/B of an environment switch on the cfg4 bench line: ab_tail.sh VAR a b [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; N=${4:-2}
for i in $(seq 1 "$N"); do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 200 python bench.py ${AB_ARGS:---no-cfg3} --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/ab.json || exit $?
    python -c "
import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print('$VAR=$v', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'],1), 'sel', round(d['selection']['us_per_pivot'],2))" | tee -a gpurun_out/ab.txt
  done
done
