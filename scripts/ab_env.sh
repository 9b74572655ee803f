#!/bin/bash
# same-box A/B of environment settings on one bench workload:
#   ab_env.sh <workload> <reps> "VAR=a VAR2=b" "VAR=c" ...   ("-" = no setting)
# one line per run into gpurun_out/ab.txt (pivots/s, sweep us, selection us/pivot)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
wl=$1; n=$2; shift 2
for i in $(seq 1 "$n"); do
  for setting in "$@"; do
    s=$setting; [ "$s" = "-" ] && s=""
    env $s timeout -k 10 200 python bench.py --workload "$wl" --no-cfg3 --no-cpu-baseline --steps 64 --warmup 5 --profile-every 1 > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$wl [$setting] rc=$rc" | tee -a gpurun_out/ab.txt; tail -3 gpurun_out/ab.err; exit $rc; fi
    python -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
ck=d['roofline'].get('shader_clock') or {}
print('$wl', '[$setting]', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'],1), 'kcyc', round(ck.get('kcycles_mean',0),1), 'GHz', round(ck.get('ghz_mean',0),3), 'frac', round(d['roofline']['frac'],3), 'sel', round(d['selection']['us_per_pivot'],2), 'fb', d['fallbacks'])" | tee -a gpurun_out/ab.txt
  done
done
