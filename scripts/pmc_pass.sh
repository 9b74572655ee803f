#!/bin/bash
# PMC passes over one bench workload: each pass its own rocprofv3 run (counters
# of one pass within gfx950's per-block slots: <= 8 SQ, <= 4 TCC, <= 2 GRBM).
# usage: bash scripts/pmc_pass.sh <outdir> <workload> "<counters pass 1>" "<counters pass 2>" ...
set -u
out=$1; wl=$2; shift 2
export TMPDIR=/tmp
mkdir -p "$out"
k=0
for ctr in "$@"; do
    k=$((k + 1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/p$k" -o run -- \
        python3 "$PWD/bench.py" --workload "$wl" --no-cfg3 --no-cpu-baseline --steps 12 --warmup 2 \
        > "$out/p$k.log" 2>&1
    rc=$?
    # a refused counter list is not a fault (go on); a kill at the limit is
    if [ $rc -ne 0 ]; then echo "pmc pass $k rc=$rc"; [ $rc -ge 124 ] && exit $rc; fi
done
