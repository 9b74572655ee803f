#!/bin/bash
# The one gpurun entry point: named steps, each under its own time limit,
# logs under gpurun_out/.  A step that faults, aborts or hits its limit ends
# the call (no later GPU step runs); a plain test failure (rc 1) goes on.
#
#   gpurun -- bash scripts/gpu.sh <step> [<step> ...]
#
# steps
#   pytest        the whole GPU suite (-m gpu)
#   smoke         __graft_entry__.smoke()
#   drv           the driver's bench command (--steps 20 --warmup 5) -> drv.json
#   bench         the default bench command -> bench.json
#   clk3 / clk4   k_sel phase stamps (variants/stamps.so) at cfg3 / cfg4 (XS)
#   ab            same-box A/B of library builds:
#                   AB_LIBS="main v1 ..." (variants/<v>.so; main = liblpgpu.so)
#                   AB_WL=cfg3|cfg4 AB_REPS=3 AB_ENV="VAR=x" -> ab.txt
#   abenv         same-box A/B of environment settings (scripts/ab_env.sh):
#                   AB_WL, AB_REPS, AB_SETTINGS="VAR=a|VAR=b|-"
#   prof          rocprofv3 --kernel-trace --stats of the drv command -> prof/
#   pmc           HBM traffic of the sweep (FETCH_SIZE / WRITE_SIZE passes) -> hbm_traffic.json
#   pmcx          other counter passes: PMC_SETS="A B|C D" AB_WL=cfg3
#   dist2         two ranks on ONE GPU over IPC, cfg4's 8-GPU rank rows (cfg4r8)
#   t:<expr>      pytest -m gpu -k <expr>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p "$OUT"
LIBDIR=$PWD/linear-program-solver_amd/lpsol_amd/_lib
run() {   # run <name> <limit-seconds> <command...>
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -4 "$OUT/$name.log"
    if grep -q -i -E "illegal memory access|memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure" "$OUT/$name.log"; then
        echo "== $name: GPU fault seen, stopping"; exit 99
    fi
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name"; exit "$rc"; fi
    return 0
}
lib() { [ "$1" = main ] && echo "$LIBDIR/liblpgpu.so" || echo "$LIBDIR/variants/$1.so"; }
summ() {   # one line from a bench JSON log
    python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = d.get("selection", {})
ck = d["roofline"].get("shader_clock") or {}
print(sys.argv[1], round(d["value"]), "sweep", round(d["roofline"]["avg_launch_us"], 1),
      "kcyc", round(ck.get("kcycles_mean", 0), 1), "GHz", round(ck.get("ghz_mean", 0), 3),
      "frac", round(d["roofline"]["frac"], 3), "sel", round(s.get("us_per_pivot", 0), 3),
      "fb", d.get("fallbacks"), "cfg3", round(d.get("cfg3", {}).get("value", 0)),
      "cfg3sel", round(d.get("cfg3", {}).get("selection", {}).get("us_per_pivot", 0), 3),
      "cfg3sweep", round(d.get("cfg3", {}).get("roofline", {}).get("avg_launch_us", 0), 1))
EOF
}
for step in "$@"; do
    case "$step" in
        pytest) run pytest_gpu 1200 python -u -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider \
                    --timeout 120 --timeout-method thread ;;
        t:*) run "pytest_k" 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider -k "${step#t:}" \
                 --timeout 120 --timeout-method thread ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        drv) run drv 300 python bench.py --steps 20 --warmup 5 && cp "$OUT/drv.log" "$OUT/drv.json" && summ drv "$OUT/drv.json" ;;
        bench) run bench 600 python bench.py && summ bench "$OUT/bench.log" ;;
        clk3) LPGPU_LIB=$(lib stamps) run clk3 300 python scripts/sel_clocks.py mixed 4096 4096 64 && cat "$OUT/clk3.log" ;;
        clk4) LPGPU_LIB=$(lib stamps) run clk4 300 python scripts/sel_clocks.py tall 32768 8192 64 && cat "$OUT/clk4.log" ;;
        ab)
            wl=${AB_WL:-cfg3}
            for rep in $(seq 1 "${AB_REPS:-3}"); do
                for v in ${AB_LIBS:-main}; do
                    run "ab_${v}_$rep" 200 env ${AB_ENV:-} LPGPU_LIB="$(lib "$v")" python bench.py --workload "$wl" \
                        --no-cfg3 --no-cpu-baseline --steps 64 --warmup 5 --profile-every 1
                    summ "$wl $v" "$OUT/ab_${v}_$rep.log" | tee -a "$OUT/ab.txt"
                done
            done ;;
        abenv)
            IFS='|' read -r -a S <<< "${AB_SETTINGS:--}"
            run abenv 900 bash scripts/ab_env.sh "${AB_WL:-cfg3}" "${AB_REPS:-3}" "${S[@]}" ;;
        prof)
            export TMPDIR=/tmp
            run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 20 --warmup 5 \
                --no-cpu-baseline ;;
        pmc)
            # HBM traffic of the sweep per workload: FETCH_SIZE and WRITE_SIZE
            # in passes of their own (they do not fit one), then the JSON
            # bench.py stamps as roofline.traffic (scripts/hbm_traffic.py)
            export TMPDIR=/tmp
            for W in ${PMC_WORKLOADS:-cfg4 cfg3}; do
                for c in FETCH_SIZE WRITE_SIZE; do
                    run "pmc_${c}_$W" 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${c}_$W" -o run -- \
                        python3 "$PWD/bench.py" --workload $W --no-cfg3 --steps 8 --warmup 2 --no-cpu-baseline \
                        --device-warmup-ms 0
                done
                run "pmc_json_$W" 120 python scripts/hbm_traffic.py "$OUT/pmc_FETCH_SIZE_$W" "$OUT/pmc_WRITE_SIZE_$W" \
                    "$OUT/hbm_traffic.json" --block 64 --kernel k_sweep_rl --workload $W
            done ;;
        pmcx)
            # other counters of one workload, one pass per PMC_SETS entry ("A B C|D E")
            export TMPDIR=/tmp
            IFS='|' read -r -a S <<< "${PMC_SETS:?}"
            k=0
            for ctr in "${S[@]}"; do
                k=$((k + 1))
                run "pmcx_$k" 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmcx_$k" -o run -- \
                    python3 "$PWD/bench.py" --workload "${AB_WL:-cfg3}" --no-cfg3 --steps 8 --warmup 2 \
                    --no-cpu-baseline --device-warmup-ms 0
            done ;;
        dist2) run dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
                   --master-port 29533 bench.py --gpus 2 --workload cfg4r8 --no-rccl --steps 64 --warmup 5 ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
