#!/bin/bash
# One GPU-box session: each step has its own time limit; a test FAILURE
# (exit 1) lets the next step run, anything else (fault, abort, timeout)
# ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p "$OUT"
run() {
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -5 "$OUT/$name.log"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name"; exit "$rc"; fi
}
for step in "$@"; do
    case "$step" in
        pytest) run pytest_gpu 1200 python -u -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        drv) run bench_drv 300 python bench.py --steps 20 --warmup 5 ;;
        benchd) run bench_default 600 python bench.py ;;
        pytestx) run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py ;;
        benchq) run benchq 300 python bench.py --no-cpu-baseline ;;
        bsweep)
            for B in 1 2 4 8 16 32; do
                run bench_b$B 300 python bench.py --no-cpu-baseline --block $B
            done ;;
        psweep)
            for B in 4 8 16 32; do
                run benchp_b$B 300 python bench.py --no-cpu-baseline --block $B
            done
            LPGPU_SELECT=kernels run benchk_b16 300 python bench.py --no-cpu-baseline --block 16 ;;
        shards)
            for S in 2 8; do
                run bench_shards$S 600 python bench.py --no-cpu-baseline --group-shards $S --steps 256
            done ;;
        cfg4one)
            for B in 16 32; do
                run bench_cfg4_1gpu_b$B 600 python bench.py --no-cpu-baseline --block $B --emulate-ranks 8 --steps 256
            done ;;
        dist2)
            # two ranks sharing the one GPU: no RCCL (it refuses that), peer exchange only
            run bench_dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 256 --warmup 32 --no-rccl ;;
        dist4)
            run bench_dist4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 256 --warmup 32 --no-rccl ;;
        prof16)
            export TMPDIR=/tmp
            run rocprof16 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof16" -o run -- python3 "$PWD/bench.py" --steps 512 --block 16 --no-cpu-baseline ;;
        prof)
            export TMPDIR=/tmp
            run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$PWD/bench.py" --steps 200 --no-cpu-baseline ;;
        pipe)
            LPGPU_PIPELINE=0 run bench_nopipe 300 python bench.py --no-cpu-baseline
            for C in 32 64 96; do
                LPGPU_SEL_CUS=$C run bench_sel$C 300 python bench.py --no-cpu-baseline
            done
            run bench_pipe_b32 300 python bench.py --no-cpu-baseline --block 32
            run bench_pipe_b8 300 python bench.py --no-cpu-baseline --block 8 ;;
        sweepvw)
            for B in 16 32; do
                LPGPU_PIPELINE=0 run bench_np_b$B 300 python bench.py --no-cpu-baseline --block $B
                run bench_p_b$B 300 python bench.py --no-cpu-baseline --block $B
            done ;;
        sweepvar)
            for V in ${SWEEP_VARIANTS:-0 1 2 3 4}; do
                for B in 16 32; do
                    LPGPU_PIPELINE=0 LPGPU_SWEEP=$V run bench_v${V}_b$B 300 python bench.py --no-cpu-baseline --block $B --steps 512
                done
            done ;;
        ab)
            # A/B of library variants built by `make -C linear-program-solver_amd/csrc variant`
            for rep in 1 2; do
                for V in ${AB_VARIANTS:-all}; do
                    L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/$V.so
                    LPGPU_LIB=$L run stamps_${V}_$rep 300 python scripts/diag_stamps.py
                    LPGPU_LIB=$L LPGPU_PIPELINE=0 run bench_${V}_$rep 300 python bench.py --no-cpu-baseline --steps 512 --block ${AB_BLOCK:-16}
                done
            done ;;
        sweepgrid)
            run sweep_grid 300 python -u -m pytest tests/test_gpu_r2.py -k sweep_grid -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        tailab)
            # A/B: k_sweep_dp2's last strip spread over all blocks (LPGPU_SWEEP_TAIL)
            # and k_sweep_dp2 at 64 pivots (LPGPU_SWEEP_DP=2, cfg4)
            for rep in 1 2; do
                for T in 1 0; do
                    LPGPU_SWEEP_TAIL=$T run bench_tail${T}_$rep 300 python bench.py --no-cpu-baseline
                    LPGPU_SWEEP_TAIL=$T LPGPU_SWEEP_DP=2 run bench_dp2_tail${T}_$rep 300 python bench.py --no-cpu-baseline --no-cfg3
                done
            done ;;
        modes)
            for rep in 1 2; do
                for B in 16 32; do
                    LPGPU_PIPELINE=0 run bench_np_b${B}_$rep 300 python bench.py --no-cpu-baseline --steps 1024 --block $B
                    LPGPU_PIPELINE=1 run bench_p_b${B}_$rep 300 python bench.py --no-cpu-baseline --steps 1024 --block $B
                done
            done ;;
        swcus)
            LPGPU_PIPELINE=0 run bench_np 300 python bench.py --no-cpu-baseline --steps 1024
            for C in 32 64 96 128 191; do
                LPGPU_PIPELINE=1 LPGPU_SWEEP_CUS=$C run bench_p_sw$C 300 python bench.py --no-cpu-baseline --steps 1024
            done ;;
        pmcsq)
            export TMPDIR=/tmp
            for B in ${PMC_BLOCKS:-16 32}; do
                run pmcsq_b$B 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS --output-format csv -d "$OUT/pmcsq_b$B" -o run -- python3 "$PWD/bench.py" --steps 128 --warmup 16 --no-cpu-baseline --block $B
                run pmcgr_b$B 600 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmcgr_b$B" -o run -- python3 "$PWD/bench.py" --steps 128 --warmup 16 --no-cpu-baseline --block $B
            done ;;
        st)
            # strip sweep: full GPU suite on one variant, then timing
            LPGPU_SWEEP=${ST_VARIANT:-21} run pytest_st 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 60 --timeout-method thread
            for V in ${ST_BENCH:-0 21 23 24}; do
                for B in 16 32; do
                    LPGPU_SWEEP=$V run bench_st${V}_b$B 300 python bench.py --no-cpu-baseline --steps 1024 --block $B
                done
            done
            grep -H -o '"avg_launch_us": [0-9.]*' "$OUT"/bench_st*.log ;;
        stvar)
            for rep in 1 2; do
                for V in ${ST_BENCH:-21 25 26 27}; do
                    LPGPU_SWEEP=$V run bench_v${V}_$rep 300 python bench.py --no-cpu-baseline --steps 1024
                done
                for C in ${ST_BPC:-2 4}; do
                    LPGPU_SWEEP_BPC=$C run bench_bpc${C}_$rep 300 python bench.py --no-cpu-baseline --steps 1024
                done
            done
            grep -H -o '"avg_launch_us": [0-9.]*' "$OUT"/bench_v*.log "$OUT"/bench_bpc*.log | awk 'NR % 2 == 1' ;;
        xcd)
            # selection blocks on one XCD with L2-local hand-offs
            LPGPU_SEL_XCD=1 run pytest_xcd 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 60 --timeout-method thread
            for rep in 1 2; do
                for X in 0 1; do
                    LPGPU_SEL_XCD=$X run bench_x${X}_$rep 300 python bench.py --no-cpu-baseline --steps 1024
                done
            done
            LPGPU_SEL_XCD=1 run stamps_x1 300 python scripts/diag_stamps.py
            grep -H -o '"value": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_x*.log ;;
        check)
            # the default build: GPU suite, two timing runs, phase stamps
            run pytest_check 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 60 --timeout-method thread
            for rep in 1 2; do
                run bench_c$rep 300 python bench.py --no-cpu-baseline --steps 1024
            done
            run stamps_c 300 python scripts/diag_stamps.py
            grep -H -o '"value": [0-9.]*\|"us_per_pivot": [0-9.]*\|"avg_launch_us": [0-9.]*' "$OUT"/bench_c*.log ;;
        xrx)
            # row-sharded selection on one XCD per rank, forced with two ranks on
            # ONE GPU (their launches must then be resident together)
            run pytest_peer 300 python -u -m pytest tests/test_gpu_peer_procs.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            LPGPU_XR_XCD=2 run pytest_peer_x 300 python -u -m pytest tests/test_gpu_peer_procs.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            run bench_dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 256 --warmup 32 --no-rccl
            LPGPU_XR_XCD=2 run bench_dist2_x 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 256 --warmup 32 --no-rccl
            grep -H -o '"value": [0-9.]*\|"us_per_pivot": [0-9.]*\|"avg_launch_us": [0-9.]*' "$OUT"/bench_dist2*.log ;;
        stamps)
            run stamps 300 python scripts/diag_stamps.py ;;
        xpipe)
            # selection on one XCD beside the sweep on the other seven
            LPGPU_PIPELINE=1 run pytest_xpipe 600 python -u -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider --timeout 60 --timeout-method thread
            run bench_xp_np 300 python bench.py --no-cpu-baseline --steps 1024
            for B in ${XP_BLOCKS:-8 12 16 20 22}; do
                LPGPU_PIPELINE=1 run bench_xp_b$B 300 python bench.py --no-cpu-baseline --steps 1024 --block $B
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_xp_*.log ;;
        xpdiag)
            LPGPU_DEBUG_XCC=1 run bench_xd_np 300 python bench.py --no-cpu-baseline --steps 1024 --block 16
            LPGPU_DEBUG_XCC=1 LPGPU_PIPELINE=1 run bench_xd_p16 300 python bench.py --no-cpu-baseline --steps 1024 --block 16
            LPGPU_DEBUG_XCC=1 LPGPU_PIPELINE=1 LPGPU_PIPE_SERIAL=1 run bench_xd_s16 300 python bench.py --no-cpu-baseline --steps 1024 --block 16
            for f in "$OUT"/bench_xd_*.log; do echo $f; grep -o 'sel_xcc [0-9]*' $f | sort | uniq -c; done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_xd_*.log ;;
        big1)
            run pytest_big 600 python -u -m pytest tests/test_gpu_parity.py -k "block_count or lds_edge or cfg3_full" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for E in 4 8; do
                run bench_big_e$E 600 python bench.py --no-cpu-baseline --emulate-ranks $E --steps 256
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_big_e*.log ;;
        tiles)
            LPGPU_SWEEP=41 run pytest_tiles 300 python -u -m pytest tests/test_gpu_parity.py -k "cfg3_full and persistent" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for rep in 1 2; do
                for V in 21 40 41; do
                    LPGPU_SWEEP=$V run bench_tl${V}_$rep 300 python bench.py --no-cpu-baseline --steps 1024
                done
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*' "$OUT"/bench_tl*.log ;;
        bsz)
            # pivots per sweep beyond 32 (BMAX 64)
            run pytest_bsz 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for rep in 1 2; do
                for B in ${BSZ:-32 40 44 48}; do
                    run bench_bsz${B}_$rep 300 python bench.py --no-cpu-baseline --steps 1056 --block $B
                done
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_bsz*.log ;;
        msw)
            LPGPU_SWEEP=50 run pytest_msw 600 python -u -m pytest tests/test_gpu_parity.py -k "cfg3_full or ragged or block_size" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for rep in 1 2; do
                for V in 21 50; do
                    LPGPU_SWEEP=$V run bench_msw${V}_$rep 300 python bench.py --no-cpu-baseline --steps 1024
                done
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*' "$OUT"/bench_msw*.log ;;
        wt)
            LPGPU_SWEEP=28 run pytest_wt 300 python -u -m pytest tests/test_gpu_parity.py -k "cfg3_full and persistent" -q -p no:cacheprovider --timeout 120 --timeout-method thread
            for rep in 1 2; do
                for V in 21 28 29; do
                    LPGPU_SWEEP=$V run bench_wt${V}_$rep 300 python bench.py --no-cpu-baseline
                done
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*' "$OUT"/bench_wt*.log ;;
        tall1)
            # the whole weak-scaling tableau of N ranks on ONE GPU (rows 4096 N)
            for E in ${TALL_RANKS:-2 4 8}; do
                run bench_tall1_e$E 600 python bench.py --no-cpu-baseline --emulate-ranks $E --steps 256
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_tall1_e*.log ;;
        pmc)
            # HBM traffic of the sweep, per workload: two --pmc passes each
            # (FETCH_SIZE and WRITE_SIZE do not fit one pass), one workload a run
            export TMPDIR=/tmp
            for W in ${PMC_WORKLOADS:-cfg4 cfg3}; do
                run pmc_fetch_$W 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$W" -o run -- python3 "$PWD/bench.py" --workload $W --no-cfg3 --steps 8 --warmup 2 --no-cpu-baseline --device-warmup-ms 0
                run pmc_write_$W 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$W" -o run -- python3 "$PWD/bench.py" --workload $W --no-cfg3 --steps 8 --warmup 2 --no-cpu-baseline --device-warmup-ms 0
                PB=64   # the engine's auto pivots per sweep (cfg4 and, since round 3, cfg3)
                run pmc_json_$W 120 python scripts/hbm_traffic.py "$OUT/pmc_fetch_$W" "$OUT/pmc_write_$W" "$OUT/hbm_traffic.json" --block $PB --kernel k_sweep_rl --workload $W
            done ;;
        proffinal)
            export TMPDIR=/tmp
            run rocprof_final 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_final" -o run -- python3 "$PWD/bench.py" --no-cpu-baseline ;;
        exp1)
            # cfg4 by pivots per sweep; phase stamps of cfg3 and cfg4
            for B in ${EXP_BLOCKS:-32 48 64}; do
                run bench_cfg4_b$B 300 python bench.py --no-cpu-baseline --no-cfg3 --block $B --steps 24 --warmup 4
            done
            L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/stamps.so
            LPGPU_LIB=$L run stamps_cfg3 300 python scripts/diag_stamps.py mixed 4096 4096 32
            LPGPU_LIB=$L run stamps_cfg4 300 python scripts/diag_stamps.py tall 32768 8192 32
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_cfg4_b*.log ;;
        exp2)
            run gather_probe 120 ./scripts/gather_probe
            LPGPU_SWEEP_WIDE=1 run pytest_wide 300 python -u -m pytest tests/test_gpu_parity.py -k "block_size or cfg3_full" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for B in 48 64; do
                LPGPU_SWEEP_WIDE=1 run bench_cfg4_w_b$B 300 python bench.py --no-cpu-baseline --no-cfg3 --block $B --steps 24 --warmup 4
            done
            for B in 32 48 64; do
                LPGPU_SWEEP_WIDE=1 run bench_cfg3_w_b$B 300 python bench.py --no-cpu-baseline --workload cfg3 --block $B --steps 64 --warmup 4
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_cfg*_w_b*.log ;;
        exp3)
            run pytest_gpu 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for B in 32 48; do
                run bench_cfg4_p_b$B 300 python bench.py --no-cpu-baseline --no-cfg3 --block $B --steps 24 --warmup 4
                LPGPU_LD_RAW=1 run bench_cfg4_raw_b$B 300 python bench.py --no-cpu-baseline --no-cfg3 --block $B --steps 24 --warmup 4
                run bench_cfg3_p_b$B 300 python bench.py --no-cpu-baseline --workload cfg3 --block $B --steps 64 --warmup 4
                LPGPU_LD_RAW=1 run bench_cfg3_raw_b$B 300 python bench.py --no-cpu-baseline --workload cfg3 --block $B --steps 64 --warmup 4
            done
            L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/stamps.so
            LPGPU_LIB=$L run stamps_cfg4_p 300 python scripts/diag_stamps.py tall 32768 8192 32
            LPGPU_LIB=$L run stamps_cfg3_p 300 python scripts/diag_stamps.py mixed 4096 4096 32
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_cfg*_p_b*.log "$OUT"/bench_cfg*_raw_b*.log ;;
        exp4)
            LPGPU_SWEEP_DP=1 run pytest_dp 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for B in 32 48 64; do
                LPGPU_SWEEP_DP=1 run bench_cfg4_dp_b$B 300 python bench.py --no-cpu-baseline --no-cfg3 --block $B --steps 24 --warmup 4
                LPGPU_SWEEP_DP=1 run bench_cfg3_dp_b$B 300 python bench.py --no-cpu-baseline --workload cfg3 --block $B --steps 64 --warmup 4
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_cfg*_dp_b*.log ;;
        exp5)
            LPGPU_SWEEP_DP=2 run pytest_dp2 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_r2.py -k "block_size or cfg3_full or cfg4 or ragged" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for D in 1 2; do
                for B in 48 64; do
                    LPGPU_SWEEP_DP=$D run bench_cfg4_d${D}_b$B 300 python bench.py --no-cpu-baseline --no-cfg3 --block $B --steps 24 --warmup 4
                done
                for B in 32 48; do
                    LPGPU_SWEEP_DP=$D run bench_cfg3_d${D}_b$B 300 python bench.py --no-cpu-baseline --workload cfg3 --block $B --steps 64 --warmup 4
                done
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*' "$OUT"/bench_cfg*_d*_b*.log ;;
        pmcsq2)
            export TMPDIR=/tmp
            for W in cfg3 cfg4; do
                run pmcsq_$W 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS --output-format csv -d "$OUT/pmcsq_$W" -o run -- python3 "$PWD/bench.py" --workload $W --no-cfg3 --steps 16 --warmup 4 --no-cpu-baseline
                run pmcsq2_$W 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmcsq2_$W" -o run -- python3 "$PWD/bench.py" --workload $W --no-cfg3 --steps 16 --warmup 4 --no-cpu-baseline
            done ;;
        quick)
            # parity subset + cfg4 / cfg3 timing (auto pivots per sweep)
            run pytest_quick 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_r2.py -k "block_size or cfg3_full or cfg4 or ragged" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for rep in 1 2; do
                run bench_q4_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
                run bench_q3_$rep 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4
            done
            grep -H -o '"value": [0-9.]*\|"avg_launch_us": [0-9.]*\|"us_per_pivot": [0-9.]*' "$OUT"/bench_q*.log ;;
        full)
            # whole GPU suite (stops at the first failure), then the quick timing
            run pytest_full 1000 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        stamps2)
            L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/stamps.so
            LPGPU_LIB=$L run stamps2_cfg4 300 python scripts/diag_stamps.py tall 32768 8192 64
            LPGPU_LIB=$L run stamps2_cfg3 300 python scripts/diag_stamps.py mixed 4096 4096 48 ;;
        abq)
            # A/B: variants/headA.so against the current build (LPGPU_GMAJ 1 / 0), cfg4 and cfg3
            for rep in 1 2; do
                for V in headA cur cur0; do
                    L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/headA.so
                    [ $V = headA ] || L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/liblpgpu.so
                    G=1; [ $V = cur0 ] && G=0
                    LPGPU_LIB=$L LPGPU_GMAJ=$G run ab4_${V}_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
                    LPGPU_LIB=$L LPGPU_GMAJ=$G run ab3_${V}_$rep 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4
                done
            done
            for f in "$OUT"/ab*_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"us_per_pivot": [0-9.]*' $f | tail -1)"; done ;;
        selg)
            # selection blocks on one XCD: 64 (rows / 64) against 128 at cfg3
            for rep in 1 2; do
                for GB in 0 128; do
                    for B in 32 48; do
                        LPGPU_SEL_BLOCKS=$GB run selg_${GB}_b${B}_$rep 300 python bench.py --no-cpu-baseline --workload cfg3 --block $B --steps 64 --warmup 4
                    done
                done
            done
            for f in "$OUT"/selg_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"us_per_pivot": [0-9.]*' $f | tail -1)"; done ;;
        lite)
            for rep in 1 2; do
                for PL in 0 1 2; do
                    LPGPU_POLL_LITE=$PL run lite4_${PL}_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
                    LPGPU_POLL_LITE=$PL run lite3_${PL}_$rep 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4
                done
            done
            for f in "$OUT"/lite*_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"us_per_pivot": [0-9.]*' $f | tail -1)"; done ;;
        dp2)
            LPGPU_SWEEP_DP=2 run pytest_dp2 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_ties.py -k "block_size or cfg3_full or cfg4 or ragged or tie" -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
            for rep in 1 2; do
                for D in 1 3; do
                    LPGPU_SWEEP_DP=$D run dp4_${D}_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
                    LPGPU_SWEEP_DP=$D run dp3_${D}_$rep 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4
                done
            done
            for f in "$OUT"/dp[34]_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"avg_launch_us": [0-9.]*' $f | head -1)"; done ;;
        swx)
            # sweep cost breakdown: diagnostic builds with parts of the sweep removed
            for rep in 1 2; do
                for V in ${SWX_VARIANTS:-base swx1 swx2 swx3 swx4}; do
                    L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/$V.so
                    [ $V = base ] && L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/liblpgpu.so
                    LPGPU_LIB=$L run swx4_${V}_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
                    LPGPU_LIB=$L run swx3_${V}_$rep 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4
                done
            done
            for f in "$OUT"/swx*_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f) $(grep -o '"avg_launch_us": [0-9.]*' $f | head -1)"; done ;;
        timing)
            # cfg4 and cfg3 timing, two runs each (auto pivots per sweep)
            for rep in 1 2; do
                run t4_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
                run t3_$rep 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4
            done
            for f in "$OUT"/t[34]_*.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'], 1), 'frac', round(d['roofline']['frac'], 3), 'sel', round(d['selection']['us_per_pivot'], 2))"; done ;;
        configs) run configs 600 python bench.py --configs ;;
        hier)
            # two-level exchange for spread selection blocks: A/B at cfg4, then phase clocks
            for rep in 1 2 3; do
                for H in 0 1; do
                    LPGPU_HIER=$H run hier_${H}_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
                done
            done
            L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/stamps.so
            LPGPU_LIB=$L run stamps_hier1 300 python scripts/diag_stamps.py tall 32768 8192 64
            LPGPU_LIB=$L LPGPU_HIER=0 run stamps_hier0 300 python scripts/diag_stamps.py tall 32768 8192 64
            for f in "$OUT"/hier_*.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'sel', round(d['selection']['us_per_pivot'], 2))"; done
            grep -H "^avg" "$OUT"/stamps_hier*.log ;;
        r3t)
            # round 3: cfg3 at 48 / 64 pivots per sweep, cfg4 default, stamps of cfg3 (k_sel)
            for rep in 1 2; do
                for B in 48 64; do
                    run t3b${B}_$rep 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4 --block $B
                done
                run t4_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
            done
            for f in "$OUT"/t3b*_*.log "$OUT"/t4_*.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'], 1), 'frac', round(d['roofline']['frac'], 3), 'sel', round(d['selection']['us_per_pivot'], 2))"; done
            L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/stamps.so
            LPGPU_LIB=$L run stamps3_48 300 python scripts/diag_stamps.py mixed 4096 4096 48
            LPGPU_LIB=$L run stamps3_64 300 python scripts/diag_stamps.py mixed 4096 4096 64
            grep -H "^avg\|^pcomp" "$OUT"/stamps3_*.log ;;
        t3q)
            # cfg3 quick: one run per pivots-per-sweep value
            for B in ${T3_BLOCKS:-32 48 64}; do
                run t3q_b$B 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4 --block $B
            done
            for f in "$OUT"/t3q_b*.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'], 1), 'frac', round(d['roofline']['frac'], 3), 'sel', round(d['selection']['us_per_pivot'], 2))"; done ;;
        vab)
            # library variants (make variant NAME=...) on cfg3 at ${VAB_BLOCK:-48} pivots per sweep
            for V in ${VAB_VARIANTS:-main}; do
                L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/$V.so
                [ "$V" = main ] && L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/liblpgpu.so
                LPGPU_LIB=$L run vab_$V 300 python bench.py --no-cpu-baseline --workload ${VAB_WORKLOAD:-cfg3} --steps 64 --warmup 4 --block ${VAB_BLOCK:-48}
            done
            for f in "$OUT"/vab_*.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'], 1), 'sel', round(d['selection']['us_per_pivot'], 3))"; done ;;
        rgtest)
            LPGPU_SWEEP_DP=${SWV:-4} run rgtest 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        rgab)
            for B in ${T3_BLOCKS:-32 48 64}; do
                run rgab_def_b$B 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4 --block $B
                LPGPU_SWEEP_DP=${SWV:-4} run rgab_rg_b$B 300 python bench.py --no-cpu-baseline --workload cfg3 --steps 64 --warmup 4 --block $B
            done
            for f in "$OUT"/rgab_*.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'], 1), 'frac', round(d['roofline']['frac'], 3), 'sel', round(d['selection']['us_per_pivot'], 3))"; done ;;
        r3new)
            run r3new 900 python -u -m pytest tests/test_gpu_r3.py -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "40000" ;;
        r3procs)
            run r3procs 1000 python -u -m pytest tests/test_gpu_r3_procs.py -v -p no:cacheprovider --timeout 900 --timeout-method thread ${R3P_K:+-k "$R3P_K"} ;;
        c4ab)
            # cfg4 on one GPU: default sweep against an LPGPU_SWEEP_DP variant
            for rep in 1 2; do
                run c4ab_def_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
                LPGPU_SWEEP_DP=${SWV:-5} run c4ab_sw_$rep 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
            done
            for f in "$OUT"/c4ab_*.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'], 1), 'frac', round(d['roofline']['frac'], 3), 'sel', round(d['selection']['us_per_pivot'], 3))"; done ;;
        c4var)
            # cfg4 on one GPU, library variants with LPGPU_SWEEP_DP=${SWV:-5}
            for V in ${C4_VARIANTS:-main}; do
                L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/$V.so
                [ "$V" = main ] && L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/liblpgpu.so
                LPGPU_LIB=$L LPGPU_SWEEP_DP=${SWV:-5} run c4var_$V 300 python bench.py --no-cpu-baseline --no-cfg3 --steps 24 --warmup 4
            done
            for f in "$OUT"/c4var_*.log; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['value']), 'sweep', round(d['roofline']['avg_launch_us'], 1), 'frac', round(d['roofline']['frac'], 3), 'sel', round(d['selection']['us_per_pivot'], 3))"; done ;;
        r3f)
            run r3f 300 python -u -m pytest tests/test_gpu_r2.py -k timeout -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
        clk)
            for V in ${CLK_VARIANTS:-stamps}; do
                L=$PWD/linear-program-solver_amd/lpsol_amd/_lib/variants/$V.so
                for B in ${CLK_BLOCKS:-48}; do
                    LPGPU_LIB=$L run clk_${V}_b$B 300 python scripts/sel_clocks.py mixed 4096 4096 $B
                    cat "$OUT/clk_${V}_b$B.log"
                done
            done ;;
        r3p)
            run r3p 600 python -u -m pytest tests/test_gpu_r3.py -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
