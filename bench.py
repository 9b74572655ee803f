#!/usr/bin/env python3
"""Benchmark of the dense simplex pivot hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One "step" = one simplex pivot (entering scan, ratio test, rank-1 update of
the whole float64 tableau) with the standard rule, all on the device (the
rank-1 updates of 32 pivots are applied in one sweep; bit-identical).
Workload (weak scaling): every GPU holds 4096 constraint rows
of an 8192-variable tableau.
  N = 1 : cfg3, G_mixed(m=4096, ns=4096, seed 3) -> a 4097 x 8193 tableau
  N > 1 : G_tall(m=4096*N, n=8192, seed 3), rows sharded 4096 per rank
          (N = 8 is cfg4, the 32768 x 8192 tableau).  Per pivot the ranks
          exchange candidates and the pivot row device-side (peer stores over
          xGMI inside one persistent selection kernel per group); RCCL
          collectives per pivot if that exchange cannot be set up.
``value`` = pivots/s x N (each pivot sweeps N shards of 4096 x 8192), i.e.
plain LP pivots/s at N = 1; ``lp_pivots_per_s`` is the LP-level rate.

Inputs are resident in HBM before the timed region.  Every sweep and
selection launch inside the timed region carries a pair of HIP events that
the launch itself records at the kernel's start and end (hipExtLaunchKernelGGL
on the engine's stream, lp_profile): the roofline's achieved bandwidth is the
sweep's algorithmic bytes over that kernel time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from lpsol_amd import _lib  # noqa: E402
from lpsol_amd import generators as gen  # noqa: E402

METRIC = "pivots/sec + achieved HBM GB/s on dense float64 tableau, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
ROWS_PER_GPU = 4096
NCOLS = 8192
SEED = 3


def pivot_bytes(m: int, n: int) -> int:
    """Algorithmic bytes of one pivot: read+write the whole
    tableau, the row-0 scan and the column+b ratio gather."""
    return 8 * (2 * (m + 1) * (n + 1) + (n + 1) + 2 * (m + 1))


SWEEP_KERNEL = "k_sweep_st"


def sweep_bytes(rows: int, n: int, block: int) -> int:
    """Algorithmic bytes of one sweep (k_sweep_st) launch on `rows` local rows applying
    `block` deferred pivots: read and write every row once, read the block's
    pivot rows P and multiplier columns M."""
    return 8 * (2 * rows * (n + 1) + block * (n + 1) + block * rows)


def workload(nranks: int, rank: int):
    """(kind, m, ns, n, row block) of this rank."""
    if nranks == 1:
        kind, m, ns = "mixed", ROWS_PER_GPU, NCOLS - ROWS_PER_GPU
    else:
        kind, m, ns = "tall", ROWS_PER_GPU * nranks, NCOLS
    _, n = gen.shape(kind, m, ns)
    rb = m * rank // nranks
    re_ = m * (rank + 1) // nranks
    return kind, m, ns, n, rb, re_


def cpu_baseline(seconds_target: float = 15.0) -> dict:
    """Exact-Fraction oracle (the reference's algorithm, oracle/exact.py) on
    the first standard-rule pivot of cfg3, applied to a bounded row sample and
    scaled to the full 4097-row tableau.  Single core."""
    from oracle import exact
    kind, m, ns = "mixed", ROWS_PER_GPU, NCOLS - ROWS_PER_GPU
    T = gen.tableau(kind, m, ns, SEED)
    # selection on the full tableau (cheap: row 0 + one column)
    c = int(np.argmin(T[0, 1:]))
    col = T[1:, 1 + c]
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(col > 0, T[1:, 0] / np.where(col > 0, col, 1), np.inf)
    r = int(np.argmin(q))
    # sample: row 0, the pivot row and the first S other rows
    t0 = time.perf_counter()
    S, total, rows_done = 16, 0.0, 0
    others = [i for i in range(m) if i != r]
    while total < seconds_target and rows_done + S <= len(others):
        pick = others[rows_done:rows_done + S]
        sub = exact.from_array(np.vstack([T[:1], T[1 + r:2 + r], T[[1 + i for i in pick]]]))
        t1 = time.perf_counter()
        exact.pivot(sub, 0, c)
        total += time.perf_counter() - t1
        rows_done += S
        S = min(2 * S, 256)
        if time.perf_counter() - t0 > 3 * seconds_target:
            break
    # rows_done updated rows (+ one row 0 and one pivot row per chunk, ignored:
    # conservative) -> seconds for the m + 1 rows of a full pivot
    sec_per_pivot = total / rows_done * (m + 1)
    return {"value": 1.0 / sec_per_pivot, "unit": "pivots/s", "cores": 1, "kind": "port",
            "sample": (f"oracle/exact.py Fraction pivot #1 of cfg3 (G_mixed 4096x8192 seed 3) "
                       f"on {rows_done} of 4097 rows ({total:.1f} s), scaled to all rows; "
                       f"host has {os.cpu_count()} cores"),
            "seconds_per_pivot": sec_per_pivot}


def config_table(cpu_budget: float = 20.0) -> None:
    """--configs: BASELINE.json's small configs on GPU 0, each next to the
    reference's algorithm on one host core (the exact-Fraction restatement,
    oracle/exact.py: the cpu_baseline leg), one JSON line per config.  GPU
    legs are whole calls (upload excluded), best of 3; CPU legs run to the end
    or for cpu_budget seconds (then per pivot)."""
    from oracle import exact

    def gpu(T, job):
        best, n = None, 0
        for _ in range(3):
            e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
            e.upload(T)
            t0 = time.perf_counter()
            if job == "solve":
                e.solve()
            else:
                e.run(_lib.RULE_STANDARD, job)
            dt = time.perf_counter() - t0
            n = len(e.log())
            e.close()
            best = dt if best is None else min(best, dt)
        return best, n

    def cpu(T, job):
        F = exact.from_array(T)
        t0 = time.perf_counter()
        if job == "solve" and T.size <= 20000:
            res = exact.solve(F)
            return time.perf_counter() - t0, len(res["seq"]), True
        done, k = 0, (1 << 30 if job == "solve" else job)
        while done < k and time.perf_counter() - t0 < cpu_budget:
            p = exact.find_standard(F)
            if isinstance(p, str):
                break
            exact.pivot(F, *p)
            done += 1
        return time.perf_counter() - t0, done, False

    cases = [
        ("cfg1", "G_pos 8 x 10 + 8 slacks, Simplex.solve", gen.tableau("pos", 8, 10, 1), "solve"),
        ("cfg2", "G_pos 512 x 512 + 512 slacks (512 x 1024), Simplex.solve",
         gen.tableau("pos", 512, 512, 2), "solve"),
        ("cfg2", "G_mixed 512 x 512 + 512 slacks (512 x 1024), 256 standard pivots",
         gen.tableau("mixed", 512, 512, 2), 256),
        ("cfg5", "degenerate Klee-Minty d = 10, Simplex.solve", gen.klee_minty(10, True), "solve"),
    ]
    for cfg, what, T, job in cases:
        tg, ng = gpu(T, job)
        tc, nc, whole = cpu(T, job)
        print(json.dumps({
            "config": cfg, "workload": what, "gpu_s": tg, "gpu_pivots": ng,
            "gpu_pivots_per_s": ng / tg,
            "cpu_s": tc, "cpu_pivots": nc, "cpu_whole_run": whole,
            "cpu_pivots_per_s": nc / tc if tc > 0 else None,
            "cpu_kind": "port: oracle/exact.py (Fraction), 1 core",
        }), flush=True)


def load_traffic(path: str | None, block: int):
    """HBM bytes per sweep launch measured by scripts/hbm_traffic.py (two
    rocprofv3 --pmc passes on this workload), or None if not measured for
    this kernel and pivots-per-sweep setting."""
    if path and os.path.exists(path):
        with open(path) as f:
            d = json.load(f)
        if d.get("block") == block and d.get("kernel", "").split("<")[0] == SWEEP_KERNEL:
            return d.get("hbm_bytes_per_launch")
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4096)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--block", type=int, default=32,
                    help="pivots deferred into one sweep of the tableau (1 = eager)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01",
                                                            "hbm_traffic.json"))
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="1-GPU diagnostic: run the N-rank job's whole tableau on one GPU")
    ap.add_argument("--exchange", choices=["auto", "peer", "rccl"], default="auto",
                    help="N > 1: device-side peer exchange per pivot (auto: if its setup "
                         "check passes on every rank) or one RCCL collective per pivot")
    ap.add_argument("--no-rccl", action="store_true",
                    help="N > 1 without an RCCL communicator (peer exchange only; lets two "
                         "ranks share one GPU for testing)")
    ap.add_argument("--group-shards", type=int, default=0,
                    help="1-GPU diagnostic: the N-rank row-sharded job as N in-process shards "
                         "on one GPU (device copies instead of RCCL)")
    ap.add_argument("--profile-every", type=int, default=8,
                    help="time every k-th launch of each kernel with HIP events (1 = all)")
    ap.add_argument("--configs", action="store_true",
                    help="instead of the benchmark: cfg1/cfg2/cfg5 on GPU 0 next to the "
                         "exact-Fraction CPU path, one JSON line each")
    args = ap.parse_args()
    if args.configs:
        config_table()
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 needs torch.distributed.run with N processes")
        raise SystemExit(f"WORLD_SIZE={world} does not match --gpus {args.gpus}")

    ndev = _lib.device_count()
    device = local % ndev if ndev else local     # one rank per GPU; wraps only on smaller boxes
    dist = None
    if world > 1:
        import torch.distributed as dist  # plumbing only: uid exchange, barriers, max
        dist.init_process_group("gloo")

    nsim = args.emulate_ranks or args.group_shards or world
    kind, m, ns, n, rb, re_ = workload(nsim, rank if world > 1 else 0)
    if world == 1:
        rb, re_ = 0, m
    shards = None
    exchange = None
    if world > 1:
        import torch
        box = [None if args.no_rccl else (_lib.comm_unique_id() if rank == 0 else None)]
        dist.broadcast_object_list(box, src=0)
        eng = _lib.create_sharded(m, n, rank, world, box[0], device=device)
        assert (eng.row_begin, eng.row_count) == (rb, re_ - rb)
        # device-side exchange between the ranks; every rank must agree on it
        ok, why = 0, "not requested"
        if args.exchange != "rccl" or args.no_rccl:
            try:
                hs = [None] * world
                dist.all_gather_object(hs, eng.peer_handle())
                eng.peer_open(b"".join(hs))
                ok, why = 1, ""
            except (_lib.DeviceError, ValueError) as ex:
                why = str(ex)
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag[0]) == 1:
            exchange = "device peer stores over xGMI (one persistent selection launch per group)"
        else:
            if args.exchange == "peer" or args.no_rccl:
                raise SystemExit(f"peer exchange unavailable on some rank: {why}")
            if ok:
                eng.peer_enable(False)
            exchange = "RCCL collectives per pivot" + (f" (peer setup failed: {why})" if why else "")
    elif args.group_shards:
        shards = _lib.create_group(m, n, args.group_shards, device=device)
        eng = shards[0]
        rb, re_ = eng.row_begin, eng.row_begin + eng.row_count
    else:
        eng = _lib.Engine(m, n, device=device)
    eng.set_block(args.block)
    blk = 2048
    for e in (shards or [eng]):
        e.put_rows(0, gen.rows(kind, m, ns, SEED, 0, 1))
        a0, a1 = (e.row_begin, e.row_begin + e.row_count) if shards else (rb, re_)
        for a in range(a0, a1, blk):
            b = min(a + blk, a1)
            e.put_rows(1 + a, gen.rows(kind, m, ns, SEED, 1 + a, 1 + b))

    def barrier():
        if dist is not None:
            dist.barrier()

    def upload():
        for e in (shards or [eng]):
            e.put_rows(0, gen.rows(kind, m, ns, SEED, 0, 1))
            a0, a1 = (e.row_begin, e.row_begin + e.row_count) if shards else (rb, re_)
            for a in range(a0, a1, blk):
                e.put_rows(1 + a, gen.rows(kind, m, ns, SEED, 1 + a, 1 + min(a + blk, a1)))

    try:
        st, done = eng.run(_lib.RULE_STANDARD, args.warmup)     # ends with a stream sync
        warm_ok = 1
    except _lib.DeviceError as ex:
        if dist is None or exchange is None or not exchange.startswith("device"):
            raise
        warm_ok, why = 0, str(ex)
    if dist is not None and exchange is not None and exchange.startswith("device"):
        import torch
        flag = torch.tensor([warm_ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag[0]) == 0:
            # the peer exchange failed on some rank: every rank starts over on
            # the RCCL per-pivot path (identical results)
            if args.no_rccl:
                raise SystemExit("peer exchange failed during warmup and there is no RCCL communicator")
            eng.peer_enable(False)
            exchange = "RCCL collectives per pivot (peer exchange failed in warmup)"
            upload()
            st, done = eng.run(_lib.RULE_STANDARD, args.warmup)
    if done != args.warmup:
        raise SystemExit(f"warmup ended early: status {st} after {done} pivots")
    barrier()
    # kernel durations: HIP events recorded by every PROFILE_EVERY-th launch of
    # each kernel inside the timed run (events on every launch cost ~3 % of
    # the rate; LPGPU_BENCH_NO_EVENTS=1 times the run with none)
    if not os.environ.get("LPGPU_BENCH_NO_EVENTS"):
        eng.profile(True, every=args.profile_every)
    t0 = time.perf_counter()
    st, done = eng.run(_lib.RULE_STANDARD, args.steps)      # enqueue + final stream sync
    t1 = time.perf_counter()
    barrier()
    if done != args.steps:
        raise SystemExit(f"timed run ended early: status {st} after {done} pivots")
    upd_ms, upd_n = eng.update_time()
    sel_ms, sel_n = eng.select_time()
    eng.profile(False)
    elapsed = t1 - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed, upd_ms / max(upd_n, 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, upd_avg_ms = float(t[0]), float(t[1])
    else:
        upd_avg_ms = upd_ms / max(upd_n, 1)

    lp_pps = args.steps / elapsed
    groups = -(-args.steps // args.block)          # sweeps (and selection launches) in the run
    local_rows = (re_ - rb) + 1
    sweep_b = sweep_bytes(local_rows, n, args.block)
    achieved = sweep_b / (upd_avg_ms * 1e-3) / 1e9 if upd_avg_ms > 0 else 0.0
    traffic = load_traffic(args.traffic_json, args.block) if world == 1 else None
    out = {
        "metric": METRIC,
        "value": lp_pps * world,
        "unit": "pivots/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (counter-based splitmix64 dyadic k/64 LP, lpsol_amd.generators)",
        "config": {
            "workload": ("cfg3: 4096x8192 float64 tableau, G_mixed seed 3" if nsim == 1 else
                         f"G_tall {m}x{n} float64 tableau seed 3, {ROWS_PER_GPU} rows per GPU"
                         + (" (cfg4)" if nsim == 8 else "")
                         + (f" [diagnostic: whole tableau on 1 GPU]" if args.emulate_ranks else "")
                         + (f" [diagnostic: {nsim} in-process shards on 1 GPU]" if args.group_shards else "")),
            "m": m, "n": n, "rows_per_gpu": re_ - rb, "rule": "standard (findPivotStandard)",
            "parallelism": f"row-shard x{world}" + (f": {exchange}" if world > 1 else ""),
        },
        "lp_pivots_per_s": lp_pps,
        "pivots_per_sweep": args.block,
        # SURVEY §8(d) bytes of one unblocked pivot x pivots/s: the bandwidth an
        # immediate-update engine would need for this rate (exceeds HBM peak
        # once pivots are deferred -- that is the point of the sweep)
        "unblocked_equivalent_GBps": pivot_bytes(m, n) * lp_pps / 1e9,
        "roofline": {
            "kernel": f"{SWEEP_KERNEL} (rank-{args.block} elimination, {args.block} deferred pivots)",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic,
            "bytes_per_launch": sweep_b,
            "avg_launch_us": upd_avg_ms * 1e3,
            "time_share": upd_avg_ms * groups / (elapsed * 1e3),
            "launches_timed": upd_n,
        },
    }
    if sel_n:
        # the other kernel of the path: one persistent launch selects a group of
        # pivots; its time is the chain of per-pivot summary exchanges and
        # dependent loads (latency), not bytes
        out["selection"] = {
            "kernel": "k_group (persistent pivot selection, latency-bound)",
            "avg_launch_us": 1e3 * sel_ms / sel_n,
            "pivots_per_launch": args.block,
            "us_per_pivot": 1e3 * sel_ms / sel_n / args.block,
            "time_share": sel_ms / max(sel_n, 1) * groups / (elapsed * 1e3),
            "launches_timed": sel_n,
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
