#!/usr/bin/env python3
"""Benchmark of the dense simplex pivot hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg4|cfg3]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A pivot is the reference's ``findPivotStandard(True)``: entering-column scan,
min-ratio test and the rank-1 elimination of the whole float64 tableau
(``lpsol/simplex.py:251-284``, ``lpsol/tableau.py:295-308``).  The engine
selects ``block`` pivots (default: the engine's automatic depth, 64 on cfg3
and cfg4) from current values and then applies
their eliminations to the stored tableau in ONE pass (bit-identical to
immediate updates).  One STEP is one such group: ``block`` pivots selected
plus one elimination pass over the whole tableau, so ``--steps K`` times
K x block pivots.  ``value`` is LP pivots per second of the whole job.

Workload (BASELINE.json config 4): cfg4, the 32768 x 8192
G_tall tableau (seed 3), STRONG scaling -- the same tableau at every N, its
constraint rows split into N contiguous row blocks, one per GPU (row 0
replicated).  At N = 1 the line also carries ``cfg3``: the 4096 x 8192
G_mixed tableau (config 3, the north star's 60 %-of-HBM-roofline case)
measured the same way.  ``--workload cfg3`` makes cfg3 the main workload.

Inputs are resident in HBM before the timed region.  Before the W warmup
steps, a device warm-up (``--device-warmup-ms``, 150 ms) runs the same
workload's groups on a SCRATCH copy of the tableau: after the idle gap of the
upload the MI355X runs the sweep 10-15 % slower for ~30 launches whatever the
data (scripts/ramp_probe2.py); the benchmarked engine still starts its warmup
steps from the initial tableau.  Every 8th sweep and selection launch (every
4th below 64 steps) inside the timed region records a pair of HIP events at the
kernel's start and end (hipExtLaunchKernelGGL on the engine's stream); the
roofline's achieved bandwidth is the sweep's algorithmic bytes over that
kernel time.
"""
from __future__ import annotations

import argparse
import hashlib
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
F64_PEAK_TFLOPS = 78.6      # float64 vector spec (half the guide's 157.3 TF FP32 vector)
SWEEP_KERNEL = "k_sweep"          # every sweep kernel's name starts so (the traffic stamp names which)
SEED = 3
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r06", "hbm_traffic.json")

# name -> (generator kind, m, ns, description)
WORKLOADS = {
    "cfg4": ("tall", 32768, 8192, "cfg4: 32768x8192 float64 tableau, G_tall seed 3"),
    "cfg3": ("mixed", 4096, 4096, "cfg3: 4096x8192 float64 tableau, G_mixed seed 3"),
    # rehearsal of one rank of the 8-GPU cfg4 job (4096 rows per rank, the
    # one-XCD cross-rank kernel k_sel<XR>, G = 64) with two ranks on ONE GPU:
    # 6144 columns, so both ranks' launches are resident at once
    "cfg4r8": ("tall", 8192, 6144, "8192x6144 G_tall seed 3: two 4096-row ranks (the 8-GPU cfg4 rank geometry)"),
    # one such rank's shape alone on one GPU (no cross-rank exchange): the
    # baseline the rehearsal's XR overhead is measured against
    "cfg4r8one": ("tall", 4096, 6144, "4096x6144 G_tall seed 3: one cfg4r8 rank's shape on one GPU"),
    # one rank's rows of the 4- and 2-GPU cfg4 job alone on one GPU (8192 /
    # 16384 rows of the 8192-column tableau; no cross-rank exchange)
    "cfg4r4one": ("tall", 8192, 8192, "8192x8192 G_tall seed 3: one 4-GPU cfg4 rank's rows on one GPU"),
    "cfg4r2one": ("tall", 16384, 8192, "16384x8192 G_tall seed 3: one 2-GPU cfg4 rank's rows on one GPU"),
}


def pivot_bytes(m: int, n: int) -> int:
    """Algorithmic bytes of one unblocked pivot: read+write
    the whole tableau, the row-0 scan and the column+b ratio gather."""
    return 8 * (2 * (m + 1) * (n + 1) + (n + 1) + 2 * (m + 1))


def sweep_bytes(rows: int, n: int, block: int) -> int:
    """Algorithmic bytes of one sweep (k_sweep_st) launch on `rows` local rows
    applying `block` deferred pivots: read and write every row once, read the
    group's pivot rows P and multiplier columns M once."""
    return 8 * (2 * rows * (n + 1) + block * (n + 1) + block * rows)


def workload(name: str, nranks: int, rank: int):
    """(kind, m, ns, n, first row, end row) of this rank's row block: the
    engine's split (lp_create_sharded) -- contiguous blocks, m * r // N."""
    kind, m, ns, _ = WORKLOADS[name]
    _, n = gen.shape(kind, m, ns)
    return kind, m, ns, n, m * rank // nranks, m * (rank + 1) // nranks


SRC_FILES = [os.path.join(ROOT, "linear-program-solver_amd", "csrc", f)
             for f in ("kernels.hip", "select.hip", "lpgpu.cpp", "engine.h", "device.h", "Makefile")] + [
    os.path.join(ROOT, "include", "lpgpu.h"), os.path.join(ROOT, "include", "lpgpu_diag.h")]


def lib_digest() -> str:
    """sha256 of the loaded library file (reported; hipcc output is not
    byte-reproducible, so the traffic stamp uses src_digest)"""
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def src_digest() -> str:
    """sha256 over the library's sources and build flags: the identity of a
    build for the PMC traffic stamp (the same sources give the same kernels)"""
    h = hashlib.sha256()
    for p in SRC_FILES:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def sweep_kernel(block: int) -> str:
    """the sweep kernel the engine launches for `block` pivots per sweep
    (kernels.hip launch_sweep: k_sweep_dp2 up to 48, k_sweep_rl at 64)"""
    return "k_sweep_dp2" if block <= 48 else "k_sweep_rl"


def load_traffic(path: str | None, block: int, workload_name: str, digest: str):
    """HBM bytes per sweep launch measured by scripts/hbm_traffic.py (two
    rocprofv3 --pmc passes of this bench), if measured on this very library
    build (sha256 stamp), workload and pivots per sweep; else None."""
    if path and os.path.exists(path):
        with open(path) as f:
            d = json.load(f)
        for e in d.get("entries", [d]):
            if (e.get("block") == block and e.get("workload") == workload_name
                    and e.get("src_sha256") == digest
                    and SWEEP_KERNEL in e.get("kernel", "")):
                return e.get("hbm_bytes_per_launch")
    return None


def first_pivots(name: str, k: int, device: int) -> list[tuple[int, int]]:
    """the workload's first k standard-rule pivots (global row, column), from
    the engine (bit-identical to the f64 oracle's, tests/test_gpu_r3.py)"""
    kind, m, ns, n, _, _ = workload(name, 1, 0)
    e = _lib.Engine(m, n, device=device)
    upload([e], kind, m, ns, [(0, m)])
    e.run(_lib.RULE_STANDARD, k)
    seq = [(int(r), int(c)) for r, c in e.log()]
    e.close()
    return seq


def _time_dense_pivot(sub, r_local: int, c: int, rows_of, nrows: int, seconds_target: float):
    """seconds per row of oracle/exact.py's dense pivot (the reference's row
    operations over every column, tableau.py:254-308) on growing slices of
    the sample rows (rows_of(i0, i1) -> exact rows); returns (seconds per
    row, rows timed, seconds)"""
    from oracle import exact
    total, done, S, i0 = 0.0, 0, 8, 0
    t0 = time.perf_counter()
    while total < seconds_target and i0 < nrows:
        blk = rows_of(i0, min(i0 + S, nrows))
        T = [list(sub[0]), list(sub[r_local])] + [list(r) for r in blk]
        t1 = time.perf_counter()
        exact.pivot_dense(T, 0, c)
        total += time.perf_counter() - t1
        done += len(blk)
        i0 += S
        S = min(2 * S, 256)
        if time.perf_counter() - t0 > 3 * seconds_target:
            break
    return total / max(done, 1), done, total


def cpu_baseline(name: str, seconds_target: float = 15.0, seq=None, k_mid: int = 16) -> dict:
    """The reference's algorithm on one host core: oracle/exact.py's
    Fraction restatement of Tableau.pivot in the reference's own order of
    operations (rowDiv, rowAddToObj, then rowSub over EVERY column of every
    other row, tableau.py:254-308), timed on a bounded sample of rows and
    scaled to all rows, at two points of the run: pivot #1 (dyadic inputs,
    the smallest denominators) and pivot #(k_mid + 1), whose exact state is
    obtained by replaying the first k_mid pivots (``seq``, the engine's) on
    row 0, the pivot rows and the sample rows -- the Fractions' denominators
    grow with every pivot, and so does the reference's cost."""
    from oracle import exact
    kind, m, ns, _ = WORKLOADS[name]
    budget = seconds_target / (2 if seq else 1)
    # pivot #1: its entering column and leaving row from the whole column (numpy)
    T0 = gen.rows(kind, m, ns, SEED, 0, 1)
    c = int(np.argmin(T0[0, 1:]))
    col = np.empty(m)
    b = np.empty(m)
    for a in range(0, m, 4096):
        R = gen.rows(kind, m, ns, SEED, 1 + a, 1 + min(a + 4096, m))
        col[a:a + len(R)] = R[:, 1 + c]
        b[a:a + len(R)] = R[:, 0]
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(col > 0, b / np.where(col > 0, col, 1), np.inf)
    r = int(np.argmin(q))
    picks = [i for i in range(0, min(m, 4096)) if i != r]
    sub = exact.from_array(np.vstack([T0, gen.rows(kind, m, ns, SEED, 1 + r, 2 + r)]))

    def rows1(i0, i1):
        return exact.from_array(np.vstack([gen.rows(kind, m, ns, SEED, 1 + i, 2 + i) for i in picks[i0:i1]]))
    sec_row1, done1, t1 = _time_dense_pivot(sub, 1, c, rows1, len(picks), budget)
    sec1 = sec_row1 * (m + 1)
    out = {"value": 1.0 / sec1, "unit": "pivots/s", "cores": 1, "kind": "port",
           "sample": (f"oracle/exact.py pivot_dense (the reference's Fraction row operations, "
                      f"every column) on pivot #1 of {name}, {done1} of {m + 1} rows "
                      f"({t1:.1f} s on one core), scaled to all rows; host has "
                      f"{os.cpu_count()} cores"),
           "seconds_per_pivot": sec1, "seconds_per_pivot_at_1": sec1}
    if seq and len(seq) > k_mid:
        # exact state after k_mid pivots of row 0, the pivot rows and a sample
        prows = sorted({rr for rr, _ in seq[:k_mid + 1]})
        sample = [i for i in range(0, m, max(1, m // 48)) if i not in set(prows)][:48]
        keep = prows + sample
        A = np.vstack([T0] + [gen.rows(kind, m, ns, SEED, 1 + i, 2 + i) for i in keep])
        X = exact.from_array(A)
        where = {g: 1 + k for k, g in enumerate(keep)}
        t0 = time.perf_counter()
        for rr, cc in seq[:k_mid]:
            exact.pivot(X, where[rr] - 1, cc)
        replay = time.perf_counter() - t0
        rk, ck = seq[k_mid]
        rows_mid = [X[where[i]] for i in sample if i != rk]
        sec_row, done, tk = _time_dense_pivot(X, where[rk], ck, lambda i0, i1: rows_mid[i0:i1], len(rows_mid),
                                              budget)
        secm = sec_row * (m + 1)
        out.update({
            "value": 1.0 / secm, "seconds_per_pivot": secm,
            "seconds_per_pivot_at_%d" % (k_mid + 1): secm,
            "sample": out["sample"] + (
                f"; pivot #{k_mid + 1} (the reported value): the first {k_mid} pivots replayed "
                f"exactly on row 0, the pivot rows and {len(sample)} sample rows ({replay:.1f} s, "
                f"not counted), then the same dense pivot on {done} of them ({tk:.1f} s), scaled "
                f"to all rows -- still a lower bound, denominators keep growing"),
        })
    return out


def config_table(cpu_budget: float = 20.0) -> None:
    """--configs: BASELINE.json's small configs on GPU 0, each next to the
    reference's algorithm on one host core (the exact-Fraction restatement,
    oracle/exact.py), one JSON line per config.  GPU legs are whole calls
    (upload excluded), best of 3; CPU legs run to the end or for cpu_budget
    seconds (then per pivot)."""
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
            exact.pivot_dense(F, *p)
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
            "cpu_kind": "port: oracle/exact.py (Fraction, the reference's row operations), 1 core",
        }), flush=True)


def upload(engines, kind, m, ns, spans, blk=2048, heaters=None):
    """rows of the workload into each engine (row 0 + its row block); a
    heater engine beside one (device_warmup) gets the same rows, locally
    numbered"""
    heaters = heaters or [None] * len(engines)
    for e, h, (a0, a1) in zip(engines, heaters, spans):
        R = gen.rows(kind, m, ns, SEED, 0, 1)
        e.put_rows(0, R)
        if h is not None:
            h.put_rows(0, R)
        for a in range(a0, a1, blk):
            R = gen.rows(kind, m, ns, SEED, 1 + a, 1 + min(a + blk, a1))
            e.put_rows(1 + a, R)
            if h is not None:
                h.put_rows(1 + a - a0, R)


def device_warmup(heater, block: int, ms: float) -> dict:
    """Keep the GPU busy for `ms` right before the warmup steps: groups of
    the same workload on a SCRATCH copy of the rank's tableau (`heater`), so
    the benchmarked engine still starts its W warmup steps from the initial
    tableau.  Why: after an idle gap (the upload) the MI355X runs the sweep
    10-15 % slower for its first ~30 launches, whatever the data -- the same
    tableau re-uploaded ramps again, the initial tableau right after another
    engine's groups does not (scripts/ramp_probe2.py, profiles/r04/README.md)."""
    if heater is None or ms <= 0:
        return {"ms": 0.0, "groups": 0}
    t0 = time.perf_counter()
    groups = 0
    while (time.perf_counter() - t0) * 1e3 < ms and groups < 4096:
        st, done = heater.run(_lib.RULE_STANDARD, 8 * block)
        groups += done // block
        if done < 8 * block:
            break                                # the scratch LP ended: warm enough or not, stop
    return {"ms": (time.perf_counter() - t0) * 1e3, "groups": groups}


def accounting(steps: int, block: int, elapsed: float, sweep_avg_ms: float, sel_avg_ms: float,
               local_rows: int, n: int) -> dict:
    """the per-launch figures of a timed run of `steps` groups of `block`
    pivots: every sweep and selection launch carries exactly `block` pivots"""
    pivots = steps * block
    sweep_b = sweep_bytes(local_rows, n, block)
    achieved = sweep_b / (sweep_avg_ms * 1e-3) / 1e9 if sweep_avg_ms > 0 else 0.0
    fma = local_rows * (n + 1) * block           # one float64 FMA per element and pivot
    return {
        "sweep_fma_per_launch": fma,
        "sweep_f64_TFLOPs": 2.0 * fma / (sweep_avg_ms * 1e-3) / 1e12 if sweep_avg_ms > 0 else 0.0,
        "pivots": pivots,
        "pivots_per_s": pivots / elapsed,
        "ms_per_step": 1e3 * elapsed / steps,
        "sweep_bytes_per_launch": sweep_b,
        "achieved_GBps": achieved,
        "sweep_time_share": sweep_avg_ms * steps / (elapsed * 1e3),
        "selection_us_per_pivot": 1e3 * sel_avg_ms / block if sel_avg_ms > 0 else None,
        "selection_time_share": sel_avg_ms * steps / (elapsed * 1e3) if sel_avg_ms > 0 else None,
    }


def dump_stamps(eng, geo: dict, block: int, rank: int) -> None:
    """diagnostic builds only (LPGPU_STAMPS=1 with variants/stamps.so): the
    last selection launch's phase clocks of this rank into
    $LPGPU_STAMPS_DUMP/stamps_rank<r>.npz (scripts/sel_clocks.py --file)"""
    d = os.environ.get("LPGPU_STAMPS_DUMP")
    if not d or os.environ.get("LPGPU_STAMPS") != "1":
        return
    import ctypes
    buf = (ctypes.c_longlong * (256 * 64 * 4))()
    if eng.lib.lpdiag_bstamps(eng.h, buf) != 0:
        return
    os.makedirs(d, exist_ok=True)
    np.savez(os.path.join(d, f"stamps_rank{rank}.npz"), buf=np.array(buf, dtype=np.int64),
             blocks=int(geo["blocks"]), block=int(block),
             geometry=np.array([geo.get(k, 0) for k in ("blocks", "ipl", "xcd_shards")]))


def profile_every_for(rows: int, n: int, steps: int, requested: int) -> int:
    """launches timed with HIP events: every one where a sweep is long (a
    local tableau beyond 1 GB: cfg4 on one GPU, ~800 us per sweep -- an
    event pair's ~2 us is 0.3 %, and sampling every 4th read a biased subset:
    VERDICT r5), else every 4th (every 8th from 64 steps; every launch costs
    cfg3's 0.4 ms groups ~2 %: 156.3k against 159.4k pivots/s)"""
    if requested > 0:
        return requested
    if 8.0 * rows * (n + 1) > 1e9:
        return 1
    return 4 if steps < 64 else 8


def sweep_clock_summary(eng, steps: int) -> dict:
    """the shader clock of the timed sweeps (k_sweep_rl's block 0 records
    cycles and 100 MHz ticks of its pass, Args::sweep_clk): with the event
    times it tells a clock effect (the same cycles at a lower clock) from a
    memory one (more cycles at the same clock)"""
    try:
        c = eng.sweep_clocks(steps)
    except Exception as ex:                      # noqa: BLE001 -- a diagnostic only
        return {"error": str(ex)}
    c = c[-steps:]
    if len(c) == 0:
        return {"launches": 0}
    ghz = c[:, 1] / (c[:, 2] / 1e8) / 1e9
    us = c[:, 2] / 100.0
    out = {"launches": int(len(c)), "ghz_mean": float(ghz.mean()), "ghz_min": float(ghz.min()),
           "ghz_max": float(ghz.max()), "block0_us_mean": float(us.mean()),
           "kcycles_mean": float(c[:, 1].mean() / 1e3)}
    if len(c) <= 64:
        out["ghz_per_launch"] = [round(float(g), 3) for g in ghz]
    return out


def timed_run(eng, steps: int, warmup: int, block: int, barrier, every: int, heater=None, heat_ms: float = 0.0):
    """device warm-up on the heater (untimed, another tableau; closed right
    after it), warmup groups, then exactly `steps` timed groups bracketed by the barrier + stream sync
    (lp_run ends with a stream sync)."""
    heat = device_warmup(heater, block, heat_ms)
    if heater is not None:
        heater.close()                           # its buffers leave before the timed groups
    barrier()                                    # ranks enter the warmup together (the exchange needs all)
    st, done = eng.run(_lib.RULE_STANDARD, warmup * block)
    if done != warmup * block:
        raise SystemExit(f"warmup ended early: status {st} after {done} pivots")
    barrier()
    if not os.environ.get("LPGPU_BENCH_NO_EVENTS"):
        eng.profile(True, every=every)
    t0 = time.perf_counter()
    st, done = eng.run(_lib.RULE_STANDARD, steps * block)
    t1 = time.perf_counter()
    barrier()
    if done != steps * block:
        raise SystemExit(f"timed run ended early: status {st} after {done} pivots")
    upd_ms, upd_n = eng.update_time()
    sel_ms, sel_n = eng.select_time()
    eng.profile(False)
    heat["sweep_clock"] = sweep_clock_summary(eng, steps)
    return t1 - t0, upd_ms / max(upd_n, 1), (sel_ms / sel_n if sel_n else 0.0), upd_n, sel_n, heat


def single_gpu_leg(name: str, steps: int, warmup: int, block: int, every: int, device: int,
                   shards: int = 0, heat_ms: float = 0.0) -> dict:
    """one workload on one GPU (or as `shards` in-process row shards of it,
    a diagnostic): timing, roofline and selection figures"""
    kind, m, ns, n, _, _ = workload(name, 1, 0)
    if shards:
        engs = _lib.create_group(m, n, shards, device=device)
        spans = [(e.row_begin, e.row_begin + e.row_count) for e in engs]
    else:
        engs = [_lib.Engine(m, n, device=device)]
        spans = [(0, m)]
    for e in engs:
        e.set_block(block)
    block = engs[0].get_block()          # the auto choice (--block 0) resolved
    heater = None
    if heat_ms > 0 and not shards:
        heater = _lib.Engine(m, n, device=device)
        heater.set_block(block)
    upload(engs, kind, m, ns, spans, heaters=[heater] if heater else None)
    xw0 = engs[0].xwait()
    every = profile_every_for(spans[0][1] - spans[0][0] + 1, n, steps, every)
    elapsed, sw_ms, sel_ms, sw_n, sel_n, heat = timed_run(engs[0], steps, warmup, block, lambda: None, every,
                                                          heater, heat_ms)
    clock = heat.pop("sweep_clock", None)
    xw1 = engs[0].xwait()
    path, fallbacks = engs[0].exchange_path()
    geo = engs[0].geometry()
    acc = accounting(steps, block, elapsed, sw_ms, sel_ms, spans[0][1] - spans[0][0] + 1, n)
    acc["selection_kernel"] = geo["kernel"]
    if geo.get("xcd_shards"):
        # k_sel as one row shard per XCD: the shards' exchange per pivot
        # (shard 0's block 0: its summary published -> every shard's seen)
        acc["selection_kernel"] += f" as {geo['xcd_shards']} XCD row shards"
        acc["xcd_hop_us_per_pivot"] = (1e6 * (xw1[0] - xw0[0]) / (xw1[1] - xw0[1])
                                       if xw1[1] > xw0[1] else 0.0)
    acc.update(block=block, path=_lib.PATH_NAMES.get(path, path), fallbacks=fallbacks, device_warmup=heat,
               sweep_avg_us=sw_ms * 1e3, sweep_launches_timed=sw_n, selection_launches_timed=sel_n,
               selection_avg_launch_us=sel_ms * 1e3, sweep_clock=clock, profile_every=every)
    for e in reversed(engs):
        e.close()
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128,
                    help="timed steps; one step = one group of --block pivots + one sweep")
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--block", type=int, default=0,
                    help="pivots deferred into one sweep of the tableau (1 = eager, 0 = the "
                         "engine's auto choice)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg4")
    ap.add_argument("--no-cfg3", action="store_true", help="N = 1: skip the cfg3 leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--traffic-json", default=TRAFFIC_JSON)
    ap.add_argument("--exchange", choices=["auto", "peer", "rccl"], default="auto",
                    help="N > 1: device-side peer exchange per pivot (auto: if its setup "
                         "check passes on every rank) or one RCCL collective per pivot")
    ap.add_argument("--no-rccl", action="store_true",
                    help="N > 1 without an RCCL communicator (peer exchange and the host "
                         "all-gather; lets ranks share one GPU for testing)")
    ap.add_argument("--group-shards", type=int, default=0,
                    help="1-GPU diagnostic: the workload as S in-process row shards on one GPU")
    ap.add_argument("--profile-every", type=int, default=0,
                    help="time every k-th launch of each kernel with HIP events (1 = all; default: "
                         "every 4th for runs under 64 steps, else every 8th)")
    ap.add_argument("--device-warmup-ms", type=float, default=150.0,
                    help="before the W warmup steps, keep the GPU busy this long with the same "
                         "workload on a scratch copy of the tableau (0: off; see device_warmup)")
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
    B = args.block
    digest = src_digest()
    kind, m, ns, n, rb, re_ = workload(args.workload, world, rank)
    out = {"metric": METRIC, "unit": "pivots/s"}

    if world == 1:
        leg = single_gpu_leg(args.workload, args.steps, args.warmup, B, args.profile_every, device,
                             args.group_shards, args.device_warmup_ms)
        elapsed_pps, devices = leg["pivots_per_s"], 1
        parallelism = (f"1 GPU ({leg['path']})" if not args.group_shards else
                       f"diagnostic: {args.group_shards} in-process row shards on 1 GPU ({leg['path']})")
        sweep_ms, local_rows = leg["sweep_avg_us"] * 1e-3, (m // (args.group_shards or 1)) + 1
        acc = leg
        B = leg["block"]
    else:
        import torch
        import torch.distributed as dist  # plumbing only: uid exchange, barriers, max
        dist.init_process_group("gloo")
        box = [None if args.no_rccl else (_lib.comm_unique_id() if rank == 0 else None)]
        dist.broadcast_object_list(box, src=0)
        eng = _lib.create_sharded(m, n, rank, world, box[0], device=device)
        assert (eng.row_begin, eng.row_count) == (rb, re_ - rb)
        if args.no_rccl:
            eng.set_host_allgather(_lib.gloo_allgather())
        ok, why = 0, "not requested (--exchange rccl)"
        if args.exchange != "rccl" or args.no_rccl:
            try:
                hs = [None] * world
                dist.all_gather_object(hs, eng.peer_handle())
                eng.peer_open(b"".join(hs))
                ok, why = 1, ""
            except (_lib.DeviceError, ValueError) as ex:
                why = f"peer_open failed: {ex}"
        # every rank's verdict on the device-side exchange (a job leaves the
        # peer path if any rank could not open it: one line says which and why)
        verdicts = [None] * world
        dist.all_gather_object(verdicts, (rank, ok, why))
        peer_fail = [(r, w) for r, o, w in verdicts if not o]
        if peer_fail:
            if args.exchange == "peer":
                raise SystemExit(f"peer exchange unavailable: rank {peer_fail[0][0]}: {peer_fail[0][1]}")
            if rank == 0:
                print(f"bench: leaving the peer exchange (one RCCL collective per pivot instead): "
                      f"rank {peer_fail[0][0]}: {peer_fail[0][1]}", file=sys.stderr, flush=True)
            if ok:
                eng.peer_enable(False)
        eng.set_block(B)
        B = eng.get_block()
        # the device warm-up: the rank's rows as a plain one-GPU tableau (no
        # exchange; load only) -- only when every rank has a GPU of its own
        # (co-located ranks' persistent selections would contend for one XCD)
        gpus = [None] * world
        dist.all_gather_object(gpus, (os.uname().nodename, device))
        heater = None
        # (LPGPU_BENCH_FORCE_HEAT=1: warm up anyway -- rehearses this path with
        # co-located ranks on a workload whose selections fit one XCD together)
        if args.device_warmup_ms > 0 and (len(set(gpus)) == world or os.environ.get("LPGPU_BENCH_FORCE_HEAT") == "1"):
            heater = _lib.Engine(re_ - rb, n, device=device)
            heater.set_block(B)
        upload([eng], kind, m, ns, [(rb, re_)], heaters=[heater])
        xw0 = eng.xwait()
        every = profile_every_for(re_ - rb + 1, n, args.steps, args.profile_every)
        elapsed, sw_ms, sel_ms, sw_n, sel_n, heat = timed_run(eng, args.steps, args.warmup, B, dist.barrier,
                                                              every, heater, args.device_warmup_ms)
        clock = heat.pop("sweep_clock", None)
        if heater is None and args.device_warmup_ms > 0:
            heat["skipped"] = "ranks share a GPU"
        xw1 = eng.xwait()
        # the cross-rank hop per pivot (block 0: its summary sent -> the
        # winner's pivot row held), over the timed pivots
        hop_us = 1e6 * (xw1[0] - xw0[0]) / (xw1[1] - xw0[1]) if xw1[1] > xw0[1] else 0.0
        t = torch.tensor([elapsed, sw_ms, sel_ms, hop_us], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, sw_ms, sel_ms, hop_us = float(t[0]), float(t[1]), float(t[2]), float(t[3])
        # distinct GPUs of the job (ranks wrap onto fewer GPUs on a small box)
        # and the selection kernel every rank actually ran (its last launch)
        path, fallbacks = eng.exchange_path()
        geo = eng.geometry()
        dump_stamps(eng, geo, B, rank)
        kern = geo["kernel"] + (f" as {geo['xcd_shards']} XCD shards" if geo.get("xcd_shards") else
                                " on one XCD" if geo.get("on_one_xcd") else "")
        ids = [None] * world
        dist.all_gather_object(ids, (os.uname().nodename, device, rank, kern, _lib.PATH_NAMES.get(path, path),
                                     fallbacks))
        devices = len(set((h, d) for h, d, *_ in ids))
        share = "" if devices == world else f", {world} ranks sharing {devices} GPU(s)"
        parallelism = (f"row-shard x{world} over {'xGMI' if devices == world else 'one GPU'}: "
                       f"{_lib.PATH_NAMES.get(path, path)}{share}")
        local_rows = (re_ - rb) + 1          # the largest block: ranks differ by <= 1 row
        sweep_ms = sw_ms
        acc = accounting(args.steps, B, elapsed, sw_ms, sel_ms, local_rows, n)
        acc.update(fallbacks=fallbacks, sweep_launches_timed=sw_n, selection_launches_timed=sel_n, device_warmup=heat,
                   selection_avg_launch_us=sel_ms * 1e3, selection_kernel=kern, sweep_clock=clock,
                   profile_every=every,
                   xrank_hop_us_per_pivot=hop_us,
                   ranks=[{"rank": r, "host": h, "device": d, "selection_kernel": k, "path": pth, "fallbacks": fb}
                          for h, d, r, k, pth, fb in ids],
                   peer_exchange={"ok": not peer_fail,
                                  "reason": (f"rank {peer_fail[0][0]}: {peer_fail[0][1]}" if peer_fail else "")})
        elapsed_pps = acc["pivots_per_s"]

    desc = WORKLOADS[args.workload][3]
    traffic = (load_traffic(args.traffic_json, B, args.workload, digest)
               if world == 1 and not args.group_shards else None)
    out.update({
        "value": elapsed_pps,
        "n_gpus": devices,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": acc["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (counter-based splitmix64 dyadic k/64 LP, lpsol_amd.generators)",
        "config": {
            "workload": desc, "m": m, "n": n, "rows_per_gpu": re_ - rb if world > 1 else m,
            "rule": "standard (findPivotStandard)",
            "step": f"{B} pivots selected + one elimination sweep of the tableau",
            "parallelism": parallelism,
        },
        "pivots_per_step": B,
        "pivots_timed": acc["pivots"],
        "us_per_pivot": 1e6 / elapsed_pps,
        "roofline": {
            "kernel": f"{sweep_kernel(B)} (rank-{B} elimination of {local_rows} local rows)",
            "bound": "hbm",
            "achieved": acc["achieved_GBps"],
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": acc["achieved_GBps"] / HBM_PEAK_GBPS,
            # the whole pivot: a GPU's sweep bytes per step over the whole
            # step (selection included) against the same peak
            "step_frac": acc["sweep_bytes_per_launch"] / (acc["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            "traffic": traffic,
            "traffic_note": ("PMC FETCH_SIZE x2 + WRITE_SIZE per launch, measured on a build of these "
                             f"sources ({os.path.relpath(args.traffic_json, ROOT)}, src_sha256)" if traffic else
                             "not measured on a build of these sources / this workload"),
            "bytes_per_launch": acc["sweep_bytes_per_launch"],
            "avg_launch_us": sweep_ms * 1e3,
            "time_share": acc["sweep_time_share"],
            # the sweep's arithmetic beside its bytes: B FMAs per element put it
            # near the float64 ridge (78.6 TF vector spec / 8 TB/s = 9.8 flop/B)
            "f64_fma_per_launch": acc["sweep_fma_per_launch"],
            "f64_TFLOPs": acc["sweep_f64_TFLOPs"],
            "f64_peak_TFLOPs": F64_PEAK_TFLOPS,
            # launches timed with events (every one at cfg4) and the shader
            # clock over them (block 0's cycles / 100 MHz ticks per launch)
            "launches_timed": acc["sweep_launches_timed"],
            "timed_every": acc.get("profile_every"),
            "shader_clock": acc.get("sweep_clock"),
        },
        "selection": {
            "kernel": f"{acc.get('selection_kernel', 'k_group')} (persistent pivot selection, latency-bound)",
            "us_per_pivot": acc["selection_us_per_pivot"],
            "avg_launch_us": acc["selection_avg_launch_us"],
            "pivots_per_launch": B,
            "time_share": acc["selection_time_share"],
            **({"xrank_hop_us_per_pivot": acc["xrank_hop_us_per_pivot"]} if world > 1 else {}),
            **({"xcd_hop_us_per_pivot": acc["xcd_hop_us_per_pivot"]} if "xcd_hop_us_per_pivot" in acc else {}),
        },
        "fallbacks": acc["fallbacks"],
        # untimed, before the W warmup steps: the same workload's groups on a
        # scratch copy of the tableau (device_warmup; --device-warmup-ms 0: off)
        "device_warmup": {**acc["device_warmup"], "on": "scratch copy of the workload's tableau"},
        **({"ranks": acc["ranks"], "peer_exchange": acc["peer_exchange"]} if world > 1 else {}),
        "src_sha256": digest,
        "lib_sha256": lib_digest(),
    })
    if world == 1 and args.workload != "cfg3" and not args.no_cfg3 and not args.group_shards:
        c3 = single_gpu_leg("cfg3", args.steps, args.warmup, args.block, args.profile_every, device,
                            heat_ms=args.device_warmup_ms)
        out["cfg3"] = {
            "workload": WORKLOADS["cfg3"][3], "value": c3["pivots_per_s"], "unit": "pivots/s",
            "ms_per_step": c3["ms_per_step"], "us_per_pivot": 1e6 / c3["pivots_per_s"],
            "pivots_per_step": c3["block"],
            "roofline": {"kernel": f"{sweep_kernel(c3['block'])} (rank-{c3['block']} elimination of 4097 rows)",
                         "bound": "hbm",
                         "achieved": c3["achieved_GBps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": c3["achieved_GBps"] / HBM_PEAK_GBPS,
                         "step_frac": c3["sweep_bytes_per_launch"] / (c3["ms_per_step"] * 1e-3) / 1e9
                         / HBM_PEAK_GBPS,
                         "traffic": load_traffic(args.traffic_json, c3["block"], "cfg3", digest),
                         "bytes_per_launch": c3["sweep_bytes_per_launch"],
                         "avg_launch_us": c3["sweep_avg_us"], "time_share": c3["sweep_time_share"],
                         "launches_timed": c3["sweep_launches_timed"], "timed_every": c3["profile_every"],
                         "shader_clock": c3["sweep_clock"]},
            "selection": {"kernel": c3["selection_kernel"], "us_per_pivot": c3["selection_us_per_pivot"],
                          "time_share": c3["selection_time_share"]},
            "path": c3["path"], "fallbacks": c3["fallbacks"],
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        seq = first_pivots(args.workload, 17, device)
        out["cpu_baseline"] = cpu_baseline(args.workload, args.cpu_seconds, seq, 16)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        eng.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
