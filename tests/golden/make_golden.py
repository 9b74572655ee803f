"""Capture golden vectors from the REFERENCE (tkoz0/linear-program-solver,
package ``lpsol``) in the build container.

Run from the repo root (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--big]
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --extra   # r2.json only
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --headline 10   # r3.json only
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --headline-prefix 64   # r4.json, checkpointed
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --headline-prefix 80 --out r5.json
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --headline-prefix 16 --workload cfg4 --out r6.json

It imports the reference, drives its own ``Tableau``/``Simplex`` on inputs
from this repo's generator (``lpsol_amd.generators``) or on hand-built LPs,
and records what the reference did: every ``Simplex._pivot(r, c)`` call in
order, how many were standard-rule pivots, the final exact objective as
``p/q`` and the final basic sequence.  Nothing of the reference's source is
stored -- only inputs (as generator specs + sha256, or exact values for
hand-built LPs) and outputs.  ``--big`` adds the slow cfg2 fixtures
(512 x 1024, about 1-3 minutes each on one core).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from fractions import Fraction

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

from lpsol import Simplex, Tableau  # noqa: E402  (the reference)
from lpsol_amd import generators as gen  # noqa: E402
from oracle import exact  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def fs(x: Fraction) -> str:
    return f"{x.numerator}/{x.denominator}"


# ---------------------------------------------------------------- reference io

def ref_tableau_from_rows(rows) -> Tableau:
    """rows: exact Fractions in the engine layout (row 0 = [_z, c...])."""
    m, n = len(rows) - 1, len(rows[0]) - 1
    t = Tableau(m, n)
    t.setZ(-rows[0][0])                     # setZ stores -z (tableau.py:128-130)
    t.setC(rows[0][1:])
    t.setB([rows[i][0] for i in range(1, m + 1)])
    t.setA([rows[i][1:] for i in range(1, m + 1)])
    t.setVarNames([f"x{j}" for j in range(n)])
    return t


def ref_rows(t: Tableau):
    m, n = t.getTableauSize()
    rows = [[-t.getZ()] + list(t.getC())]
    for i in range(m):
        rows.append([t.getBi(i)] + list(t.getA()[i]))
    return rows


class LoggingSimplex(Simplex):
    """Reference Simplex that records each pivot and which rule chose it."""

    def __init__(self, tab, log):
        self._log = log
        self._rule = "init"
        super().__init__(tab)

    def _pivot(self, r, c):
        self._log.append((r, c, self._rule))
        super()._pivot(r, c)

    def findPivotStandard(self, do_pivot=False):
        self._rule = "std"
        return super().findPivotStandard(do_pivot)

    def findPivotMinIndex(self, do_pivot=False):
        self._rule = "min"
        return super().findPivotMinIndex(do_pivot)


def bare_simplex(tab, log):
    """Simplex without phase 1 (harness-only bypass)."""
    s = LoggingSimplex.__new__(LoggingSimplex)
    s._log = log
    s._rule = "init"
    s._tab = tab
    s._bfs = [-1] * tab.getNumCons()
    return s


# ---------------------------------------------------------------- fixtures

def source_of(spec):
    if "gen" in spec:
        g = spec["gen"]
        T = gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
        return T, exact.from_array(T)
    if "exact" in spec:
        e = spec["exact"]
        rows = exact.from_strings(e["z"], e["c"], e["b"], e["a"])
        T = np.array([[float(x) for x in r] for r in rows])
        return T, rows
    if "phase1" in spec:
        g = spec["phase1"]
        T = gen.phase1_lp(g["kind"], g["m"], g["ns"], g["seed"])
        return T, exact.from_array(T)
    T = np.asarray(spec["array"], dtype=np.float64)
    return T, exact.from_array(T)


def solve_fixture(name, spec, check_oracle=True):
    T, rows = source_of(spec)
    t = ref_tableau_from_rows(rows)
    log = []
    t0 = time.time()
    s = LoggingSimplex(t, log)
    init_pivots = len(log)
    s.solve()
    dt = time.time() - t0
    seq = [[r, c] for r, c, _ in log]
    nstd = sum(1 for _, _, k in log[init_pivots:] if k == "std")
    fx = {
        "name": name, "mode": "solve", **spec,
        "m": int(T.shape[0] - 1), "n": int(T.shape[1] - 1),
        "sha256": gen.digest(T),
        "seq": seq, "nstd": nstd, "init_pivots": init_pivots,
        "objective": fs(s.getObjValue()),
        "objective_float": float(s.getObjValue()),
        "bfs": list(s.getBasicSequence()),
        "ref_seconds": round(dt, 4),
    }
    if T.size <= 400:
        fx["final"] = [[fs(x) for x in row] for row in ref_rows(t)]
    if check_oracle and init_pivots == 0:
        orow = [list(r) for r in rows]
        res = exact.solve(orow)
        assert [list(p) for p in res["seq"]] == seq, f"{name}: oracle sequence differs"
        assert res["nstd"] == nstd, f"{name}: oracle nstd differs"
        assert fs(exact.objective(orow)) == fx["objective"], f"{name}: oracle objective"
    print(f"{name}: {len(seq)} pivots ({nstd} std) in {dt:.3f}s obj={fx['objective_float']}",
          flush=True)
    return fx


def standard_k_fixture(name, spec, k, check_oracle=True):
    """k pivots of findPivotStandard(True) with no phase 1 / stall logic."""
    T, rows = source_of(spec)
    t = ref_tableau_from_rows(rows)
    log = []
    s = bare_simplex(t, log)
    end = None
    t0 = time.time()
    for _ in range(k):
        res = s.findPivotStandard(True)
        if isinstance(res, str):
            end = res
            break
    dt = time.time() - t0
    seq = [[r, c] for r, c, _ in log]
    fx = {
        "name": name, "mode": "standard_k", "k": k, **spec,
        "m": int(T.shape[0] - 1), "n": int(T.shape[1] - 1),
        "sha256": gen.digest(T), "seq": seq, "end": end,
        "objective": fs(t.getZ()), "objective_float": float(t.getZ()),
        "ref_seconds": round(dt, 4),
    }
    if check_oracle:
        orow = [list(r) for r in rows]
        oseq = exact.run_standard(orow, k)
        oend = oseq[-1] if oseq and isinstance(oseq[-1], str) else None
        oseq = [list(p) for p in oseq if not isinstance(p, str)]
        assert oseq == seq and oend == end, f"{name}: oracle sequence differs"
        assert fs(exact.objective(orow)) == fx["objective"], f"{name}: oracle objective"
    print(f"{name}: {len(seq)} std pivots end={end} in {dt:.3f}s", flush=True)
    return fx


def selection_fixture(name, spec, npiv):
    """Reference findPivot* results (no pivot) at successive states of a
    standard-rule walk: pins the selection rules, max-increase and find-all."""
    T, rows = source_of(spec)
    t = ref_tableau_from_rows(rows)
    s = bare_simplex(t, [])
    states = []
    for _ in range(npiv):
        st = {
            "standard": s.findPivotStandard(False),
            "min_index": s.findPivotMinIndex(False),
            "max_increase": s.findPivotMaxIncrease(False),
            "all": [list(p) for p in s.findPivotAll()],
            "is_optimal": t.isOptimal(),
            "is_unbounded": t.isUnbounded(),
            "is_infeasible": t.isInfeasible(),
            "is_degenerate": t.isDegenerate(),
        }
        bc = [0] * t.getNumCons()
        st["is_canonical"] = t.isCanonical(bc)
        st["bcols"] = bc
        for k in ("standard", "min_index", "max_increase"):
            if isinstance(st[k], tuple):
                st[k] = list(st[k])
        states.append(st)
        res = s.findPivotStandard(True)
        if isinstance(res, str):
            break
    print(f"{name}: {len(states)} selection states", flush=True)
    return {"name": name, "mode": "selection", **spec,
            "m": int(T.shape[0] - 1), "n": int(T.shape[1] - 1),
            "sha256": gen.digest(T), "states": states}


def phase1_fixture(name, spec):
    """Simplex(tab) on an LP that needs artificial variables: the phase-1
    pivots made by the constructor (simplex.py:36-108), the basis and size
    it leaves, then solve() -- or the exception the reference raises."""
    T, rows = source_of(spec)
    t = ref_tableau_from_rows(rows)
    log = []
    fx = {"name": name, "mode": "phase1", **spec, "m": int(T.shape[0] - 1),
          "n": int(T.shape[1] - 1), "sha256": gen.digest(T)}
    try:
        s = LoggingSimplex(t, log)
        fx["init_seq"] = [[r, c] for r, c, _ in log]
        fx["init_bfs"] = list(s.getBasicSequence())
        fx["init_size"] = list(t.getTableauSize())
        k0 = len(log)
        s.solve()
        fx["seq"] = [[r, c] for r, c, _ in log[k0:]]
        fx["objective"] = fs(s.getObjValue())
        fx["bfs"] = list(s.getBasicSequence())
    except Exception as ex:                      # noqa: BLE001 -- recorded as the outcome
        fx["error"] = type(ex).__name__
        fx["message"] = str(ex)[:120]
        fx["init_seq"] = [[r, c] for r, c, _ in log]
    return fx


def kat_fixture():
    """The reference's own known-answer pivot test (test_tableau.py:9-29,
    :220-227) recorded as exact values."""
    tab1a = exact.from_strings("0", ["-40", "-30", "0", "0"], ["12", "16"],
                               [["1", "1", "1", "0"], ["2", "1", "0", "1"]])
    t = ref_tableau_from_rows(tab1a)
    t.pivot(1, 0)
    after1 = ref_rows(t)
    t.pivot(0, 1)
    after2 = ref_rows(t)
    return {"name": "kat_tab1", "mode": "kat",
            "start": [[fs(x) for x in r] for r in tab1a],
            "pivots": [[1, 0], [0, 1]],
            "after": [[[fs(x) for x in r] for r in after1],
                      [[fs(x) for x in r] for r in after2]]}


def raises_fixture(name, rows, new_b):
    """Simplex(tab) on a canonical tableau, then setB(new_b) with a negative
    entry and solve(): the reference's solve() asserts (simplex.py:133 /
    :125).  Records the pivots made before the assertion, the exception and
    the tableau it leaves."""
    t = ref_tableau_from_rows(rows)
    log = []
    s = LoggingSimplex(t, log)
    k0 = len(log)
    t.setB([Fraction(x) for x in new_b])
    fx = {"name": name, "mode": "raises",
          "start": [[fs(x) for x in r] for r in rows], "new_b": [str(x) for x in new_b]}
    try:
        s.solve()
        fx["error"] = None
    except AssertionError as ex:
        fx["error"] = type(ex).__name__
        fx["message"] = str(ex)
    fx["seq"] = [[r, c] for r, c, _ in log[k0:]]
    fx["final"] = [[fs(x) for x in r] for r in ref_rows(t)]
    print(f"{name}: {fx['error']} {fx.get('message')} after {len(fx['seq'])} pivots", flush=True)
    return fx


def json_fixture(name, spec):
    """Tableau.saveJson() of the reference before and after Simplex(t).solve()
    (tableau.py:322-360), with variable names and the basis marks."""
    T, rows = source_of(spec)
    t = ref_tableau_from_rows(rows)
    before = t.saveJson()
    s = Simplex(t)
    s.solve()
    after = t.saveJson()
    dyadic = all(Fraction(x).denominator & (Fraction(x).denominator - 1) == 0
                 for x in [after["z"]] + after["c"] + after["b"] + [v for r in after["a"] for v in r])
    print(f"{name}: saveJson {after['m']}x{after['n']} dyadic={dyadic}", flush=True)
    return {"name": name, "mode": "json", **spec, "before": before, "after": after,
            "dyadic": dyadic, "bfs": list(s.getBasicSequence()), "objective": fs(s.getObjValue())}


def extra_main():
    """tests/golden/r2.json: solve() assertions and saveJson round trips."""
    out = {"raises": [], "json": []}
    # canonical 2 x 4 (slack basis); b_1 made negative: the ratio test picks
    # row 1 (ratio -1) and the objective rises to 1 (simplex.py:133)
    base = exact.from_strings("0", ["-1", "-1", "0", "0"], ["2", "3"],
                              [["1", "1", "1", "0"], ["1", "2", "0", "1"]])
    out["raises"].append(raises_fixture("obj_increase_2x4", base, ["2", "-1"]))
    # a larger one: the assertion after a few ordinary pivots
    T, rows = source_of({"gen": {"kind": "pos", "m": 6, "ns": 6, "seed": 5}})
    nb = [str(x) for x in [rows[i][0] for i in range(1, 7)]]
    nb[4] = "-1/64"
    out["raises"].append(raises_fixture("obj_increase_pos6_s5", rows, nb))
    z, c, b, a = gen.beale_exact()
    out["json"].append(json_fixture("json_beale", {"exact": {"z": z, "c": c, "b": b, "a": a}}))
    out["json"].append(json_fixture("json_kat", {"exact": {
        "z": "0", "c": ["-40", "-30", "0", "0"], "b": ["12", "16"],
        "a": [["1", "1", "1", "0"], ["2", "1", "0", "1"]]}}))
    for seed in (1, 2, 3):
        out["json"].append(json_fixture(f"json_cfg1_mixed_s{seed}",
                                        {"gen": {"kind": "mixed", "m": 8, "ns": 10, "seed": seed}}))
    out["json"].append(json_fixture("json_pos_12x12_s4", {"gen": {"kind": "pos", "m": 12, "ns": 12, "seed": 4}}))
    out["json"].append(json_fixture("json_km_deg_d6", {"array": gen.klee_minty(6, True).tolist()}))
    with open(os.path.join(OUT, "r2.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))


def headline_main(k: int):
    """tests/golden/r3.json: a prefix of the reference's own standard-rule
    pivot sequence on the benchmark's cfg3 tableau (4096 x 8192, G_mixed seed
    3; bench.py WORKLOADS), with the exact objective after it.  About 90 s per
    pivot of the reference on one core; the oracle check is skipped (it would
    double that) -- the GPU test compares the engine with this directly."""
    spec = {"gen": {"kind": "mixed", "m": 4096, "ns": 4096, "seed": 3}}
    fx = standard_k_fixture(f"cfg3_mixed_4096x4096_s3_k{k}", spec, k, check_oracle=False)
    with open(os.path.join(OUT, "r3.json"), "w") as f:
        json.dump({"standard_k": [fx]}, f, separators=(",", ":"))


HEADLINE_WORKLOADS = {
    # bench.py WORKLOADS, by name: (generator spec, fixture name)
    "cfg3": ({"gen": {"kind": "mixed", "m": 4096, "ns": 4096, "seed": 3}}, "cfg3_mixed_4096x4096_s3_prefix"),
    "cfg4": ({"gen": {"kind": "tall", "m": 32768, "ns": 8192, "seed": 3}}, "cfg4_tall_32768x8192_s3_prefix"),
}


def interned_rows(T):
    """exact.from_array with one Fraction object per distinct float value:
    the generators draw from a few hundred values, and at cfg4 (268 M cells)
    separate objects would cost ~33 GB before the first pivot.  Fractions are
    immutable, so sharing them changes nothing the reference computes."""
    cache = {}
    out = []
    for row in T:
        r = []
        for x in row.tolist():
            f = cache.get(x)
            if f is None:
                f = cache[x] = Fraction(x)
            r.append(f)
        out.append(r)
    return out


def headline_prefix_main(k: int, out: str = "r4.json", workload: str = "cfg3"):
    """tests/golden/r4.json: the same reference walk as ``headline_main`` on
    the cfg3 bench tableau, extended towards one full 64-pivot bench group and
    CHECKPOINTED: after every reference pivot the prefix so far (sequence and
    exact objective ``-_z`` of the reference, ``tableau.py:82-84``) is written
    atomically, so a run stopped after any number of pivots leaves a valid
    fixture.  Several hours on one core (denominators grow with the pivots)."""
    spec, name = HEADLINE_WORKLOADS[workload]
    g = spec["gen"]
    T = gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
    shape, sha = T.shape, gen.digest(T)
    rows = interned_rows(T)
    del T
    t = ref_tableau_from_rows(rows)
    del rows
    log = []
    s = bare_simplex(t, log)
    path = os.path.join(OUT, out)
    t0 = time.time()
    end = None
    times = []
    for i in range(k):
        res = s.findPivotStandard(True)
        if isinstance(res, str):
            end = res
        times.append(round(time.time() - t0, 1))
        fx = {
            "name": name, "mode": "standard_k", "k": len(log), "workload": workload,
            **spec, "m": int(shape[0] - 1), "n": int(shape[1] - 1),
            "sha256": sha, "seq": [[r, c] for r, c, _ in log], "end": end,
            "objective": fs(t.getZ()), "objective_float": float(t.getZ()),
            "ref_seconds": times[-1], "ref_seconds_cumulative": times,
        }
        with open(path + ".tmp", "w") as f:
            json.dump({"standard_k": [fx]}, f, separators=(",", ":"))
        os.replace(path + ".tmp", path)
        print(f"pivot {len(log)}: {log[-1][:2] if log else None} at {times[-1]} s", flush=True)
        if end is not None:
            break


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--extra", action="store_true",
                    help="only tests/golden/r2.json (solve assertions, saveJson round trips)")
    ap.add_argument("--headline", type=int, default=0, metavar="K",
                    help="only tests/golden/r3.json: K reference pivots on the cfg3 bench tableau")
    ap.add_argument("--headline-prefix", type=int, default=0, metavar="K",
                    help="only tests/golden/r4.json: up to K reference pivots on the cfg3 bench "
                         "tableau, rewritten after every pivot")
    ap.add_argument("--workload", default="cfg3", choices=sorted(HEADLINE_WORKLOADS),
                    help="--headline-prefix: the bench workload whose tableau the reference pivots "
                         "(cfg4: r6.json, 32768 x 8192 G_tall seed 3, ~25 min per reference pivot)")
    ap.add_argument("--out", default="r4.json",
                    help="--headline-prefix: the fixture file under tests/golden/ (r5.json: K = 80, across "
                         "the first sweep boundary)")
    args = ap.parse_args()
    if args.headline_prefix:
        headline_prefix_main(args.headline_prefix, args.out, args.workload)
        return
    if args.extra:
        extra_main()
        return
    if args.headline:
        headline_main(args.headline)
        return

    small = {"kat": [kat_fixture()], "solve": [], "standard_k": [], "selection": [], "phase1": []}
    z, c, b, a = gen.beale_exact()
    small["solve"].append(solve_fixture("beale", {"exact": {"z": z, "c": c, "b": b, "a": a}}))
    for d in (3, 4, 5, 6, 8, 10):
        small["solve"].append(solve_fixture(f"km_std_d{d}", {"array": gen.klee_minty(d).tolist()}))
    for d in (4, 6, 8, 10):
        small["solve"].append(solve_fixture(f"km_deg_d{d}",
                                            {"array": gen.klee_minty(d, True).tolist()}))
    for seed in range(1, 9):
        small["solve"].append(solve_fixture(f"cfg1_mixed_s{seed}",
                                            {"gen": {"kind": "mixed", "m": 8, "ns": 10, "seed": seed}}))
    for seed in range(1, 5):
        small["solve"].append(solve_fixture(f"cfg1_pos_s{seed}",
                                            {"gen": {"kind": "pos", "m": 8, "ns": 10, "seed": seed}}))
    for (m, ns) in ((16, 16), (24, 32), (32, 24), (40, 40)):
        for seed in (11, 12, 13):
            small["solve"].append(solve_fixture(f"mixed_{m}x{ns}_s{seed}",
                                                {"gen": {"kind": "mixed", "m": m, "ns": ns, "seed": seed}}))
    for (m, ns) in ((32, 32), (64, 64)):
        for seed in (21, 22):
            small["solve"].append(solve_fixture(f"pos_{m}x{ns}_s{seed}",
                                                {"gen": {"kind": "pos", "m": m, "ns": ns, "seed": seed}}))
    for seed in range(1, 7):
        small["standard_k"].append(standard_k_fixture(
            f"tall_64x16_s{seed}", {"gen": {"kind": "tall", "m": 64, "ns": 16, "seed": seed}}, 400))
    small["standard_k"].append(standard_k_fixture(
        "mixed_64x64_k120", {"gen": {"kind": "mixed", "m": 64, "ns": 64, "seed": 31}}, 120))
    small["selection"].append(selection_fixture(
        "sel_mixed_8x10", {"gen": {"kind": "mixed", "m": 8, "ns": 10, "seed": 3}}, 12))
    small["selection"].append(selection_fixture(
        "sel_tall_16x8", {"gen": {"kind": "tall", "m": 16, "ns": 8, "seed": 4}}, 12))
    small["selection"].append(selection_fixture(
        "sel_km_deg_d6", {"array": gen.klee_minty(6, True).tolist()}, 12))
    small["selection"].append(selection_fixture(
        "sel_beale", {"exact": {"z": z, "c": c, "b": b, "a": a}}, 12))
    for kind in ("eq", "ge", "neg"):
        for (m, ns) in ((4, 5), (6, 8), (10, 12), (16, 20)):
            for seed in (1, 2, 3):
                small["phase1"].append(phase1_fixture(
                    f"p1_{kind}_{m}x{ns}_s{seed}",
                    {"phase1": {"kind": kind, "m": m, "ns": ns, "seed": seed}}))
    for seed in (1, 2):
        small["phase1"].append(phase1_fixture(
            f"p1_dep_6x8_s{seed}", {"phase1": {"kind": "dep", "m": 6, "ns": 8, "seed": seed}}))
    small["phase1"].append(phase1_fixture(
        "p1_infeasible_4", {"phase1": {"kind": "infeasible", "m": 2, "ns": 4, "seed": 0}}))
    with open(os.path.join(OUT, "small.json"), "w") as f:
        json.dump(small, f, separators=(",", ":"))

    if args.big:
        big = {"solve": [], "standard_k": []}
        big["solve"].append(solve_fixture(
            "cfg2_pos_512x512_s7", {"gen": {"kind": "pos", "m": 512, "ns": 512, "seed": 7}},
            check_oracle=False))
        big["standard_k"].append(standard_k_fixture(
            "cfg2_mixed_512x512_s7_k64", {"gen": {"kind": "mixed", "m": 512, "ns": 512, "seed": 7}},
            64, check_oracle=False))
        with open(os.path.join(OUT, "big.json"), "w") as f:
            json.dump(big, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
