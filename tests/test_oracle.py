"""Pin the oracles to the reference (CPU only).

Golden vectors were captured by running the reference itself in the build
container (tests/golden/make_golden.py).  Both oracles must reproduce them:
  * oracle/exact.py  (Fraction restatement): identical pivot sequences,
    identical exact objectives, identical final tableaux;
  * oracle/lp_f64.c  (float64 restatement with the engine's semantics):
    identical pivot sequences, objective within 1e-9 relative.
"""
from fractions import Fraction

import numpy as np
import pytest

from conftest import fixture_exact, fixture_input, load_golden

from lpsol_amd import generators as gen
from oracle import exact
from oracle.f64 import F64Tableau

SMALL = load_golden("small.json")
BIG = load_golden("big.json")
REL = 1e-9   # north star: objective within 1e-9 relative of the rational answer


def _ids(fxs):
    return [fx["name"] for fx in fxs]


def test_kat_reference_pivot_pair():
    """tableau.py test_pivot (test_tableau.py:220-227) on the exact oracle."""
    kat = SMALL["kat"][0]
    T = [[Fraction(x) for x in r] for r in kat["start"]]
    for (r, c), after in zip(kat["pivots"], kat["after"]):
        exact.pivot(T, r, c)
        assert T == [[Fraction(x) for x in row] for row in after]


@pytest.mark.parametrize("fx", SMALL["solve"] + BIG["solve"] + SMALL["standard_k"] + BIG["standard_k"],
                         ids=_ids(SMALL["solve"] + BIG["solve"] + SMALL["standard_k"] + BIG["standard_k"]))
def test_fixture_input_pinned(fx):
    """the generator / hand-built inputs are byte-identical to the captured ones"""
    assert gen.digest(fixture_input(fx)) == fx["sha256"]


@pytest.mark.parametrize("fx", SMALL["solve"], ids=_ids(SMALL["solve"]))
def test_exact_solve_matches_reference(fx):
    T = fixture_exact(fx)
    res = exact.solve(T)
    assert [list(p) for p in res["seq"]] == fx["seq"]
    assert res["nstd"] == fx["nstd"]
    assert exact.frac_str(exact.objective(T)) == fx["objective"]
    if "final" in fx:
        assert T == [[Fraction(x) for x in row] for row in fx["final"]]
    bfs = [-1] * (len(T) - 1)
    ok, bcols = exact.is_canonical(fixture_exact(fx))
    assert ok
    bfs = list(bcols)
    for r, c in res["seq"]:
        bfs[r] = c
    assert bfs == fx["bfs"]


@pytest.mark.parametrize("fx", SMALL["standard_k"], ids=_ids(SMALL["standard_k"]))
def test_exact_standard_k_matches_reference(fx):
    T = fixture_exact(fx)
    seq = exact.run_standard(T, fx["k"])
    end = seq[-1] if seq and isinstance(seq[-1], str) else None
    assert [list(p) for p in seq if not isinstance(p, str)] == fx["seq"]
    assert end == fx["end"]
    assert exact.frac_str(exact.objective(T)) == fx["objective"]


@pytest.mark.parametrize("fx", SMALL["selection"], ids=_ids(SMALL["selection"]))
def test_exact_selection_rules_match_reference(fx):
    """findPivotStandard/MinIndex/MaxIncrease/All and the form checks at every
    state of a standard-rule walk."""
    T = fixture_exact(fx)
    for st in fx["states"]:
        def norm(x):
            return list(x) if isinstance(x, tuple) else x
        assert norm(exact.find_standard(T)) == st["standard"]
        assert norm(exact.find_min_index(T)) == st["min_index"]
        assert norm(exact.find_max_increase(T)) == st["max_increase"]
        assert [list(p) for p in exact.find_all(T)] == st["all"]
        assert exact.is_optimal(T) == st["is_optimal"]
        assert exact.is_unbounded(T) == st["is_unbounded"]
        assert exact.is_infeasible(T) == st["is_infeasible"]
        assert exact.is_degenerate(T) == st["is_degenerate"]
        ok, bcols = exact.is_canonical(T)
        assert ok == st["is_canonical"]
        if ok or any(b != 0 for b in st["bcols"]):
            assert bcols == st["bcols"]
        res = exact.find_standard(T)
        if isinstance(res, str):
            break
        exact.pivot(T, *res)


@pytest.mark.parametrize("fx", SMALL["selection"], ids=_ids(SMALL["selection"]))
def test_f64_oracle_selection_rules_match_reference(fx):
    """the float64 restatement's findPivotStandard/MinIndex/MaxIncrease/All at
    every state of the reference's standard-rule walk"""
    t = F64Tableau(fixture_input(fx))
    for st in fx["states"]:
        def norm(x):
            return list(x) if isinstance(x, tuple) else x
        assert norm(t.find(0)) == st["standard"]
        assert norm(t.find(1)) == st["min_index"]
        assert norm(t.find_max_increase()) == st["max_increase"]
        assert [list(p) for p in t.find_all()] == st["all"]
        res = t.find(0)
        if isinstance(res, str):
            break
        t.pivot(*res)


@pytest.mark.parametrize("fx", SMALL["solve"] + BIG["solve"], ids=_ids(SMALL["solve"] + BIG["solve"]))
def test_f64_oracle_solve_matches_reference(fx):
    t = F64Tableau(fixture_input(fx))
    st, log, nstd = t.solve()
    assert st == 1
    assert log.tolist() == fx["seq"]
    assert nstd == fx["nstd"]
    obj = float(Fraction(fx["objective"]))
    assert abs(t.objective() - obj) <= REL * max(1.0, abs(obj))


@pytest.mark.parametrize("fx", SMALL["standard_k"] + BIG["standard_k"],
                         ids=_ids(SMALL["standard_k"] + BIG["standard_k"]))
def test_f64_oracle_standard_k_matches_reference(fx):
    t = F64Tableau(fixture_input(fx))
    st, log = t.run(0, fx["k"])
    assert log.tolist() == fx["seq"]
    assert (fx["end"] == "optimal") == (st == 1)
    obj = float(Fraction(fx["objective"]))
    assert abs(t.objective() - obj) <= REL * max(1.0, abs(obj))


def test_f64_oracle_cycling_without_switch():
    """Beale's LP cycles under the pure standard rule: the stall switch of
    solve() is what ends it."""
    t = F64Tableau(gen.beale())
    st, log = t.run(0, 40)
    assert st == 0 and len(log) == 40          # still pivoting: a cycle
    assert [tuple(p) for p in log[:6]] == [tuple(p) for p in log[6:12]]


def test_generator_is_counter_based():
    """any row block can be generated independently (sharded ranks)"""
    full = gen.tableau("tall", 40, 24, 5)
    parts = [gen.rows("tall", 40, 24, 5, a, b) for a, b in ((0, 7), (7, 20), (20, 41))]
    assert np.array_equal(full, np.vstack(parts))
    T = gen.tableau("mixed", 16, 16, 3)
    assert np.all(T[1:, 0] > 0) and np.all(T[0, 1:17] < 0)
    assert np.array_equal(T[1:, 17:], np.eye(16))
    assert np.all(np.abs(T * 64 - np.round(T * 64)) == 0)      # dyadic k/64


@pytest.mark.parametrize("fx", SMALL["selection"], ids=_ids(SMALL["selection"]))
def test_host_form_checks_match_reference(fx):
    """the front-end's numpy predicates (lpsol_amd.Tableau host path) on the
    float64 states of the reference's walk answer what the reference did"""
    from lpsol_amd import Tableau
    t = F64Tableau(fixture_input(fx))
    for st in fx["states"]:
        h = Tableau.fromArray(t.T)
        bc = [-2] * t.m
        assert h.isCanonical(bc) == st["is_canonical"]
        if st["is_canonical"]:
            assert bc == st["bcols"]
        assert h.isOptimal() == st["is_optimal"]
        assert h.isUnbounded() == st["is_unbounded"]
        assert h.isInfeasible() == st["is_infeasible"]
        assert h.isDegenerate() == st["is_degenerate"]
        res = t.find(0)
        if isinstance(res, str):
            break
        t.pivot(*res)


@pytest.mark.parametrize("fx", SMALL["phase1"], ids=_ids(SMALL["phase1"]))
def test_phase1_oracle_matches_reference(fx):
    """oracle/phase1.py (Simplex._find_bfs on the float64 contract) against
    the reference run on the same LP: every phase-1 pivot (artificial solve
    and drive-out), the basis and size it leaves, then solve()."""
    from oracle import phase1
    o = phase1.solve_lp(fixture_input(fx))
    assert o["init_seq"] == fx["init_seq"]
    if fx.get("error") == "ValueError":              # infeasible: same exception
        assert o.get("error") == "ValueError"
        return
    if fx.get("error") == "IndexError":
        # the reference's _m bug (simplex.py:93) after dropping a dependent
        # row; the restatement drops it and solves the LP without it
        assert o["init_size"] == [fx["m"] - 1, fx["n"]]
        twin = next(f for f in SMALL["phase1"] if f.get("phase1") == dict(fx["phase1"], kind="eq"))
        obj = float(Fraction(twin["objective"]))
        assert abs(o["objective"] - obj) <= REL * max(1.0, abs(obj))
        return
    assert o["init_bfs"] == fx["init_bfs"]
    assert o["init_size"] == fx["init_size"]
    assert o["seq"] == fx["seq"]
    assert o["bfs"] == fx["bfs"]
    obj = float(Fraction(fx["objective"]))
    assert abs(o["objective"] - obj) <= REL * max(1.0, abs(obj))


def test_phase1_golden_covers_every_outcome():
    kinds = {fx["phase1"]["kind"] for fx in SMALL["phase1"]}
    assert kinds == {"eq", "ge", "neg", "dep", "infeasible"}
    assert {fx.get("error") for fx in SMALL["phase1"]} == {None, "IndexError", "ValueError"}
    # phase 1 made drive-out pivots somewhere (artificial basic at value 0)
    assert any(len(fx["init_seq"]) > 0 for fx in SMALL["phase1"] if fx["phase1"]["kind"] == "ge")


def test_oracle_under_sanitizers():
    """oracle/lp_f64.c built with -fsanitize=address,undefined (no recovery)
    and run over exact-size tableaux (random dyadic LPs, Klee-Minty d=2..8):
    no sanitizer report, and its solve/scan invariants hold
    (oracle/sanitize_main.c)."""
    import os
    import shutil
    import subprocess
    if shutil.which(os.environ.get("CC", "gcc")) is None:
        pytest.skip("no C compiler")
    root = os.path.join(os.path.dirname(__file__), "..", "oracle")
    subprocess.run(["make", "-s", "-C", root, "sanitize"], check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([os.path.join(root, "build", "lpf64_sanitize")], capture_output=True,
                         text=True, timeout=300, env=env)
    assert run.returncode == 0, run.stdout + run.stderr
    assert "clean" in run.stdout
