"""Round-2 CPU tests: the reference's solve() assertions and its saveJson
output, both pinned by tests/golden/r2.json (captured from the reference by
tests/golden/make_golden.py --extra)."""
import json
from fractions import Fraction

import numpy as np
import pytest

from conftest import fixture_exact, load_golden

from lpsol_amd import Tableau, _lib
from lpsol_amd.simplex import optimal_row0
from oracle import exact
from oracle.f64 import F64Tableau

R2 = load_golden("r2.json")


def _ids(fxs):
    return [fx["name"] for fx in fxs]


def _raised_start(fx):
    rows = [[Fraction(x) for x in r] for r in fx["start"]]
    for i, b in enumerate(fx["new_b"]):
        rows[1 + i][0] = Fraction(b)
    return rows


@pytest.mark.parametrize("fx", R2["raises"], ids=_ids(R2["raises"]))
def test_exact_solve_objective_assertion(fx):
    """oracle/exact.py raises where the reference's solve() asserts
    (simplex.py:133), after the same pivots, leaving the same tableau"""
    assert fx["error"] == "AssertionError"
    T = _raised_start(fx)
    seq = []
    with pytest.raises(exact.ObjectiveIncreased, match="objective value increased"):
        exact.solve(T, log=seq)
    assert [list(p) for p in seq] == fx["seq"]
    assert T == [[Fraction(x) for x in r] for r in fx["final"]]


@pytest.mark.parametrize("fx", R2["raises"], ids=_ids(R2["raises"]))
def test_f64_solve_objective_status(fx):
    """oracle/lp_f64.c stops with LP_OBJ_INCREASED after the same pivots"""
    T = np.array([[float(x) for x in r] for r in _raised_start(fx)])
    o = F64Tableau(T)
    st, log, _ = o.solve()
    assert st == _lib.OBJ_INCREASED
    assert log.tolist() == fx["seq"]
    want = np.array([[float(Fraction(x)) for x in r] for r in fx["final"]])
    assert np.allclose(o.T, want, rtol=1e-12, atol=1e-12)


def test_final_optimality_check():
    """the float64 form of simplex.py:148 (every c_j >= -tol.cost)"""
    assert optimal_row0([5.0, 0.0, 1.0, -1e-12], 1e-9)
    assert not optimal_row0([5.0, 0.0, 1.0, -1e-6], 1e-9)


@pytest.mark.parametrize("fx", R2["json"], ids=_ids(R2["json"]))
def test_load_save_json_is_the_reference_format(fx, tmp_path):
    """loadJson(reference saveJson) -> saveJson gives back the reference's
    dict key by key (dyadic inputs are exact in float64), also through a file"""
    t = Tableau(1, 1)
    t.loadJson(fx["before"])
    assert t.saveJson() == fx["before"]
    p = tmp_path / "t.json"
    t.saveFile(str(p))
    with open(p) as f:
        assert json.load(f) == fx["before"]
    u = Tableau(1, 1)
    u.loadFile(str(p))
    assert u.saveJson() == fx["before"]


@pytest.mark.parametrize("fx", R2["json"], ids=_ids(R2["json"]))
def test_exact_oracle_reproduces_reference_json(fx):
    """the exact oracle's solve of the saved tableau ends in the reference's
    saved tableau (pins the 'after' fixtures the GPU test compares with)"""
    T = fixture_exact(fx)
    exact.solve(T)
    a = fx["after"]
    want = [[Fraction(a["z"])] + [Fraction(x) for x in a["c"]]]
    want += [[Fraction(a["b"][i])] + [Fraction(x) for x in a["a"][i]] for i in range(a["m"])]
    assert T == want
