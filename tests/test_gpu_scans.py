"""Device column scans and phase 1 on the MI355X.

  * findPivotMaxIncrease / findPivotAll (simplex.py:286-360) as one device
    scan of every column (k_colstat + k_colband) -- compared with the
    reference's answers at every state of its own walk (golden
    "selection" states) and with oracle/lp_f64.c on random tableaus,
    single device and row-sharded;
  * isCanonical / isOptimal / isUnbounded / isInfeasible / isDegenerate
    (tableau.py:466-518) as device reductions -- equal to the reference's
    answers and to the host numpy predicates on the same float64 bits;
  * Simplex._find_bfs (simplex.py:36-108) driven by the device engine --
    every pivot, the basis, the size, the phase-2 sequence and objective
    equal to the reference's (golden "phase1" fixtures) and the final
    tableau bit-identical to oracle/phase1.py.
"""
from fractions import Fraction

import numpy as np
import pytest

from conftest import fixture_input, load_golden

from lpsol_amd import Simplex, Tableau, _lib
from lpsol_amd import generators as gen
from oracle import phase1
from oracle.f64 import F64Tableau

pytestmark = pytest.mark.gpu

SMALL = load_golden("small.json")
REL = 1e-9


@pytest.fixture(scope="module", autouse=True)
def gpu():
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"


@pytest.fixture(params=["peer", "rccl"])
def shard_mode(request, monkeypatch):
    monkeypatch.setenv("LPGPU_PEER", "1" if request.param == "peer" else "0")
    return request.param


def _ids(fxs):
    return [fx["name"] for fx in fxs]


def _norm(x):
    return list(x) if isinstance(x, tuple) else x


def _group(T, nshards):
    m, n = T.shape[0] - 1, T.shape[1] - 1
    if nshards == 1:
        e = _lib.Engine(m, n)
        e.upload(T)
        return [e]
    grp = _lib.create_group(m, n, nshards)
    for g in grp:
        g.upload(T)
    return grp


def _close(grp):
    for g in reversed(grp):
        g.close()


def _host_checks(D):
    """the host (numpy) predicates of lpsol_amd.Tableau on the same bits"""
    t = Tableau.fromArray(D)
    bc = [-2] * (D.shape[0] - 1)
    return dict(canonical=t.isCanonical(bc), optimal=t.isOptimal(), unbounded=t.isUnbounded(),
                infeasible=t.isInfeasible(), degenerate=t.isDegenerate(), bcols=bc)


# ------------------------------------------------- reference selection states
@pytest.mark.parametrize("nshards", [1, 3])
@pytest.mark.parametrize("fx", SMALL["selection"], ids=_ids(SMALL["selection"]))
def test_scans_match_reference_states(fx, nshards):
    """at every state of the reference's standard-rule walk: the four
    selection rules and the five form checks answer what the reference did"""
    T = fixture_input(fx)
    if nshards > T.shape[0] - 1:
        pytest.skip("fewer rows than shards")
    grp = _group(T, nshards)
    e = grp[0]
    for st in fx["states"]:
        assert _norm(e.find(_lib.RULE_STANDARD, False)) == st["standard"]
        assert _norm(e.find(_lib.RULE_MIN_INDEX, False)) == st["min_index"]
        assert _norm(e.find_max_increase(False)) == st["max_increase"]
        assert [list(p) for p in e.find_all()] == st["all"]
        f = e.form_checks()
        assert f["canonical"] == st["is_canonical"]
        assert f["optimal"] == st["is_optimal"]
        assert f["unbounded"] == st["is_unbounded"]
        assert f["infeasible"] == st["is_infeasible"]
        assert f["degenerate"] == st["is_degenerate"]
        if st["is_canonical"]:
            assert f["bcols"] == st["bcols"]
        if e.find(_lib.RULE_STANDARD, True) in ("optimal", "unbounded"):
            break
    _close(grp)


# ------------------------------------------------------ random, vs oracle
@pytest.mark.parametrize("nshards", [1, 2, 5])
@pytest.mark.parametrize("kind,m,ns,seed,Q", [
    ("mixed", 40, 30, 1, 64), ("mixed", 130, 70, 2, 64), ("degenerate", 96, 64, 3, 64),
    ("pos", 64, 64, 4, 2), ("tall", 700, 20, 5, 64), ("mixed", 16, 300, 6, 64),
    ("pos", 300, 200, 7, 4)])
def test_scans_match_oracle_along_walk(kind, m, ns, seed, Q, nshards, shard_mode):
    """max-increase pivots driven on the device; after each one the device
    answer of both scans equals the oracle's and the rows are bit-identical
    (pos with Q = 2, 4: many tied costs, ratios and increases)"""
    if kind == "degenerate":
        T = gen.tableau("mixed", m, ns, seed, Q)
        T[1::3, 0] = 0.0                              # b_i = 0 on every third row
    else:
        T = gen.tableau(kind, m, ns, seed, Q)
    grp = _group(T, nshards)
    o = F64Tableau(T)
    for _ in range(25):
        assert [list(p) for p in grp[0].find_all()] == [list(p) for p in o.find_all()]
        want = o.find_max_increase()
        got = grp[0].find_max_increase(True)
        assert _norm(got) == _norm(want)
        if isinstance(want, str):
            break
        o.pivot(*want)
    for g in grp:
        b, c = g.row_begin, g.row_count
        assert np.array_equal(g.rows(0, 1), o.T[:1])
        assert np.array_equal(g.rows(1 + b, c), o.T[1 + b:1 + b + c])
    _close(grp)


@pytest.mark.parametrize("nshards", [1, 4])
def test_scans_unbounded_and_optimal(nshards):
    # unbounded: column 1 has negative cost and no positive entry
    T = np.array([[0.0, -1.0, -2.0, 0.0],
                  [4.0, 1.0, -1.0, 1.0],
                  [6.0, 2.0, 0.0, 0.0],
                  [1.0, 0.0, -3.0, 0.0],
                  [2.0, 1.0, -1.0, 0.0]])
    grp = _group(T, nshards)
    assert grp[0].find_max_increase(False) == F64Tableau(T).find_max_increase() == "unbounded"
    f = grp[0].form_checks()
    assert f["unbounded"] and not f["optimal"]
    _close(grp)
    T2 = T.copy()
    T2[0, 1:] = [1.0, 0.0, 0.0]
    grp = _group(T2, nshards)
    assert grp[0].find_max_increase(True) == "optimal"
    assert grp[0].form_checks()["optimal"]
    _close(grp)


@pytest.mark.parametrize("nshards", [1, 3])
def test_form_checks_match_host_predicates(nshards):
    """device predicates == host numpy predicates on the same float64 bits,
    through a walk that passes canonical, degenerate and infeasible states"""
    deg = gen.tableau("mixed", 48, 40, 7)
    deg[2::5, 0] = 0.0
    cases = [deg, gen.tableau("mixed", 60, 50, 8)]
    inf = gen.tableau("mixed", 30, 20, 9)
    inf[5, 0] = 3.0
    inf[5, 1:] = -np.abs(inf[5, 1:])                 # b > 0, every a <= 0: infeasible row
    cases.append(inf)
    neg = gen.tableau("mixed", 30, 20, 10)
    neg[3, 0] = -1.0                                 # b < 0: not canonical, bcols untouched
    cases.append(neg)
    for T in cases:
        grp = _group(T, nshards)
        for _ in range(12):
            D = np.concatenate([grp[0].rows(0, 1)] +
                               [g.rows(1 + g.row_begin, g.row_count) for g in grp])
            f = grp[0].form_checks()
            h = _host_checks(D)
            for k in ("canonical", "optimal", "unbounded", "infeasible", "degenerate"):
                assert f[k] == h[k], k
            if f["bcols"] is not None:
                assert f["bcols"] == h["bcols"]
            else:
                assert h["bcols"] == [-2] * (D.shape[0] - 1)
            if grp[0].find(_lib.RULE_STANDARD, True) in ("optimal", "unbounded"):
                break
        _close(grp)


# ----------------------------------------------------------- front-end
class _LogSimplex(Simplex):
    def __init__(self, tab, log):
        self._plog = log
        super().__init__(tab)

    def _mark(self, r, c):
        self._plog.append([int(r), int(c)])
        super()._mark(r, c)


def test_frontend_max_increase_and_all():
    T = gen.tableau("mixed", 50, 40, 11)
    t = Tableau.fromArray(T)
    s = Simplex(t)
    o = F64Tableau(T)
    assert s.findPivotAll() == [tuple(p) for p in o.find_all()]
    for _ in range(10):
        want = o.find_max_increase()
        got = s.findPivotMaxIncrease(True)
        assert got == want
        if isinstance(want, str):
            break
        o.pivot(*want)
        r, c = want
        assert s.getBasicSequence()[r] == c and t.getVarMark(c)
    assert np.array_equal(t.toArray(), o.T)
    # the form checks of the device copy (host mirror stale) agree with numpy's
    f = {k: getattr(t, "is" + k)() for k in ("Canonical", "Optimal", "Unbounded",
                                             "Infeasible", "Degenerate")}
    h = _host_checks(o.T)
    for k, v in f.items():
        assert v == h[k.lower()], k


@pytest.mark.parametrize("fx", SMALL["phase1"], ids=_ids(SMALL["phase1"]))
def test_phase1_matches_reference(fx):
    """Simplex(tab) then solve(): phase-1 pivots, the basis and size it leaves,
    the phase-2 sequence, objective and basis -- as the reference; tableau bit
    for bit as oracle/phase1.py.  Dependent rows: the reference raises
    IndexError (simplex.py:93); here the row is dropped and the LP solved."""
    T = fixture_input(fx)
    t = Tableau.fromArray(T)
    log = []
    if fx.get("error") == "ValueError":
        with pytest.raises(ValueError, match="infeasible problem"):
            _LogSimplex(t, log)
        assert log == fx["init_seq"]
        return
    s = _LogSimplex(t, log)
    init = list(log)
    assert list(t.getTableauSize()) == [fx["m"] - (fx.get("error") == "IndexError"),
                                        fx["n"]]
    o = phase1.solve_lp(T)
    if fx.get("error") == "IndexError":
        assert init == fx["init_seq"]                # everything up to the reference's failure
        assert init == o["init_seq"]
    else:
        assert init == fx["init_seq"]
        assert list(s.getBasicSequence()) == fx["init_bfs"]
        assert list(t.getTableauSize()) == fx["init_size"]
    del log[:]
    s.solve()
    assert log == o["seq"]
    assert list(s.getBasicSequence()) == o["bfs"]
    assert np.array_equal(t.toArray(), o["T"])
    if "objective" in fx:
        assert log == fx["seq"]
        assert list(s.getBasicSequence()) == fx["bfs"]
        obj = float(Fraction(fx["objective"]))
        assert abs(s.getObjValue() - obj) <= REL * max(1.0, abs(obj))
    else:
        # same LP without the repeated row (the "eq" fixture of that seed)
        g = fx["phase1"]
        twin = next(f for f in SMALL["phase1"] if f.get("phase1") == dict(g, kind="eq"))
        obj = float(Fraction(twin["objective"]))
        assert abs(s.getObjValue() - obj) <= REL * max(1.0, abs(obj))
