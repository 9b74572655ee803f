"""Parity of the HIP engine with the oracles and the reference (MI355X).

Every test calls through the C-ABI (liblpgpu.so).  Bars:
  * pivot sequences identical to the reference's (golden vectors);
  * objective within 1e-9 relative of the reference's exact rational;
  * the whole device tableau BIT-IDENTICAL to oracle/lp_f64.c, which
    restates the same float64 operations on the host.
"""
from fractions import Fraction

import numpy as np
import pytest

from conftest import fixture_input, load_golden

from lpsol_amd import Simplex, Tableau, _lib
from lpsol_amd import generators as gen
from oracle.f64 import F64Tableau

pytestmark = pytest.mark.gpu

SMALL = load_golden("small.json")
BIG = load_golden("big.json")
REL = 1e-9


@pytest.fixture(scope="module", autouse=True)
def gpu():
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"


def _ids(fxs):
    return [fx["name"] for fx in fxs]


def _obj_ok(z, fx):
    obj = float(Fraction(fx["objective"]))
    return abs(z - obj) <= REL * max(1.0, abs(obj))


def _initial_basis(T):
    bc = [0] * (T.shape[0] - 1)
    assert Tableau.fromArray(T).isCanonical(bc)
    return bc


@pytest.fixture(params=["persistent", "kernels"])
def select_mode(request, monkeypatch):
    """single-device selection path: one persistent k_group launch per group
    followed by the in-place sweep (default), or the per-pivot k_ratio/k_prow
    launches (the sharded path's kernels)"""
    monkeypatch.setenv("LPGPU_SELECT", "kernels" if request.param == "kernels" else "persistent")
    return request.param


def no_fallback(e):
    """the run took no timed-out persistent group (each is redone on the
    per-pivot kernels: correct, but never expected)"""
    assert e.exchange_path()[1] == 0


def engine_of(T, block=8):
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(block)
    return e


# ------------------------------------------------------------------ KAT
def test_reference_kat_pivot_pair():
    """lpsol/test_tableau.py:220-227 through the front-end on the GPU"""
    def tab(z, c, b, a):
        t = Tableau(2, 4)
        t.setVarNames(["x1", "x2", "s1", "s2"])
        t.setZ(-Fraction(z))
        t.setC(c)
        t.setB(b)
        t.setA(a)
        return t
    t1a = tab("0", ["-40", "-30", "0", "0"], [12, 16], [[1, 1, 1, 0], [2, 1, 0, 1]])
    t1b = tab("320", [0, -10, 0, 20], [4, 8], [[0, "1/2", 1, "-1/2"], [1, "1/2", 0, "1/2"]])
    t1c = tab("400", [0, 0, 20, 10], [8, 4], [[0, 1, 2, -1], [1, 0, -1, 1]])
    t1a.pivot(1, 0)
    assert t1a == t1b
    t1b.pivot(0, 1)
    assert t1b == t1c
    t1a.pivot(0, 1)
    assert t1a == t1c


# ----------------------------------------------------------- golden solves
@pytest.mark.parametrize("block", [1, 8])
@pytest.mark.parametrize("fx", SMALL["solve"] + BIG["solve"], ids=_ids(SMALL["solve"] + BIG["solve"]))
def test_solve_matches_reference(fx, block, select_mode):
    T = fixture_input(fx)
    e = engine_of(T, block)
    st, npiv, nstd = e.solve()
    assert st == _lib.OPTIMAL
    assert e.log().tolist() == fx["seq"]
    assert nstd == fx["nstd"]
    assert _obj_ok(e.objective(), fx)
    o = F64Tableau(T)
    o.solve()
    assert np.array_equal(e.download(), o.T), "tableau differs from the f64 oracle"


@pytest.mark.parametrize("fx", SMALL["standard_k"] + BIG["standard_k"],
                         ids=_ids(SMALL["standard_k"] + BIG["standard_k"]))
@pytest.mark.parametrize("block", [1, 5, 32])
def test_standard_k_matches_reference(fx, block, select_mode):
    T = fixture_input(fx)
    e = engine_of(T, block)
    st, done = e.run(_lib.RULE_STANDARD, fx["k"])
    assert e.log().tolist() == fx["seq"]
    assert (st == _lib.OPTIMAL) == (fx["end"] == "optimal")
    assert _obj_ok(e.objective(), fx)
    o = F64Tableau(T)
    o.run(0, fx["k"])
    assert np.array_equal(e.download(), o.T)


@pytest.mark.parametrize("fx", SMALL["selection"], ids=_ids(SMALL["selection"]))
def test_selection_rules_match_reference(fx):
    e = engine_of(fixture_input(fx))
    for st in fx["states"]:
        def norm(x):
            return list(x) if isinstance(x, tuple) else x
        assert norm(e.find(_lib.RULE_STANDARD, False)) == st["standard"]
        assert norm(e.find(_lib.RULE_MIN_INDEX, False)) == st["min_index"]
        if isinstance(e.find(_lib.RULE_STANDARD, True), str):
            break


def test_frontend_simplex_solve_bfs():
    for fx in SMALL["solve"][:12]:
        t = Tableau.fromArray(fixture_input(fx))
        s = Simplex(t)
        s.solve()
        assert s.getBasicSequence() == fx["bfs"], fx["name"]
        assert _obj_ok(s.getObjValue(), fx)
        # marks follow _pivot's bookkeeping only (simplex.py:192-197): a
        # canonical start returns before any mark is set (simplex.py:46-47)
        marks = [False] * t.getNumVars()
        bfs = _initial_basis(fixture_input(fx))
        for r, c in fx["seq"]:
            marks[bfs[r]] = False
            bfs[r] = c
            marks[c] = True
        assert t.getVarMarks() == marks
        bfs = s.getBFS()
        assert set(bfs) == set(fx["bfs"])


def test_frontend_find_and_validated_pivot():
    fx = SMALL["solve"][12]
    T = fixture_input(fx)
    t = Tableau.fromArray(T)
    s = Simplex(t)
    r, c = fx["seq"][0]
    assert s.findPivotStandard(False) == (r, c)
    wrong = next(i for i in range(t.getNumCons()) if i != r and t.getAij(i, c) > 0)
    with pytest.raises(ValueError):
        s.pivot(wrong, c)
    s.pivot(r, c)
    assert s.getBasicSequence()[r] == c and t.getVarMark(c)
    assert s.findPivotStandard(True) == tuple(fx["seq"][1])


# --------------------------------------------------------------- errors
def test_zero_pivot_raises():
    t = Tableau.fromArray(gen.beale())
    before = t.toArray()
    with pytest.raises(ZeroDivisionError):
        t.pivot(2, 1)            # a_{2,1} == 0
    assert np.array_equal(t.toArray(), before)


def test_unbounded_raises_assertion():
    T = np.array([[0.0, -1.0, 0.0], [1.0, -1.0, 1.0]])   # min -x, x - s... x unbounded
    t = Tableau.fromArray(T)
    s = Simplex(t)
    assert s.findPivotStandard() == "unbounded"
    with pytest.raises(AssertionError, match="unbounded"):
        s.solve()


def test_optimal_at_start_and_cap():
    T = gen.tableau("mixed", 40, 40, 12)
    e = engine_of(T)
    st, npiv, _ = e.solve(max_pivots=5)
    assert st == _lib.CAP_REACHED and npiv == 5
    e2 = engine_of(T)
    st, npiv, _ = e2.solve()
    assert st == _lib.OPTIMAL
    st, npiv, _ = e2.solve()
    assert st == _lib.OPTIMAL and npiv == 0


# ------------------------------------------------- sizes, ragged edges
@pytest.mark.parametrize("kind,m,ns,k", [
    ("tall", 1, 1, 3), ("mixed", 1, 5, 3), ("mixed", 3, 60, 10), ("tall", 5, 63, 10),
    ("tall", 257, 64, 30), ("mixed", 300, 191, 30), ("tall", 513, 7, 20),
    ("tall", 1000, 2, 10), ("tall", 2, 5000, 10), ("mixed", 255, 129, 40),
    # two rows per lane (> 256 blocks x 64 rows), 32768 rows, past it (four
    # rows per lane since round 3), past 256 x 256 columns
    ("tall", 16500, 3, 12), ("tall", 32768, 9, 8), ("tall", 32769, 3, 6), ("tall", 2, 66000, 6),
])
@pytest.mark.parametrize("block", [1, 7, 32, 48])
def test_ragged_shapes_bit_exact(kind, m, ns, k, block, select_mode):
    T = gen.tableau(kind, m, ns, 77)
    e = engine_of(T, block)
    st, done = e.run(_lib.RULE_STANDARD, k)
    o = F64Tableau(T)
    ost, olog = o.run(0, k)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    no_fallback(e)


@pytest.mark.parametrize("block", [1, 32, 44, 64])
def test_cfg3_full_size_bit_exact(block, select_mode):
    """4096 x 8192 (the 1-GPU roofline config): 40 standard pivots, whole
    268 MB tableau bit-identical to the f64 oracle."""
    T = gen.tableau("mixed", 4096, 4096, 3)
    e = engine_of(T, block)
    st, done = e.run(_lib.RULE_STANDARD, 40)
    assert st == _lib.PIVOTED and done == 40
    o = F64Tableau(T)
    _, olog = o.run(0, 40)
    assert e.log().tolist() == olog.tolist()
    D = e.download()
    assert np.array_equal(D, o.T)
    # size-independent properties: basic columns are exact unit vectors
    for r, c in e.log().tolist()[-3:]:
        col = D[:, 1 + c]
        assert col[1 + r] == 1.0 and np.count_nonzero(col) == 1


# ------------------------------------------------------------ sharding
@pytest.fixture(params=["peer", "rccl"])
def shard_mode(request, monkeypatch):
    """row-sharded pivot selection: one persistent kernel per shard with the
    device-side exchange (default), or the per-pivot kernels with one
    (emulated) RCCL collective per pivot"""
    monkeypatch.setenv("LPGPU_PEER", "1" if request.param == "peer" else "0")
    return request.param


@pytest.mark.parametrize("block", [1, 6, 32, 48])
@pytest.mark.parametrize("nshards", [1, 2, 3, 5, 8])
def test_sharded_group_invariance(nshards, block, shard_mode):
    """Row-sharded protocol (allreduce-min + slot allgather) emulated in one
    process: identical sequence and bit-identical rows for any shard count."""
    T = gen.tableau("mixed", 300, 200, 9)
    m, n = T.shape[0] - 1, T.shape[1] - 1
    ref = engine_of(T)
    st0, npiv0, nstd0 = ref.solve()
    grp = _lib.create_group(m, n, nshards)
    for g in grp:
        g.upload(T)
    grp[0].set_block(block)
    st, npiv, nstd = grp[0].solve()
    assert (st, npiv, nstd) == (st0, npiv0, nstd0)
    assert grp[0].log().tolist() == ref.log().tolist()
    D = ref.download()
    for g in grp:
        b, c = g.row_begin, g.row_count
        assert np.array_equal(g.rows(0, 1), D[:1])
        assert np.array_equal(g.rows(1 + b, c), D[1 + b:1 + b + c])
    for g in reversed(grp):
        g.close()


def test_sharded_group_explicit_and_checked_pivots():
    T = gen.tableau("mixed", 64, 64, 4)
    m, n = T.shape[0] - 1, T.shape[1] - 1
    grp = _lib.create_group(m, n, 4)
    for g in grp:
        g.upload(T)
    o = F64Tableau(T)
    r, c = o.find(0)
    assert grp[0].find(_lib.RULE_STANDARD, False) == (r, c)
    wrong = next(i for i in range(m) if i != r and T[1 + i, 1 + c] > 0)
    assert grp[0].pivot_checked(wrong, c) == _lib.BAD_PIVOT
    assert grp[0].pivot_checked(r, c) == _lib.PIVOTED
    o.pivot(r, c)
    assert grp[2].pivot(5, 3) == _lib.PIVOTED
    o.pivot(5, 3)
    for g in grp:
        b, cnt = g.row_begin, g.row_count
        assert np.array_equal(g.rows(1 + b, cnt), o.T[1 + b:1 + b + cnt])
    for g in reversed(grp):
        g.close()


def test_rccl_single_rank_communicator():
    """The RCCL transport with a 1-rank communicator drives the sharded
    kernels end to end (the 8-rank job differs only in nranks)."""
    T = gen.tableau("mixed", 200, 150, 21)
    m, n = T.shape[0] - 1, T.shape[1] - 1
    uid = _lib.comm_unique_id()
    e = _lib.create_sharded(m, n, 0, 1, uid)
    e.upload(T)
    st, npiv, _ = e.solve()
    ref = engine_of(T)
    ref.solve()
    assert e.log().tolist() == ref.log().tolist()
    assert np.array_equal(e.rows(0, m + 1), ref.download())


def test_sweep_kernel_event_timing():
    T = gen.tableau("mixed", 512, 512, 7)
    e = engine_of(T, 4)
    e.profile(True)
    e.run(_lib.RULE_STANDARD, 10)      # sweeps after pivots 4, 8 and 10
    ms, n = e.update_time()
    assert n == 3 and ms > 0


def test_block_size_invariance(select_mode):
    """every deferral depth gives the same bits (the sweep replays the exact
    per-pivot float64 operations)"""
    T = gen.tableau("mixed", 200, 300, 5)
    outs = []
    for block in (1, 2, 3, 8, 13, 31, 32, 33, 44, 48, 57, 64):
        e = engine_of(T, block)
        e.run(_lib.RULE_STANDARD, 70)
        outs.append((e.log().tolist(), e.download()))
    for log, D in outs[1:]:
        assert log == outs[0][0]
        assert np.array_equal(D, outs[0][1])


def test_find_without_pivot_leaves_tableau_untouched(shard_mode):
    T = gen.tableau("mixed", 64, 64, 8)
    for grp in ([engine_of(T)], _lib.create_group(64, 128, 3)):
        for g in grp:
            g.upload(T)
        o = F64Tableau(T)
        assert grp[0].find(_lib.RULE_STANDARD, False) == o.find(0)
        assert grp[0].find(_lib.RULE_MIN_INDEX, False) == o.find(1)
        st, done = grp[0].run(_lib.RULE_STANDARD, 5)
        o.run(0, 5)
        for g in grp:
            b, c = g.row_begin, g.row_count
            assert np.array_equal(g.rows(1 + b, c), o.T[1 + b:1 + b + c])
        for g in reversed(grp):
            g.close()


def _straddle_tableau():
    T = np.zeros((5, 6))
    T[0, 1] = -1.0
    T[1:, 0] = [1.2, 1.0, 0.9, 2.0]
    T[1:, 1] = 1.0
    T[1:, 2:] = np.eye(4)
    return T


@pytest.mark.parametrize("kind,tie,nshards,k", [
    ("straddle", 0.25, 2, 1), ("mixed", 0.25, 3, 40), ("mixed", 0.02, 4, 60), ("tall", 0.1, 5, 40),
])
def test_sharded_one_exchange_band_and_straddle(kind, tie, nshards, k, shard_mode):
    """The one-allgather protocol's band test, and its rare two-exchange
    recovery when a near-tie straddles the band (oracle/sharded_model.py)."""
    T = _straddle_tableau() if kind == "straddle" else gen.tableau(kind, 48, 32, 23)
    m, n = T.shape[0] - 1, T.shape[1] - 1
    grp = _lib.create_group(m, n, nshards)
    for g in grp:
        g.upload(T)
    grp[0].set_tol(ratio_tie=tie)
    grp[0].set_block(4)
    st, done = grp[0].run(_lib.RULE_STANDARD, k)
    o = F64Tableau(T, {"ratio_tie": tie})
    ost, olog = o.run(0, k)
    assert grp[0].log().tolist() == olog.tolist()
    for g in grp:
        b, c = g.row_begin, g.row_count
        assert np.array_equal(g.rows(1 + b, c), o.T[1 + b:1 + b + c])
    if kind == "straddle":
        assert olog.tolist() == [[1, 0]]
    for g in reversed(grp):
        g.close()


@pytest.mark.parametrize("ns", [12200, 13300])
def test_one_xcd_selection_at_lds_edge(ns):
    """wide tableaux whose persistent selection blocks need 66-73 KB of LDS
    each (two per CU on one XCD, the edge of group_blocks_xcd's sizing):
    the launch must not stall and the rows stay bit-identical to the oracle"""
    T = gen.tableau("tall", 4096, ns, 17)
    e = engine_of(T, 32)
    st, done = e.run(_lib.RULE_STANDARD, 40)
    o = F64Tableau(T)
    ost, olog = o.run(0, 40)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    no_fallback(e)
    e.close()


@pytest.mark.parametrize("m,ns,block", [(10000, 300, 32), (16000, 600, 7), (8192, 2000, 16)])
def test_one_xcd_selection_block_count(m, ns, block, select_mode):
    """tall, narrow tableaux: 125-250 selection blocks whose LDS would let
    far more than four share a CU; one XCD holds them only if at most one
    single-wave block per SIMD is assumed (otherwise the launch stalls and
    times out) -- same pivots and bit-identical rows as the oracle"""
    T = gen.tableau("tall", m, ns, 23)
    e = engine_of(T, block)
    st, done = e.run(_lib.RULE_STANDARD, 48)
    o = F64Tableau(T)
    ost, olog = o.run(0, 48)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    no_fallback(e)
    e.close()
