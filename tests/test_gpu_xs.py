"""The XCD-sharded persistent selection (k_sel<XS>, select.hip) on ONE device,
through the C-ABI: a tableau too tall for one XCD's 64 x 64 rows runs as 8 row
shards, one per XCD, in one launch.  Each shard's blocks own its rows and all
the variable columns; the shards exchange their leaving-row candidates and
every shard forms the winner's pivot row from the shared tableau.  The pivot
sequence and every row must stay bit-identical to oracle/lp_f64.c, which
restates /root/reference/lpsol/simplex.py:251-284 (findPivotStandard),
:218-249 (findPivotMinIndex), :110-148 (solve) and tableau.py:295-308 (pivot).
"""
import numpy as np
import pytest

from lpsol_amd import _lib
from lpsol_amd import generators as gen
from oracle.f64 import F64Tableau

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu():
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"


def _engine(T, block, tie=None):
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(block)
    if tie is not None:
        e.set_tol(cost_tie=tie, ratio_tie=tie)
    return e


def _xs(e):
    geo = e.geometry()
    assert geo["kernel"] == "k_sel" and geo["xcd_shards"] == 8, geo
    assert geo["xcd_shards_engaged"], geo
    return geo


@pytest.mark.parametrize("kind,m,ns,seed", [
    ("tall", 4097, 40, 41),        # the shortest XS tableau: 513-row shards of 9 blocks
    ("mixed", 4160, 900, 42),      # ragged last shard, one own column per lane
    ("mixed", 9000, 500, 43),      # n = 9500: 64 blocks per shard (fewer leave too little LDS)
    ("tall", 20000, 200, 44),
    ("tall", 32768, 40, 45),       # the tallest: 4096-row shards of 64 blocks
])
@pytest.mark.parametrize("block", [48, 64])
def test_xs_shapes_bit_exact(kind, m, ns, seed, block):
    T = gen.tableau(kind, m, ns, seed)
    e = _engine(T, block)
    st, done = e.run(_lib.RULE_STANDARD, 150)
    o = F64Tableau(T)
    ost, olog = o.run(0, 150)
    assert done == len(olog)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
    _xs(e)
    e.close()


@pytest.mark.parametrize("rule", [_lib.RULE_STANDARD, _lib.RULE_MIN_INDEX])
@pytest.mark.parametrize("kind,tie", [("pos", 0.3), ("tall", 0.05), ("pos", 1e-12)])
def test_xs_wide_tie_bands(rule, kind, tie):
    """wide tie bands: the first shard inside the global band often offers a
    candidate outside it (a straddle answered by that shard's rescan), and
    blocks' candidates straddle inside a shard"""
    T = gen.tableau(kind, 6000, 60, 46)
    e = _engine(T, 64, tie)
    st, done = e.run(rule, 80)
    o = F64Tableau(T, {"cost_tie": tie, "ratio_tie": tie})
    ost, olog = o.run(0 if rule == _lib.RULE_STANDARD else 1, 80)
    assert done == len(olog)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
    _xs(e)
    e.close()


@pytest.mark.parametrize("kind,seed", [("pos", 47), ("mixed", 48)])
def test_xs_solve(kind, seed):
    """a whole Simplex.solve on the XCD shards (stall counter, min-index
    switch, optimality): status, standard-rule count, sequence, tableau"""
    T = gen.tableau(kind, 5000, 120, seed)
    e = _engine(T, 0)
    st, npiv, nstd = e.solve()
    o = F64Tableau(T)
    ost, olog, onstd = o.solve()
    assert (st, nstd) == (ost, onstd)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    assert e.get_block() == 64
    _xs(e)
    e.close()


def test_xs_objective_increased():
    """Simplex.solve's 'objective value increased' stop (simplex.py:133) on
    the XCD shards: a negative b makes the first pivot raise the objective"""
    T = gen.tableau("tall", 16500, 40, 36)
    o0 = F64Tableau(T)
    r, c = o0.find(0)
    T[1 + r, 0] = -1.0 / 64
    e = _engine(T, 64)
    st, npiv, nstd = e.solve()
    o = F64Tableau(T)
    ost, olog, onstd = o.solve()
    assert st == ost == _lib.OBJ_INCREASED
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    _xs(e)
    e.close()


def test_xs_timeout_recovery(monkeypatch):
    """fault injection: shard 0's block 1 withholds a ratio summary, every
    shard's exchange times out, the host redoes the group on the per-pivot
    kernels -- sequence and tableau as without it"""
    monkeypatch.setenv("LPGPU_FAULT", "1:3")
    monkeypatch.setenv("LPGPU_SPIN_MAX", "20000")
    monkeypatch.delenv("LPGPU_STRICT", raising=False)
    T = gen.tableau("tall", 16500, 40, 36)
    e = _engine(T, 64)
    assert e.geometry()["xcd_shards"] == 8
    st, done = e.run(_lib.RULE_STANDARD, 40)
    o = F64Tableau(T)
    ost, olog = o.run(0, 40)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    assert e.exchange_path() == (_lib.PATH_KERNELS, 1)
    e.close()


def test_xs_and_k_group_agree_with_explicit_pivots():
    """explicit pivots (Tableau.pivot) between chained runs on a tall tableau:
    the XCD shards and k_group give the same rows as the oracle"""
    T = gen.tableau("mixed", 8200, 500, 49)
    o = F64Tableau(T)
    _, l1 = o.run(0, 30)
    r, c = o.find(0)
    for xs in (True, False):
        e = _engine(T, 64)
        e.set_xcd_shards(xs)
        e.run(_lib.RULE_STANDARD, 30)
        assert e.log().tolist() == l1.tolist()
        e.pivot(r, c)
        e.run(_lib.RULE_STANDARD, 20)
        if xs:
            _xs(e)
        want = F64Tableau(T)
        want.run(0, 30)
        want.pivot(r, c)
        want.run(0, 20)
        assert np.array_equal(e.download(), want.T)
        e.close()


def test_xs_frontend_simplex_solve():
    """the lpsol-compatible front-end on a tableau taller than one XCD:
    Simplex.solve (simplex.py:110-148) runs lp_solve on the XCD shards and
    replays the device log through _pivot; the basis follows the oracle's
    pivot sequence, the objective and the downloaded tableau match it"""
    from lpsol_amd import Simplex, Tableau
    T = gen.tableau("pos", 4500, 60, 50)
    tab = Tableau.fromArray(T)
    s = Simplex(tab)
    s.solve()
    o = F64Tableau(T)
    ost, olog, _ = o.solve()
    eng = tab._engine()
    assert eng.log().tolist() == olog.tolist()
    assert eng.geometry()["xcd_shards"] == 8
    assert abs(s.getObjValue() - o.objective()) <= 1e-9 * max(1.0, abs(o.objective()))
    assert np.array_equal(tab.toArray(), o.T)
    bfs = list(range(T.shape[1] - 1 - (T.shape[0] - 1), T.shape[1] - 1))   # the slacks start basic
    for r, c in olog.tolist():
        bfs[r] = c
    assert s.getBasicSequence() == bfs
