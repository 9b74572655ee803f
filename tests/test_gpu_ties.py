"""Wide tie bands on ONE device (MI355X, through the C-ABI): the rare
branches of the persistent selection.

With cost_tie / ratio_tie far above their 1e-12 defaults, the first block
whose slice minimum lies inside the global tie band often reports a
candidate (the first entry inside ITS OWN, wider band) that lies outside the
global band, and the kernel must rescan that block's slice of row 0
(entering column) or its rows (leaving row) -- `combine_loaded` /
`first_in_band` in kernels.hip.  The pivot sequence and every row must stay
bit-identical to oracle/lp_f64.c, which applies the same two-pass rule
(exact minimum g, then the first index with value <= g + tie |g|) over the
whole column / row.  Covers one and two own rows per lane and every deferral
depth the auto choice uses.
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


@pytest.mark.parametrize("kind,m,ns,seed,k", [
    ("mixed", 300, 200, 31, 60),      # 64 blocks, one own row per lane
    ("pos", 700, 400, 32, 50),        # many equal costs and ratios (Q = 64 grid)
    ("tall", 16500, 40, 33, 24),      # 258+ blocks -> two own rows per lane
])
@pytest.mark.parametrize("tie", [0.05, 0.3])
@pytest.mark.parametrize("block", [8, 48, 64])
def test_single_device_wide_tie_bands(kind, m, ns, seed, k, tie, block):
    T = gen.tableau(kind, m, ns, seed)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(block)
    e.set_tol(cost_tie=tie, ratio_tie=tie)
    st, done = e.run(_lib.RULE_STANDARD, k)
    o = F64Tableau(T, {"cost_tie": tie, "ratio_tie": tie})
    ost, olog = o.run(0, k)
    assert done == len(olog)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    assert e.exchange_path()[1] == 0          # no timed-out group
    e.close()


@pytest.mark.parametrize("tie", [0.05, 0.3])
def test_single_device_wide_tie_solve(tie):
    """a whole solve (stall counter, min-index switch) under wide bands"""
    T = gen.tableau("pos", 400, 300, 34)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_tol(cost_tie=tie, ratio_tie=tie)
    st, npiv, nstd = e.solve()
    o = F64Tableau(T, {"cost_tie": tie, "ratio_tie": tie})
    ost, olog, onstd = o.solve()
    assert (st, nstd) == (ost, onstd)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    e.close()


@pytest.mark.parametrize("rule", [_lib.RULE_STANDARD, _lib.RULE_MIN_INDEX])
@pytest.mark.parametrize("tie", [1e-12, 0.3])
def test_spread_selection_two_level_exchange(rule, tie):
    """blocks spread over the XCDs (16500 rows: 136 blocks, two own rows per
    lane) exchange through their XCD's L2 and one summary per XCD
    (k_group's two-level exchange): with wide bands the group summaries'
    candidates often lie outside the global band and the kernel rescans a
    whole XCD group's rows or row-0 columns"""
    T = gen.tableau("tall", 16500, 40, 36)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(64)
    e.set_xcd_shards(False)            # k_group (the XCD-sharded k_sel: test_gpu_xs.py)
    e.set_tol(cost_tie=tie, ratio_tie=tie)
    st, done = e.run(rule, 40)
    o = F64Tableau(T, {"cost_tie": tie, "ratio_tie": tie})
    ost, olog = o.run(0 if rule == _lib.RULE_STANDARD else 1, 40)
    assert done == len(olog)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
    geo = e.geometry()                 # the two-level exchange really engaged
    assert geo["kernel"] == "k_group" and geo["two_level_engaged"], geo
    e.close()
