"""Round 3 parity on the exact timed configurations (MI355X, through the C-ABI).

* the reference's own pivots at the headline size: tests/golden/r3.json holds
  the first 10 standard-rule pivots and the exact objective the reference
  (lpsol, exact Fractions) produced on the bench's cfg3 tableau
  (make_golden.py --headline; /root/reference/lpsol/simplex.py:251-284,
  tableau.py:295-308);
* the bench's own configurations -- cfg3 and cfg4 at the engine's automatic
  pivots per sweep, the persistent selection kernel the bench times, two
  full groups and a partial one -- bit-exact against oracle/lp_f64.c;
* cfg4 as 8 in-process row shards (the 8-GPU layout on one device) the same.
"""
from fractions import Fraction

import numpy as np
import pytest

from conftest import load_golden

from lpsol_amd import _lib
from lpsol_amd import generators as gen
from oracle.f64 import F64Tableau

pytestmark = pytest.mark.gpu

R3 = load_golden("r3.json")
REL = 1e-9
CFG3 = ("mixed", 4096, 4096, 3)
CFG4 = ("tall", 32768, 8192, 3)


@pytest.fixture(scope="module", autouse=True)
def gpu():
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"


def _engine(T, block=0, xcd_shards=True):
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(block)
    if not xcd_shards:
        e.set_xcd_shards(False)
    return e


@pytest.fixture(scope="module")
def cfg3():
    return gen.tableau(*CFG3)


def test_cfg3_reference_prefix(cfg3):
    """the reference's own first 10 pivots of the cfg3 bench tableau: same
    (row, column) sequence, objective within 1e-9 of its exact rational, and
    the whole tableau bit-identical to the f64 restatement"""
    fx = R3["standard_k"][0]
    assert gen.digest(cfg3) == fx["sha256"]
    e = _engine(cfg3)
    st, done = e.run(_lib.RULE_STANDARD, fx["k"])
    assert st == _lib.PIVOTED and done == fx["k"]
    assert e.log().tolist() == fx["seq"]
    obj = float(Fraction(fx["objective"]))
    assert abs(e.objective() - obj) <= REL * max(1.0, abs(obj))
    o = F64Tableau(cfg3)
    o.run(0, fx["k"])
    assert np.array_equal(e.download(), o.T)
    e.close()


@pytest.mark.parametrize("block", [0, 48])
def test_cfg3_timed_configuration(cfg3, block):
    """cfg3 as the bench runs it: the automatic pivots per sweep (and 48),
    the one-XCD selection kernel, 136 pivots (two full groups and a partial
    one at 64; 2 x 48 + 40 at 48), no fallback, bit-exact"""
    e = _engine(cfg3, block)
    k = 136
    st, done = e.run(_lib.RULE_STANDARD, k)
    assert st == _lib.PIVOTED and done == k
    assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
    geo = e.geometry()
    assert geo["kernel"] == "k_sel" and geo["on_one_xcd"], geo
    if block == 0:
        assert e.get_block() in (48, 64)
    o = F64Tableau(cfg3)
    _, olog = o.run(0, k)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    e.close()


@pytest.fixture(scope="module")
def cfg4_136():
    """cfg4 after 136 standard pivots on the f64 oracle (host threads)"""
    T = gen.tableau(*CFG4)
    o = F64Tableau(T)
    _, olog = o.run(0, 136)
    return T, o.T, olog


@pytest.mark.parametrize("xcd_shards", [True, False])
def test_cfg4_timed_configuration(cfg4_136, xcd_shards):
    """cfg4 on one GPU as the bench runs it: 64 pivots per sweep (auto),
    the persistent selection as 8 XCD shards of k_sel (the default) or
    k_group's two-level exchange, 136 pivots, no fallback, bit-exact"""
    T, want, olog = cfg4_136
    e = _engine(T, 0, xcd_shards)
    st, done = e.run(_lib.RULE_STANDARD, 136)
    assert st == _lib.PIVOTED and done == 136
    assert e.get_block() == 64
    assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
    geo = e.geometry()
    if xcd_shards:
        assert geo["kernel"] == "k_sel" and geo["xcd_shards"] == 8 and geo["xcd_shards_engaged"], geo
    else:
        assert geo["kernel"] == "k_group" and geo["two_level_engaged"], geo
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), want)
    e.close()


def test_cfg4_eight_shards_timed(cfg4_136):
    """cfg4 as 8 in-process row shards of 4096 rows at the automatic pivots
    per sweep: 136 pivots, no fallback, every shard's rows bit-exact"""
    T, want, olog = cfg4_136
    grp = _lib.create_group(T.shape[0] - 1, T.shape[1] - 1, 8)
    for g in grp:
        g.upload(T)
    st, done = grp[0].run(_lib.RULE_STANDARD, 136)
    assert done == 136
    assert grp[0].exchange_path() == (_lib.PATH_PEER, 0)
    assert grp[0].log().tolist() == olog.tolist()
    assert np.array_equal(grp[0].rows(0, 1), want[:1])
    for g in grp:
        b, c = g.row_begin, g.row_count
        assert np.array_equal(g.rows(1 + b, c), want[1 + b:1 + b + c])
    for g in reversed(grp):
        g.close()


@pytest.mark.parametrize("m,ns,kind", [(4096, 40, "tall"), (1000, 3000, "mixed"), (64, 100, "mixed"),
                                       (4000, 200, "mixed")])
@pytest.mark.parametrize("block", [8, 32, 64])
def test_sel_shapes_bit_exact(m, ns, kind, block):
    """the one-XCD kernel on other shapes and depths (1, 2 and 4 columns per
    lane, blocks with no own columns, ragged last blocks)"""
    T = gen.tableau(kind, m, ns, 7)
    e = _engine(T, block)
    o = F64Tableau(T)
    st, done = e.run(_lib.RULE_STANDARD, 150)
    ost, olog = o.run(0, 150)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    assert e.geometry()["kernel"] == "k_sel"
    e.close()


# ------------------------------------------- the two-level exchange's rare paths
TALL = ("tall", 16500, 40, 36)


def test_two_level_timeout_recovery(monkeypatch):
    """fault injection on a shape that takes k_group's two-level
    exchange (16500 rows, blocks spread over the XCDs): block 1 withholds a
    ratio summary, its XCD group's combine times out, the host redoes the
    group on the per-pivot kernels -- sequence and tableau as without it"""
    monkeypatch.setenv("LPGPU_FAULT", "1:3")
    monkeypatch.setenv("LPGPU_SPIN_MAX", "20000")
    monkeypatch.delenv("LPGPU_STRICT", raising=False)
    T = gen.tableau(*TALL)
    e = _engine(T, 64, False)
    st, done = e.run(_lib.RULE_STANDARD, 40)
    o = F64Tableau(T)
    ost, olog = o.run(0, 40)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    assert e.exchange_path() == (_lib.PATH_KERNELS, 1)
    e.close()


def test_two_level_objective_increased():
    """Simplex.solve's 'objective value increased' stop
    (simplex.py:133) on the two-level exchange: a negative b makes the first
    pivot raise the objective; status, pivots and tableau as the f64 oracle's"""
    T = gen.tableau(*TALL)
    o0 = F64Tableau(T)
    r, c = o0.find(0)
    T[1 + r, 0] = -1.0 / 64           # the row the ratio test picks first
    e = _engine(T, 64, False)
    st, npiv, nstd = e.solve()
    o = F64Tableau(T)
    ost, olog, onstd = o.solve()
    assert st == ost == _lib.OBJ_INCREASED
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    geo = e.geometry()
    assert geo["kernel"] == "k_group" and geo["two_level_engaged"], geo
    e.close()


def test_tall_40000_rows_persistent():
    """the persistent selection past 32768 rows per device (four
    own rows per lane): a 40000 x 64 tall tableau stays on PATH_PERSISTENT,
    150 pivots bit-exact (auto pivots per sweep and 64)"""
    T = gen.tableau("tall", 40000, 64, 5)
    o = F64Tableau(T)
    ost, olog = o.run(0, 150)
    for block in (0, 64):
        e = _engine(T, block)
        st, done = e.run(_lib.RULE_STANDARD, 150)
        assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
        assert e.geometry()["rpl"] == 4, e.geometry()
        assert e.log().tolist() == olog.tolist()
        assert np.array_equal(e.download(), o.T)
        e.close()


_COOP_CHILD = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1] + "/linear-program-solver_amd", sys.argv[1]]
from lpsol_amd import _lib, generators as gen
from oracle.f64 import F64Tableau
_lib.load()
kind, m, ns, block, kernel = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
T = gen.tableau(kind, m, ns, 9)
e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
e.upload(T)
e.set_block(block)
st, done = e.run(_lib.RULE_STANDARD, 70)
o = F64Tableau(T)
ost, olog = o.run(0, 70)
assert e.log().tolist() == olog.tolist()
assert np.array_equal(e.download(), o.T)
assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0), e.exchange_path()
assert e.geometry()["kernel"] == kernel, e.geometry()
print("ok", e.geometry())
"""


@pytest.mark.parametrize("kind,m,ns,block,kernel", [
    ("mixed", 4096, 4096, 0, "k_sel"),     # cfg3's one-XCD geometry
    ("tall", 32768, 8192, 0, "k_sel"),     # cfg4's XCD shards (512 blocks, 2 per CU)
    ("tall", 36000, 300, 64, "k_group"),   # k_group spread, two rows per lane
    ("tall", 40000, 64, 64, "k_group"),    # four rows per lane
])
def test_persistent_geometry_admitted_by_cooperative_launch(kind, m, ns, block, kernel):
    """the occupancy sizing of every persistent selection kind, checked by the
    runtime: LPGPU_COOP=1 launches them cooperatively, which the runtime
    refuses (hipErrorCooperativeLaunchTooLarge -> LP_DEVICE_ERROR) unless every
    block of the grid is resident at once; results bit-exact, no fallback"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LPGPU_COOP="1", LPGPU_STRICT="1")
    r = subprocess.run([sys.executable, "-c", _COOP_CHILD, root, kind, str(m), str(ns), str(block), kernel],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
