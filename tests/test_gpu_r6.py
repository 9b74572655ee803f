"""Round 6 GPU tests (MI355X, through the C-ABI).

* ADVICE r5 (low, out of place): the unforced fallbacks of the out-of-place
  sweep -- too little free memory for the second buffer, or its allocation
  failing -- run in place and stay bit-exact (tests/_oop_fallback_worker.py).
* ADVICE r5 (low, ballots): a ratio-test minimum so close to DBL_MAX that
  g + tie |g| overflows.  The band is clamped to DBL_MAX (device.h
  tie_band), so lanes and blocks without a candidate (+inf) never pass the
  ballot and the leaving row is the first candidate, as oracle/lp_f64.c's
  +inf band picks it -- on the one-XCD selection and on the XCD shards.
* The 4-wave sweep's unequal row runs (launch_sweep, SWEEP_SPLIT: each
  CU's older workgroup takes the longer run): at several splits, equal runs
  included, on shapes whose runs come out even, against the f64 oracle.

Reference: /root/reference/lpsol/simplex.py:251-284 (findPivotStandard: the
ratio test's first row with the minimum ratio), tableau.py:269-280 (rowAdd).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from lpsol_amd import _lib
from oracle.f64 import F64Tableau

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("env,buffers", [({}, 2), ({"LPGPU_OOP_ROOM_MB": "100000000"}, 1),
                                         ({"LPGPU_OOP_FAIL_ALLOC": "1"}, 1)],
                         ids=["out-of-place", "no-room", "alloc-fails"])
def test_out_of_place_fallbacks(env, buffers):
    worker = os.path.join(os.path.dirname(__file__), "_oop_fallback_worker.py")
    e = dict(os.environ, EXPECT_BUFFERS=str(buffers), **env)
    e.pop("LPGPU_SWEEP_OOP", None)
    run = subprocess.run([sys.executable, "-u", worker], env=e, capture_output=True, text=True, timeout=110)
    assert run.returncode == 0 and "ALL OK" in run.stdout, run.stdout + run.stderr


def _huge_ratio_lp(m, first_candidate):
    """m constraint rows, 8 variables: column 1 enters (c_1 = -1, the most
    negative); rows before `first_candidate` have a_1 <= 0 (no ratio), the
    rest ratios b / a within a few ulps of DBL_MAX (finite) -- the band
    g + tie |g| overflows"""
    n = 8
    T = np.zeros((m + 1, n + 1))
    T[0, 1:] = [-1.0, -0.5, 0.25, 0.0, -0.25, 0.5, 0.0, 0.125]
    big = np.finfo(np.float64).max
    rng = np.random.default_rng(7)
    for i in range(1, m + 1):
        T[i, 2:] = rng.integers(-4, 5, size=n - 1) / 4.0
        if i < first_candidate:
            T[i, 0] = 1.0
            T[i, 1] = -float(rng.integers(0, 3)) / 2.0        # a <= 0: no candidate
        else:
            T[i, 0] = np.nextafter(big, 0.0) if i % 3 else big
            T[i, 1] = 1.0
    return T


@pytest.mark.parametrize("m,first", [(3000, 1700), (3000, 2), (6000, 5200)], ids=["one-xcd", "first-rows", "xcd-shards"])
def test_ratio_band_overflow_picks_first_candidate(m, first):
    T = _huge_ratio_lp(m, first)
    o = F64Tableau(T.copy())
    _, olog = o.run(0, 1)
    assert olog.tolist() == [[first - 1, 0]]
    e = _lib.Engine(m, 8)
    e.upload(T)
    e.set_block(64)
    st, done = e.run(_lib.RULE_STANDARD, 1)
    assert done == 1 and e.log().tolist() == olog.tolist(), (e.log(), olog, e.geometry())
    geo = e.geometry()
    assert geo["kernel"] == "k_sel" and (geo["xcd_shards"] == 8) == (m > 4096), geo
    e.close()


def test_sweep_clock_records():
    """the sweep's per-launch and per-block clock records (Args::sweep_clk,
    lpdiag_sweep_clocks / lpdiag_sweep_block_clocks; bench.py's
    roofline.shader_clock): one record per 64-pivot sweep launch, in launch
    order, cycles and 100 MHz ticks giving a plausible shader clock; every
    block of the latest launch recorded once"""
    from lpsol_amd import generators as gen
    T = gen.tableau("mixed", 1500, 1000, 3)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(64)
    st, done = e.run(_lib.RULE_STANDARD, 3 * 64)
    assert done == 3 * 64
    c = e.sweep_clocks()
    assert len(c) >= 2 and all(c[i + 1, 0] > c[i, 0] for i in range(len(c) - 1))
    ghz = c[:, 1] / (c[:, 2] / 1e8) / 1e9
    assert ((ghz > 0.3) & (ghz < 4.0)).all(), ghz
    b = e.sweep_block_clocks()
    assert len(b) > 0 and len(set(b[:, 0].tolist())) == len(b)
    assert (b[:, 2] >= b[:, 1]).all() and (b[:, 3] > 0).all()
    e.close()


def test_sweep_clock_ring_wraps():
    """more sweep launches than the ring holds (SWEEP_CLK_RING = 1024): the
    latest 1024 records come back, oldest first, in launch order"""
    from lpsol_amd import generators as gen
    T = gen.tableau("mixed", 512, 512, 3)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.set_block(64)
    for _ in range(20):                        # 20 x 56 = 1120 sweep launches
        e.upload(T)
        st, done = e.run(_lib.RULE_STANDARD, 56 * 64)
        assert done == 56 * 64, (st, done)
    c = e.sweep_clocks(4096)
    assert len(c) == 1024, len(c)
    assert (np.diff(c[:, 0]) > 0).all()
    assert c[-1, 0] >= 1100 and c[-1, 0] - c[0, 0] >= 1023
    ghz = c[:, 1] / (c[:, 2] / 1e8) / 1e9
    assert ((ghz > 0.3) & (ghz < 4.0)).all()
    e.close()


# (kind, m, ns, pivots, pivots per sweep): 16-32 row runs of two workgroups per
# CU (nrun even), row counts off the 8-row batch
SPLIT_SHAPES = "mixed,3001,2100,130,64;pos,2300,1500,70,64;mixed,5003,2100,70,64"


@pytest.mark.parametrize("split,oop", [("0", "0"), ("0.55", "0"), ("0.7", "0"), ("0.62", "1")])
def test_sweep_run_split_bit_exact(split, oop):
    """k_sweep_rl with the grid's first half of row runs longer than the
    second (LPGPU_SWEEP_SPLIT; the default 0.62 runs in every other test):
    the pivot sequence and every bit of the tableau as oracle/lp_f64.c's,
    in place and out of place (tableau.py:269-280)"""
    worker = os.path.join(os.path.dirname(__file__), "_sweep_env_worker.py")
    env = dict(os.environ, LPGPU_SWEEP_SPLIT=split, LPGPU_SWEEP_OOP=oop, SWEEP_SHAPES=SPLIT_SHAPES)
    run = subprocess.run([sys.executable, "-u", worker], env=env, capture_output=True, text=True, timeout=110)
    assert run.returncode == 0 and "ALL OK" in run.stdout, run.stdout + run.stderr
