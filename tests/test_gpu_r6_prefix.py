"""Round 6 GPU test (MI355X, through the C-ABI), VERDICT r5 (next 3): the
reference's own first pivots on the HEADLINE tableau (cfg4, 32768 x 8192
G_tall seed 3; tests/golden/r6.json, captured from /root/reference by
make_golden.py --headline-prefix --workload cfg4) through the engine exactly
as bench.py runs it: the XCD-sharded k_sel, the automatic depth (64), the
out-of-place k_sweep_rl.

* 128 pivots (two full bench groups, each closed by a 64-pivot sweep): the
  first K are the reference's (row, column) sequence, and the whole tableau
  is bit-identical to the f64 restatement (oracle/lp_f64.c) after them;
* the same tableau re-uploaded, K pivots: the objective within 1e-9
  (relative) of the reference's exact rational.

Reference: /root/reference/lpsol/simplex.py:251-284, tableau.py:295-308."""
import os
from fractions import Fraction

import numpy as np
import pytest
from conftest import GOLDEN, load_golden

from lpsol_amd import _lib, generators as gen
from oracle.f64 import F64Tableau

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(os.path.join(GOLDEN, "r6.json")),
                                 reason="tests/golden/r6.json not captured")]


def test_cfg4_reference_prefix_as_the_bench_runs():
    fx = load_golden("r6.json")["standard_k"][0]
    k = fx["k"]
    assert k >= 8
    g = fx["gen"]
    T = gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
    assert gen.digest(T) == fx["sha256"]
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(0)
    assert e.get_block() == 64
    assert e.sweep_buffers() == 2                    # out of place, as the bench
    st, done = e.run(_lib.RULE_STANDARD, 128)
    assert st == _lib.PIVOTED and done == 128
    geo = e.geometry()
    assert geo["kernel"] == "k_sel" and geo["xcd_shards"] == 8, geo
    assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
    log = e.log().tolist()
    assert log[:k] == fx["seq"]
    o = F64Tableau(T.copy())
    _, olog = o.run(0, 128)
    assert log == olog.tolist()
    assert np.array_equal(e.download().view(np.uint64), o.T.view(np.uint64))
    del o
    # the reference's objective after its last captured pivot
    e.upload(T)
    st, done = e.run(_lib.RULE_STANDARD, k)
    assert done == k and e.log().tolist() == fx["seq"]
    obj = float(Fraction(fx["objective"]))
    assert abs(e.objective() - obj) <= 1e-9 * max(1.0, abs(obj))
    e.close()
