"""Round 5 GPU test (MI355X, through the C-ABI), VERDICT r4 (next 7): the
reference's own 80 cfg3 pivots (tests/golden/r5.json) through the engine as
the bench runs it, across the boundary between the first bench group and the
second."""
from fractions import Fraction

import numpy as np
import pytest
from conftest import load_golden

from lpsol_amd import _lib, generators as gen
from oracle.f64 import F64Tableau

pytestmark = pytest.mark.gpu


def test_cfg3_reference_prefix_across_group_boundary():
    """the reference's first 80 standard-rule pivots on the bench's cfg3
    tableau (tests/golden/r5.json, captured from /root/reference,
    make_golden.py --headline-prefix 80): automatic depth 64, the one-XCD
    k_sel, no fallback -- group 1 of 64 pivots, a whole sweep, then group 2
    -- the same (row, column) sequence, the objective within 1e-9 of the
    reference's exact rational, the tableau bit-identical to the f64
    restatement (simplex.py:251-284, tableau.py:295-308)"""
    fx = load_golden("r5.json")["standard_k"][0]
    assert fx["k"] >= 72
    g = fx["gen"]
    T = gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
    assert gen.digest(T) == fx["sha256"]
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(0)
    assert e.get_block() == 64
    st, done = e.run(_lib.RULE_STANDARD, fx["k"])
    assert st == _lib.PIVOTED and done == fx["k"]
    assert e.geometry()["kernel"] == "k_sel" and e.geometry()["on_one_xcd"]
    assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
    assert e.log().tolist() == fx["seq"]
    obj = float(Fraction(fx["objective"]))
    assert abs(e.objective() - obj) <= 1e-9 * max(1.0, abs(obj))
    o = F64Tableau(T)
    o.run(0, fx["k"])
    assert np.array_equal(e.download().view(np.uint64), o.T.view(np.uint64))
    e.close()
