"""Round 3, CPU: the f64 oracle against the reference's own pivots at the
headline size (tests/golden/r3.json: the first 10 standard-rule pivots of the
bench's cfg3 tableau, 4096 x 8192, and the exact objective after them, captured
from /root/reference by make_golden.py --headline), and the selection
geometry query without a GPU."""
from fractions import Fraction

import pytest

from conftest import load_golden

from lpsol_amd import generators as gen
from oracle.f64 import F64Tableau

R3 = load_golden("r3.json")


@pytest.mark.parametrize("fx", R3["standard_k"], ids=[f["name"] for f in R3["standard_k"]])
def test_f64_oracle_matches_reference_at_cfg3(fx):
    g = fx["gen"]
    T = gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
    assert gen.digest(T) == fx["sha256"]
    t = F64Tableau(T)
    st, log = t.run(0, fx["k"])
    assert log.tolist() == fx["seq"]
    obj = float(Fraction(fx["objective"]))
    assert abs(t.objective() - obj) <= 1e-9 * max(1.0, abs(obj))
