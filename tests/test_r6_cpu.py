"""Round 6, CPU: the reference's own pivots on the HEADLINE tableau -- cfg4,
32768 x 8192 G_tall seed 3, the bench's default workload (tests/golden/r6.json:
make_golden.py --headline-prefix K --workload cfg4 --out r6.json, the
reference lpsol run in the build container, checkpointed after every pivot;
/root/reference/lpsol/simplex.py:251-284, tableau.py:295-308).

The float64 oracle (oracle/lp_f64.c, the engine's contract) reproduces the
reference's sequence on the full 32769 x 8193 tableau, its objective within
1e-9 (relative) of the reference's exact rational after the last captured
pivot.  (missing 3: parity at the benched shape rested on
lp_f64.c alone.)"""
import os
from fractions import Fraction

import pytest
from conftest import GOLDEN, load_golden

from lpsol_amd import generators as gen
from oracle.f64 import F64Tableau

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(GOLDEN, "r6.json")),
                                reason="tests/golden/r6.json not captured")


def _fixture():
    return load_golden("r6.json")["standard_k"][0]


def test_r6_fixture_is_the_bench_workload():
    fx = _fixture()
    assert fx["workload"] == "cfg4" and fx["gen"] == {"kind": "tall", "m": 32768, "ns": 8192, "seed": 3}
    assert (fx["m"], fx["n"]) == (32768, 8192)
    assert fx["k"] == len(fx["seq"]) >= 8 and fx["end"] is None
    assert len(fx["ref_seconds_cumulative"]) == fx["k"]


def test_f64_oracle_matches_reference_at_cfg4():
    fx = _fixture()
    g = fx["gen"]
    T = gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
    assert gen.digest(T) == fx["sha256"]
    t = F64Tableau(T)
    st, log = t.run(0, fx["k"])
    assert log.tolist() == fx["seq"]
    obj = float(Fraction(fx["objective"]))
    assert abs(t.objective() - obj) <= 1e-9 * max(1.0, abs(obj))
