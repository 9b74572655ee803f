"""Round 4, CPU: the reference's own pivots on the bench's cfg3 tableau extended
to one full bench group (tests/golden/r4.json: make_golden.py --headline-prefix,
the reference lpsol run in the build container, its exact objective after
every pivot -- /root/reference/lpsol/simplex.py:251-284, tableau.py:295-308).

* the fixture agrees with round 3's independent 10-pivot capture (r3.json);
* the float64 oracle (oracle/lp_f64.c, the engine's contract) reproduces the
  reference's whole pivot sequence, and its objective is within 1e-9
  (relative) of the reference's exact rational."""
from fractions import Fraction

import pytest

from conftest import load_golden

from lpsol_amd import generators as gen
from oracle.f64 import F64Tableau

R3 = load_golden("r3.json")["standard_k"][0]
R4 = load_golden("r4.json")["standard_k"][0]


def test_prefix_fixture_consistent_with_round3_capture():
    assert R4["sha256"] == R3["sha256"] and R4["gen"] == R3["gen"]
    assert R4["k"] == len(R4["seq"]) >= 64
    assert R4["seq"][:R3["k"]] == R3["seq"]
    assert len(R4["ref_seconds_cumulative"]) == R4["k"]


def test_f64_oracle_matches_reference_full_group_at_cfg3():
    g = R4["gen"]
    T = gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
    assert gen.digest(T) == R4["sha256"]
    t = F64Tableau(T)
    st, log = t.run(0, R4["k"])
    assert log.tolist() == R4["seq"]
    obj = float(Fraction(R4["objective"]))
    assert abs(t.objective() - obj) <= 1e-9 * max(1.0, abs(obj))
