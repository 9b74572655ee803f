"""Round 5, CPU: the reference's own pivots on the bench's cfg3 tableau past
the first bench group -- 80 pivots, the second group (pivots 65..80) starting
after a whole sweep (tests/golden/r5.json: make_golden.py --headline-prefix 80
--out r5.json, the reference lpsol run in the build container with its exact
objective after every pivot; /root/reference/lpsol/simplex.py:251-284,
tableau.py:295-308).

* the fixture agrees with round 4's 64-pivot capture (r4.json) on its prefix;
* the float64 oracle (oracle/lp_f64.c, the engine's contract) reproduces the
  reference's whole sequence across the group boundary, its objective within
  1e-9 (relative) of the reference's exact rational."""
from fractions import Fraction

from conftest import load_golden

from lpsol_amd import generators as gen
from oracle.f64 import F64Tableau

R4 = load_golden("r4.json")["standard_k"][0]
R5 = load_golden("r5.json")["standard_k"][0]


def test_r5_prefix_fixture_extends_round4_capture():
    assert R5["sha256"] == R4["sha256"] and R5["gen"] == R4["gen"]
    assert R5["k"] == len(R5["seq"]) >= 72                  # past pivot 64: a sweep boundary
    assert R5["seq"][:R4["k"]] == R4["seq"]
    assert len(R5["ref_seconds_cumulative"]) == R5["k"]


def test_f64_oracle_matches_reference_across_group_boundary_at_cfg3():
    g = R5["gen"]
    T = gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
    assert gen.digest(T) == R5["sha256"]
    t = F64Tableau(T)
    st, log = t.run(0, R5["k"])
    assert log.tolist() == R5["seq"]
    obj = float(Fraction(R5["objective"]))
    assert abs(t.objective() - obj) <= 1e-9 * max(1.0, abs(obj))
