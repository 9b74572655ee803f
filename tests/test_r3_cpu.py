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


def test_lost_tableau_recovers_on_load():
    """a device failure while the device copy was the only current
    one marks the tableau lost; loading a whole new tableau clears that (the
    reference has no such state), and a failed non-pivoting call never marks
    it.  Host logic only: the failure is simulated."""
    from lpsol_amd import Tableau, _lib
    from lpsol_amd.simplex import Simplex

    t = Tableau(2, 3)
    saved = t.saveJson()
    t._host_ok = False                 # the device held the only current copy
    t._device_failed()
    with pytest.raises(_lib.DeviceError):
        t.getZ()
    t.loadJson(saved)
    assert t.getZ() == 0 and t.getTableauSize() == (2, 3)

    class Boom:
        m, n = 2, 3

        def find(self, rule, do_pivot):
            raise _lib.DeviceError("injected")

    s = Simplex.__new__(Simplex)
    s._tab = t
    t._host_ok, t._dev_ok = False, True
    t._engine = lambda: Boom()
    with pytest.raises(_lib.DeviceError):
        s.findPivotStandard(False)     # no pivot: the tableau is not lost
    assert not t._lost
    with pytest.raises(_lib.DeviceError):
        s.findPivotStandard(True)      # a pivoting call: it is
    assert t._lost
