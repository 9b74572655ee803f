"""Child process of test_gpu_r2.py::test_sweep_grid_modes_bit_exact (and
test_gpu_r5.py's tail test): the sweep's grid switches (LPGPU_SWEEP_TAIL,
LPGPU_SWEEP_CUS) are read once per process, so each setting
runs here, over several shapes (or SWEEP_SHAPES), against the f64 oracle.
Prints one line per shape and "ALL OK" at the end."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
sys.path.insert(0, ROOT)

from lpsol_amd import _lib, generators as gen  # noqa: E402
from oracle.f64 import F64Tableau  # noqa: E402

# (kind, m, ns, pivots, pivots per sweep): strips of 1, 2, 9 and 17 x 128
# columns, row counts off the 4-row batch, tall and square
SHAPES = [("tall", 777, 64, 20, 8), ("mixed", 333, 100, 24, 16), ("tall", 4099, 700, 24, 16),
          ("mixed", 1500, 1000, 30, 48), ("pos", 2050, 2000, 20, 64)]


def main():
    shapes = SHAPES
    if os.environ.get("SWEEP_SHAPES"):           # "kind,m,ns,pivots,block[,rule];..."
        shapes = [(f[0], int(f[1]), int(f[2]), int(f[3]), int(f[4])) + ((int(f[5]),) if len(f) > 5 else ())
                  for f in (x.split(",") for x in os.environ["SWEEP_SHAPES"].split(";"))]
    expect_nr = int(os.environ.get("EXPECT_NR", "0"))   # the persistent selection's summaries per lane
    for shape in shapes:
        kind, m, ns, k, block = shape[:5]
        rule = shape[5] if len(shape) > 5 else 0
        T = gen.tableau(kind, m, ns, 11)
        o = F64Tableau(T.copy())
        _, olog = o.run(rule, k)
        e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
        e.upload(T)
        e.set_block(block)
        st, done = e.run(_lib.RULE_MIN_INDEX if rule else _lib.RULE_STANDARD, k)
        ok = done == len(olog) and e.log().tolist() == olog.tolist() and np.array_equal(e.download(), o.T)
        geo = e.geometry()
        if expect_nr and (geo["nr"] != expect_nr or e.exchange_path()[1] != 0):
            print(kind, m, ns, "geometry", geo, "path", e.exchange_path(), flush=True)
            ok = False
        print(kind, m, ns, "rule", rule, "pivots", done, "ok" if ok else "MISMATCH", flush=True)
        if ok and os.environ.get("SOLVE_TOO") == "1":
            # the whole solve (stall counter, min-index switch, stop rules)
            # from the same tableau, against the oracle's solve
            e.upload(T)
            o2 = F64Tableau(T.copy())
            ost, olog2, _ = o2.solve(cap=20000)
            est = e.solve(20000)
            ok = e.log().tolist() == olog2.tolist() and np.array_equal(e.download(), o2.T)
            print(kind, m, ns, "solve", len(olog2), "pivots", "ok" if ok else "MISMATCH", est, ost, flush=True)
        e.close()
        if not ok:
            sys.exit(1)
    print("ALL OK")


if __name__ == "__main__":
    main()
