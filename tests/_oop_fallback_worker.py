"""Child process of test_gpu_r6.py::test_out_of_place_fallbacks:
a tableau beyond 512 MiB takes out-of-place sweeps only where the second
buffer fits with room to spare, and falls back to in-place sweeps when it
does not.  The knobs are read once per process, so each setting runs here:

* no knob: two buffers (out of place);
* LPGPU_OOP_ROOM_MB=<huge>: hipMemGetInfo shows too little room -> in place;
* LPGPU_OOP_FAIL_ALLOC=1: the second buffer's allocation fails -> in place.

EXPECT_BUFFERS names the expected count; the run (136 pivots at the
automatic depth: two full groups and a padded one) must match
oracle/lp_f64.c bit for bit either way.  Prints "ALL OK" at the end."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
sys.path.insert(0, ROOT)

from lpsol_amd import _lib, generators as gen  # noqa: E402
from oracle.f64 import F64Tableau  # noqa: E402


def main():
    want = int(os.environ["EXPECT_BUFFERS"])
    T = gen.tableau("tall", 8500, 8192, 23)       # 8501 x 8320 x 8 B = 566 MB > 512 MiB
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    nbuf = e.sweep_buffers()
    print("sweep buffers", nbuf, "expected", want, flush=True)
    st, done = e.run(_lib.RULE_STANDARD, 136)
    o = F64Tableau(T.copy())
    _, olog = o.run(0, 136)
    ok_seq = done == len(olog) and e.log().tolist() == olog.tolist()
    got = e.download()
    ok_bits = np.array_equal(got.view(np.uint64), o.T.view(np.uint64))
    print("pivots", done, "sequence", "ok" if ok_seq else "MISMATCH", "tableau", "ok" if ok_bits else "MISMATCH",
          "path", e.exchange_path(), flush=True)
    e.close()
    if nbuf != want or not ok_seq or not ok_bits:
        sys.exit(1)
    print("ALL OK")


if __name__ == "__main__":
    main()
