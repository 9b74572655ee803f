"""Child process of test_gpu_r4.py::test_out_of_place_sweep_worker: the
engine with LPGPU_SWEEP_OOP=1 (read once per process) -- k_sweep_rl reads one
tableau buffer and writes the other, and the host follows the buffer the last
sweep that ran wrote.  Every case against oracle/lp_f64.c, bit for bit:

* 136 pivots at depth 64 (two full groups, a padded one), then more runs;
* solves that end inside a batch (the later sweeps of the batch are skipped:
  the host must stay on the last buffer written);
* explicit pivots and findPivot(True) between runs (in-place sweeps on the
  current buffer), a re-upload between runs;
* a timed-out persistent group (LPGPU_FAULT, set per handle before
  set_block): its sweep is skipped, the host redoes it on the per-pivot
  kernels from the buffer that holds the group's start.
Prints one line per case and "ALL OK" at the end."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
sys.path.insert(0, ROOT)

from lpsol_amd import _lib, generators as gen  # noqa: E402
from oracle.f64 import F64Tableau  # noqa: E402


def bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint64), np.ascontiguousarray(b).view(np.uint64))


def check(name, ok):
    print(name, "ok" if ok else "MISMATCH", flush=True)
    if not ok:
        sys.exit(1)


def runs():
    T = gen.tableau("mixed", 700, 900, 41)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(64)
    o = F64Tableau(T)
    for k in (136, 70, 5, 64):
        st, done = e.run(_lib.RULE_STANDARD, k)
        _, olog = o.run(0, k)
        check(f"run {k}", done == len(olog) and bits(e.download(), o.T))
    for _ in range(3):
        want = o.find(0)
        if isinstance(want, str):
            break
        e.pivot(*want)
        o.pivot(*want)
    check("explicit pivots", bits(e.download(), o.T))
    got = e.find(_lib.RULE_STANDARD, True)
    want = o.find(0)
    if not isinstance(want, str):
        o.pivot(*want)
    check("findPivot(True)", (list(got) if isinstance(got, tuple) else got) ==
          (list(want) if isinstance(want, tuple) else want) and bits(e.download(), o.T))
    st, done = e.run(_lib.RULE_STANDARD, 100)
    _, olog = o.run(0, 100)
    check("run after explicit", done == len(olog) and bits(e.download(), o.T))
    e.upload(T)
    o = F64Tableau(T)
    st, done = e.run(_lib.RULE_STANDARD, 130)
    _, olog = o.run(0, 130)
    check("re-upload", done == len(olog) and bits(e.download(), o.T))
    assert e.exchange_path()[1] == 0
    e.close()


def solves():
    for kind, m, ns, seed in (("pos", 300, 300, 5), ("pos", 500, 420, 7), ("mixed", 120, 200, 3)):
        T = gen.tableau(kind, m, ns, seed)
        e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
        e.upload(T)
        e.set_block(64)
        o = F64Tableau(T)
        st, npiv, nstd = e.solve()
        ost, olog, onstd = o.solve()
        check(f"solve {kind} {m}x{ns}: {npiv} pivots", st == ost and npiv == len(olog) and bits(e.download(), o.T))
        e.close()


def timeout_recovery():
    T = gen.tableau("mixed", 400, 800, 13)
    os.environ["LPGPU_FAULT"] = "2:40"      # launch 2, pivot 40: a summary withheld
    os.environ["LPGPU_SPIN_MAX"] = "20000"
    os.environ.pop("LPGPU_STRICT", None)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(0)                          # (reads the fault settings)
    os.environ.pop("LPGPU_FAULT")
    o = F64Tableau(T)
    st, done = e.run(_lib.RULE_STANDARD, 200)
    _, olog = o.run(0, 200)
    check("timeout recovery", done == len(olog) and e.log().tolist() == olog.tolist() and bits(e.download(), o.T)
          and e.exchange_path() == (_lib.PATH_KERNELS, 1))
    e.close()


def shard_group():
    """in-process row shards (one k_group launch for all members): each
    member's sweep flips its own buffers"""
    T = gen.tableau("tall", 3000, 300, 19)
    o = F64Tableau(T)
    _, olog = o.run(0, 150)
    grp = _lib.create_group(T.shape[0] - 1, T.shape[1] - 1, 2)
    for g in grp:
        g.upload(T)
        g.set_block(64)
    st, done = grp[0].run(_lib.RULE_STANDARD, 150)
    ok = done == len(olog) and grp[0].log().tolist() == olog.tolist()
    ok = ok and bits(grp[0].rows(0, 1), o.T[:1])
    for g in grp:
        b, c = g.row_begin, g.row_count
        ok = ok and bits(g.rows(1 + b, c), o.T[1 + b:1 + b + c])
    check("2 in-process shards", ok)
    for g in reversed(grp):
        g.close()


if __name__ == "__main__":
    assert os.environ.get("LPGPU_SWEEP_OOP") == "1"
    runs()
    solves()
    timeout_recovery()
    shard_group()
    print("ALL OK")
