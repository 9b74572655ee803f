"""ORACLE -- test infrastructure only (tests/, make_golden.py).  Phase 1 of
the reference (``Simplex._find_bfs``, lpsol/simplex.py:36-108) restated on
the float64 contract of oracle/lp_f64.c: exact comparisons against zero
become the tolerance tests of that contract, the artificial solve is
``lpf_solve``, and host row edits are the same numpy expressions the
front-end uses (lpsol_amd/tableau.py rowMult / rowAddToObj).

The one deliberate difference from the reference: after dropping linearly
dependent rows the row count is corrected (the reference keeps ``_m = m``,
simplex.py:93, and then fails with IndexError -- SURVEY §5 quirk 5).
"""
from __future__ import annotations

import numpy as np

from .f64 import DEFAULT_TOL, OPTIMAL, F64Tableau


def basic_columns(T: np.ndarray) -> tuple[bool, list[int]]:
    """``Tableau.isCanonical(bcols)`` (lpsol/tableau.py:466-496): a column is
    basic for row i when its reduced cost is 0, a_ij == 1 at the first 1 and
    every other entry is 0; the first such column per row is recorded.
    Returns (canonical, bcols); bcols is all -1 when some b_i < 0 (the
    reference returns before filling it, :474-475)."""
    m, n = T.shape[0] - 1, T.shape[1] - 1
    bcols = [-1] * m
    if any(T[1 + i, 0] < 0.0 for i in range(m)):
        return False, bcols
    for j in range(n):
        if T[0, 1 + j] != 0.0:
            continue
        onei = -1
        for i in range(m):
            if T[1 + i, 1 + j] == 1.0:
                onei = i
                break
        if onei == -1:
            continue
        if all(i == onei or T[1 + i, 1 + j] == 0.0 for i in range(m)):
            if bcols[onei] == -1:
                bcols[onei] = j
    return all(j != -1 for j in bcols), bcols


def find_bfs(T, tol=None) -> dict:
    """Run phase 1 on a copy of T.  Returns {"T", "bfs", "init_seq"} or
    {"error": "ValueError", "init_seq"} for an infeasible problem.  init_seq
    lists every pivot made: the artificial solve, then the pivots that move
    basic artificials out (simplex.py:82)."""
    tl = dict(DEFAULT_TOL, **(tol or {}))
    T = np.array(T, dtype=np.float64, copy=True)
    m, n = T.shape[0] - 1, T.shape[1] - 1
    for i in range(m):                                   # simplex.py:43-45
        if T[1 + i, 0] < 0.0:
            T[1 + i] *= -1.0
    ok, bfs = basic_columns(T)                           # :46-47
    if ok:
        return {"T": T, "bfs": bfs, "init_seq": []}
    # getZ() is -T[0,0] + 0.0 and setZ(z) stores -z (tableau.py:82-84,
    # front-end tableau.py getZ/setZ): mirrored so signed zeros agree
    orig_c, orig_z = T[0, 1:].copy(), -T[0, 0] + 0.0     # :49-52
    missing = [i for i, j in enumerate(bfs) if j == -1]
    W = np.zeros((m + 1, n + 1 + len(missing)))
    W[:, :n + 1] = T
    W[0, 1:] = 0.0
    W[0, 0] = -0.0
    for ind, i in enumerate(missing):                    # :56-60
        W[0, 1 + n + ind] = 1.0
        W[1 + i, 1 + n + ind] = 1.0
        W[0] += -1.0 * W[1 + i]
        bfs[i] = n + ind
    ft = F64Tableau(W, tol)
    st, log, _ = ft.solve()                              # :62
    assert st == OPTIMAL, "unbounded artificial problem (internal error)"
    seq = [[int(r), int(c)] for r, c in log]
    for r, c in seq:
        bfs[r] = c
    if abs(ft.T[0, 0]) > tl["zero"]:                     # :64-67
        return {"error": "ValueError", "init_seq": seq}
    keep = [True] * m
    for i in range(m):                                   # :68-84
        j = bfs[i]
        if j < n:
            continue
        assert abs(ft.T[1 + i, 0]) <= tl["zero"], "invalid artificial solution"
        nz = [k for k in range(n) if abs(ft.T[1 + i, 1 + k]) > tl["pivot"]]
        if not nz:
            keep[i] = False
        else:
            ft.pivot(i, nz[0])
            bfs[i] = nz[0]
            seq.append([i, nz[0]])
    rows = [0] + [1 + i for i in range(m) if keep[i]]    # :87-100
    T = np.ascontiguousarray(ft.T[rows, :n + 1])
    bfs = [j for i, j in enumerate(bfs) if keep[i]]
    # rows whose artificial left the basis at value 0 can carry a rounding
    # residue of either sign; exactly 0 in the reference, snapped to +0 here
    # so the canonical-form check (b >= 0) holds as it does there
    small = np.abs(T[1:, 0]) <= tl["zero"]
    T[1:, 0][small] = 0.0
    T[0, 0] = -orig_z                                    # :102-105
    T[0, 1:] = orig_c
    for i, j in enumerate(bfs):
        T[0] += -T[0, 1 + j] * T[1 + i]
    assert basic_columns(T)[0], "tableau not canonical (internal error)"
    return {"T": T, "bfs": bfs, "init_seq": seq}


def solve_lp(T, tol=None) -> dict:
    """``Simplex(tab)`` followed by ``solve()``: phase 1, then the
    standard/min-index loop of lpf_solve.  Adds "seq", "objective" and the
    final "bfs" to find_bfs's result."""
    out = find_bfs(T, tol)
    if "error" in out:
        return out
    out["init_bfs"] = list(out["bfs"])
    out["init_size"] = [out["T"].shape[0] - 1, out["T"].shape[1] - 1]
    ft = F64Tableau(out["T"], tol)
    st, log, _ = ft.solve()
    assert st == OPTIMAL, f"phase-2 status {st}"
    bfs = list(out["bfs"])
    for r, c in log:
        bfs[int(r)] = int(c)
    out.update(seq=[[int(r), int(c)] for r, c in log], objective=ft.objective(), bfs=bfs,
               T=ft.T)
    return out
