"""ORACLE -- test infrastructure only.

Host model of the engine's ROW-SHARDED pivot protocol (one rank per GPU in
the product; here one process per rank over torch.distributed/gloo), built
from the float64 pieces of oracle/lp_f64.c so every number is bit-identical
to the single-process restatement.  tests/test_sharded_cpu.py runs it with
world_size 2 and 3 and checks that the pivot sequence and every row equal an
unsharded run: the protocol (not just the kernels) is order-independent.

Layout per rank: row 0 (replicated) + constraint rows [rb, rb + rc).
Per pivot (the same steps as csrc/kernels.hip k_ratio/k_pick/k_prow):
  1. entering column from the replicated row 0            (no communication)
  2. local ratio test: l = local minimum ratio; cand = first local row with
     q <= band(l), its ratio q
  3. ONE allgather of [cand global index, l, q, cand's row]
  4. g = min l over ranks; the first rank (= first rows) with l <= band(g)
     holds the winner: its candidate when q <= band(g)          (fast path)
     otherwise (a near-tie straddling the band -- rare): every rank takes
     the first local row with q <= band(g) and a second allgather settles it
  5. every rank normalises the winning row and applies the pivot locally.
band(x) = x + tol.ratio_tie * |x| (oracle/lp_f64.c header).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .f64 import Tol, _tol, lib

_PD = C.POINTER(C.c_double)
NONE = -1


def _ptr(a):
    return a.ctypes.data_as(_PD)


def _setup():
    L = lib()
    L.lpf_prow.argtypes = [_PD, C.c_int64, C.c_int64, _PD]
    L.lpf_prow.restype = None
    L.lpf_apply.argtypes = [_PD, C.c_int64, C.c_int64, C.c_int64, _PD, C.c_int64, C.c_int64]
    L.lpf_apply.restype = None
    L.lpf_min_ratio.argtypes = [_PD, C.c_int64, C.c_int64, C.c_int64, C.POINTER(Tol)]
    L.lpf_min_ratio.restype = C.c_double
    L.lpf_first_within.argtypes = [_PD, C.c_int64, C.c_int64, C.c_int64, C.POINTER(Tol),
                                   C.c_double, _PD]
    L.lpf_first_within.restype = C.c_int64
    L.lpf_entering.argtypes = [_PD, C.c_int64, C.c_int, C.POINTER(Tol)]
    L.lpf_entering.restype = C.c_int64
    return L


def band(x: float, tie: float) -> float:
    return x + tie * abs(x)


class ShardState:
    """One rank's rows of the tableau (row 0 replicated)."""

    def __init__(self, T, rank: int, nranks: int, tol=None):
        T = np.asarray(T, dtype=np.float64)
        self.m, self.n = T.shape[0] - 1, T.shape[1] - 1
        self.rb = self.m * rank // nranks
        self.rc = self.m * (rank + 1) // nranks - self.rb
        self.row0 = np.ascontiguousarray(T[0].copy())
        self.rows = np.ascontiguousarray(T[1 + self.rb:1 + self.rb + self.rc].copy())
        self.tol = _tol(tol)
        self.L = _setup()
        self.slow_path = 0          # how often step 4's rare branch ran

    def local_candidate(self, col: int, thr: float | None = None):
        """(global index or NONE, local min l, candidate ratio q)"""
        L, ld = self.L, self.n + 1
        if self.rc == 0:
            return NONE, float("inf"), 0.0
        l = L.lpf_min_ratio(_ptr(self.rows), self.rc, ld, col, C.byref(self.tol))
        if not np.isfinite(l):
            return NONE, float("inf"), 0.0
        q = C.c_double()
        t = band(l, self.tol.ratio_tie) if thr is None else thr
        i = L.lpf_first_within(_ptr(self.rows), self.rc, ld, col, C.byref(self.tol), t, C.byref(q))
        return (NONE if i < 0 else self.rb + i), l, q.value

    def apply(self, P: np.ndarray, col: int, r: int):
        L, ld = self.L, self.n + 1
        # row 0 (never the pivot row)
        row0 = self.row0.reshape(1, -1)
        L.lpf_apply(_ptr(row0), 1, self.n, ld, _ptr(P), col, -1)
        self.row0 = row0.reshape(-1)
        Rloc = r - self.rb if self.rb <= r < self.rb + self.rc else -1
        if self.rc:
            L.lpf_apply(_ptr(self.rows), self.rc, self.n, ld, _ptr(P), col, Rloc)

    def row_of(self, r: int) -> np.ndarray:
        return self.rows[r - self.rb]


def pivot_step(st: ShardState, allgather, rule: int = 0):
    """One pivot of the protocol.  allgather(np.ndarray) -> list of arrays (one
    per rank, rank order).  Returns (r, c) or 'optimal' / 'unbounded'."""
    L = st.L
    c = L.lpf_entering(_ptr(st.row0), st.n, rule, C.byref(st.tol))
    if c < 0:
        return "optimal"
    Ccol = c + 1
    idx, l, q = st.local_candidate(Ccol)
    msg = np.zeros(3 + st.n + 1)
    msg[:3] = (idx, l, q)
    if idx != NONE:
        msg[3:] = st.row_of(idx)
    got = allgather(msg)
    ls = [float(x[1]) for x in got]
    g = min(ls)
    if not np.isfinite(g):
        return "unbounded"
    thr = band(g, st.tol.ratio_tie)
    first = next(k for k, lv in enumerate(ls) if lv <= thr)
    if got[first][2] <= thr:
        r = int(got[first][0])
        row = got[first][3:]
    else:
        # rare: a near-tie straddles the band -- each rank offers its first
        # row inside the GLOBAL band, the lowest index wins
        st.slow_path += 1
        idx2, _, _ = st.local_candidate(Ccol, thr)
        msg2 = np.zeros(1 + st.n + 1)
        msg2[0] = idx2 if idx2 != NONE else np.inf
        if idx2 != NONE:
            msg2[1:] = st.row_of(idx2)
        got2 = allgather(msg2)
        k = int(np.argmin([x[0] for x in got2]))
        r = int(got2[k][0])
        row = got2[k][1:]
    P = np.empty(st.n + 1)
    L.lpf_prow(_ptr(np.ascontiguousarray(row)), st.n, Ccol, _ptr(P))
    st.apply(P, Ccol, r)
    return r, c


def run(st: ShardState, allgather, k: int, rule: int = 0):
    seq = []
    for _ in range(k):
        res = pivot_step(st, allgather, rule)
        if isinstance(res, str):
            return seq, res
        seq.append(res)
    return seq, None
