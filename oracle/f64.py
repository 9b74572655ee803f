"""ORACLE -- test infrastructure only (tests/, __graft_entry__.smoke(),
bench.py's cpu_baseline).  ctypes wrapper of oracle/lp_f64.c: the scalar
float64 restatement with the engine's exact floating-point semantics, used to
check the GPU tableau bit for bit (see lp_f64.c's header for the contract)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liblpf64.so")

OPTIMAL, UNBOUNDED, CAP = 1, 2, -4
_I64, _PD, _P64 = C.c_int64, C.POINTER(C.c_double), C.POINTER(C.c_int64)


class Tol(C.Structure):
    _fields_ = [("cost", C.c_double), ("cost_tie", C.c_double), ("pivot", C.c_double),
                ("zero", C.c_double), ("ratio_tie", C.c_double), ("stall", C.c_double)]


DEFAULT_TOL = dict(cost=1e-9, cost_tie=1e-12, pivot=1e-9, zero=1e-9, ratio_tie=1e-12,
                   stall=1e-12)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle`")
        L = C.CDLL(LIB)
        L.lpf_pivot.argtypes = [_PD, _I64, _I64, _I64, _I64, _I64]
        L.lpf_find.argtypes = [_PD, _I64, _I64, _I64, C.c_int, C.POINTER(Tol), _P64, _P64]
        L.lpf_run.argtypes = [_PD, _I64, _I64, _I64, C.c_int, C.POINTER(Tol), _I64, _P64, _P64]
        L.lpf_solve.argtypes = [_PD, _I64, _I64, _I64, C.POINTER(Tol), _I64, _P64, _P64, _P64]
        L.lpf_find_max_increase.argtypes = [_PD, _I64, _I64, _I64, C.POINTER(Tol), _P64, _P64]
        L.lpf_find_all.argtypes = [_PD, _I64, _I64, _I64, C.POINTER(Tol), _P64, _I64]
        L.lpf_find_all.restype = _I64
        for f in (L.lpf_pivot, L.lpf_find, L.lpf_run, L.lpf_solve, L.lpf_find_max_increase):
            f.restype = C.c_int
        _lib = L
    return _lib


def _tol(tol):
    d = dict(DEFAULT_TOL)
    if tol:
        d.update(tol)
    return Tol(**d)


class F64Tableau:
    """(m+1) x (n+1) float64 tableau driven by the C restatement."""

    def __init__(self, T, tol=None):
        self.T = np.array(T, dtype=np.float64, order="C", copy=True)
        self.m, self.n = self.T.shape[0] - 1, self.T.shape[1] - 1
        self.tol = _tol(tol)

    def _p(self):
        return self.T.ctypes.data_as(_PD)

    def pivot(self, r, c):
        return lib().lpf_pivot(self._p(), self.m, self.n, self.n + 1, r, c)

    def find(self, rule):
        r, c = C.c_int64(), C.c_int64()
        st = lib().lpf_find(self._p(), self.m, self.n, self.n + 1, rule, C.byref(self.tol),
                            C.byref(r), C.byref(c))
        if st == OPTIMAL:
            return "optimal"
        if st == UNBOUNDED:
            return "unbounded"
        return r.value, c.value

    def find_max_increase(self):
        r, c = C.c_int64(), C.c_int64()
        st = lib().lpf_find_max_increase(self._p(), self.m, self.n, self.n + 1, C.byref(self.tol),
                                         C.byref(r), C.byref(c))
        if st == OPTIMAL:
            return "optimal"
        if st == UNBOUNDED:
            return "unbounded"
        return r.value, c.value

    def find_all(self):
        cnt = lib().lpf_find_all(self._p(), self.m, self.n, self.n + 1, C.byref(self.tol), None, 0)
        out = np.zeros(2 * max(cnt, 1), dtype=np.int64)
        lib().lpf_find_all(self._p(), self.m, self.n, self.n + 1, C.byref(self.tol),
                           out.ctypes.data_as(_P64), cnt)
        return [(int(out[2 * k]), int(out[2 * k + 1])) for k in range(cnt)]

    def run(self, rule, k):
        log = np.zeros(2 * max(k, 1), dtype=np.int64)
        npiv = C.c_int64()
        st = lib().lpf_run(self._p(), self.m, self.n, self.n + 1, rule, C.byref(self.tol), k,
                           log.ctypes.data_as(_P64), C.byref(npiv))
        return st, log[:2 * npiv.value].reshape(-1, 2)

    def solve(self, cap=-1, logcap=1 << 20):
        log = np.zeros(2 * logcap, dtype=np.int64)
        npiv, nstd = C.c_int64(), C.c_int64()
        lim = cap if cap >= 0 else logcap
        st = lib().lpf_solve(self._p(), self.m, self.n, self.n + 1, C.byref(self.tol), lim,
                             log.ctypes.data_as(_P64), C.byref(npiv), C.byref(nstd))
        return st, log[:2 * npiv.value].reshape(-1, 2), nstd.value

    def objective(self):
        return -self.T[0, 0]
