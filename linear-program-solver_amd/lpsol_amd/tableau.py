"""``Tableau`` with the reference's API (``lpsol/tableau.py:16-521``), backed by
a float64 tableau that lives in GPU memory.

Storage: one (m+1) x (n+1) float64 array in the engine layout (row 0 =
``[_z, c...]``, row 1+i = ``[b_i, a_i...]``; ``_z`` is the stored NEGATED
objective exactly like the reference, ``tableau.py:46,82-84``).  Two copies
may exist -- the device tableau inside an ``Engine`` and a host mirror for
element access -- and each is refreshed lazily from the other when it is
stale.  Pivots always run on the device (``Engine.pivot``); nothing here
computes a pivot on the host.

Differences from the reference: values are float64, so
getters return ``float`` instead of ``Fraction`` (dyadic inputs such as the
reference's own test tableaux are exact either way); setters accept anything
``Fraction()`` accepts (ints, floats, ``'1/2'`` strings, Fractions).
"""
from __future__ import annotations

import csv
import io
import json
from fractions import Fraction
from typing import Any

import numpy as np

from . import _lib


def _num(x) -> float:
    if isinstance(x, float):
        return x
    return float(Fraction(x))


def _json_num(x) -> str:
    """saveJson text of a float64: the simplest fraction that round-trips."""
    x = float(x)
    f = Fraction(x)
    g = f.limit_denominator(1 << 20)
    return str(g if float(g) == x else f)


def _fmt(x: float) -> str:
    """Reference-style number text: Fractions print as 'p/q' or 'p'."""
    f = Fraction(x)
    if f.denominator <= (1 << 20):
        return str(f)
    return repr(float(x))


class Tableau:
    """Full simplex tableau (m constraints, n variables) -- reference
    ``lpsol.Tableau``."""

    def __init__(self, m: int, n: int):
        if m <= 0:
            raise ValueError(f'need m > 0, provided m = {m}')
        if n <= 0:
            raise ValueError(f'need n > 0, provided n = {n}')
        self._m = m
        self._n = n
        self._T = np.zeros((m + 1, n + 1), dtype=np.float64)
        self._cl: list[str] = [''] * n
        self._cm: list[bool] = [False] * n
        self._eng: _lib.Engine | None = None
        self._host_ok = True     # host mirror is current
        self._dev_ok = False     # device tableau is current
        self._lost = False       # a device failure took the only current copy
        self._tol: dict = {}

    # ------------------------------------------------------------------ sync
    def _host(self) -> np.ndarray:
        """Current host mirror (downloads from the device if stale)."""
        self._check_lost()
        if not self._host_ok:
            self._T = self._eng.download()
            self._host_ok = True
        return self._T

    def _touch(self):
        """Host mirror was modified: the device copy is stale."""
        self._host()
        self._dev_ok = False

    def _engine(self) -> _lib.Engine:
        """Device engine holding the current tableau (uploads if stale)."""
        self._check_lost()
        if self._eng is None or (self._eng.m, self._eng.n) != (self._m, self._n):
            if self._eng is not None:
                self._host()
                self._eng.close()
            self._eng = _lib.Engine(self._m, self._n)
            if self._tol:
                self._eng.set_tol(**self._tol)
            self._dev_ok = False
        if not self._dev_ok:
            self._eng.upload(self._host())
            self._dev_ok = True
        return self._eng

    def _device_changed(self):
        """A device operation modified the tableau."""
        self._host_ok = False
        self._dev_ok = True

    def _device_failed(self):
        """A device call that changes the tableau raised DeviceError part way
        through: the device copy can no longer be trusted.  If the host
        mirror is current it is the state before the call (the next device
        call re-uploads it; Simplex._bfs was not touched either); otherwise
        the tableau is lost and every later access says so."""
        if self._host_ok:
            self._dev_ok = False
        else:
            self._lost = True

    def _check_lost(self):
        if self._lost:
            raise _lib.DeviceError('tableau lost in an earlier device failure')

    def setTolerances(self, **kw):
        """Extension: float64 comparison tolerances (``lp_tol`` fields)."""
        self._tol.update(kw)
        if self._eng is not None:
            self._eng.set_tol(**self._tol)

    def toArray(self) -> np.ndarray:
        """Extension: copy of the (m+1) x (n+1) engine-layout array."""
        return self._host().copy()

    @classmethod
    def fromArray(cls, T, names=None, marks=None) -> 'Tableau':
        """Extension: tableau from an engine-layout array."""
        T = np.asarray(T, dtype=np.float64)
        t = cls(T.shape[0] - 1, T.shape[1] - 1)
        t._T = T.copy()
        if names is not None:
            t.setVarNames(names)
        if marks is not None:
            t.setVarMarks(marks)
        return t

    # ------------------------------------------------------------ comparison
    def __eq__(self, t) -> bool:
        if not isinstance(t, Tableau):
            raise TypeError(f'cannot compare to type {type(t)}')
        return (self._m == t._m and self._n == t._n
                and bool(np.array_equal(self._host(), t._host()))
                and self._cl == t._cl and self._cm == t._cm)

    # --------------------------------------------------------------- getters
    def getNumCons(self) -> int:
        return self._m

    def getNumVars(self) -> int:
        return self._n

    def getTableauSize(self) -> tuple[int, int]:
        return self.getNumCons(), self.getNumVars()

    def getZ(self) -> float:
        ''' objective value (-z) '''
        self._check_lost()
        if not self._host_ok:
            return self._eng.objective()
        return float(-self._T[0, 0]) + 0.0

    def getC(self) -> list[float]:
        return self._host()[0, 1:].tolist()

    def getCj(self, j: int) -> float:
        self._check_j(j)
        return float(self._host()[0, 1 + self._wrap(j, self._n)])

    def getB(self) -> list[float]:
        return self._host()[1:, 0].tolist()

    def getBi(self, i: int) -> float:
        self._check_i(i)
        return float(self._host()[1 + self._wrap(i, self._m), 0])

    def getA(self) -> list[list[float]]:
        return self._host()[1:, 1:].tolist()

    def getAij(self, i: int, j: int) -> float:
        self._check_i(i)
        self._check_j(j)
        return float(self._host()[1 + self._wrap(i, self._m), 1 + self._wrap(j, self._n)])

    def getVarNames(self) -> list[str]:
        return self._cl

    def getVarName(self, j: int) -> str:
        return self._cl[j]

    def getVarMarks(self) -> list[bool]:
        return self._cm

    def getVarMark(self, j: int) -> bool:
        return self._cm[j]

    def _check_i(self, i):
        if not -self._m <= i < self._m:
            raise IndexError('list index out of range')

    def _check_j(self, j):
        if not -self._n <= j < self._n:
            raise IndexError('list index out of range')

    @staticmethod
    def _wrap(k, size):
        return k + size if k < 0 else k

    # --------------------------------------------------------------- setters
    def setZ(self, z):
        ''' set objective value, the value stored is -z '''
        self._touch()
        self._T[0, 0] = -_num(z)

    def setC(self, c: list[Any]):
        self._touch()
        self._T[0, 1:] = [_num(c[j]) for j in range(self._n)]

    def setCj(self, j: int, cj):
        self._check_j(j)
        self._touch()
        self._T[0, 1 + self._wrap(j, self._n)] = _num(cj)

    def setB(self, b: list[Any]):
        self._touch()
        self._T[1:, 0] = [_num(b[i]) for i in range(self._m)]

    def setBi(self, i: int, bi):
        self._check_i(i)
        self._touch()
        self._T[1 + self._wrap(i, self._m), 0] = _num(bi)

    def setA(self, a: list[list[Any]]):
        self._touch()
        self._T[1:, 1:] = [[_num(a[i][j]) for j in range(self._n)] for i in range(self._m)]

    def setAij(self, i: int, j: int, aij):
        self._check_i(i)
        self._check_j(j)
        self._touch()
        self._T[1 + self._wrap(i, self._m), 1 + self._wrap(j, self._n)] = _num(aij)

    def setVarNames(self, cl: list[str]):
        for j in range(self._n):
            self._cl[j] = cl[j]

    def setVarName(self, j: int, l: str):
        self._cl[j] = l

    def setVarMarks(self, cm: list[bool]):
        for j in range(self._n):
            self._cm[j] = cm[j]

    def setVarMark(self, j: int, m: bool):
        self._cm[j] = m

    def toggleVarMark(self, j: int):
        self._cm[j] = not self._cm[j]

    # ------------------------------------------------------- data management
    # (host-side reshaping of the mirror; the device copy is rebuilt lazily)
    def addVar(self, v: str = ''):
        self.addVars([v])

    def addVars(self, vs: list[str]):
        T = self._host()
        self._T = np.hstack([T, np.zeros((self._m + 1, len(vs)))])
        self._n += len(vs)
        self._cl += list(vs)
        self._cm += [False] * len(vs)
        self._dev_ok = False

    def addCon(self):
        self.addCons(1)

    def addCons(self, count: int):
        if count <= 0:
            raise ValueError(f'need count > 0, provided count = {count}')
        T = self._host()
        self._T = np.vstack([T, np.zeros((count, self._n + 1))])
        self._m += count
        self._dev_ok = False

    def permuteRows(self, perm: list[int]):
        m = self._m
        if len(perm) != m or set(perm) != set(range(m)):
            raise ValueError(f'not a permutation of 0..{m-1}')
        self._touch()
        self._T[1:] = self._T[1:][np.asarray(perm)]

    def permuteCols(self, perm: list[int]):
        n = self._n
        if len(perm) != n or set(perm) != set(range(n)):
            raise ValueError(f'not a permutation of 0..{n-1}')
        self._touch()
        self._T[:, 1:] = self._T[:, 1:][:, np.asarray(perm)]
        self._cl = [self._cl[j] for j in perm]
        self._cm = [self._cm[j] for j in perm]

    def copy(self) -> 'Tableau':
        ret = Tableau(self._m, self._n)
        ret._T = self._host().copy()
        ret._cl = self._cl[:]
        ret._cm = self._cm[:]
        ret._tol = dict(self._tol)
        return ret

    def _drop(self, keep_rows: list[int], ncols: int):
        """Keep constraint rows keep_rows and the first ncols variables
        (phase-1 clean-up, the reference's private-field edit at
        simplex.py:88-100)."""
        T = self._host()
        self._T = np.ascontiguousarray(T[[0] + [1 + i for i in keep_rows], :ncols + 1])
        self._m = len(keep_rows)
        self._n = ncols
        self._cl = self._cl[:ncols]
        self._cm = self._cm[:ncols]
        self._dev_ok = False

    def _snap_b(self, zero: float):
        """Set b_i with |b_i| <= zero to +0 (phase-1 clean-up)."""
        T = self._host()
        small = np.abs(T[1:, 0]) <= zero
        if small.any():
            self._touch()
            self._T[1:, 0][small] = 0.0

    # ------------------------------------------------------- row operations
    # Host edits of the mirror used by phase 1 and user code (tableau.py:254-293).
    # The pivot (below) never goes through them: it runs on the device.
    def rowMult(self, r: int, m):
        m = _num(m)
        if m == 1.0:
            return
        self._touch()
        self._T[1 + r] *= m

    def rowDiv(self, r: int, d):
        d = _num(d)
        if d == 0.0:
            raise ZeroDivisionError('cannot divide row by zero')
        self._touch()
        self._T[1 + r] /= d

    def rowAdd(self, rd: int, rs: int, m: Any = 1):
        m = _num(m)
        if m == 0.0:
            return
        self._touch()
        self._T[1 + rd] += m * self._T[1 + rs]

    def rowSub(self, rd: int, rs: int, m: Any = 1):
        self.rowAdd(rd, rs, -_num(m))

    def rowAddToObj(self, r: int, m: Any = 1):
        m = _num(m)
        if m == 0.0:
            return
        self._touch()
        self._T[0] += m * self._T[1 + r]

    def rowSubFromObj(self, r: int, m: Any = 1):
        self.rowAddToObj(r, -_num(m))

    def pivot(self, r: int, c: int):
        '''
        simplex pivot on r,c on the GPU (tableau.py:295-308)
        '''
        if not (0 <= r < self._m and 0 <= c < self._n):
            raise IndexError('list index out of range')
        eng = self._engine()
        try:
            st = eng.pivot(r, c)
        except _lib.DeviceError:
            self._device_failed()
            raise
        if st == _lib.ZERO_PIVOT:
            raise ZeroDivisionError(f'zero pivot {r},{c}')
        self._device_changed()

    # ---------------------------------------------------------- input/output
    def loadFile(self, file: str):
        with open(file, 'r') as f:
            self.loadJson(json.loads(f.read()))

    def saveFile(self, file: str):
        with open(file, 'w') as f:
            f.write(json.dumps(self.saveJson(), separators=(',', ':')))

    def loadJson(self, data: dict[str, Any]):
        ''' same keys and number strings as the reference (tableau.py:322-346) '''
        assert isinstance(data['m'], int) and data['m'] > 0
        assert isinstance(data['n'], int) and data['n'] > 0
        m, n = data['m'], data['n']
        T = np.zeros((m + 1, n + 1))
        T[0, 0] = _num(data['z'])          # stored cell, as in the reference
        T[0, 1:] = [_num(data['c'][j]) for j in range(n)]
        T[1:, 0] = [_num(data['b'][i]) for i in range(m)]
        T[1:, 1:] = [[_num(data['a'][i][j]) for j in range(n)] for i in range(m)]
        self._m, self._n = m, n
        self._T = T
        self._cl = [str(data['cl'][j]) for j in range(n)]
        self._cm = [bool(data['cm'][j]) for j in range(n)]
        # a whole new tableau: whatever an earlier device failure lost is gone
        self._host_ok, self._dev_ok, self._lost = True, False, False

    def saveJson(self) -> dict[str, Any]:
        ''' same keys and number strings as the reference (tableau.py:348-360);
        a float64 value is written as the simplest fraction (denominator <=
        2^20) that converts back to the same float64, else as its exact binary
        fraction -- loadJson of the text gives back the same tableau, and
        short rationals (the reference's own test data, 1/25, ...) print as
        the reference prints them '''
        T = self._host()
        return {
            'm': self._m, 'n': self._n,
            'z': _json_num(T[0, 0]),
            'c': [_json_num(x) for x in T[0, 1:]],
            'b': [_json_num(x) for x in T[1:, 0]],
            'a': [[_json_num(x) for x in row] for row in T[1:, 1:]],
            'cl': list(self._cl),
            'cm': list(self._cm),
        }

    def printGrid(self, labels: bool = True, rownums: bool = True,
                  mpre: str = '(', msuf: str = ')') -> list[list[str]]:
        T = self._host()
        data: list[list[str]] = []
        if labels:
            row = ['', ''] if rownums else ['']
            row += [f'{mpre}{l}{msuf}' if self._cm[j] else l for j, l in enumerate(self._cl)]
            data.append(row)
        row = ['', _fmt(T[0, 0])] if rownums else [_fmt(T[0, 0])]
        data.append(row + [_fmt(x) for x in T[0, 1:]])
        for i in range(self._m):
            row = [f'{i}', _fmt(T[1 + i, 0])] if rownums else [_fmt(T[1 + i, 0])]
            data.append(row + [_fmt(x) for x in T[1 + i, 1:]])
        return data

    def printText(self, labels: bool = True, rownums: bool = False, spacing: int = 2,
                  left: bool = False, mpre: str = '(', msuf: str = ')') -> str:
        if spacing < 1:
            raise ValueError(f'spacing must be positive, provided {spacing}')
        grid = self.printGrid(labels, rownums, mpre, msuf)
        width = [max(len(r[k]) for r in grid) for k in range(len(grid[0]))]
        cells = [[(s.ljust if left else s.rjust)(width[k]) for k, s in enumerate(r)] for r in grid]
        gap = ' ' * spacing
        rule = '-' * (spacing * (len(grid[0]) + 2) + sum(width) + 3)
        head = 2 if labels else 1
        split = 2 if rownums else 1
        out = [rule]
        for k, r in enumerate(cells):
            if k == head:
                out.append(rule)
            out.append('|' + gap + gap.join(r[:split] + ['|'] + r[split:]) + gap + '|')
        out.append(rule)
        return '\n'.join(out) + '\n'

    def printLatex(self, labels: bool = True, rownums: bool = False,
                   mpre: str = '(', msuf: str = ')') -> str:
        grid = self.printGrid(labels, rownums, mpre, msuf)
        head = 2 if labels else 1
        out = ['\\begin{tabular}{' + ('|c' * head) + '|' + ('c' * self._n) + '|} \\hline']
        grid = [[f'${s}$' if s else s for s in r] for r in grid]
        for k, r in enumerate(grid):
            line = ' & '.join(r) + ' \\\\'
            if k < head or k == len(grid) - 1:
                line += '\\hline'
            out.append(line)
        out.append('\\end{tabular}')
        return '\n'.join(out) + '\n'

    def printCSV(self, labels: bool = True, rownums: bool = False,
                 mpre: str = '(', msuf: str = ')') -> str:
        buf = io.StringIO()
        csv.writer(buf).writerows(self.printGrid(labels, rownums, mpre, msuf))
        return buf.getvalue()

    def __str__(self) -> str:
        return self.printText()

    def __repr__(self) -> str:
        return f'<{type(self).__name__} object at {hex(id(self))}, m = {self._m}, n = {self._n}>'

    # ------------------------------------------------------------ form checks
    # Read-only scans of the mirrored tableau (tableau.py:466-521).
    # form checks (tableau.py:466-521), exact comparisons of the float64
    # values.  When the device copy is the current one (after pivots) they run
    # as one device column scan instead of downloading the tableau.
    def _device_form(self):
        if self._dev_ok and not self._host_ok and self._eng is not None:
            return self._eng.form_checks()
        return None

    def isCanonical(self, bcols: list[int] | None = None) -> bool:
        f = self._device_form()
        if f is not None:
            if bcols is not None and f["bcols"] is not None:
                for i in range(self._m):
                    bcols[i] = f["bcols"][i]
            return f["canonical"]
        T = self._host()
        m = self._m
        A = T[1:, 1:]
        found = [-1] * m
        ok_b = not bool(np.any(T[1:, 0] < 0.0))
        if ok_b:
            zero_c = T[0, 1:] == 0.0
            ones = A == 1.0
            nz = np.count_nonzero(A, axis=0)
            for j in np.nonzero(zero_c & (nz == 1) & ones.any(axis=0))[0]:
                i = int(np.argmax(ones[:, j]))
                if found[i] == -1:
                    found[i] = int(j)
        if not ok_b:           # the reference returns before touching bcols (:474-475)
            return False
        if bcols is not None:
            for i in range(m):
                bcols[i] = found[i]
        return all(j != -1 for j in found)

    def isOptimal(self) -> bool:
        f = self._device_form()
        if f is not None:
            return f["optimal"]
        return bool(np.all(self._host()[0, 1:] >= 0.0))

    def isUnbounded(self) -> bool:
        f = self._device_form()
        if f is not None:
            return f["unbounded"]
        T = self._host()
        return bool(np.any((T[0, 1:] < 0.0) & np.all(T[1:, 1:] <= 0.0, axis=0)))

    def isInfeasible(self) -> bool:
        f = self._device_form()
        if f is not None:
            return f["infeasible"]
        T = self._host()
        return bool(np.any((T[1:, 0] > 0.0) & np.all(T[1:, 1:] <= 0.0, axis=1)))

    def isDegenerate(self) -> bool:
        f = self._device_form()
        if f is not None:
            return f["degenerate"]
        return bool(np.any(self._host()[1:, 0] == 0.0))
