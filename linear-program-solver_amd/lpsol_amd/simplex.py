"""``Simplex`` with the reference's API (``lpsol/simplex.py:16-379``); every
pivot, pivot selection and the whole ``solve()`` loop run on the GPU.

The reference selects pivots through per-element Tableau getters
(``simplex.py:229,238,241,263,273,276``); here each selection is one C-ABI
call (``lp_find_pivot``) and ``solve()`` is one device-resident loop
(``lp_solve``) that returns the pivot log, which is replayed on the host to
maintain ``_bfs`` and the variable marks exactly like ``_pivot``
(``simplex.py:192-197``).
"""
from __future__ import annotations

from . import _lib
from .tableau import Tableau

L_opt = 'optimal'
L_unb = 'unbounded'


def optimal_row0(row0, cost_tol: float) -> bool:
    """isOptimal of a row 0 ``[_z, c_0 .. c_{n-1}]`` with the float64
    contract's comparison (``tableau.py:500-502``: every c_j >= 0 in exact
    arithmetic; here c_j >= -tol.cost, the device's own 'optimal' test)."""
    import numpy as np
    c = np.asarray(row0, dtype=np.float64)[1:]
    return bool(np.all(c >= -cost_tol))


class Simplex:
    '''
    state of the simplex algorithm with canonical form tableaus and pivoting
    between basic feasible solutions (reference ``lpsol.Simplex``)
    '''

    def __init__(self, tab: Tableau):
        self._tab: Tableau = tab
        self._bfs: list[int] = [-1] * tab.getNumCons()
        self.last_solve: dict = {}
        self._find_bfs()

    # ----------------------------------------------------------- phase 1
    def _find_bfs(self):
        '''
        initial basic feasible solution by the method of artificial variables
        (simplex.py:36-108); artificial columns only for rows without a basic
        column.  Its pivots and its solve run on the device; the row edits
        around them are host edits of the mirrored tableau.
        '''
        tab = self._tab
        m, n = tab.getTableauSize()
        for i in range(m):
            if tab.getBi(i) < 0.0:
                tab.rowMult(i, -1)
        if tab.isCanonical(self._bfs):
            return
        tol = tab._engine().get_tol()
        orig_c = tab.getC()[:]
        orig_z = tab.getZ()
        tab.setC([0] * n)
        tab.setZ(0)
        missing = [i for i, j in enumerate(self._bfs) if j == -1]
        tab.addVars([f'$a{i}' for i in missing])
        for ind, i in enumerate(missing):
            tab.setCj(n + ind, 1)
            tab.setAij(i, n + ind, 1)
            tab.rowSubFromObj(i, 1)
            self._bfs[i] = n + ind
        self.solve()
        z = tab.getZ()
        if abs(z) > tol.zero:
            raise ValueError(f'infeasible problem, artificial opt = {z}')
        keep = [True] * m
        for i in range(m):
            j = self._bfs[i]
            if j < n:
                continue
            assert abs(tab.getBi(i)) <= tol.zero, 'invalid artificial solution (internal error)'
            row = tab._host()[1 + i, 1:1 + n]
            nz = [k for k in range(n) if abs(row[k]) > tol.pivot]
            if not nz:                       # linearly dependent constraint
                keep[i] = False
            else:
                self._pivot(i, nz[0])
        # drop dependent rows and the artificial columns.  The reference keeps
        # _m = m here (simplex.py:93) and then fails with
        # IndexError; the row count is corrected instead.
        self._bfs = [j for i, j in enumerate(self._bfs) if keep[i]]
        assert all(0 <= j < n for j in self._bfs), \
            'invalid basic feasible solution (internal error)'
        tab._drop([i for i in range(m) if keep[i]], n)
        # b_i of rows whose artificial left the basis at 0 can carry a rounding
        # residue of either sign (exactly 0 in the reference): snap to +0 so
        # the canonical-form check below (b >= 0) holds as it does there
        tab._snap_b(tol.zero)
        tab.setZ(orig_z)
        tab.setC(orig_c)
        for i, j in enumerate(self._bfs):
            tab.rowSubFromObj(i, tab.getCj(j))
        assert tab.isCanonical(), 'tableau not canonical (internal error)'
        for j in self._bfs:
            tab.setVarMark(j, True)

    # ------------------------------------------------------------ solve
    def solve(self, max_pivots: int | None = None):
        '''
        pivot to an optimal solution on the device: standard-rule pivots,
        switching to min-index pivots if the objective seems stuck
        (simplex.py:110-148).  ``max_pivots`` is an extension (the reference
        can cycle forever).
        '''
        tab = self._tab
        eng = tab._engine()
        try:
            st, npiv, nstd = eng.solve(-1 if max_pivots is None else int(max_pivots))
        except _lib.DeviceError:
            tab._device_failed()
            raise
        if npiv:
            tab._device_changed()
            self._replay(eng.log())
        self.last_solve = {'status': _lib.STATUS_NAMES.get(st, st), 'npiv': npiv, 'nstd': nstd}
        if st == _lib.UNBOUNDED:
            raise AssertionError('unbounded artificial problem (internal error)')
        if st == _lib.OBJ_INCREASED:
            # simplex.py:133; the offending pivot has been made, as there
            raise AssertionError('objective value increased (internal error)')
        if st == _lib.CAP_REACHED:
            raise RuntimeError(f'pivot cap reached after {npiv} pivots')
        if st != _lib.OPTIMAL:
            raise _lib.DeviceError(f'solve ended with status {st}')
        # simplex.py:148 -- with the float64 contract's comparison: no reduced
        # cost below -tol.cost (the device's 'optimal' test, read back here
        # from the device's row 0)
        if not optimal_row0(eng.rows(0, 1)[0], eng.get_tol().cost):
            raise AssertionError('solver failed (internal error)')

    def _replay(self, log):
        for r, c in log:
            self._mark(int(r), int(c))

    def _mark(self, r: int, c: int):
        self._tab.setVarMark(self._bfs[r], False)
        self._bfs[r] = c
        self._tab.setVarMark(c, True)

    # ----------------------------------------------------------- getters
    def getBasicSequence(self) -> list[int]:
        return self._bfs

    def getBasicSequenceNames(self) -> list[str]:
        return [self._tab.getVarName(j) for j in self._bfs]

    def getBFS(self) -> dict[int, float]:
        b = self._tab.getB()
        return {j: b[i] for i, j in enumerate(self._bfs)}

    def getObjValue(self) -> float:
        return self._tab.getZ()

    def getBFSNames(self) -> dict[str, float]:
        b = self._tab.getB()
        return {name: b[i] for i, name in enumerate(self.getBasicSequenceNames())}

    # ------------------------------------------------------------ pivots
    def _pivot(self, r: int, c: int):
        ''' pivot without checking validity (internal use only) '''
        self._tab.pivot(r, c)
        self._mark(r, c)

    def pivot(self, r: int, c: int):
        '''
        pivot only if row r attains the minimum ratio in column c
        (simplex.py:199-216)
        '''
        tab = self._tab
        if not (0 <= r < tab.getNumCons() and 0 <= c < tab.getNumVars()):
            raise IndexError('list index out of range')
        try:
            st = tab._engine().pivot_checked(r, c)
        except _lib.DeviceError:
            tab._device_failed()
            raise
        if st == _lib.ZERO_PIVOT:
            raise ZeroDivisionError('Fraction(%s, 0)' % tab.getBi(r))
        if st == _lib.BAD_PIVOT:
            raise ValueError(f'bad pivot by min ratio test, r = {r}, c = {c}')
        tab._device_changed()
        self._mark(r, c)

    def _find(self, rule: int, do_pivot: bool):
        tab = self._tab
        try:
            res = tab._engine().find(rule, do_pivot)
        except _lib.DeviceError:
            if do_pivot:                   # only a pivoting call can have changed the tableau
                tab._device_failed()
            raise
        if do_pivot and isinstance(res, tuple):
            tab._device_changed()
            self._mark(*res)
        return res

    def findPivotMinIndex(self, do_pivot: bool = False):
        '''
        first negative reduced cost, first row of minimum ratio
        (simplex.py:218-249); 'optimal' / 'unbounded' otherwise
        '''
        return self._find(_lib.RULE_MIN_INDEX, do_pivot)

    def findPivotStandard(self, do_pivot: bool = False):
        '''
        most negative reduced cost, first row of minimum ratio
        (simplex.py:251-284); 'optimal' / 'unbounded' otherwise
        '''
        return self._find(_lib.RULE_STANDARD, do_pivot)

    def findPivotMaxIncrease(self, do_pivot: bool = False):
        '''
        the pivot with the largest objective increase among negative reduced
        costs (simplex.py:286-328): one device scan of every column.
        'unbounded' as soon as any negative-cost column has no positive
        entry (:319-320); 'optimal' if there is no negative cost.
        '''
        tab = self._tab
        try:
            res = tab._engine().find_max_increase(do_pivot)
        except _lib.DeviceError:
            if do_pivot:
                tab._device_failed()
            raise
        if do_pivot and isinstance(res, tuple):
            tab._device_changed()
            self._mark(*res)
        return res

    def findPivotAll(self) -> list[tuple[int, int]]:
        '''
        every min-ratio pivot of every column, column-major, rows in order
        (simplex.py:330-360): one device scan of every column.
        '''
        return self._tab._engine().find_all()

    # ---------------------------------------------------------- printing
    def __str__(self) -> str:
        out = str(self._tab)
        names = [self._tab.getVarName(j) for j in self._bfs]
        b = self._tab.getB()
        vals = [str(b[i]) for i in range(len(self._bfs))]
        w = [max(len(a), len(v)) for a, v in zip(names, vals)]
        names = [a.rjust(w[i]) for i, a in enumerate(names)]
        vals = [v.rjust(w[i]) for i, v in enumerate(vals)]
        out += f'BFS: ({",".join(names)})\n'
        out += f'   = ({",".join(vals)})\n'
        return out

    def __repr__(self) -> str:
        return (f'<{type(self).__name__} object at {hex(id(self))}, '
                f'm = {self._tab._m}, n = {self._tab._n}')
