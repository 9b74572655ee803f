"""ORACLE -- test infrastructure only, never part of the product path.

Exact-rational (``fractions.Fraction``) restatement of the reference's dense
simplex hot path, used as the correctness checker for the HIP engine.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module.

Parity is PINNED: ``tests/test_oracle.py`` checks every function here against
the golden vectors in ``tests/golden/`` that ``tests/golden/make_golden.py``
captured by running the reference (tkoz0/linear-program-solver, package
``lpsol``) in the build container, plus the reference's own known-answer test
(``lpsol/test_tableau.py:220-227``).

Representation: one list of rows of ``Fraction``.  Row 0 is
``[_z, c_0 .. c_{n-1}]`` where ``_z`` is the stored NEGATED objective
(``lpsol/tableau.py:46,82-84``); row 1+i is ``[b_i, a_i0 .. a_i,n-1]``.  This
is the device layout, not the reference's split fields.
"""
from __future__ import annotations

from fractions import Fraction
from typing import Iterable

ZERO = Fraction(0)
ONE = Fraction(1)


# --------------------------------------------------------------------------
# construction / conversion
# --------------------------------------------------------------------------

def from_array(T) -> list[list[Fraction]]:
    """Exact copy of a float64 tableau (``Fraction(float)`` is exact)."""
    return [[Fraction(float(x)) for x in row] for row in T]


def from_strings(z, c, b, a) -> list[list[Fraction]]:
    """Rows from reference-style values: z is the STORED cell (-objective)."""
    rows = [[Fraction(z)] + [Fraction(x) for x in c]]
    for bi, ai in zip(b, a):
        rows.append([Fraction(bi)] + [Fraction(x) for x in ai])
    return rows


def to_floats(T) -> list[list[float]]:
    return [[float(x) for x in row] for row in T]


def size(T) -> tuple[int, int]:
    return len(T) - 1, len(T[0]) - 1


def objective(T) -> Fraction:
    """getZ(): the objective value, i.e. minus the stored cell
    (``lpsol/tableau.py:82-84``)."""
    return -T[0][0]


# --------------------------------------------------------------------------
# Tableau.pivot  (lpsol/tableau.py:295-308 via rowMult/rowAdd/rowAddToObj
# at :254-293)
# --------------------------------------------------------------------------

def pivot(T, r: int, c: int) -> None:
    """In-place pivot on constraint row r, variable column c (0-based).

    Order of operations follows ``tableau.py:300-308``: zero check, normalise
    row r (skipped when the factor is one, :257), fold it into the objective
    row with multiplier -c_c (skipped when zero, :285), then eliminate column
    c from every other constraint row (each skipped when its multiplier is
    zero, :272).  Multipliers are read before their row changes."""
    R, C = r + 1, c + 1
    prow = T[R]
    a = prow[C]
    if a == ZERO:
        raise ZeroDivisionError(f"zero pivot {r},{c}")
    if a != ONE:
        inv = ONE / a
        prow = [x * inv for x in prow]
        T[R] = prow
    nz = [k for k, x in enumerate(prow) if x != ZERO]
    for rr in range(len(T)):
        if rr == R:
            continue
        row = T[rr]
        f = row[C]
        if f == ZERO:
            continue
        for k in nz:
            row[k] = row[k] - f * prow[k]


def pivot_dense(T, r: int, c: int) -> None:
    """``Tableau.pivot`` in the reference's own order of operations and with
    its full row walks (``tableau.py:254-308``): ``rowDiv`` multiplies the
    pivot row by 1/a (skipped when that is one, :257), ``rowAddToObj(r,
    -c_c)`` and ``rowSub(rr, r, a_rr,c)`` for every other row (each skipped
    when its multiplier is zero, :272,:285) add m * source[j] to EVERY entry
    j of the destination row, zeros included.  Same result as ``pivot``;
    this is the cost model of the reference's CPU path (bench.py's
    cpu_baseline)."""
    R, C = r + 1, c + 1
    a = T[R][C]
    if a == ZERO:
        raise ZeroDivisionError(f"zero pivot {r},{c}")
    inv = ONE / a
    if inv != ONE:
        T[R] = [x * inv for x in T[R]]
    prow = T[R]
    width = len(prow)
    for rr in range(len(T)):
        if rr == R:
            continue
        row = T[rr]
        mult = -row[C]
        if mult == ZERO:
            continue
        for k in range(width):
            row[k] += mult * prow[k]


# --------------------------------------------------------------------------
# pivot selection  (lpsol/simplex.py:218-284)
# --------------------------------------------------------------------------

def _ratio_row(T, c: int):
    """First constraint row attaining the minimum b_i / a_ic over a_ic > 0;
    strict ``<`` keeps the first minimum (``simplex.py:237-244,272-279``).
    Returns None when no a_ic is positive."""
    C = c + 1
    best = None
    best_i = -1
    for i in range(1, len(T)):
        a = T[i][C]
        if a <= ZERO:
            continue
        q = T[i][0] / a
        if best is None or q < best:
            best, best_i = q, i - 1
    return None if best is None else best_i


def find_standard(T):
    """findPivotStandard (``simplex.py:251-284``): most negative reduced cost,
    first index on ties (strict ``<`` at :266)."""
    c0 = T[0]
    j = -1
    for k in range(1, len(c0)):
        v = c0[k]
        if v < ZERO and (j == -1 or v < c0[j + 1]):
            j = k - 1
    if j == -1:
        return "optimal"
    i = _ratio_row(T, j)
    if i is None:
        return "unbounded"
    return i, j


def find_min_index(T):
    """findPivotMinIndex (``simplex.py:218-249``): first negative reduced cost;
    ratio ties go to the first ROW (not textbook Bland)."""
    c0 = T[0]
    j = next((k - 1 for k in range(1, len(c0)) if c0[k] < ZERO), -1)
    if j == -1:
        return "optimal"
    i = _ratio_row(T, j)
    if i is None:
        return "unbounded"
    return i, j


def find_max_increase(T):
    """findPivotMaxIncrease (``simplex.py:286-328``), including its early
    'unbounded' return on the first column with no positive entry (:319-320)
    and its tie branch that can never fire (:316-318)."""
    m, n = size(T)
    inc = None
    sel = (-1, -1)
    any_neg = False
    for j in range(n):
        cj = T[0][j + 1]
        if cj >= ZERO:
            continue
        any_neg = True
        ratio = None
        isel = -1
        colinc = None
        for i in range(m):
            a = T[i + 1][j + 1]
            if a <= ZERO:
                continue
            q = T[i + 1][0] / a
            if ratio is None or q < ratio:
                ratio, colinc, isel = q, -cj * q, i
            elif q == ratio and colinc is not None and -cj * q > colinc:
                colinc, isel = -cj * q, i
        if colinc is None:
            return "unbounded"
        if inc is None or colinc > inc:
            inc, sel = colinc, (isel, j)
    if not any_neg:
        return "optimal"
    return sel


def find_all(T) -> list[tuple[int, int]]:
    """findPivotAll (``simplex.py:330-360``): every min-ratio pivot of every
    column, in column-major order, ties in row order."""
    m, n = size(T)
    out = []
    for j in range(n):
        ratio = None
        lst: list[tuple[int, int]] = []
        for i in range(m):
            a = T[i + 1][j + 1]
            if a <= ZERO:
                continue
            q = T[i + 1][0] / a
            if ratio is None or q < ratio:
                ratio, lst = q, [(i, j)]
            elif q == ratio:
                lst.append((i, j))
        out += lst
    return out


def validated_pivot_ok(T, r: int, c: int) -> bool:
    """Simplex.pivot's min-ratio check (``simplex.py:204-215``)."""
    m, _ = size(T)
    best = None
    for i in range(m):
        a = T[i + 1][c + 1]
        if a <= ZERO:
            continue
        q = T[i + 1][0] / a
        if best is None or q < best:
            best = q
    return T[r + 1][0] / T[r + 1][c + 1] == best


# --------------------------------------------------------------------------
# Simplex.solve  (lpsol/simplex.py:110-148)
# --------------------------------------------------------------------------

class Unbounded(AssertionError):
    pass


class ObjectiveIncreased(AssertionError):
    """simplex.py:133: a standard-rule pivot of solve() raised the objective
    above its value at the start of the call (possible only on a tableau
    whose b has negative entries: the ratio test then picks a negative ratio)."""


def solve(T, cap: int | None = None, log: list | None = None) -> dict:
    """Standard-rule pivots until ``steps_stuck`` reaches m+n, then min-index
    pivots to optimality (``simplex.py:116-148``).

    Quirks kept: ``obj_val`` is read once at the start and never
    refreshed (:118), so the stall counter counts pivots that leave the
    objective equal to its INITIAL value; m and n are captured at the start
    (:116).  ``cap`` is an extension: stop after that many pivots.

    Returns {'status': 'optimal'|'cap', 'npiv', 'nstd', 'seq': [(r, c), ...]}.
    """
    m, n = size(T)
    seq = [] if log is None else log
    obj_val = objective(T)
    if all(x >= ZERO for x in T[0][1:]):
        return {"status": "optimal", "npiv": 0, "nstd": 0, "seq": seq}
    stuck = 0
    nstd = 0
    while stuck < m + n:
        if cap is not None and len(seq) >= cap:
            return {"status": "cap", "npiv": len(seq), "nstd": nstd, "seq": seq}
        res = find_standard(T)
        if res == "unbounded":
            raise Unbounded("unbounded artificial problem (internal error)")
        if res == "optimal":
            return {"status": "optimal", "npiv": len(seq), "nstd": nstd, "seq": seq}
        pivot(T, *res)
        seq.append(res)
        nstd += 1
        z = objective(T)
        if z > obj_val:                       # simplex.py:133
            raise ObjectiveIncreased("objective value increased (internal error)")
        stuck = stuck + 1 if z == obj_val else 0
    while True:
        if cap is not None and len(seq) >= cap:
            return {"status": "cap", "npiv": len(seq), "nstd": nstd, "seq": seq}
        res = find_min_index(T)
        if res == "unbounded":
            raise Unbounded("unbounded artificial problem (internal error)")
        if res == "optimal":
            return {"status": "optimal", "npiv": len(seq), "nstd": nstd, "seq": seq}
        pivot(T, *res)
        seq.append(res)


def run_standard(T, k: int) -> list:
    """k pivots of findPivotStandard(do_pivot=True) (no stall logic): the
    fixed-K timing loop of bench.py.  Stops early on optimal/unbounded and
    appends that string."""
    seq = []
    for _ in range(k):
        res = find_standard(T)
        if isinstance(res, str):
            seq.append(res)
            break
        pivot(T, *res)
        seq.append(res)
    return seq


# --------------------------------------------------------------------------
# form checks  (lpsol/tableau.py:466-521)
# --------------------------------------------------------------------------

def is_canonical(T) -> tuple[bool, list[int]]:
    """isCanonical (``tableau.py:466-496``): b >= 0 and, for every row, some
    column with zero reduced cost that is a unit vector with its one there.
    bcols[i] = first such column, -1 if none."""
    m, n = size(T)
    bcols = [-1] * m
    if any(T[i][0] < ZERO for i in range(1, m + 1)):
        return False, bcols
    for j in range(n):
        if T[0][j + 1] != ZERO:
            continue
        one = next((i for i in range(m) if T[i + 1][j + 1] == ONE), -1)
        if one == -1:
            continue
        if all(i == one or T[i + 1][j + 1] == ZERO for i in range(m)):
            if bcols[one] == -1:
                bcols[one] = j
    return all(x != -1 for x in bcols), bcols


def is_optimal(T) -> bool:
    return all(x >= ZERO for x in T[0][1:])


def is_unbounded(T) -> bool:
    m, n = size(T)
    return any(T[0][j + 1] < ZERO and all(T[i + 1][j + 1] <= ZERO for i in range(m))
               for j in range(n))


def is_infeasible(T) -> bool:
    m, n = size(T)
    return any(T[i + 1][0] > ZERO and all(T[i + 1][j + 1] <= ZERO for j in range(n))
               for i in range(m))


def is_degenerate(T) -> bool:
    return any(T[i][0] == ZERO for i in range(1, len(T)))


def frac_str(x: Fraction) -> str:
    return f"{x.numerator}/{x.denominator}"


def parse_frac(s: str) -> Fraction:
    return Fraction(s)


def seq_pairs(seq: Iterable) -> list[list[int]]:
    return [[int(r), int(c)] for r, c in seq]
