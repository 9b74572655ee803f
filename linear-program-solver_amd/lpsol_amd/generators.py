"""Deterministic synthetic dense LPs in the engine's tableau layout.

The reference ships no benchmark inputs, so the build fixes its
own generator.  Every value is a dyadic rational k/Q (Q = 64 by default), which
is exact in float64 and keeps the exact-Fraction oracle's denominators small.

Layout (SURVEY.md §8 conventions, reference `lpsol/tableau.py:44-52`):
    T[0, 0]      = stored objective cell ``_z`` (the NEGATED objective,
                   `tableau.py:82-84,128-130`); 0 for a fresh LP
    T[0, 1 + j]  = reduced cost c_j
    T[1 + i, 0]  = b_i
    T[1 + i, 1 + j] = a_ij

The random stream is counter-based (splitmix64 finaliser of seed/stream/index),
so any row block of a tableau can be produced independently -- a rank of the
row-sharded engine generates only its own rows.
"""
from __future__ import annotations

import hashlib

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# stream ids for the independent fields of one LP
S_A, S_B, S_C = 1, 2, 3


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def draw(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """64-bit pseudo-random words for counter indices ``idx`` (uint64)."""
    with np.errstate(over="ignore"):
        word = (seed * 0x100000001B3 + stream) & 0xFFFFFFFFFFFFFFFF
        key = _mix(np.asarray([word], dtype=np.uint64) * _GOLD)[0]
        return _mix(key + (np.asarray(idx, dtype=np.uint64) + np.uint64(1)) * _GOLD)


def uint_range(seed: int, stream: int, idx: np.ndarray, lo: int, hi: int) -> np.ndarray:
    """Integers in [lo, hi] (inclusive) as int64."""
    span = np.uint64(hi - lo + 1)
    return (draw(seed, stream, idx) % span).astype(np.int64) + lo


# ---------------------------------------------------------------------------
# generator kinds
#   mixed : A_ij = U{-Q..Q}/Q, first constraint row all ones with b_0 = ns
#           (bounds the LP), b_i = U{1..Q}/Q, c_j = -U{1..Q}/Q, slack basis.
#           Many pivots (good for fixed-K timing).            SURVEY §8(d)
#   pos   : A_ij = U{1..Q}/Q, b_i in [1, ns/4 + 1], c_j = -U{1..Q}/Q, slacks.
#           Solves in tens of pivots (good for full-solve parity).
#   tall  : no slack columns; A_ij = U{-Q..Q}/Q (row 0 of A all ones,
#           b_0 = ncols), b_i in [1, 2], c_j = -U{1..Q}/Q.  Not canonical:
#           driven by a fixed number of standard-rule pivots.
# ---------------------------------------------------------------------------

KINDS = ("mixed", "pos", "tall")


def shape(kind: str, m: int, ns: int) -> tuple[int, int]:
    """(m, n) of the constraint matrix for a generator call."""
    if kind == "tall":
        return m, ns
    return m, ns + m


def rows(kind: str, m: int, ns: int, seed: int, r0: int, r1: int,
         Q: int = 64) -> np.ndarray:
    """Tableau rows [r0, r1) (row 0 = objective) as float64, width n + 1."""
    if kind not in KINDS:
        raise ValueError(f"unknown generator kind {kind!r}")
    m_, n = shape(kind, m, ns)
    if not (0 <= r0 <= r1 <= m_ + 1):
        raise ValueError("row range out of bounds")
    out = np.zeros((r1 - r0, n + 1), dtype=np.float64)
    q = float(Q)
    for R in range(r0, r1):
        row = out[R - r0]
        if R == 0:
            j = np.arange(ns, dtype=np.uint64)
            row[1:1 + ns] = -uint_range(seed, S_C, j, 1, Q) / q
            continue
        i = R - 1
        j = np.arange(ns, dtype=np.uint64) + np.uint64(i * ns)
        if kind == "pos":
            row[1:1 + ns] = uint_range(seed, S_A, j, 1, Q) / q
            row[0] = uint_range(seed, S_B, np.asarray([i], np.uint64),
                                0, Q * (ns // 4))[0] / q + 1.0
        else:
            if i == 0:
                row[1:1 + ns] = 1.0
            else:
                row[1:1 + ns] = uint_range(seed, S_A, j, -Q, Q) / q
            if i == 0:
                row[0] = float(ns)
            elif kind == "mixed":
                row[0] = uint_range(seed, S_B, np.asarray([i], np.uint64), 1, Q)[0] / q
            else:
                row[0] = uint_range(seed, S_B, np.asarray([i], np.uint64), 0, Q)[0] / q + 1.0
        if kind != "tall":
            row[1 + ns + i] = 1.0
    return out


def tableau(kind: str, m: int, ns: int, seed: int, Q: int = 64) -> np.ndarray:
    m_, _ = shape(kind, m, ns)
    return rows(kind, m, ns, seed, 0, m_ + 1, Q)


def digest(T: np.ndarray) -> str:
    """sha256 of the float64 little-endian bytes (fixture identity)."""
    return hashlib.sha256(np.ascontiguousarray(T, dtype="<f8").tobytes()).hexdigest()


# --- hand-built classic LPs (small, exact) ---------------------------------

def beale() -> np.ndarray:
    """Beale's cycling LP (3 x 7) with slack basis x1..x3.

    min -3/4 x4 + 150 x5 - 1/50 x6 + 6 x7
        x1 + 1/4 x4 -  60 x5 - 1/25 x6 + 9 x7 = 0
        x2 + 1/2 x4 -  90 x5 - 1/50 x6 + 3 x7 = 0
        x3                  +      x6        = 1
    """
    T = np.zeros((4, 8))
    T[0, 1:] = [0, 0, 0, -0.75, 150, -1 / 50, 6]
    T[1, :] = [0, 1, 0, 0, 0.25, -60, -1 / 25, 9]
    T[2, :] = [0, 0, 1, 0, 0.5, -90, -1 / 50, 3]
    T[3, :] = [1, 0, 0, 1, 0, 0, 1, 0]
    return T


def beale_exact():
    """Beale's LP as exact strings (1/50, 1/25 are not dyadic)."""
    z = "0"
    c = ["0", "0", "0", "-3/4", "150", "-1/50", "6"]
    b = ["0", "0", "1"]
    a = [["1", "0", "0", "1/4", "-60", "-1/25", "9"],
         ["0", "1", "0", "1/2", "-90", "-1/50", "3"],
         ["0", "0", "1", "0", "0", "1", "0"]]
    return z, c, b, a


def klee_minty(d: int, degenerate: bool = False) -> np.ndarray:
    """Klee-Minty cube in standard form with slacks: m = d, n = 2d.

    max sum_j 2^(d-j) x_j  (as min of the negation)
    s.t. 2 * sum_{j<i} 2^(i-j) x_j + x_i <= 5^i,   i = 1..d
    degenerate=True sets b_i = 0 for even i (a degenerate, stalling variant).
    """
    T = np.zeros((d + 1, 2 * d + 1))
    for j in range(1, d + 1):
        T[0, j] = -float(2 ** (d - j))
    for i in range(1, d + 1):
        for j in range(1, i):
            T[i, j] = float(2 ** (i - j + 1))
        T[i, i] = 1.0
        T[i, d + i] = 1.0
        T[i, 0] = 0.0 if (degenerate and i % 2 == 0) else float(5 ** i)
    return T


# ---------------------------------------------------------------------------
# LPs that need phase 1 (Simplex._find_bfs, simplex.py:36-108): general
# constraints with x0 >= 0 a known feasible point, all values dyadic.
#   eq   : A x = b (no slacks), plus sum x = S (bounds the region)
#   ge   : A x >= b with surplus columns (-1), plus sum x <= S with a slack
#   neg  : A x <= b with slacks, some b_i < 0 (phase 1 flips those rows)
#   dep  : eq plus a repeated row (linearly dependent: the reference raises
#          IndexError there, simplex.py:93)
#   infeasible : sum x = 1 and sum x = 2
# ---------------------------------------------------------------------------

def phase1_lp(kind: str, m: int, ns: int, seed: int, Q: int = 64) -> np.ndarray:
    if kind == "infeasible":
        T = np.zeros((3, ns + 1))
        T[0, 1:] = -1.0
        T[1:, 1:] = 1.0
        T[1, 0], T[2, 0] = 1.0, 2.0
        return T
    idx = np.arange(m * ns, dtype=np.uint64)
    A = uint_range(seed, S_A, idx, -Q, Q).reshape(m, ns) / Q
    x0 = uint_range(seed, 7, np.arange(ns, dtype=np.uint64), 0, 4) / 4.0
    c = -uint_range(seed, S_C, np.arange(ns, dtype=np.uint64), 1, Q) / Q
    S = float(np.sum(x0)) + 1.0
    if kind in ("eq", "dep"):
        b = A @ x0
        rows_a = [A, np.ones((1, ns))]
        rows_b = [b, [float(np.sum(x0))]]
        if kind == "dep":
            rows_a.append(A[:1])
            rows_b.append(b[:1])
        Af = np.vstack(rows_a)
        bf = np.concatenate([np.asarray(r, dtype=np.float64) for r in rows_b])
        cf = c
    elif kind == "ge":
        b = A @ x0 - uint_range(seed, S_B, np.arange(m, dtype=np.uint64), 0, 2) / 4.0
        Af = np.zeros((m + 1, ns + m + 1))
        Af[:m, :ns] = A
        Af[:m, ns:ns + m] = -np.eye(m)
        Af[m, :ns] = 1.0
        Af[m, ns + m] = 1.0
        bf = np.concatenate([b, [S]])
        cf = np.concatenate([c, np.zeros(m + 1)])
    elif kind == "neg":
        b = A @ x0 + uint_range(seed, S_B, np.arange(m, dtype=np.uint64), 0, 2) / 4.0
        Af = np.zeros((m + 1, ns + m + 1))
        Af[:m, :ns] = A
        Af[:m, ns:ns + m] = np.eye(m)
        Af[m, :ns] = 1.0
        Af[m, ns + m] = 1.0
        bf = np.concatenate([b, [S]])
        cf = np.concatenate([c, np.zeros(m + 1)])
    else:
        raise ValueError(kind)
    T = np.zeros((Af.shape[0] + 1, Af.shape[1] + 1))
    T[0, 1:] = cf
    T[1:, 0] = bf
    T[1:, 1:] = Af
    assert np.all(T * 4096 == np.round(T * 4096))     # dyadic: exact in float64
    return T
