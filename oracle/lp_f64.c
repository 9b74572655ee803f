/*
 * ORACLE -- test infrastructure only, never part of the product path.
 *
 * Scalar float64 restatement of the reference's dense simplex hot path with
 * EXACTLY the floating-point semantics the HIP engine implements, so the
 * engine's whole tableau can be compared BIT FOR BIT at sizes where the
 * exact-Fraction oracle (oracle/exact.py) is too slow.  Its own agreement
 * with the reference (pivot sequences, objectives) is pinned by the golden
 * vectors in tests/golden/ (tests/test_oracle.py).
 *
 * Reference being restated (tkoz0/linear-program-solver, package lpsol):
 *   lpf_pivot      <- Tableau.pivot            lpsol/tableau.py:295-308
 *   lpf_find (0)   <- findPivotStandard        lpsol/simplex.py:251-284
 *   lpf_find (1)   <- findPivotMinIndex        lpsol/simplex.py:218-249
 *   lpf_solve      <- Simplex.solve            lpsol/simplex.py:110-148
 *   lpf_find_max_increase <- findPivotMaxIncrease  lpsol/simplex.py:286-328
 *   lpf_find_all   <- findPivotAll             lpsol/simplex.py:330-360
 *
 * Float semantics (the contract shared with linear-program-solver_amd/csrc):
 *   pivot(r,c): R=r+1, C=c+1, a=T[R][C] (a==0 -> ZERO_PIVOT)
 *     P[j] = T[R][j] / a (IEEE division), P[C] = 1
 *     for every row i != R, f = T[i][C]:
 *         T[i][j] = fma(-f, P[j], T[i][j])  for all j (at j = C this is exactly +0)
 *     T[R] = P
 *   The reference skips rows whose multiplier is zero (tableau.py:272); in
 *   float64 fma(-0, p, x) == x for every finite x (only the sign of a zero x
 *   can differ), so rows are not skipped -- the branch-free form lets the
 *   engine's deferred sweep be pure FMAs.
 *   entering, standard : g = min c_j; optimal unless g < -tol.cost;
 *                        c = first j with c_j <= g + tol.cost_tie*|g|
 *   entering, min-index: c = first j with c_j < -tol.cost
 *   ratio test         : rows with a_ic > tol.pivot; num = |b_i| <= tol.zero ? 0 : b_i
 *                        q_i = num / a_ic; g = min q; r = first i with
 *                        q_i <= g + tol.ratio_tie*|g|
 *   stall (solve)      : |z - z0| <= tol.stall * max(1, |z0|); z - z0 above
 *                        that band stops the solve with LP_OBJ_INCREASED
 *                        (simplex.py:133 asserts z <= obj_val)
 *   max increase       : over columns with c_j < -tol.cost: g_j = min ratio of
 *                        the column (ratio test above); 'unbounded' if any such
 *                        column has no row with a > tol.pivot (the reference
 *                        returns at the first one, :319-320); inc_j = -c_j * g_j;
 *                        M = max inc; j = first column with inc_j >= M - tol.ratio_tie*|M|,
 *                        i = its ratio-test row; 'optimal' if no such column
 *   all pivots         : for every column (any c_j), every row with
 *                        q_i <= g_j + tol.ratio_tie*|g_j|, column-major, rows in order
 * Build with -ffp-contract=off (no implicit fusing anywhere).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lpgpu.h"

static double *row(double *T, int64_t ld, int64_t i) { return T + i * ld; }

int lpf_pivot(double *T, int64_t m, int64_t n, int64_t ld, int64_t r, int64_t c)
{
    if (r < 0 || r >= m || c < 0 || c >= n) return LP_BAD_ARG;
    const int64_t R = r + 1, C = c + 1;
    double *p = row(T, ld, R);
    const double a = p[C];
    if (a == 0.0) return LP_ZERO_PIVOT;
    for (int64_t j = 0; j <= n; ++j) p[j] = p[j] / a;
    p[C] = 1.0;
    /* rows are independent: split over host threads for the headline sizes
       (each element gets the same operations whichever thread runs it) */
#pragma omp parallel for schedule(static) if ((m + 1) * (n + 1) > (1 << 22))
    for (int64_t i = 0; i <= m; ++i) {
        if (i == R) continue;
        double *t = row(T, ld, i);
        const double f = t[C];
        for (int64_t j = 0; j <= n; ++j) t[j] = fma(-f, p[j], t[j]);
    }
    return LP_PIVOTED;
}

static int64_t entering(const double *T, int64_t n, int rule, const lp_tol *tol)
{
    const double *c0 = T;
    if (rule == LP_RULE_MIN_INDEX) {
        for (int64_t j = 1; j <= n; ++j)
            if (c0[j] < -tol->cost) return j - 1;
        return -1;
    }
    double g = INFINITY;
    for (int64_t j = 1; j <= n; ++j)
        if (c0[j] < g) g = c0[j];
    if (!(g < -tol->cost)) return -1;
    const double thr = g + tol->cost_tie * fabs(g);
    for (int64_t j = 1; j <= n; ++j)
        if (c0[j] <= thr) return j - 1;
    return -1; /* unreachable */
}

static double ratio_of(const double *t, int64_t C, const lp_tol *tol, int *ok)
{
    const double a = t[C];
    if (!(a > tol->pivot)) { *ok = 0; return 0.0; }
    *ok = 1;
    const double b = t[0];
    const double num = fabs(b) <= tol->zero ? 0.0 : b;
    return num / a;
}

static int64_t leaving(const double *T, int64_t m, int64_t ld, int64_t c, const lp_tol *tol)
{
    const int64_t C = c + 1;
    double g = INFINITY;
    int any = 0;
    for (int64_t i = 1; i <= m; ++i) {
        int ok;
        const double q = ratio_of(T + i * ld, C, tol, &ok);
        if (ok && (!any || q < g)) { g = q; any = 1; }
    }
    if (!any) return -1;
    const double thr = g + tol->ratio_tie * fabs(g);
    for (int64_t i = 1; i <= m; ++i) {
        int ok;
        const double q = ratio_of(T + i * ld, C, tol, &ok);
        if (ok && q <= thr) return i - 1;
    }
    return -1; /* unreachable */
}

int lpf_find(const double *T, int64_t m, int64_t n, int64_t ld, int rule,
             const lp_tol *tol, int64_t *r, int64_t *c)
{
    *r = -1;
    *c = entering(T, n, rule, tol);
    if (*c < 0) return LP_OPTIMAL;
    *r = leaving(T, m, ld, *c, tol);
    if (*r < 0) return LP_UNBOUNDED;
    return LP_PIVOTED;
}

/* k pivots with one fixed rule (no stall logic); log gets 2 entries per pivot */
int lpf_run(double *T, int64_t m, int64_t n, int64_t ld, int rule, const lp_tol *tol,
            int64_t k, int64_t *log, int64_t *npiv)
{
    *npiv = 0;
    for (int64_t t = 0; t < k; ++t) {
        int64_t r, c;
        const int st = lpf_find(T, m, n, ld, rule, tol, &r, &c);
        if (st != LP_PIVOTED) return st;
        lpf_pivot(T, m, n, ld, r, c);
        if (log) { log[2 * t] = r; log[2 * t + 1] = c; }
        ++*npiv;
    }
    return LP_PIVOTED;
}

int lpf_solve(double *T, int64_t m, int64_t n, int64_t ld, const lp_tol *tol,
              int64_t cap, int64_t *log, int64_t *npiv, int64_t *nstd)
{
    *npiv = 0;
    *nstd = 0;
    const double z0 = -T[0];
    int64_t stuck = 0;
    int rule = LP_RULE_STANDARD;
    for (;;) {
        if (rule == LP_RULE_STANDARD && stuck >= m + n) rule = LP_RULE_MIN_INDEX;
        if (cap >= 0 && *npiv >= cap) return LP_CAP_REACHED;
        int64_t r, c;
        const int st = lpf_find(T, m, n, ld, rule, tol, &r, &c);
        if (st != LP_PIVOTED) return st;
        lpf_pivot(T, m, n, ld, r, c);
        if (log) { log[2 * *npiv] = r; log[2 * *npiv + 1] = c; }
        ++*npiv;
        if (rule == LP_RULE_STANDARD) {
            ++*nstd;
            const double z = -T[0];
            const double band = tol->stall * fmax(1.0, fabs(z0));
            if (z - z0 > band) return LP_OBJ_INCREASED;   /* simplex.py:133, after the pivot */
            if (fabs(z - z0) <= band) ++stuck;
            else stuck = 0;
        }
    }
}

/* ---- pieces of one pivot, for the row-sharded protocol model ------------- */

/* P = row / row[C], P[C] = 1  (the normalised pivot row) */
void lpf_prow(const double *row, int64_t n, int64_t C, double *P)
{
    const double a = row[C];
    for (int64_t j = 0; j <= n; ++j) P[j] = row[j] / a;
    P[C] = 1.0;
}

/* apply the pivot (P, tableau column C) to `rows` stored rows; local row
 * Rloc (or -1) becomes P, every other row gets fma(-f, P[j], x) */
void lpf_apply(double *T, int64_t rows, int64_t n, int64_t ld, const double *P, int64_t C,
               int64_t Rloc)
{
    for (int64_t i = 0; i < rows; ++i) {
        double *t = T + i * ld;
        if (i == Rloc) {
            for (int64_t j = 0; j <= n; ++j) t[j] = P[j];
            continue;
        }
        const double f = t[C];
        for (int64_t j = 0; j <= n; ++j) t[j] = fma(-f, P[j], t[j]);
    }
}

/* ratio-test pieces over `rows` stored constraint rows (no row 0):
 * *lmin = min ratio (INFINITY if none eligible); returns the first row with
 * ratio <= thr (or -1) and its ratio in *q */
double lpf_min_ratio(const double *T, int64_t rows, int64_t ld, int64_t C, const lp_tol *tol)
{
    double g = INFINITY;
    for (int64_t i = 0; i < rows; ++i) {
        int ok;
        const double q = ratio_of(T + i * ld, C, tol, &ok);
        if (ok && q < g) g = q;
    }
    return g;
}

int64_t lpf_first_within(const double *T, int64_t rows, int64_t ld, int64_t C, const lp_tol *tol,
                         double thr, double *q_out)
{
    for (int64_t i = 0; i < rows; ++i) {
        int ok;
        const double q = ratio_of(T + i * ld, C, tol, &ok);
        if (ok && q <= thr) { *q_out = q; return i; }
    }
    return -1;
}

int64_t lpf_entering(const double *row0, int64_t n, int rule, const lp_tol *tol)
{
    return entering(row0, n, rule, tol);
}

/* findPivotMaxIncrease (simplex.py:286-328).  The reference's tie branch at
 * :316-318 can never fire (equal ratios give equal increases), so the first
 * column of the maximum wins. */
int lpf_find_max_increase(const double *T, int64_t m, int64_t n, int64_t ld, const lp_tol *tol,
                          int64_t *r, int64_t *c)
{
    *r = -1;
    *c = -1;
    double M = -INFINITY;
    int any_neg = 0;
    double *inc = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    for (int64_t j = 0; j < n; ++j) {
        inc[j] = -INFINITY;
        if (!(T[1 + j] < -tol->cost)) continue;
        any_neg = 1;
        const double g = lpf_min_ratio(T + ld, m, ld, j + 1, tol);
        if (!(g < INFINITY)) {
            free(inc);
            return LP_UNBOUNDED;
        }
        inc[j] = -T[1 + j] * g;
        if (inc[j] > M) M = inc[j];
    }
    if (!any_neg) {
        free(inc);
        return LP_OPTIMAL;
    }
    const double thr = M - tol->ratio_tie * fabs(M);
    for (int64_t j = 0; j < n; ++j)
        if (inc[j] >= thr) {
            *c = j;
            *r = leaving(T, m, ld, j, tol);
            break;
        }
    free(inc);
    return LP_PIVOTED;
}

/* findPivotAll (simplex.py:330-360): writes up to cap (r, c) pairs, returns
 * how many there are */
int64_t lpf_find_all(const double *T, int64_t m, int64_t n, int64_t ld, const lp_tol *tol,
                     int64_t *rc, int64_t cap)
{
    int64_t cnt = 0;
    for (int64_t j = 0; j < n; ++j) {
        const double g = lpf_min_ratio(T + ld, m, ld, j + 1, tol);
        if (!(g < INFINITY)) continue;
        const double thr = g + tol->ratio_tie * fabs(g);
        for (int64_t i = 0; i < m; ++i) {
            int ok;
            const double q = ratio_of(T + (i + 1) * ld, j + 1, tol, &ok);
            if (ok && q <= thr) {
                if (cnt < cap) {
                    rc[2 * cnt] = i;
                    rc[2 * cnt + 1] = j;
                }
                ++cnt;
            }
        }
    }
    return cnt;
}
