/*
 * ORACLE self-check under AddressSanitizer + UndefinedBehaviorSanitizer
 * (test infrastructure only; `make -C oracle sanitize`, run by
 * tests/test_oracle.py::test_oracle_under_sanitizers).
 *
 * Every tableau is malloc'ed at its exact size (ld = n + 1, no padding), so an
 * out-of-bounds row or column access in lp_f64.c is an ASan report, and any
 * signed overflow / bad shift / misaligned access is a UBSan abort
 * (-fno-sanitize-recover=all).  Besides running clean, it checks invariants
 * that hold for the reference's algorithm (lpsol/tableau.py:295-308,
 * lpsol/simplex.py:110-148, :251-284, :286-360):
 *   - lpf_prow + lpf_apply is bit-identical to lpf_pivot,
 *   - lpf_solve ends OPTIMAL (or UNBOUNDED) with no negative reduced cost
 *     below -tol.cost, a non-negative RHS, and an objective (-T[0]) that did
 *     not increase,
 *   - lpf_run with the standard rule replays lpf_solve's pivot log while the
 *     solve has not switched to the min-index rule,
 *   - lpf_find_all lists the pivot lpf_find picks, lpf_find_max_increase's
 *     pivot is among lpf_find_all's.
 * Exit status 0 = clean; the failing check is printed otherwise.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lpgpu.h"

int lpf_pivot(double *T, int64_t m, int64_t n, int64_t ld, int64_t r, int64_t c);
int lpf_find(const double *T, int64_t m, int64_t n, int64_t ld, int rule, const lp_tol *tol,
             int64_t *r, int64_t *c);
int lpf_run(double *T, int64_t m, int64_t n, int64_t ld, int rule, const lp_tol *tol, int64_t k,
            int64_t *log, int64_t *npiv);
int lpf_solve(double *T, int64_t m, int64_t n, int64_t ld, const lp_tol *tol, int64_t cap,
              int64_t *log, int64_t *npiv, int64_t *nstd);
void lpf_prow(const double *row, int64_t n, int64_t C, double *P);
void lpf_apply(double *T, int64_t rows, int64_t n, int64_t ld, const double *P, int64_t C,
               int64_t Rloc);
int lpf_find_max_increase(const double *T, int64_t m, int64_t n, int64_t ld, const lp_tol *tol,
                          int64_t *r, int64_t *c);
int64_t lpf_find_all(const double *T, int64_t m, int64_t n, int64_t ld, const lp_tol *tol,
                     int64_t *rc, int64_t cap);

static int failures;
#define CHECK(cond, ...)                                                                   \
    do {                                                                                   \
        if (!(cond)) {                                                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                           \
            fprintf(stderr, __VA_ARGS__);                                                  \
            fputc('\n', stderr);                                                           \
            ++failures;                                                                    \
        }                                                                                  \
    } while (0)

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint64_t next_u64(void)
{
    uint64_t z = (rng += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
/* dyadic k/64 in [lo, hi] (exact in float64, like lpsol_amd.generators) */
static double dyadic(int lo, int hi) { return (double)(lo * 64 + (int)(next_u64() % (uint64_t)((hi - lo) * 64 + 1))) / 64.0; }

/* canonical max c.x s.t. A x <= b, x >= 0 with slacks: row 0 = [0 | -c | 0],
 * row i = [b_i | A_i | e_i]  (the reference's Tableau layout, tableau.py:44-52) */
static double *random_lp(int64_t m, int64_t nv, int64_t *n_out)
{
    const int64_t n = nv + m, ld = n + 1;
    double *T = calloc((size_t)((m + 1) * ld), sizeof(double));
    for (int64_t j = 0; j < nv; ++j) T[1 + j] = -dyadic(0, 4);
    for (int64_t i = 1; i <= m; ++i) {
        double *t = T + i * ld;
        t[0] = dyadic(1, 16);
        for (int64_t j = 0; j < nv; ++j) t[1 + j] = (next_u64() % 4 == 0) ? 0.0 : dyadic(-1, 4);
        t[1 + nv + (i - 1)] = 1.0;
    }
    *n_out = n;
    return T;
}

/* Klee-Minty cube of dimension d (max sum 2^(d-i) x_i; degenerate-free but
 * exponential for Dantzig's rule) */
static double *klee_minty(int64_t d, int64_t *n_out)
{
    const int64_t m = d, n = 2 * d, ld = n + 1;
    double *T = calloc((size_t)((m + 1) * ld), sizeof(double));
    for (int64_t j = 0; j < d; ++j) T[1 + j] = -ldexp(1.0, (int)(d - 1 - j));
    for (int64_t i = 1; i <= d; ++i) {
        double *t = T + i * ld;
        t[0] = ldexp(1.0, (int)(2 * i));   /* 5^i scaled to powers of two keeps it exact */
        for (int64_t j = 0; j < i - 1; ++j) t[1 + j] = ldexp(1.0, (int)(i - j));
        t[i] = 1.0;
        t[1 + d + (i - 1)] = 1.0;
    }
    *n_out = n;
    return T;
}

static void check_pivot_split(const double *T0, int64_t m, int64_t n, const lp_tol *tol)
{
    const int64_t ld = n + 1;
    const size_t sz = (size_t)((m + 1) * ld) * sizeof(double);
    int64_t r, c;
    if (lpf_find(T0, m, n, ld, LP_RULE_STANDARD, tol, &r, &c) != LP_PIVOTED) return;
    double *A = malloc(sz), *B = malloc(sz), *P = malloc((size_t)ld * sizeof(double));
    memcpy(A, T0, sz);
    memcpy(B, T0, sz);
    CHECK(lpf_pivot(A, m, n, ld, r, c) == LP_PIVOTED, "pivot (%lld,%lld)", (long long)r, (long long)c);
    lpf_prow(B + (r + 1) * ld, n, c + 1, P);
    lpf_apply(B, m + 1, n, ld, P, c + 1, r + 1);
    CHECK(memcmp(A, B, sz) == 0, "prow+apply differs from pivot at (%lld,%lld)", (long long)r, (long long)c);
    CHECK(lpf_pivot(A, m, n, ld, m, 0) == LP_BAD_ARG, "row m accepted");
    CHECK(lpf_pivot(A, m, n, ld, 0, n) == LP_BAD_ARG, "column n accepted");
    free(A);
    free(B);
    free(P);
}

static void check_solve(const double *T0, int64_t m, int64_t n, const lp_tol *tol, const char *what)
{
    const int64_t ld = n + 1;
    const size_t sz = (size_t)((m + 1) * ld) * sizeof(double);
    const int64_t cap = 4 * (m + n) + 4096;
    double *T = malloc(sz), *U = malloc(sz);
    int64_t *log = malloc((size_t)(2 * cap) * sizeof(int64_t));
    int64_t *log2 = malloc((size_t)(2 * cap) * sizeof(int64_t));
    memcpy(T, T0, sz);
    int64_t npiv, nstd;
    const int st = lpf_solve(T, m, n, ld, tol, cap, log, &npiv, &nstd);
    CHECK(st == LP_OPTIMAL || st == LP_UNBOUNDED, "%s: solve status %d", what, st);
    CHECK(-T[0] <= -T0[0] + tol->stall * fmax(1.0, fabs(T0[0])), "%s: objective rose", what);   /* simplex.py:133 */
    if (st == LP_OPTIMAL) {
        for (int64_t j = 1; j <= n; ++j) CHECK(!(T[j] < -tol->cost), "%s: c_%lld < 0 at optimum", what, (long long)j);
        for (int64_t i = 1; i <= m; ++i) CHECK(T[i * ld] >= -1e-9, "%s: b_%lld < 0", what, (long long)i);
    }
    /* the standard-rule prefix of the solve replays with lpf_run */
    memcpy(U, T0, sz);
    int64_t nrun;
    lpf_run(U, m, n, ld, LP_RULE_STANDARD, tol, nstd, log2, &nrun);
    CHECK(nrun == nstd, "%s: run made %lld of %lld pivots", what, (long long)nrun, (long long)nstd);
    CHECK(memcmp(log, log2, (size_t)(2 * nrun) * sizeof(int64_t)) == 0, "%s: pivot logs differ", what);
    free(T);
    free(U);
    free(log);
    free(log2);
}

static void check_scans(const double *T0, int64_t m, int64_t n, const lp_tol *tol, const char *what)
{
    const int64_t ld = n + 1;
    int64_t r, c, rm, cm;
    const int st = lpf_find(T0, m, n, ld, LP_RULE_STANDARD, tol, &r, &c);
    const int64_t cnt = lpf_find_all(T0, m, n, ld, tol, NULL, 0);
    int64_t *rc = malloc((size_t)(2 * (cnt > 0 ? cnt : 1)) * sizeof(int64_t));
    CHECK(lpf_find_all(T0, m, n, ld, tol, rc, cnt) == cnt, "%s: find_all count", what);
    int found = 0, found_mi = 0;
    const int smi = lpf_find_max_increase(T0, m, n, ld, tol, &rm, &cm);
    for (int64_t k = 0; k < cnt; ++k) {
        if (rc[2 * k] == r && rc[2 * k + 1] == c) found = 1;
        if (rc[2 * k] == rm && rc[2 * k + 1] == cm) found_mi = 1;
    }
    if (st == LP_PIVOTED) CHECK(found, "%s: find_all lacks (%lld,%lld)", what, (long long)r, (long long)c);
    if (smi == LP_PIVOTED) CHECK(found_mi, "%s: find_all lacks max-increase pivot", what);
    free(rc);
}

int main(void)
{
    const lp_tol tol = {1e-9, 1e-12, 1e-9, 1e-9, 1e-12, 1e-12};   /* lp_default_tol's values */
    static const int64_t shapes[][2] = {{1, 1}, {2, 3}, {8, 10}, {17, 5}, {31, 64}, {64, 33}, {100, 100}};
    char what[64];
    for (size_t s = 0; s < sizeof shapes / sizeof shapes[0]; ++s)
        for (int rep = 0; rep < 3; ++rep) {
            int64_t n;
            double *T = random_lp(shapes[s][0], shapes[s][1], &n);
            snprintf(what, sizeof what, "random %lldx%lld #%d", (long long)shapes[s][0],
                     (long long)shapes[s][1], rep);
            check_pivot_split(T, shapes[s][0], n, &tol);
            check_scans(T, shapes[s][0], n, &tol, what);
            check_solve(T, shapes[s][0], n, &tol, what);
            free(T);
        }
    for (int64_t d = 2; d <= 8; ++d) {
        int64_t n;
        double *T = klee_minty(d, &n);
        snprintf(what, sizeof what, "klee-minty d=%lld", (long long)d);
        check_pivot_split(T, d, n, &tol);
        check_scans(T, d, n, &tol, what);
        check_solve(T, d, n, &tol, what);
        free(T);
    }
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("oracle sanitizer self-check: clean\n");
    return 0;
}
