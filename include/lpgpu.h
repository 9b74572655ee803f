/*
 * lpgpu.h -- C-ABI of the MI355X dense simplex pivot engine (liblpgpu.so).
 *
 * The reference (tkoz0/linear-program-solver, package lpsol) is pure Python
 * with no FFI: its "operator API" for the hot path is the method surface
 * Simplex calls on Tableau.  Per-element getters cannot
 * cross a device boundary cheaply, so the boundary is lifted one level: each
 * entry point below replaces a whole reference method (cited file:line), and
 * the Python front-end (linear-program-solver_amd/lpsol_amd) binds them with
 * ctypes behind the reference's own class and method names.
 *
 * Conventions
 *   - The tableau is (m+1) x (n+1) float64, row-major.  Row 0 is
 *     [_z, c_0..c_{n-1}] with _z the stored NEGATED objective
 *     (lpsol/tableau.py:46,82-84); row 1+i is [b_i, a_i0..a_i,n-1].
 *   - r indexes constraints (0..m-1), c indexes variables (0..n-1), exactly
 *     like the reference's pivot(r, c).
 *   - Host buffers are caller-owned and copied synchronously.  The library
 *     owns all device memory.  A handle is used by one host thread at a time.
 *   - No exceptions cross the ABI: every call returns an lp_status; the
 *     front-end maps them to the reference's exceptions.
 */
#ifndef LPGPU_H
#define LPGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum lp_status {
    LP_PIVOTED = 0,      /* a pivot was found (and performed, where asked)   */
    LP_OPTIMAL = 1,      /* 'optimal'   simplex.py:233-234,268-269            */
    LP_UNBOUNDED = 2,    /* 'unbounded' simplex.py:245-246,280-281            */
    LP_ZERO_PIVOT = -1,  /* ZeroDivisionError('zero pivot r,c') tableau.py:300-301 */
    LP_BAD_ARG = -2,     /* ValueError / IndexError in the reference          */
    LP_DEVICE_ERROR = -3,/* HIP or RCCL failure; see lp_last_error            */
    LP_CAP_REACHED = -4, /* extension: pivot cap hit before optimality        */
    LP_BAD_PIVOT = -5,   /* ValueError('bad pivot by min ratio test') simplex.py:214-215 */
    LP_OBJ_INCREASED = -6 /* AssertionError('objective value increased') simplex.py:133:
                            a standard-rule pivot of lp_solve left the objective above
                            its value at the start of the call by more than the stall
                            tolerance; the solve stops after that pivot */
} lp_status;

typedef enum lp_rule {
    LP_RULE_STANDARD = 0,  /* findPivotStandard   simplex.py:251-284 */
    LP_RULE_MIN_INDEX = 1  /* findPivotMinIndex   simplex.py:218-249 */
} lp_rule;

/* Float64 stand-ins for the reference's exact rational comparisons. */
typedef struct lp_tol {
    double cost;      /* c_j is negative iff c_j < -cost     (simplex.py:229,264)  */
    double cost_tie;  /* standard rule: first j with c_j <= g + cost_tie*|g|,
                         g = min c_j                        (simplex.py:266)       */
    double pivot;     /* a_ij is positive iff a_ij > pivot  (simplex.py:239,274)  */
    double zero;      /* |b_i| <= zero counts as b_i = 0 in the ratio             */
    double ratio_tie; /* first i with q_i <= g + ratio_tie*|g| (simplex.py:242,277) */
    double stall;     /* |z - z0| <= stall*max(1,|z0|) is "unchanged" (simplex.py:134) */
} lp_tol;

typedef struct lp_handle lp_handle;

/* Defaults: cost 1e-9, cost_tie 1e-12, pivot 1e-9, zero 1e-9, ratio_tie 1e-12,
 * stall 1e-12. */
void lp_default_tol(lp_tol *tol);

/* Number of visible GPUs. */
int lp_device_count(int *count);

/* Tableau(m, n) on one GPU (lpsol/tableau.py:36-52): allocates a zeroed
 * (m+1) x ld device tableau, ld = n+1 rounded up to 64 doubles.
 * m <= 0 or n <= 0 -> LP_BAD_ARG (the reference raises ValueError, :40-43). */
int lp_create(int64_t m, int64_t n, int device, lp_handle **out);

/* Row-sharded tableau for one rank of an nranks-process job (one GPU per
 * process).  Constraint rows are split in contiguous blocks; row 0 (the
 * objective) is replicated on every rank.  uid is the 128-byte RCCL unique id
 * from lp_comm_unique_id on rank 0, broadcast to all ranks by the caller;
 * uid NULL creates no RCCL communicator (the device-side peer exchange below
 * must then be set up, or the host's all-gather given with
 * lp_set_host_allgather, for the per-pivot exchanges). */
int lp_comm_unique_id(void *uid128);
int lp_create_sharded(int64_t m, int64_t n, int device, int rank, int nranks,
                      const void *uid128, lp_handle **out);
/* In-process emulation of an nshards-rank job on ONE device: nshards handles
 * (written to out[0..nshards-1]) that share a stream and exchange through
 * device copies instead of RCCL.  Driving any member (lp_solve, lp_run,
 * lp_find_pivot, lp_pivot, ...) drives all of them in lock-step.  Used by the
 * test-suite to prove the pivot sequence is independent of the shard count. */
int lp_create_group(int64_t m, int64_t n, int device, int nshards, lp_handle **out);
/* This rank's constraint-row block [*row_begin, *row_begin + *row_count). */
int lp_shard_rows(const lp_handle *h, int64_t *row_begin, int64_t *row_count);

/* Device-side exchange between the ranks of a sharded job (one GPU per
 * rank): the pivot selection runs as one persistent kernel per rank and
 * group of pivots, exchanging the leaving-row candidates and the pivot row
 * through the ranks' exchange buffers (peer stores over xGMI) instead of one
 * RCCL collective per pivot.  Setup is collective:
 *   lp_peer_handle  -> this rank's exchange-buffer IPC handle (LP_PEER_HANDLE_BYTES)
 *   (the caller all-gathers the handles in rank order)
 *   lp_peer_open    -> opens the peers' buffers and checks the exchange with
 *                      a ping between all ranks; LP_DEVICE_ERROR if it fails
 * If any rank fails, every rank calls lp_peer_enable(h, 0): the RCCL
 * per-pivot path stays in use (identical results).  In-process shard groups
 * (lp_create_group) set this up themselves. */
#define LP_PEER_HANDLE_BYTES 64
int lp_peer_handle(lp_handle *h, void *handle);
int lp_peer_open(lp_handle *h, const void *handles);
int lp_peer_enable(lp_handle *h, int enable);

/* The host's own all-gather for a multi-process sharded handle (gloo, MPI,
 * ...): fn(ctx, send, recv, bytes) must gather `bytes` from every rank into
 * recv in rank order (nranks * bytes) and return 0.  It combines the column
 * scans' per-column results (lp_find_pivot_max_increase, lp_find_pivot_all,
 * lp_form_checks; RCCL is used when this is not set) and, on a handle
 * created without an RCCL communicator, carries the per-pivot exchanges of
 * the per-pivot path (explicit and validated pivots, peer exchange disabled)
 * synchronously.  No reference counterpart (the reference is one process);
 * it replaces the collective the scans of simplex.py:286-360 and
 * tableau.py:466-521 need once the rows are split across processes.
 * LP_BAD_ARG on a handle that is not a multi-process shard. */
typedef int (*lp_allgather_fn)(void *ctx, const void *send, void *recv, int64_t bytes);
int lp_set_host_allgather(lp_handle *h, lp_allgather_fn fn, void *ctx);

int lp_destroy(lp_handle *h);

int lp_set_tol(lp_handle *h, const lp_tol *tol);
int lp_get_tol(const lp_handle *h, lp_tol *tol);

/* Bulk copies of tableau rows [row0, row0+nrows) (row 0 = objective) to and
 * from a host row-major buffer with leading dimension ldh >= n+1.  Replace the
 * reference's setZ/setC/setB/setA (tableau.py:128-158) and getZ/getC/getB/getA
 * (tableau.py:82-108).  On a sharded handle the rows are GLOBAL indices and
 * must be row 0 or lie inside this rank's block. */
int lp_upload_rows(lp_handle *h, int64_t row0, int64_t nrows, const double *src, int64_t ldh);
int lp_download_rows(lp_handle *h, int64_t row0, int64_t nrows, double *dst, int64_t ldh);

/* Tableau.pivot(r, c) (tableau.py:295-308).  a_rc == 0 -> LP_ZERO_PIVOT and
 * the tableau is untouched. */
int lp_pivot(lp_handle *h, int64_t r, int64_t c);

/* findPivotStandard / findPivotMinIndex (simplex.py:218-284): selects (r, c)
 * by rule and, if do_pivot, performs it.  Returns LP_PIVOTED (found),
 * LP_OPTIMAL or LP_UNBOUNDED. */
int lp_find_pivot(lp_handle *h, int rule, int do_pivot, int64_t *r, int64_t *c);

/* Simplex.pivot(r, c) (simplex.py:199-216): pivot only if row r attains the
 * minimum ratio in column c, else LP_BAD_PIVOT and nothing changes. */
int lp_pivot_checked(lp_handle *h, int64_t r, int64_t c);

/* Simplex.solve (simplex.py:110-148) entirely on the device: standard-rule
 * pivots until the stall counter (pivots leaving the objective equal to its
 * value at the start of the call) reaches m+n, then min-index pivots to
 * optimality.  max_pivots < 0 means no cap.  Returns LP_OPTIMAL, LP_UNBOUNDED
 * (the reference raises AssertionError there) or LP_CAP_REACHED.
 * *npiv = pivots done, *nstd = of which standard-rule. */
int lp_solve(lp_handle *h, int64_t max_pivots, int64_t *npiv, int64_t *nstd);

/* k pivots of one rule with no stall logic (the fixed-K benchmark loop, i.e.
 * findPivot*(do_pivot=True) called k times).  Stops early on optimal or
 * unbounded.  Returns the last status; *done = pivots performed. */
int lp_run(lp_handle *h, int rule, int64_t k, int64_t *done);

/* findPivotMaxIncrease (simplex.py:286-328): over columns with c_j < -cost,
 * the largest objective increase -c_j * (min ratio of column j); ties to the
 * first column, its ratio-test row.  LP_UNBOUNDED if any such column has no
 * eligible row (the reference returns at the first one, :319-320),
 * LP_OPTIMAL if no column qualifies; performs the pivot if do_pivot.  On a
 * multi-process sharded handle every rank calls it (collective: the ranks'
 * per-column results are all-gathered, see lp_set_host_allgather). */
int lp_find_pivot_max_increase(lp_handle *h, int do_pivot, int64_t *r, int64_t *c);

/* findPivotAll (simplex.py:330-360): every min-ratio pivot of every column,
 * column-major, rows in order; writes up to cap (r, c) pairs, *count = all.
 * Collective on a multi-process sharded handle (every rank gets all pairs). */
int lp_find_pivot_all(lp_handle *h, int64_t *rc, int64_t cap, int64_t *count);

/* Form checks of the current tableau, exact comparisons of the float64 values
 * (tableau.py:466-521): flags[0] isCanonical, [1] isOptimal, [2] isUnbounded,
 * [3] isInfeasible, [4] isDegenerate.  bcols (m entries, may be NULL) gets
 * isCanonical's basic column per row (-1: none) unless some b_i < 0, where
 * the reference leaves it untouched.  Collective on a multi-process sharded
 * handle. */
int lp_form_checks(lp_handle *h, int32_t *flags, int64_t *bcols);

/* Pivot log of the last lp_solve / lp_run: (r, c) pairs, oldest first.  The
 * front-end replays it to maintain Simplex._bfs and the variable marks
 * (simplex.py:192-197).  *count = pivots available (may exceed cap). */
int lp_pivot_log(lp_handle *h, int64_t *rc, int64_t cap, int64_t *count);

/* Objective value getZ() = -T[0][0] (tableau.py:82-84, simplex.py:175-179). */
int lp_objective(lp_handle *h, double *z);

/* Pivots deferred into one sweep of the tableau (1..64; 0 = auto, the
 * default: the deepest of 64 / 48 / 32 whose persistent selection still fits
 * one XCD, else 64; lp_get_block reports the value in use).  Each
 * pivot's selection and pivot row use current values computed on the fly; the
 * rank-1 eliminations of `pivots_per_sweep` pivots are applied to the stored
 * tableau in one pass (the same float64 operations in the same order, so the
 * results are identical for every setting).  1 = immediate elimination. */
int lp_set_block(lp_handle *h, int pivots_per_sweep);
int lp_get_block(const lp_handle *h, int *pivots_per_sweep);

/* Device-time accounting of the elimination sweep kernel (for the roofline):
 * enable = 0 off, 1 every launch, k > 1 every k-th launch of each kernel
 * (sampled: fewer events inside a timed loop).  A timed launch records HIP
 * events on the stream it runs on, as part of the launch itself.
 * lp_update_time returns the summed milliseconds and timed launches since the
 * last reset. */
int lp_profile(lp_handle *h, int enable);
int lp_update_time(lp_handle *h, double *ms, int64_t *launches);
/* The same for the pivot-selection launches (one per group of
 * pivots_per_sweep pivots on the single-device path). */
int lp_select_time(lp_handle *h, double *ms, int64_t *launches);

/* Which pivot path the last lp_solve / lp_run of this handle took (extension;
 * the reference is one process on one CPU):
 *   LP_PATH_KERNELS     single device, per-pivot selection kernels
 *   LP_PATH_PERSISTENT  single device, one persistent selection launch per group
 *   LP_PATH_PEER        row-sharded, persistent selection per rank with the
 *                       device-side peer exchange between ranks
 *   LP_PATH_COLLECTIVE  row-sharded, per-pivot kernels + one collective
 *                       exchange per pivot (RCCL, or the host's all-gather)
 * A persistent group whose exchange times out (never expected: the launch is
 * sized from the kernel's occupancy) is redone on the per-pivot kernels and
 * counted in *fallbacks. */
#define LP_PATH_KERNELS 0
#define LP_PATH_PERSISTENT 1
#define LP_PATH_PEER 2
#define LP_PATH_COLLECTIVE 3
int lp_exchange_path(const lp_handle *h, int *path, int *fallbacks);

/* Row-sharded persistent selection (LP_PATH_PEER): the cross-rank hop as
 * this rank's block 0 saw it -- from sending its leaving-row summary (and
 * speculative pivot row) to holding the winner's pivot row -- summed over
 * the handle's pivots: *ticks of the 100 MHz device real-time clock over
 * *pivots pivots (both cumulative since lp_create; read after a call). */
int lp_xwait(const lp_handle *h, int64_t *ticks, int64_t *pivots);

/* Human-readable description of the last failure on this handle (or of the
 * last failed lp_create* when h is NULL). */
const char *lp_last_error(const lp_handle *h);

#ifdef __cplusplus
}
#endif
#endif /* LPGPU_H */
