// Device kernels of the dense simplex pivot engine (gfx950 / CDNA4).
//
// Deferred ("blocked") pivots.  A pivot is selected and its normalised row
// computed from CURRENT values, but the rank-1 elimination of the whole
// tableau is postponed: up to BMAX pivots (a "group") are later applied in
// one sweep that reads and writes the tableau once (a rank-B update: B FMAs
// per 16 bytes of HBM traffic instead of 1).  Every element goes through
// exactly the same float64 operations, in the same order, as with an
// immediate update (oracle/lp_f64.c) -- upd() below is that operation -- so
// results are bit-identical for any group size B (B = 1 is the plain pivot).
//
// Per pivot t of a group (single device), two launches:
//   k_ratio   combines k_prow's row-0 summaries into the entering column
//             (every block redundantly: the summaries are tiny), then the
//             current column C (stored value + deferred pivots 0..t-1) ->
//             multipliers M[t] and per-block min-ratio summaries
//                                  simplex.py:228-232 / :262-267, :235-246 / :270-281
//   k_prow    combines the ratio summaries into the leaving row (again in
//             every block), current pivot row / a -> P[t]; pivot t applied to
//             row 0 and column 0 (kept current eagerly); per-block row-0
//             summaries for the next entering column
//                                  tableau.py:300-303
// Every B pivots (and at the end of every call):
//   k_sweep   T <- T with pivots 0..ndef-1 applied  tableau.py:305-308 -> :269-289
// No atomics or grid-wide hand-offs on this path: each kernel consumes the
// previous kernel's records after the kernel boundary.
// Row-sharded (one rank per GPU) replaces the leaving-row choice with
//   k_ratio(LOCAL) -> allreduce-min(g) -> k_pick -> allgather(slots) -> k_prow
//
// Local storage: row 0 (objective, replicated on every rank) + this rank's
// constraint rows, row-major, leading dimension ld (a multiple of 64 doubles
// = 512 B: every row starts on a cache-line boundary, 16-byte accesses are
// aligned).
#include "engine.h"
#include "device.h"

#include <hip/hip_ext.h>

#include <array>
#include <cstdlib>
#include <map>
#include <mutex>

namespace lpk {


// ---------------------------------------------------------------------------
// control
// ---------------------------------------------------------------------------

__global__ void k_reset(Args A, int mode, int rule, int chain, long long cap, long long r,
                        long long c)
{
    Ctl *ctl = A.ctl;
    ctl->status = LP_PIVOTED;
    ctl->mode = mode;
    ctl->rule = rule;
    ctl->chain = chain;
    ctl->cap = cap;
    ctl->r = r;
    ctl->c = c;
    ctl->npiv = 0;
    ctl->nstd = 0;
    ctl->stuck = 0;
    ctl->ndef[0] = 0;
    ctl->ndef[1] = 0;
    ctl->z0 = -A.row0[0];
    ctl->ticket = 0;
    ctl->bar[0] = 0;
    ctl->bar[1] = 0;
    ctl->bar_timeout = 0;
    A.dR[0] = r >= 0 ? local_of(A, r) : -1;
}

// row0 / col0 <- the stored tableau (after an upload)
__global__ void k_load_eager(Args A)
{
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long j = g; j < A.ld; j += stride) A.row0[j] = A.T[j];
    for (long long i = g; i < A.rows; i += stride) A.col0[i] = A.T[i * A.ld];
}

// entering column from the current row 0 (one workgroup): first pivot of a call
__global__ void __launch_bounds__(ENTER_THREADS) k_enter(Args A)
{
    __shared__ double sd[16];
    __shared__ long long sl[16];
    __shared__ int s_go;
    Ctl *ctl = A.ctl;
    if (threadIdx.x == 0) {
        int go = ctl->status == LP_PIVOTED;
        if (go && ctl->cap >= 0 && ctl->npiv >= ctl->cap) {
            ctl->status = LP_CAP_REACHED;
            go = 0;
        }
        s_go = go;
    }
    __syncthreads();
    if (!s_go) return;
    const int rule = ctl->rule;
    const double *c0 = A.row0;
    const long long n = A.n;
    long long j = NONE;
    if (rule == LP_RULE_MIN_INDEX) {
        for (long long k = 1 + threadIdx.x; k <= n; k += blockDim.x)
            if (c0[k] < -A.tol.cost) { j = k; break; }
        j = block_min_ll(j, sl);
    } else {
        double g = INFINITY;
        for (long long k = 1 + threadIdx.x; k <= n; k += blockDim.x) g = fmin(g, c0[k]);
        g = block_min(g, sd);
        if (g < -A.tol.cost) {
            const double thr = tie_band(g, A.tol.cost_tie);
            for (long long k = 1 + threadIdx.x; k <= n; k += blockDim.x)
                if (c0[k] <= thr) { j = k; break; }
            j = block_min_ll(j, sl);
        }
    }
    if (threadIdx.x == 0) {
        if (j == NONE) ctl->status = LP_OPTIMAL;
        else ctl->c = j - 1;
    }
}

// entering column from per-block row-0 summaries (block-wide; every block
// gets the same answer): two-pass semantics of oracle/lp_f64.c's entering().
// Summary b covers row-0 columns [b*width, (b+1)*width).  The first summary
// inside the global band holds the answer -- its own candidate, or a rescan
// of its slice of row 0.  sc1 loads: valid right after a grid barrier too.
__device__ long long combine_entering(const Args &A, int rule, unsigned nb, long long width,
                                      double *sd, long long *sl)
{
    if (rule == LP_RULE_MIN_INDEX) {
        long long j = NONE;
        for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) {
            const long long f = ld_sc1(&A.erec[b].fneg);
            j = f < j ? f : j;
        }
        return block_min_ll(j, sl);
    }
    double g = INFINITY;
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) g = fmin(g, ld_sc1(&A.erec[b].l));
    g = block_min(g, sd);
    if (!(g < -A.tol.cost)) return NONE;
    const double thr = tie_band(g, A.tol.cost_tie);
    long long bsel = NONE;
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x)
        if (ld_sc1(&A.erec[b].l) <= thr) { bsel = b; break; }
    bsel = block_min_ll(bsel, sl);
    if (ld_sc1(&A.erec[bsel].q) <= thr) return ld_sc1(&A.erec[bsel].i);
    long long best = NONE;
    const long long k0 = bsel * width;
    for (long long k = k0 + threadIdx.x; k < k0 + width; k += blockDim.x)
        if (k >= 1 && k <= A.n && ld_sc1(&A.row0[k]) <= thr) { best = k; break; }
    return block_min_ll(best, sl);
}

// ---------------------------------------------------------------------------
// K1: entering column (chained pivots), ratio test over this rank's
// constraint rows, multiplier snapshot M[t], per-block summaries
//   (local min l_b, first row within the tie band of l_b, its ratio).
// Every earlier row of a block has a ratio above tie_band(l_b) >=
// tie_band(g), so the first block with l_b <= tie_band(g) holds the leaving
// row: its own candidate if inside the global band, else a rescan of that
// block alone -- equal to the two-pass scan of oracle/lp_f64.c.
// ---------------------------------------------------------------------------

// first local row in [li0, li1) with ratio <= thr (block-wide), NONE if none
__device__ long long rescan_rows(const Args &A, int t, long long C, long long li0, long long li1,
                                 double thr, long long *scratch)
{
    long long best = NONE;
    for (long long li = li0 + threadIdx.x; li < li1; li += blockDim.x) {
        bool ok;
        const double a = current(A, t, li, C, A.T[li * A.ld + C]);
        const double q = row_ratio(a, A.col0[li], A.tol, ok);
        if (ok && q <= thr) { best = li; break; }
    }
    return block_min_ll(best, scratch);
}

// first local row within tie_band(g), from the ratio summaries (block-wide)
__device__ long long pick_from_records(const Args &A, int t, long long C, double g,
                                       long long *scratch)
{
    const double thr = tie_band(g, A.tol.ratio_tie);
    const unsigned nb = (unsigned)ratio_blocks(A.rows);
    long long bsel = NONE;
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x)
        if (A.rec[b].l <= thr) { bsel = b; break; }
    bsel = block_min_ll(bsel, scratch);
    if (bsel == NONE) return NONE;
    if (A.rec[bsel].q <= thr) return A.rec[bsel].i;
    const long long b0 = 1 + bsel * RATIO_CHUNK;
    return rescan_rows(A, t, C, b0, min(b0 + RATIO_CHUNK, A.rows), thr, scratch);
}

// minimum over the ratio summaries (block-wide)
__device__ double records_min(const Args &A, double *sd)
{
    const unsigned nb = (unsigned)ratio_blocks(A.rows);
    double g = INFINITY;
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) g = fmin(g, A.rec[b].l);
    return block_min(g, sd);
}

template <int TP>
__global__ void __launch_bounds__(RATIO_THREADS)
k_ratio(Args A, int t, int grp, int mode, int from_erec, long long check_row)
{
    __shared__ double sd[16];
    __shared__ long long sl[16];
    __shared__ long long sR[TP > 0 ? TP : 1];
    __shared__ double sPc[TP > 0 ? TP : 1];
    __shared__ double s_q;
    __shared__ int s_last;
    Ctl *ctl = A.ctl;
    // the previous group's sweep is complete (stream order): recycle its counter
    if (t == 0 && blockIdx.x == 0 && threadIdx.x == 0) ctl->ndef[grp ^ 1] = 0;
    if (ctl->status != LP_PIVOTED) {
        if (mode == RATIO_LOCAL && blockIdx.x == 0 && threadIdx.x == 0) *A.xg = INFINITY;
        return;
    }
    long long C;
    if (from_erec) {
        if (ctl->cap >= 0 && ctl->npiv >= ctl->cap) {
            if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_CAP_REACHED;
            if (mode == RATIO_LOCAL && blockIdx.x == 0 && threadIdx.x == 0) *A.xg = INFINITY;
            return;
        }
        C = combine_entering(A, ctl->rule, (unsigned)prow_blocks(A.ld), PROW_THREADS, sd, sl);
        if (C == NONE) {
            if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_OPTIMAL;
            if (mode == RATIO_LOCAL && blockIdx.x == 0 && threadIdx.x == 0) *A.xg = INFINITY;
            return;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) ctl->c = C - 1;
    } else {
        C = ctl->c + 1;
    }
    if (threadIdx.x < TP && threadIdx.x < t) {
        sR[threadIdx.x] = A.dR[threadIdx.x];
        sPc[threadIdx.x] = A.P[threadIdx.x * A.ld + C];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // row 0's multiplier (+ the sweep's copy)
        A.M[mi(A.rows, 0, t)] = A.row0[C];
        A.MQ[mq(0, t)] = A.row0[C];
    }
    __syncthreads();

    const long long li0 = 1 + (long long)blockIdx.x * RATIO_CHUNK;
    const long long li1 = min(li0 + RATIO_CHUNK, A.rows);
    const long long li = li0 + threadIdx.x;      // one row per thread
    bool ok = false;
    double q = 0.0;
    if (li < li1) {
        const double a = current_col<TP>(A, t, li, A.T[li * A.ld + C], sR, sPc);
        A.M[mi(A.rows, li, t)] = a;
        A.MQ[mq(li, t)] = a;
        q = row_ratio(a, A.col0[li], A.tol, ok);
    }
    const double lb = block_min(ok ? q : INFINITY, sd);
    long long ib = NONE;
    if (lb < INFINITY) ib = block_min_ll(ok && q <= tie_band(lb, A.tol.ratio_tie) ? li : NONE, sl);
    if (threadIdx.x == 0) s_q = 0.0;
    __syncthreads();
    if (ib != NONE && li == ib) s_q = q;
    __syncthreads();
    if (mode == RATIO_FULL) {
        if (threadIdx.x == 0) {
            A.rec[blockIdx.x].l = lb;
            A.rec[blockIdx.x].i = ib;
            A.rec[blockIdx.x].q = s_q;
        }
        return;
    }
    // LOCAL / CHECK: the last block needs every summary within this launch
    if (threadIdx.x == 0) {
        st_sc1(&A.rec[blockIdx.x].l, lb);
        st_sc1(&A.rec[blockIdx.x].i, ib);
        st_sc1(&A.rec[blockIdx.x].q, (double)s_q);
    }
    if (!arrive_last(&ctl->ticket, &s_last)) return;
    double g = INFINITY;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) g = fmin(g, ld_sc1(&A.rec[b].l));
    g = block_min(g, sd);
    if (threadIdx.x == 0) {
        if (mode == RATIO_LOCAL) {
            *A.xg = g;
        } else {
            // Simplex.pivot(r, c): row r must attain the minimum ratio (simplex.py:204-215)
            bool okr;
            const double a = current(A, t, check_row, C, A.T[check_row * A.ld + C]);
            const double qr = row_ratio(a, A.col0[check_row], A.tol, okr);
            if (a == 0.0) ctl->status = LP_ZERO_PIVOT;
            else if (!(g < INFINITY) || !okr || !(qr <= tie_band(g, A.tol.ratio_tie)))
                ctl->status = LP_BAD_PIVOT;
        }
        st_sc1(&ctl->ticket, 0u);
    }
}

// ---------------------------------------------------------------------------
// K1s (sharded): after the allreduce-min of the ratio, each rank offers its
// first row within the global tie band (or the requested row) in its slot,
// as CURRENT values.  Every block recomputes the (cheap) candidate and copies
// a slice of the row.
// ---------------------------------------------------------------------------

template <int TP>
__global__ void __launch_bounds__(256) k_pick(Args A, int t, int mode)
{
    __shared__ long long sl[16];
    Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) return;
    const long long C = ctl->c + 1;
    long long li = -1;
    long long code = 0;
    double lloc = INFINITY, qloc = 0.0;
    if (mode == PICK_LOCAL) {
        // one-exchange protocol: this rank's minimum and first in-band row
        __shared__ double sd[16];
        lloc = records_min(A, sd);
        if (lloc < INFINITY) {
            const long long w = pick_from_records(A, t, C, lloc, sl);
            li = w;
            bool ok;
            const double a = current(A, t, w, C, A.T[w * A.ld + C]);
            qloc = row_ratio(a, A.col0[w], A.tol, ok);
        }
    } else if (mode == PICK_RATIO) {
        const double g = *A.xg;
        if (!(g < INFINITY)) {
            // every rank holds the same global minimum: unbounded everywhere
            if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_UNBOUNDED;
            return;
        }
        const long long w = pick_from_records(A, t, C, g, sl);
        li = (w == NONE) ? -1 : w;
    } else {
        li = local_of(A, ctl->r);
        if (li >= 0 && mode == PICK_CHECK) {
            bool okr;
            const double g = *A.xg;
            const double a = current(A, t, li, C, A.T[li * A.ld + C]);
            const double qr = row_ratio(a, A.col0[li], A.tol, okr);
            if (a == 0.0) code = LP_ZERO_PIVOT;
            else if (!(g < INFINITY) || !okr || !(qr <= tie_band(g, A.tol.ratio_tie)))
                code = LP_BAD_PIVOT;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.xs[0] = as_d(li < 0 ? NONE : li - 1 + A.rb);
        A.xs[1] = as_d(code);
        A.xs[2] = lloc;
        A.xs[3] = qloc;
    }
    if (li < 0) return;
    for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < A.ld;
         j += (long long)gridDim.x * blockDim.x)
        A.xs[SLOT_HDR + j] = current_row<TP>(A, t, li, j, A.T[li * A.ld + j]);
}

// explicit pivot (Tableau.pivot): multiplier snapshot of the (current) column
__global__ void k_gather(Args A, int t)
{
    Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) return;
    const long long C = ctl->c + 1;
    for (long long li = blockIdx.x * (long long)blockDim.x + threadIdx.x; li < A.rows;
         li += (long long)gridDim.x * blockDim.x) {
        const double mv = li == 0 ? A.row0[C] : current(A, t, li, C, A.T[li * A.ld + C]);
        A.M[mi(A.rows, li, t)] = mv;
        A.MQ[mq(li, t)] = mv;
    }
}

// ---------------------------------------------------------------------------
// K2: leaving row (from the ratio summaries, the caller or the rank slots);
// pivot row P[t] = current row R / a, P[t][C] = 1 (tableau.py:300-302);
// pivot t applied to the current row 0 and column 0; per-block row-0
// summaries; block 0 records the pivot (log, counters, stall test).
// ---------------------------------------------------------------------------

template <int TP>
__global__ void __launch_bounds__(PROW_THREADS) k_prow(Args A, int t, int grp, int rsrc, int peek)
{
    __shared__ double sd[16];
    __shared__ long long sl[16];
    __shared__ double s_q;
    Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) return;
    const long long C = ctl->c + 1;
    long long R, rglob;
    double a;
    const double *src = nullptr;   // sharded: the current pivot row from its owner
    if (rsrc == RSRC_SLOTS || rsrc == RSRC_BAND) {
        const long long slot = SLOT_HDR + A.ld;
        long long best = NONE, code = 0;
        int who = -1;
        if (rsrc == RSRC_BAND) {
            // ranks hold consecutive row blocks: the first rank whose minimum
            // is inside the global band holds the first in-band row, provided
            // its own first in-band row is inside the global band too
            double g = INFINITY;
            for (int k = 0; k < A.nranks; ++k) g = fmin(g, A.xr[k * slot + 2]);
            if (!(g < INFINITY)) {
                if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_UNBOUNDED;
                return;
            }
            const double thr = tie_band(g, A.tol.ratio_tie);
            int k = 0;
            while (!(A.xr[k * slot + 2] <= thr)) ++k;
            if (!(A.xr[k * slot + 3] <= thr)) {
                if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = ST_STRADDLE;
                return;
            }
            best = as_ll(A.xr[k * slot]);
            who = k;
        } else {
            for (int k = 0; k < A.nranks; ++k) {
                const long long idx = as_ll(A.xr[k * slot]);
                const long long cd = as_ll(A.xr[k * slot + 1]);
                if (cd != 0) code = cd;
                if (idx < best) { best = idx; who = k; }
            }
        }
        if (code != 0 || best == NONE) {
            if (blockIdx.x == 0 && threadIdx.x == 0)
                ctl->status = code != 0 ? (int)code : LP_UNBOUNDED;
            return;
        }
        if (peek) {   // findPivot*(False): report the row only
            if (blockIdx.x == 0 && threadIdx.x == 0) ctl->r = best;
            return;
        }
        src = A.xr + who * slot + SLOT_HDR;
        rglob = best;
        R = local_of(A, best);
        a = src[C];
    } else {
        if (rsrc == RSRC_RECORDS) {
            const double g = records_min(A, sd);
            if (!(g < INFINITY)) {
                if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_UNBOUNDED;
                return;
            }
            R = pick_from_records(A, t, C, g, sl);
        } else {
            R = A.dR[t];
        }
        rglob = R - 1 + A.rb;
        if (peek) {
            if (blockIdx.x == 0 && threadIdx.x == 0) ctl->r = rglob;
            return;
        }
        a = A.M[mi(A.rows, R, t)];
    }
    if (a == 0.0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_ZERO_PIVOT;
        return;
    }
    const double f0 = A.M[mi(A.rows, 0, t)];   // row 0's multiplier (its current value at C)
    const long long j = blockIdx.x * (long long)PROW_THREADS + threadIdx.x;
    double v = INFINITY;
    if (j < A.ld) {
        const double x = src ? src[j] : current_row<TP>(A, t, R, j, A.T[R * A.ld + j]);
        const double p = (j == C) ? 1.0 : x / a;
        A.P[t * A.ld + j] = p;
        v = upd(0, -1, f0, p, A.row0[j]);
        A.row0[j] = v;
        if (j == 0) A.col0[0] = v;
    }
    // column 0 of the local constraint rows (column 0 is never the pivot column)
    {
        const double x0 = src ? src[0] : current_row<TP>(A, t, R, 0, A.T[R * A.ld]);
        const double p0 = x0 / a;
        const long long stride = (long long)gridDim.x * blockDim.x;
        for (long long li = 1 + blockIdx.x * (long long)blockDim.x + threadIdx.x; li < A.rows;
             li += stride)
            A.col0[li] = upd(li, R, A.M[mi(A.rows, li, t)], p0, A.col0[li]);
    }
    // entering-column summary of this slice of the new row 0
    const bool cand = j >= 1 && j <= A.n;
    const double lb = block_min(cand ? v : INFINITY, sd);
    const long long ib =
        block_min_ll(cand && lb < INFINITY && v <= tie_band(lb, A.tol.cost_tie) ? j : NONE, sl);
    const long long fn = block_min_ll(cand && v < -A.tol.cost ? j : NONE, sl);
    if (threadIdx.x == 0) s_q = 0.0;
    __syncthreads();
    if (ib != NONE && j == ib) s_q = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        A.erec[blockIdx.x].l = lb;
        A.erec[blockIdx.x].i = ib;
        A.erec[blockIdx.x].q = s_q;
        A.erec[blockIdx.x].fneg = fn;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // j == 0: v is the new row0[0]
        A.dR[t] = R;
        A.dC[t] = C;
        ctl->r = rglob;
        const long long k = ctl->npiv;
        if (k < A.logcap) {
            A.log[2 * k] = rglob;
            A.log[2 * k + 1] = C - 1;
        }
        ctl->npiv = k + 1;
        ctl->ndef[grp] = t + 1;
        if (ctl->mode == MODE_SOLVE && ctl->rule == LP_RULE_STANDARD) {
            ctl->nstd += 1;
            // stall bookkeeping (simplex.py:132-137) and the switch to the
            // min-index rule (simplex.py:123,138)
            const double z = -v;
            const double z0 = ctl->z0;
            const double band = A.tol.stall * fmax(1.0, fabs(z0));
            if (z - z0 > band) ctl->status = LP_OBJ_INCREASED;   // simplex.py:133
            if (fabs(z - z0) <= band) ctl->stuck += 1;
            else ctl->stuck = 0;
            if (ctl->stuck >= A.m + A.n) ctl->rule = LP_RULE_MIN_INDEX;
        }
    }
}

// ---------------------------------------------------------------------------
// K-group: every selection of one group of chained pivots in ONE persistent
// launch (single device).  G co-resident single-wave workgroups; block b owns
// a slice of the constraint rows (at most one per lane: ratio test) and a
// slice of the columns (pivot row, row 0).  Per pivot two all-to-all
// exchanges of tiny per-block summaries:
//   entering column  <- row-0 summaries of every block
//   ratio test on own rows -> ratio summary
//   leaving row      <- ratio summaries of every block
//   pivot row and row 0 on own columns -> row-0 summary
// A summary travels as tagged 8-byte granules {payload u32, tag u32}, each
// written by ONE sc1 store; a reader polls the granules of every block with
// sc1 loads until every tag is the expected one -- the wait and the data are
// the same round trip (MI355X_MICROARCH price list: granule hand-offs, no
// counter).  Larger data a phase publishes for the other blocks (pivot-row
// values, multipliers, row 0) is stored sc1 and drained before the block's
// granules, and read with sc1 loads only after all granules matched
// ("Valid forms" row 1: the granules are the flag).
// Same float64 operations as k_ratio + k_prow; no host round trips.
// ---------------------------------------------------------------------------


// NR = summaries per lane (G <= 64 NR); IPL = own columns per lane (cpb <= 64 IPL);
// RPL = own rows per lane (rpb <= 64 RPL: lane l owns rows lr0 + l + 64k, so
// the first row with a property is again the lowest lane of the first k);
// XR = one rank of a row-sharded job (leaving row and pivot row exchanged
// between ranks through the peers' exchange buffers).
// first (the first launch of a call): bit 0 resets the loop state (mode,
// rule, cap = fmode, frule, fcap; k_reset's work), bit 1 loads the eager row 0
// / column 0 from the stored tableau (k_load_eager's), bit 2 picks the first
// entering column from the row-0 slices with one extra exchange (k_enter's).
template <int NR, int IPL, int RPL, bool XR, bool HK = false>
__global__ void __launch_bounds__(GROUP_THREADS)
k_group(Args A0, const Args *As, int gper, int grp, int count, int from_erec, unsigned seq, int bmax,
        int xmode, int first, int fmode, int frule, long long fcap)
{
    // xmode: the grid is 8 x gper and only blocks 0, 8, 16, ... work; they
    // share one XCD under the round-robin dealing of workgroups over the 8
    // XCDs (speed only: checked below, correct either way)
    unsigned bid = blockIdx.x;
    if (xmode) {
        if (bid & 7u) return;
        bid >>= 3;
    }
    // As: in-process shards of one device in ONE launch (gper blocks each, so
    // every shard's blocks are co-resident); otherwise this device's A0
    const Args A = As ? As[bid / gper] : A0;
    constexpr int NGRX = XR ? 7 : NGR;   // XR: the candidate's pivot element too
    __shared__ double sd[16];
    __shared__ long long sl[16];
    __shared__ long long sR[BMAX + CH];     // local pivot rows of this group
    __shared__ double sPc[BMAX + CH];       // P[s][C] for the current entering column
    __shared__ double sMr[BMAX + CH];       // M[R][s] for the current leaving row
    // dynamic LDS, per own row / own column contiguous over the pivots with an
    // odd stride cs (lanes 2-way over the banks; a chunk of pivots is one base
    // address plus immediate offsets): this block's rows' multipliers, its
    // columns' pivot-row values, its slices of row 0 / column 0.  Own data
    // never leaves LDS for a re-read; it is also published for the other
    // blocks and the sweep.
    extern __shared__ __attribute__((aligned(16))) double dyn[];
    Ctl *ctl = A.ctl;
    const unsigned G = gper, b = bid % gper;
    const int tid = threadIdx.x;
    constexpr int nth = GROUP_THREADS;
    const bool reset = (first & 1) != 0, eager = (first & 2) != 0, enter = (first & 4) != 0;
    if (b == 0 && tid == 0) *gp(&ctl->ndef[grp]) = 0;
    // a stopped loop, or an earlier group of the batch that timed out
    if (!reset && (ld_sc1(&ctl->status) != LP_PIVOTED || ld_sc1(&ctl->bar_timeout) != 0u)) return;
    const long long cap = reset ? fcap : *gp(&ctl->cap);
    const int mode = reset ? fmode : *gp(&ctl->mode);
    // counters live in registers for the launch (block 0 publishes them)
    long long npiv = reset ? 0 : ld_sc1(&ctl->npiv);
    int rule = reset ? frule : ld_sc1(&ctl->rule);
    long long nstd = 0, stuck = 0;
    if (!reset) {
        nstd = ld_sc1(&ctl->nstd);
        stuck = ld_sc1(&ctl->stuck);
    }
    if (tid == 0) {
        // the loop state before this group: what a timed-out group is redone
        // from (written before anything of this launch can time out)
        st_sc1(&ctl->g_npiv, npiv);
        st_sc1(&ctl->g_nstd, nstd);
        st_sc1(&ctl->g_stuck, stuck);
        st_sc1(&ctl->g_rule, rule);
        st_sc1(&ctl->g_seq, seq);
    }
    // summary regions of GROUP_MAXBLOCKS x GSLOT granules: ratio, row 0, XCD check
    u64 *grR = A.gran;
    u64 *grE = A.gran + GROUP_MAXBLOCKS * GSLOT;
    const int xs = (xmode && A.gmaj) ? 0 : 1;  // 0: granule-major (one XCD), 1: block-major
    bool fast = false;
    if (xmode) {
        // every block publishes its XCD; plain hand-off stores only if all match
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        u64 *grX = A.gran + 2 * GROUP_MAXBLOCKS * GSLOT;
        if (threadIdx.x == 0) st_sc1(&grX[gslot(0, b, 0)], ((u64)gtag(seq, 0, 7) << 32) | xcc);
        unsigned wx[NRMAX][1];
        if (!gather<NRMAX, 1>(grX, G, gtag(seq, 0, 7), wx, &ctl->bar_timeout, A.spin_max)) {
            if (b == 0 && threadIdx.x == 0) st_sc1(&ctl->status, (int)LP_DEVICE_ERROR);
            return;
        }
        bool same = true;
#pragma unroll
        for (int k = 0; k < NRMAX; ++k)
            if (threadIdx.x + k * GROUP_THREADS < G) same = same && wx[k][0] == xcc;
        // wave-uniform in a scalar register: st_x branches on it without
        // exec masking (a divergent-looking branch around each store made
        // the compiler wait for the stores before the next one)
        fast = __builtin_amdgcn_readfirstlane(__all(same) ? 1 : 0) != 0;
    }
    // Two-level exchange for blocks spread over the 8 XCDs (single device): the
    // G / 8 blocks of one XCD (b % 8 equal under the round-robin dealing,
    // checked here) exchange their summaries through that XCD's L2 (level 1,
    // plain stores, granule-major), the XCD's last block combines them into
    // one summary of the same format and publishes it write-through (level 2),
    // and every block polls the 8 level-2 summaries -- instead of every block
    // polling all G summaries across the XCDs.  Blocks are numbered XCD-major
    // (logical L: rows and columns in L order), so the first summary within
    // the band is found group first, then member: a group's summary carries
    // its first member within ITS band, which is the answer whenever that
    // candidate is inside the global band (every earlier row is above it);
    // otherwise (q = INFINITY: a rescan) the group's rows / columns are
    // rescanned against the global band, as a block's are in the flat form.
    bool hier = false;
    const unsigned G8 = G / 8;
    // (HK: the variant compiled with it, launched for spread single-device groups)
    if (HK && !XR && !As && !xmode && A.hier && G % 8 == 0 && G8 >= 8 && G8 <= (unsigned)GROUP_THREADS) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        u64 *grX = A.gran + 2 * GROUP_MAXBLOCKS * GSLOT;
        if (threadIdx.x == 0) st_sc1(&grX[gslot(0, b, 0)], ((u64)gtag(seq, 0, 7) << 32) | xcc);
        unsigned wx[NRMAX][1];
        if (!gather<NRMAX, 1>(grX, G, gtag(seq, 0, 7), wx, &ctl->bar_timeout, A.spin_max)) {
            if (b == 0 && threadIdx.x == 0) st_sc1(&ctl->status, (int)LP_DEVICE_ERROR);
            return;
        }
        // block l + 64k shares an XCD with block (l + 64k) % 8 (lane l % 8 of k = 0)
        bool same = true;
#pragma unroll
        for (int k = 0; k < NRMAX; ++k) {
            const unsigned x0 = (unsigned)__shfl((int)wx[0][0], (int)(threadIdx.x & 7));
            if (threadIdx.x + k * GROUP_THREADS < G) same = same && wx[k][0] == x0;
        }
        hier = __builtin_amdgcn_readfirstlane(__all(same) ? 1 : 0) != 0;
    }
    if (b == 0 && tid == 0) *gp(&ctl->sel_flags) = (fast ? 1u : 0u) | (hier ? 2u : 0u);   // diagnostics
    const unsigned L = hier ? (b % 8) * G8 + b / 8 : b;     // logical block: rows, columns, flat slots
    const unsigned Geff = hier ? 8u : G;                    // summaries in the final combine
    const long long rpb = (A.rc + G - 1) / G;               // rows per block (<= RPL nth)
    const long long lr0 = 1 + L * rpb, lr1 = min(lr0 + rpb, A.rows);
    const long long cpb = (A.ld + G - 1) / G;               // columns per block (<= IPL nth)
    const long long jc0 = L * cpb, jc1 = min(jc0 + cpb, A.ld);
    const long long smul = hier ? (long long)G8 : 1;        // blocks per final summary (rescans)
    u64 *grR2 = A.gran + 3 * GROUP_MAXBLOCKS * GSLOT;       // level 2: 8 slots x 8 granules, block-major
    u64 *grE2 = grR2 + 8 * GSLOT;
    // publication of a block's summary (+ the level-1 combine by an XCD's
    // first block) and the wait for the summaries to combine
    auto pub2 = [&](u64 *g1, u64 *g2, unsigned tag, unsigned wv, int n, double tie, bool entering) -> bool {
        if (!hier) {
            publish(g1, L, tag, wv, n, fast, xs);
            return true;
        }
        publish(g1, L, tag, wv, n, true, 0);
        if (b / 8 != G8 - 1) return true;      // the group's last block combines (block 0 has its own duties)
        return entering ? hier_combine<NGE>(g1, g2, b % 8, G8, tag, tie, true, &ctl->bar_timeout, A.spin_max)
                        : hier_combine<NGR>(g1, g2, b % 8, G8, tag, tie, false, &ctl->bar_timeout, A.spin_max);
    };
    const int cs = bmax + 1;
    double *lM = dyn;                        // [rpb][cs]  M[own row][s]
    double *lP = lM + rpb * cs;              // [cpb][cs]  P[s][own column]
    double *l0 = lP + cpb * cs;              // [cpb]      row 0 slice
    double *lc = l0 + cpb;                   // [rpb]      column 0 slice
    long long li[RPL];                       // this lane's own rows
    bool own[RPL];
    double *mrow[RPL];
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        li[k] = lr0 + tid + k * nth;
        own[k] = li[k] < lr1;
        mrow[k] = lM + min((long long)tid + k * nth, rpb - 1) * cs;
    }
    long long kc[IPL];                       // own columns jc0 + kc[k] (clamped into the slice)
    const double *pcol[IPL];
#pragma unroll
    for (int k = 0; k < IPL; ++k) {
        kc[k] = min((long long)tid + k * nth, cpb - 1);
        pcol[k] = lP + kc[k] * cs;
    }
    // row 0 / column 0: the eager copies, or (first launch after an upload)
    // the stored tableau's, which become the eager copies
    for (long long j = jc0 + tid; j < jc1; j += nth) {
        const double v = eager ? *gp(A.T + j) : *gp(A.row0 + j);
        l0[j - jc0] = v;
        if (eager) st_x(&A.row0[j], v, fast);
    }
#pragma unroll
    for (int k = 0; k < RPL; ++k)
        if (own[k]) {
            const double v = eager ? *gp(A.T + li[k] * A.ld) : *gp(A.col0 + li[k]);
            lc[tid + k * nth] = v;
            if (eager) st_x(&A.col0[li[k]], v, fast);
        }
    if (eager && b == 0 && tid == 0) st_x(&A.col0[0], *gp(A.T), fast);
    double z0 = 0.0;
    __syncthreads();
    if (b == 0 && tid == 0) {
        if (reset) {
            z0 = -l0[0];                     // obj_val at the start (simplex.py:118)
            st_x(&ctl->status, (int)LP_PIVOTED, fast);
            st_x(&ctl->mode, mode, fast);
            st_x(&ctl->rule, rule, fast);
            st_x(&ctl->chain, 1, fast);
            st_x(&ctl->cap, cap, fast);
            st_x(&ctl->r, -1LL, fast);
            st_x(&ctl->c, -1LL, fast);
            st_x(&ctl->npiv, 0LL, fast);
            st_x(&ctl->nstd, 0LL, fast);
            st_x(&ctl->stuck, 0LL, fast);
            st_x(&ctl->z0, z0, fast);
            st_x(&ctl->ndef[grp ^ 1], 0LL, fast);
            // a flag left by an unrecovered earlier call (a block of this
            // launch that times out sets it again)
            st_sc1(&ctl->bar_timeout, 0u);
        } else {
            z0 = *gp(&ctl->z0);
        }
    }
    int status = LP_PIVOTED;
    int pending = -1;                 // pivot whose column-0 update is still due
    long long pendR = -1;
    double p0 = 0.0;                  // its P[.][0]
    u64 ownpiv[RPL];                  // pivots s whose pivot row is the lane's k-th row
#pragma unroll
    for (int k = 0; k < RPL; ++k) ownpiv[k] = 0;
    int stop = 0;                     // block 0: the objective increased (simplex.py:133)
    int ndone = 0;                    // pivots of this launch completed (their M in lM)
    unsigned long long xwait = 0;     // XR: cross-rank waits of this block (Ctl::xwait_ticks)
    for (int tv = 0; tv < count; ++tv) {
        // the pivot index is wave-uniform; saying so keeps the chains'
        // trip counts and bounds in SGPRs (scalar branches, no exec masking:
        // the loop's exits look divergent to the compiler)
        const int t = __builtin_amdgcn_readfirstlane(tv);
        stamp(A, b, t, 0);
        // ---- entering column
        long long C;
        if (t == 0 && !from_erec && !enter) {
            C = ld_sc1(&ctl->c) + 1;
        } else {
            const bool capped = cap >= 0 && npiv >= cap;
            double el[NR], eq[NR];
            long long ei[NR];
            long long ef = NONE;
            double emin = INFINITY;
            bool halt = false;
            if (t == 0 && from_erec) {   // previous launch's summaries (kernel boundary: plain data)
#pragma unroll
                for (int k = 0; k < NR; ++k) {
                    const unsigned bb = tid + k * nth;
                    el[k] = INFINITY;
                    eq[k] = 0.0;
                    ei[k] = NONE;
                    if (bb < G) {
                        el[k] = ld_sc1(&A.erec[bb].l);
                        ei[k] = ld_sc1(&A.erec[bb].i);
                        eq[k] = ld_sc1(&A.erec[bb].q);
                        const long long f = ld_sc1(&A.erec[bb].fneg);
                        ef = f < ef ? f : ef;
                        emin = fmin(emin, el[k]);
                    }
                }
                rule = (int)__builtin_amdgcn_readfirstlane((int)ld_sc1(&A.erec[0].rule));
            } else {
                const unsigned etag = t == 0 ? gtag(seq, 0, 0) : gtag(seq, t - 1, 1);
                if (t == 0) {
                    // first pivot of a call: every block's summary of its
                    // row-0 slice, exchanged like a pivot's (k_enter's work)
                    double vv[IPL], vmin = INFINITY;
#pragma unroll
                    for (int k = 0; k < IPL; ++k) {
                        const long long j = jc0 + tid + k * nth;
                        vv[k] = INFINITY;
                        if (j < jc1 && j >= 1 && j <= A.n) {
                            vv[k] = l0[kc[k]];
                            vmin = fmin(vmin, vv[k]);
                        }
                    }
                    double sel_, seq_;
                    long long sei_, sfn_;
                    row0_summary<IPL>(vv, vmin, jc0, A.tol, sel_, sei_, seq_, sfn_);
                    unsigned wv = 0;
                    if (tid == 0) wv = lo32(sel_);
                    else if (tid == 1) wv = hi32(sel_);
                    else if (tid == 2) wv = lo32(seq_);
                    else if (tid == 3) wv = hi32(seq_);
                    else if (tid == 4) wv = idx32(sei_);
                    else if (tid == 5) wv = idx32(sfn_) & 0x7fffffffu;
                    if (!pub2(grE, grE2, etag, wv, NGE, A.tol.cost_tie, true)) {
                        status = LP_DEVICE_ERROR;
                        break;
                    }
                }
                unsigned w[NR][NGE];
                if (!(hier ? gather<NR, NGE, false>(grE2, 8, etag, w, &ctl->bar_timeout, A.spin_max)
                           : gather<NR, NGE>(grE, G, etag, w, &ctl->bar_timeout, A.spin_max, xs))) {
                    status = LP_DEVICE_ERROR;
                    break;
                }
#pragma unroll
                for (int k = 0; k < NR; ++k) {
                    const unsigned bb = tid + k * nth;
                    el[k] = INFINITY;
                    eq[k] = 0.0;
                    ei[k] = NONE;
                    if (bb < Geff) {
                        el[k] = mk_d(w[k][0], w[k][1]);
                        eq[k] = mk_d(w[k][2], w[k][3]);
                        ei[k] = un_idx(w[k][4] & 0x7fffffffu);
                        const long long f = un_idx(w[k][5] & 0x7fffffffu);
                        ef = f < ef ? f : ef;
                        emin = fmin(emin, el[k]);
                    }
                }
                if (t > 0) {
                    // block 0's summary (lane 0) carries the rule, the stop
                    // flag and P[t-1][0]
                    rule = (int)((unsigned)__builtin_amdgcn_readfirstlane(w[0][5]) >> 31);
                    halt = ((unsigned)__builtin_amdgcn_readfirstlane(w[0][4]) >> 31) != 0;
                    p0 = mk_d(__builtin_amdgcn_readfirstlane(w[0][6]),
                              __builtin_amdgcn_readfirstlane(w[0][7]));
                }
            }
            if (halt || capped) {
                C = NONE;
            } else if (rule == LP_RULE_MIN_INDEX) {
                C = block_min_ll(ef, sl);
            } else {
                const double g = block_min(emin, sd);
                if (!(g < -A.tol.cost)) {
                    C = NONE;
                } else {
                    const double ethr = tie_band(g, A.tol.cost_tie);
                    // the summaries combined: every block's (previous launch's
                    // records) or, two-level, the 8 XCD groups'
                    const bool rec = t == 0 && from_erec;
                    C = combine_loaded(el, ei, eq, rec ? G : Geff, ethr);
                    if (C < 0) {   // rare: rescan that slice of row 0
                        const long long wsl = cpb * (rec ? 1 : smul);
                        const long long k0 = (-1 - C) * wsl;
                        long long best = NONE;
                        for (long long k = k0 + tid; k < k0 + wsl; k += nth)
                            if (k >= 1 && k <= A.n && ld_sc1(&A.row0[k]) <= ethr) { best = k; break; }
                        C = block_min_ll(best, sl);
                    }
                }
            }
            if (C == NONE) status = halt ? LP_OBJ_INCREASED : capped ? LP_CAP_REACHED : LP_OPTIMAL;
        }
        stamp(A, b, t, 1);
        bstamp(A, b, t, 2);
        if (pending >= 0) {
#pragma unroll
            for (int k = 0; k < RPL; ++k)
                if (own[k]) {
                    const double c0 = upd(li[k], pendR, mrow[k][pending], p0, lc[tid + k * nth]);
                    lc[tid + k * nth] = c0;
                    st_x(&A.col0[li[k]], c0, fast);
                }
            pending = -1;
        }
        if (status != LP_PIVOTED) break;
        stamp(A, b, t, 2);
        // ---- ratio test over own rows; M[t] of own rows.  The tableau column
        //      loads are issued before the cross-block loads (one round trip).
        double a[RPL];
#pragma unroll
        for (int k = 0; k < RPL; ++k) a[k] = own[k] ? *gp(A.T + li[k] * A.ld + C) : 0.0;
        if (tid < t) sPc[tid] = ld_sc1(&A.P[tid * A.ld + C]);
        if (tid == 0) {
            if (b == 0) st_x(&ctl->c, C - 1, fast);
            if (C >= jc0 && C < jc1) {   // row 0's multiplier (+ the sweep's copy, read after the launch)
                st_x(&A.M[mi(A.rows, 0, t)], l0[C - jc0], fast);
                *gp(&A.MQ[mq(0, t)]) = l0[C - jc0];
            }
        }
        __syncthreads();
        stamp(A, b, t, 3);
        if (STAMPS && A.stamps) {   // diagnostic: the column elements have arrived
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            bstamp(A, b, t, 3);
        }
        // deferred pivots 0..t-1 on the own rows' elements of column C, CH at
        // a time.  A lane whose row was an earlier pivot row takes the select;
        // otherwise plain FMAs.
        {
            bool anyp = false;
#pragma unroll
            for (int k = 0; k < RPL; ++k) anyp = anyp || (own[k] && ownpiv[k] != 0);
            const bool sel = __ballot(anyp) != 0;
            // whole chunks without a pivot row among the own rows: no
            // per-pivot branch (the common case), the rest guarded
            const int tfull = sel ? 0 : (t & ~(CH - 1));
            for (int s0 = 0; s0 < tfull; s0 += CH) {
                double pc[CH], mm[RPL][CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    pc[u] = sPc[s0 + u];
#pragma unroll
                    for (int k = 0; k < RPL; ++k) mm[k][u] = mrow[k][s0 + u];
                }
#pragma unroll
                for (int u = 0; u < CH; ++u)
#pragma unroll
                    for (int k = 0; k < RPL; ++k) a[k] = fma(-mm[k][u], pc[u], a[k]);
            }
            for (int s0 = tfull; s0 < t; s0 += CH) {
                double pc[CH], mm[RPL][CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    pc[u] = sPc[s0 + u];
#pragma unroll
                    for (int k = 0; k < RPL; ++k) mm[k][u] = mrow[k][s0 + u];
                }
                if (!sel) {
#pragma unroll
                    for (int u = 0; u < CH; ++u)
                        if (s0 + u < t) {
#pragma unroll
                            for (int k = 0; k < RPL; ++k) a[k] = fma(-mm[k][u], pc[u], a[k]);
                        }
                } else {
#pragma unroll
                    for (int u = 0; u < CH; ++u)
                        if (s0 + u < t) {
#pragma unroll
                            for (int k = 0; k < RPL; ++k)
                                a[k] = ((ownpiv[k] >> (s0 + u)) & 1) ? pc[u] : fma(-mm[k][u], pc[u], a[k]);
                        }
                }
            }
        }
        double qown[RPL];
        bool okown[RPL];
        double mloc = INFINITY;
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            qown[k] = 0.0;
            okown[k] = false;
            if (own[k]) {
                mrow[k][t] = a[k];
                st_x(&A.M[mi(A.rows, li[k], t)], a[k], fast);
                qown[k] = row_ratio(a[k], lc[tid + k * nth], A.tol, okown[k]);
                okown[k] = okown[k] && own[k];
                if (okown[k]) mloc = fmin(mloc, qown[k]);
            }
        }
        const double lb = wave_min(mloc);
        stamp(A, b, t, 4);
        long long ib = NONE;
        double qb = 0.0, ab = 0.0;
        if (lb < INFINITY) {
            // own rows are lanes in row order (per k): the first row inside
            // the band is the lowest lane of the first k that has one
            const double thr = tie_band(lb, A.tol.ratio_tie);
            bool found = false;
#pragma unroll
            for (int k = 0; k < RPL; ++k) {
                const u64 mask = __ballot(okown[k] && qown[k] <= thr);
                if (!found && mask) {
                    found = true;
                    const int f = __builtin_ctzll(mask);
                    ib = lr0 + k * nth + f;
                    qb = rl_d(lo32(qown[k]), hi32(qown[k]), f);
                    if constexpr (XR) ab = rl_d(lo32(a[k]), hi32(a[k]), f);
                }
            }
        }
        if (!(A.fault == t + 1 && b == 1)) {   // fault injection (tests): block 1 never publishes
            unsigned wv = idx32(ib);
            if (tid == 0) wv = lo32(lb);
            else if (tid == 1) wv = hi32(lb);
            else if (tid == 2) wv = lo32(qb);
            else if (tid == 3) wv = hi32(qb);
            else if (tid == 5) wv = lo32(ab);
            else if (tid == 6) wv = hi32(ab);
            if (!pub2(grR, grR2, gtag(seq, t, 0), wv, NGRX, A.tol.ratio_tie, false)) {
                status = LP_DEVICE_ERROR;
                break;
            }
        }
        bstamp(A, b, t, 0);
        stamp(A, b, t, 5);

        // ---- leaving row (combine the ratio summaries)
        double rl[NR];
        double rmin = INFINITY;
        unsigned w[NR][NGRX];
        if (!(hier ? gather<NR, NGRX, false>(grR2, 8, gtag(seq, t, 0), w, &ctl->bar_timeout, A.spin_max)
                   : gather<NR, NGRX>(grR, G, gtag(seq, t, 0), w, &ctl->bar_timeout, A.spin_max, xs))) {
            status = LP_DEVICE_ERROR;
            break;
        }
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            const unsigned bb = tid + k * nth;
            rl[k] = INFINITY;
            if (bb < Geff) {
                rl[k] = mk_d(w[k][0], w[k][1]);
                rmin = fmin(rmin, rl[k]);
            }
        }
        stamp(A, b, t, 6);
        const double g = block_min(rmin, sd);
        long long R = NONE;           // local row: this device's leaving row / candidate
        double qR = 0.0, aR = 0.0;    // its ratio and pivot element (XR)
        if (g < INFINITY) {
            const double thr = tie_band(g, A.tol.ratio_tie);
            const int bs = first_in_band(rl, Geff, thr);
            const int k = bs / nth, f = bs % nth;
            double q = 0.0, av_ = 0.0;
            unsigned wi = 0;
#pragma unroll
            for (int kk = 0; kk < NR; ++kk)
                if (kk == k) {
                    q = rl_d(w[kk][2], w[kk][3], f);
                    wi = rl32(w[kk][4], f);
                    if constexpr (XR) av_ = rl_d(w[kk][5], w[kk][6], f);
                }
            if (q <= thr) {
                R = un_idx(wi);
                qR = q;
                aR = av_;
            } else {   // rare: rescan the selected block's (group's) rows (their M[t], col0 are published)
                const long long r0 = 1 + (long long)bs * rpb * smul, r1 = min(r0 + rpb * smul, A.rows);
                long long mine = NONE;
                double qm = 0.0, am = 0.0;
                for (long long lj = r0 + tid; lj < r1; lj += nth) {
                    bool ok;
                    const double mv = ld_sc1(&A.M[mi(A.rows, lj, t)]);
                    const double qq = row_ratio(mv, ld_sc1(&A.col0[lj]), A.tol, ok);
                    if (ok && qq <= thr) { mine = lj; qm = qq; am = mv; break; }
                }
                R = block_min_ll(mine, sl);
                const int fr = __builtin_ctzll(__ballot(mine == R));
                qR = rl_d(lo32(qm), hi32(qm), fr);
                aR = rl_d(lo32(am), hi32(am), fr);
            }
        } else if (!XR) {
            status = LP_UNBOUNDED;
            break;
        }
        stamp(A, b, t, 7);
        // ---- pivot row on own columns.  prow(Rl, av): the current values of
        //      local row Rl (stored row + this group's deferred pivots)
        //      divided by the pivot element.  Tableau row loads first, then
        //      the cross-block loads (one round trip).
        double pv_[IPL];                  // this pivot's normalised row on own columns
        const double f0 = ld_sc1(&A.M[mi(A.rows, 0, t)]);
        auto prow = [&](long long Rl, double avv) {
            double xv[IPL];
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const long long j = jc0 + tid + k * nth;
                xv[k] = j < jc1 ? *gp(A.T + Rl * A.ld + j) : 0.0;
            }
            if (tid <= t) sMr[tid] = ld_sc1(&A.M[mi(A.rows, Rl, tid)]);
            // pivots s whose pivot row is Rl: the select instead of the FMA (uniform)
            const u64 rpiv = __ballot(tid < t && sR[tid] == Rl);
            __syncthreads();
            stamp(A, b, t, 8);
            const double av = XR ? avv : sMr[t];
            // whole chunks when row Rl was no earlier pivot row: no per-pivot
            // branch (the common case), the rest guarded
            const int tfull = rpiv ? 0 : (t & ~(CH - 1));
            for (int s0 = 0; s0 < tfull; s0 += CH) {
                double mr[CH], pv[CH][IPL];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    mr[u] = sMr[s0 + u];
#pragma unroll
                    for (int k = 0; k < IPL; ++k) pv[u][k] = pcol[k][s0 + u];
                }
#pragma unroll
                for (int u = 0; u < CH; ++u)
#pragma unroll
                    for (int k = 0; k < IPL; ++k) xv[k] = fma(-mr[u], pv[u][k], xv[k]);
            }
            for (int s0 = tfull; s0 < t; s0 += CH) {
                double mr[CH], pv[CH][IPL];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    mr[u] = sMr[s0 + u];
#pragma unroll
                    for (int k = 0; k < IPL; ++k) pv[u][k] = pcol[k][s0 + u];
                }
#pragma unroll
                for (int u = 0; u < CH; ++u)
                    if (s0 + u < t) {
                        if ((rpiv >> (s0 + u)) & 1) {     // row Rl was pivot row s
#pragma unroll
                            for (int k = 0; k < IPL; ++k) xv[k] = pv[u][k];
                        } else {
#pragma unroll
                            for (int k = 0; k < IPL; ++k) xv[k] = fma(-mr[u], pv[u][k], xv[k]);
                        }
                    }
            }
            if (STAMPS && A.stamps) {   // diagnostic: the chain's results exist
                asm volatile("" ::"v"(xv[0]), "v"(xv[IPL - 1]));
                stamp(A, b, t, 12);
            }
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const long long j = jc0 + tid + k * nth;
                pv_[k] = (j == C) ? 1.0 : xv[k] / av;
            }
            if (STAMPS && A.stamps) {
                asm volatile("" ::"v"(pv_[0]), "v"(pv_[IPL - 1]));
                stamp(A, b, t, 13);
            }
            __syncthreads();      // sMr is reused
        };
        bool win = true;              // this rank holds the leaving row
        long long rglob = R - 1 + A.rb;
        if constexpr (XR) {
            // ---- leaving row across ranks.  Every rank sends (local minimum,
            //      candidate's ratio, global row, pivot element) to all ranks
            //      and, without waiting for the verdict, its candidate's
            //      normalised row: the winner's row is then already on its way.
            const int par = t & 1;
            const int N = A.nranks;
            const unsigned long long xticks = (unsigned long long)A.xwait_ms * 100000ull;
            u64 *xs = A.xbuf + par * XS_SUM_PAR;           // local slots, written by the peers
            if (b == 0 && tid < 7) {
                const unsigned long long tg = (u64)gtag(seq, t, 2) << 32;
                unsigned wv = 0;
                if (tid == 0) wv = lo32(g);
                else if (tid == 1) wv = hi32(g);
                else if (tid == 2) wv = lo32(qR);
                else if (tid == 3) wv = hi32(qR);
                else if (tid == 4) wv = R == NONE ? 0xffffffffu : (unsigned)rglob;
                else if (tid == 5) wv = lo32(aR);
                else wv = hi32(aR);
                for (int p = 0; p < N; ++p)
                    st_sys(&(*gp(A.peer + p))[par * XS_SUM_PAR + A.rank * 8 + tid], tg | wv);
            }
            // this rank's slot of pivot-row slices in every peer's buffer
            auto send_row = [&](int ph) {
                const unsigned long long tg = (u64)gtag(seq, t, ph) << 32;
                for (int p = 0; p < N; ++p) {
                    if (p == A.rank) continue;
                    u64 *dst = (*gp(A.peer + p)) + XS_PROW + (long long)(par * N + A.rank) * XS_PROW_RANK +
                               (long long)b * XS_PROW_BLOCK;
#pragma unroll
                    for (int k = 0; k < IPL; ++k) {
                        const int kk = tid + k * nth;
                        if (jc0 + kk < jc1) {
                            st_sys(&dst[2 * kk], tg | lo32(pv_[k]));
                            st_sys(&dst[2 * kk + 1], tg | hi32(pv_[k]));
                        }
                    }
                }
            };
            if (R != NONE) {
                prow(R, aR);
                send_row(3);
            }
            unsigned x[7];
            const unsigned long long xw0 = __builtin_amdgcn_s_memrealtime();
            if (!gather_x<7>(xs, N, gtag(seq, t, 2), x, &ctl->bar_timeout, xticks)) {
                status = LP_DEVICE_ERROR;
                break;
            }
            const double lp = (int)tid < N ? mk_d(x[0], x[1]) : INFINITY;
            const double gg = wave_min(lp);
            if (!(gg < INFINITY)) { status = LP_UNBOUNDED; break; }
            const double thr = tie_band(gg, A.tol.ratio_tie);
            const int ps = __builtin_ctzll(__ballot((int)tid < N && lp <= thr));
            const double qs = rl_d(x[2], x[3], ps);
            long long rg;
            double as;
            int ph = 3;                   // the tag of the winner's row slices
            if (qs <= thr) {
                rg = (long long)rl32(x[4], ps);
                as = rl_d(x[5], x[6], ps);
            } else {
                // rare: a near-tie straddles the band across ranks.  Rank ps
                // (the first with a row inside it) finds its first such row:
                // each block offers its first own row, block 0 sends the lowest
                // to every rank (the straddle slot); rank ps then ships that
                // row's normalised values instead of its candidate's
                if (A.rank == ps) {
                    long long ir = NONE;
                    double ar = 0.0;
                    bool found = false;
#pragma unroll
                    for (int k = 0; k < RPL; ++k) {
                        const u64 mk = __ballot(okown[k] && qown[k] <= thr);
                        if (!found && mk) {
                            found = true;
                            const int fr = __builtin_ctzll(mk);
                            ir = lr0 + k * nth + fr;
                            ar = rl_d(lo32(a[k]), hi32(a[k]), fr);
                        }
                    }
                    u64 *loc = A.xbuf + XS_PROW + 2LL * N * XS_PROW_RANK;
                    if (tid < 3) {
                        const unsigned wv = tid == 0 ? idx32(ir) : tid == 1 ? lo32(ar) : hi32(ar);
                        st_sc1(&loc[b * 8 + tid], ((u64)gtag(seq, t, 4) << 32) | wv);
                    }
                    unsigned wl[NR][3];
                    if (!gather<NR, 3, false>(loc, G, gtag(seq, t, 4), wl, &ctl->bar_timeout, A.spin_max)) {
                        status = LP_DEVICE_ERROR;
                        break;
                    }
                    double il[NR];
#pragma unroll
                    for (int k = 0; k < NR; ++k)
                        il[k] = (tid + k * nth < G && wl[k][0] != 0x7fffffffu) ? 0.0 : INFINITY;
                    const int bf = first_in_band(il, G, 0.0);
                    const int kf = bf / nth, ff = bf % nth;
                    unsigned r0w = 0, a0 = 0, a1 = 0;
#pragma unroll
                    for (int kk = 0; kk < NR; ++kk)
                        if (kk == kf) {
                            r0w = rl32(wl[kk][0], ff);
                            a0 = rl32(wl[kk][1], ff);
                            a1 = rl32(wl[kk][2], ff);
                        }
                    if (b == 0 && tid < 3) {
                        const unsigned wv = tid == 0 ? (unsigned)((long long)r0w - 1 + A.rb) : tid == 1 ? a0 : a1;
                        for (int p = 0; p < N; ++p)
                            st_sys(&(*gp(A.peer + p))[par * XS_SUM_PAR + NRANK_MAX * 8 + tid],
                                   ((u64)gtag(seq, t, 5) << 32) | wv);
                    }
                }
                unsigned y[3];
                if (!gather_x<3>(xs + NRANK_MAX * 8, 1, gtag(seq, t, 5), y, &ctl->bar_timeout, xticks)) {
                    status = LP_DEVICE_ERROR;
                    break;
                }
                rg = (long long)__builtin_amdgcn_readfirstlane(y[0]);
                as = mk_d(__builtin_amdgcn_readfirstlane(y[1]), __builtin_amdgcn_readfirstlane(y[2]));
                ph = 6;
                if (A.rank == ps) {
                    prow(rg - A.rb + 1, as);
                    send_row(6);
                }
            }
            win = A.rank == ps;
            rglob = rg;
            R = win ? rg - A.rb + 1 : -1;
            aR = as;
            if (!win) {
                // the winning rank's block b sent these columns
                const u64 *src = A.xbuf + XS_PROW + (long long)(par * N + ps) * XS_PROW_RANK +
                                 (long long)b * XS_PROW_BLOCK;
                const unsigned tg = gtag(seq, t, ph);
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    bool ok = true;
#pragma unroll
                    for (int k = 0; k < IPL; ++k) {
                        const int kk = min((long long)tid + k * nth, cpb - 1);
                        const u64 lo = ld_sys(&src[2 * kk]), hi = ld_sys(&src[2 * kk + 1]);
                        pv_[k] = mk_d((unsigned)lo, (unsigned)hi);
                        ok = ok && (jc0 + kk >= jc1 ||
                                    ((unsigned)(lo >> 32) == tg && (unsigned)(hi >> 32) == tg));
                    }
                    if (__all(ok)) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > xticks) {
                        st_sc1(&ctl->bar_timeout, 1u);
                        status = LP_DEVICE_ERROR;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (status != LP_PIVOTED) break;
            }
            xwait += __builtin_amdgcn_s_memrealtime() - xw0;
        } else {
            prow(R, 0.0);
        }
#pragma unroll
        for (int k = 0; k < RPL; ++k)
            if (li[k] == R) ownpiv[k] |= 1ull << t;
        if (tid == 0) sR[t] = R;
        double vmin = INFINITY, v0 = 0.0;
        double vv[IPL];                   // new row 0 on own columns (INFINITY: not a variable column)
        double vn[IPL];                   // new row 0 on own columns
        // every LDS read and all arithmetic first, then the LDS writes, then
        // the global stores: no register of a pending store is rewritten in
        // between (the compiler would wait for the store to complete)
#pragma unroll
        for (int k = 0; k < IPL; ++k) vn[k] = upd(0, -1, f0, pv_[k], l0[kc[k]]);
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            const long long j = jc0 + tid + k * nth;
            vv[k] = INFINITY;
            if (j == 0) v0 = vn[k];
            if (j < jc1 && j >= 1 && j <= A.n) {
                vmin = fmin(vmin, vn[k]);
                vv[k] = vn[k];
            }
        }
#pragma unroll
        for (int k = 0; k < IPL; ++k)
            if (jc0 + tid + k * nth < jc1) {
                lP[kc[k] * cs + t] = pv_[k];
                l0[kc[k]] = vn[k];
            }
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            const long long j = jc0 + tid + k * nth;
            if (j < jc1) {
                st_x(&A.P[t * A.ld + j], pv_[k], fast);
                st_x(&A.row0[j], vn[k], fast);
            }
        }
        __syncthreads();
        stamp(A, b, t, 9);
        double el, eq;
        long long ei, efn;
        row0_summary<IPL>(vv, vmin, jc0, A.tol, el, ei, eq, efn);
        stamp(A, b, t, 10);
        // stall bookkeeping (simplex.py:132-137), min-index switch (:123,138)
        // and the objective check (:133) by block 0 (column 0 is in its
        // slice: v0 = new row0[0]); rule and stop flag travel in its summary,
        // the records are stored after the publish
        if (b == 0 && tid == 0 && mode == MODE_SOLVE && rule == LP_RULE_STANDARD) {
            nstd += 1;
            const double z = -v0;
            const double band = A.tol.stall * fmax(1.0, fabs(z0));
            if (z - z0 > band) stop = 1;   // 'objective value increased'
            if (fabs(z - z0) <= band) stuck += 1;
            else stuck = 0;
            if (stuck >= A.m + A.n) rule = LP_RULE_MIN_INDEX;
        }
        rule = __builtin_amdgcn_readfirstlane(rule);   // block 0 lane 0 may have switched it
        stop = __builtin_amdgcn_readfirstlane(stop);
        const double p0n = b == 0 ? lP[t] : 0.0;       // P[t][0] (column 0 is block 0's first)
        {
            unsigned wv = 0;
            if (tid == 0) wv = lo32(el);
            else if (tid == 1) wv = hi32(el);
            else if (tid == 2) wv = lo32(eq);
            else if (tid == 3) wv = hi32(eq);
            else if (tid == 4) wv = (idx32(ei) & 0x7fffffffu) | ((unsigned)stop << 31);
            else if (tid == 5) wv = (idx32(efn) & 0x7fffffffu) | ((unsigned)rule << 31);
            else if (tid == 6) wv = lo32(p0n);
            else if (tid == 7) wv = hi32(p0n);
            if (!pub2(grE, grE2, gtag(seq, t, 1), wv, NGE, A.tol.cost_tie, true)) {
                status = LP_DEVICE_ERROR;
                break;
            }
        }
        // records read after the launch only (host, sweep, next launch): one
        // store instruction of the last block (block 0 already carries the
        // stall bookkeeping and column 0), one record per lane
        if (b == G - 1 && tid < 7) {
            long long *adr = &A.dR[t];
            long long val = R;
            if (tid == 1) { adr = &A.dC[t]; val = C; }
            else if (tid == 2) { adr = &ctl->r; val = rglob; }
            else if (tid == 3) { adr = &ctl->npiv; val = npiv + 1; }
            else if (tid == 4) { adr = &ctl->ndef[grp]; val = t + 1; }
            else if (tid == 5) { adr = A.log + 2 * min(npiv, A.logcap - 1); val = rglob; }
            else if (tid == 6) { adr = A.log + 2 * min(npiv, A.logcap - 1) + 1; val = C - 1; }
            if (tid < 5 || npiv < A.logcap) st_x(adr, val, fast);
        }
        if (b == 0 && tid == 0 && mode == MODE_SOLVE) {
            st_x(&ctl->nstd, nstd, fast);
            st_x(&ctl->stuck, stuck, fast);
            st_x(&ctl->rule, (int)rule, fast);
        }
        if (t == count - 1 && tid == 0) {     // the next launch reads plain summaries
            st_x(&A.erec[L].l, el, fast);
            st_x(&A.erec[L].i, ei, fast);
            st_x(&A.erec[L].q, eq, fast);
            st_x(&A.erec[L].fneg, efn, fast);
            if (b == 0) st_x(&A.erec[0].rule, (long long)rule, fast);
        }
        bstamp(A, b, t, 1);
        ++npiv;
        ++ndone;
        stamp(A, b, t, 11);
        pending = t;
        pendR = R;
    }
    // the last pivot's column-0 update: P[pending][0] arrives in block 0's
    // row-0 summary
    if (pending >= 0) {
        unsigned w[NR][NGE];
        if (hier ? gather<NR, NGE, false>(grE2, 8, gtag(seq, pending, 1), w, &ctl->bar_timeout, A.spin_max)
                 : gather<NR, NGE>(grE, G, gtag(seq, pending, 1), w, &ctl->bar_timeout, A.spin_max, xs)) {
            const double pl = mk_d(__builtin_amdgcn_readfirstlane(w[0][6]),
                                   __builtin_amdgcn_readfirstlane(w[0][7]));
#pragma unroll
            for (int k = 0; k < RPL; ++k)
                if (own[k]) st_x(&A.col0[li[k]], upd(li[k], pendR, mrow[k][pending], pl, lc[tid + k * nth]), fast);
        } else {
            status = LP_DEVICE_ERROR;
        }
    }
    // the sweep's copy of the group's multipliers of the own rows (MQ, 4-row
    // quads) from LDS: consecutive lanes store consecutive doubles of the
    // block's quads (the quads shared with a neighbour block: own rows only);
    // read after the launch, so plain stores (issued before the last
    // exchange's wait instead: 0.1 us per pivot slower)
    {
        const int nds = __builtin_amdgcn_readfirstlane(ndone);
        const long long e0 = (lr0 >> 2) * (4 * BMAX), e1 = (((lr1 - 1) >> 2) + 1) * (4 * BMAX);
        for (long long e = e0 + tid; e < e1 && nds > 0; e += nth) {
            const long long row = e / (4 * BMAX) * 4 + (e & 3);
            const int s = (int)(e % (4 * BMAX) >> 2);
            if (row >= lr0 && row < lr1 && s < nds) *gp(&A.MQ[e]) = lM[(row - lr0) * cs + s];
        }
    }
    if (XR && b == 0 && tid == 0) {
        *gp(&ctl->xwait_ticks) += xwait;
        *gp(&ctl->xwait_pivots) += ndone;
    }
    if (b == 0 && tid == 0) {
        // an increase at the launch's last pivot: nothing read the flag yet
        if (stop && status == LP_PIVOTED) status = LP_OBJ_INCREASED;
        if (status != LP_PIVOTED) st_sc1(&ctl->status, status);
    }
}

// ---------------------------------------------------------------------------
// K3: the sweep (tableau.py:305-308 -> :269-289 for a whole group).  T <- T
//   with the group's deferred pivots 0..ndef-1 applied.  Two kernels:
//   k_sweep_rl (below) for groups of 49..64 pivots -- the automatic depth of
//   cfg3 and cfg4, so the bench's kernel -- and k_sweep_dp2 for shorter ones
//   (a call's short last group, explicit pivots, the per-pivot path's 32).
//   Pivots nd..NB-1 are padding with P = 0 and multiplier 0: fma(-0, 0, x)
//   == x for every x.  Every element gets exactly the float64 operations of
//   an immediate update in pivot order (upd()): bit-identical to
//   oracle/lp_f64.c for every group size.  (Rounds 1-2's k_sweep_st and
//   k_sweep_dp, LDS- and register-broadcast strips, were removed in round 6:
//   k_sweep_rl replaced them at 64 pivots)
// ---------------------------------------------------------------------------

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
// raw buffer over a wave-uniform base: loads and stores then address with
// one 32-bit lane offset (VGPR) + a uniform byte offset (SGPR)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7fffffff, 0x00020000);
}

// ---------------------------------------------------------------------------
// The multipliers broadcast by DPP: a 4-pivot chunk's multipliers of a 4-row
// batch sit in one register, value v = 4 s' + k (pivot 4 c + s', batch row
// k) in lane v of each 16-lane row, and the FMA reads the one it needs with a
// row_newbcast DPP operand:
//     v_fmac_f64_dpp x, -m, p row_newbcast:v      (x <- fma(-m[v], p, x))
// -- no instruction is spent on the broadcast.
// ---------------------------------------------------------------------------

// pivots 4c + 2h, 4c + 2h + 1 of one batch (4 rows x 2 columns per lane): 16
// FMAs whose multiplier operand is lane (4 s' + k) of the lane's 16-lane row
// of m.  The s_nop (first half only) covers the VALU-write -> DPP-read hazard
// should the compiler copy m into place right before the block.
#define DPF(XR, PV, L) "v_fmac_f64_dpp " XR ", -%8, " PV " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
#define DPP_PIVOT(L0, L1, L2, L3, PX, PY)                                                     \
    DPF("%0", PX, L0) DPF("%1", PY, L0) DPF("%2", PX, L1) DPF("%3", PY, L1) DPF("%4", PX, L2) \
    DPF("%5", PY, L2) DPF("%6", PX, L3) DPF("%7", PY, L3)
#define DPP_OUTS(x)                                                                                       \
    "+v"(x[0].x), "+v"(x[0].y), "+v"(x[1].x), "+v"(x[1].y), "+v"(x[2].x), "+v"(x[2].y), "+v"(x[3].x), \
        "+v"(x[3].y)
__device__ __forceinline__ void dp_half(double2 (&x)[4], double m, double2 p0, double2 p1, int h)
{
    if (h == 0)
        asm("s_nop 1\n" DPP_PIVOT(0, 1, 2, 3, "%9", "%10") DPP_PIVOT(4, 5, 6, 7, "%11", "%12")
            : DPP_OUTS(x) : "v"(m), "v"(p0.x), "v"(p0.y), "v"(p1.x), "v"(p1.y));
    else
        asm(DPP_PIVOT(8, 9, 10, 11, "%9", "%10") DPP_PIVOT(12, 13, 14, 15, "%11", "%12")
            : DPP_OUTS(x) : "v"(m), "v"(p0.x), "v"(p0.y), "v"(p1.x), "v"(p1.y));
}
#undef DPP_OUTS
#undef DPP_PIVOT
#undef DPF

// ---------------------------------------------------------------------------
// K3'': k_sweep_dp2, the sweep of groups of up to 48 pivots: a workgroup of
//   W waves owns a 128-column strip (2 columns per lane, 16-byte accesses) of
//   a run of rows, the strip's slice of P staged in LDS once, each wave on
//   4-row batches with the next batch in flight.  A batch's 4 x NB multipliers
//   arrive with 2 coalesced 16-byte loads per lane (lane l: pivot l's four
//   rows, half a batch per 32 lanes) instead of NB/4 replicated 8-byte loads,
//   are written to the slot half a batch at a time, and each 4-pivot chunk's
//   register is read back just in time (one ds_read_b64, 16 addresses
//   broadcast over the four 16-lane rows) -- about 80 VGPRs instead of 125,
//   6 waves per SIMD instead of 4.  Same FMAs in the same order.
// ---------------------------------------------------------------------------
template <int W, int NB, int SA>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(5, 8)))
k_sweep_dp2(const double *T, double *Tout, const double *__restrict__ P, const double *__restrict__ M,
            const long long *__restrict__ dR, const Ctl *__restrict__ ctl, long long ld, long long rows, int grp,
            int nstrips, long long run, long long tail)
{
    constexpr int RW = 4;                        // rows per batch
    constexpr int NM = NB / 4;                   // 4-pivot chunks
    constexpr int NH = NB / 2;                   // pivots per staged half
    static_assert(NB % 8 == 0 && NB <= BMAX && NH <= 32, "k_sweep_dp2: pivots per sweep");
    __shared__ double2 sp[NB][64];               // the strip's slice of P
    __shared__ double sm[W][NH * RW];            // per wave: half a batch's multipliers, [chunk][16]
    __shared__ long long sr[NB];
    const int nd = (int)ctl->ndef[grp];
    if (nd == 0 || ctl->bar_timeout) return;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ldb = (int)(ld * 8);
    if (threadIdx.x < NB) sr[threadIdx.x] = (int)threadIdx.x < nd ? dR[threadIdx.x] : -2;
    // lane l stages pivot h NH + (l & 31) of half h = l >> 5 (pivots past nd
    // read pivot nd - 1's: finite, and their P is 0)
    const int hl = lane >> 5, sl = lane & 31;
    const bool stager = sl < NH;
    const int sv = min(hl * NH + sl, nd - 1);
    const int nch = (nd + 3) >> 2;
    double *smw = &sm[wave][0];
    // rows [r0, r1) of one strip
    auto piece = [&](int strip, long long r0, long long r1) {
        const long long c0 = (long long)strip * 128;
        const int lo = min(lane * 2, (int)(ld - c0) - 2);
        const int lob = lo * 8;
        const double *Ts = T + c0;
        double *Tos = Tout + c0;
        for (int s = wave; s < NB; s += W)
            sp[s][lane] = s < nd ? *reinterpret_cast<const double2 *>(P + s * ld + c0 + lo) : make_double2(0.0, 0.0);
        auto load_m = [&](double2 (&mv)[2], long long rb) {
            const int kmax = (int)(r1 - 1 - rb);
            const __amdgpu_buffer_rsrc_t rm = buf_rsrc(M + (rb >> 2) * (4 * BMAX));
            const int base = sv * 4 * 8;                  // pivot sv's 4 rows: 32 contiguous bytes
            if (kmax >= 3) {
                mv[0] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rm, base, 0, 0));
                mv[1] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rm, base + 16, 0, 0));
            } else {   // the last batch of a piece: rows past r1 repeat row r1 - 1
                double v[4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    v[k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rm, base + min(k, kmax) * 8, 0, 0));
                mv[0] = make_double2(v[0], v[1]);
                mv[1] = make_double2(v[2], v[3]);
            }
        };
        auto load_x = [&](double2 (&x)[RW], long long rb) {
            const int kmax = (int)(r1 - 1 - rb);
            const __amdgpu_buffer_rsrc_t rt = buf_rsrc(Ts + rb * ld);
#pragma unroll
            for (int k = 0; k < RW; ++k)
                x[k] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rt, lob, min(k, kmax) * ldb, 0));
        };
        // half h of the batch's multipliers into the wave's slot: chunk c, value
        // 4 s' + k at [c * 16 + 4 s' + k] = [s * 4 + k] for the half's pivot s
        auto stage = [&](const double2 (&mv)[2], int h) {
            if (hl == h && stager) {
                reinterpret_cast<double2 *>(smw)[2 * sl] = mv[0];
                reinterpret_cast<double2 *>(smw)[2 * sl + 1] = mv[1];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        const long long step = (long long)W * RW;
        long long rb = r0 + (long long)wave * RW;
        double2 xn[RW], mv[2];
        if (rb < r1) {
            load_x(xn, rb);
            load_m(mv, rb);
        }
        __syncthreads();                         // sp (and sr) staged
        for (; rb < r1; rb += step) {
            double2 x[RW];
#pragma unroll
            for (int k = 0; k < RW; ++k) x[k] = xn[k];
            const long long rn = rb + step;
            const bool more = rn < r1;
            if (more) load_x(xn, rn);
            const int kmax = (int)min((long long)RW - 1, r1 - 1 - rb);
            // a whole chunk's P (4 pivots) is read from LDS while the previous
            // chunk's 32 FMAs run
            double2 pc[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) pc[u] = sp[u][lane];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                stage(mv, h);
                if (h == 1 && more) load_m(mv, rn);   // the next batch's, in flight from here
                double m = smw[lane & 15];
#pragma unroll
                for (int cl = 0; cl < NM / 2; ++cl) {
                    const int c = h * (NM / 2) + cl;
                    const double mn = smw[((cl + 1) % (NM / 2)) * 16 + (lane & 15)];
                    double2 pn[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) pn[u] = sp[(4 * c + 4 + u) % NB][lane];
                    if (c < nch) {               // wave-uniform
                        dp_half(x, m, pc[0], pc[1], 0);
                        dp_half(x, m, pc[2], pc[3], 1);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) pc[u] = pn[u];
                    m = mn;
                }
            }
            // a row that was pivot row s of the group: recomputed from P (rare)
            const long long R = sr[lane % NB];
            if (__builtin_expect(__ballot(R >= rb && R < rb + RW) != 0, 0)) {
#pragma unroll
                for (int k = 0; k < RW; ++k) {
                    const long long row = rb + min(k, kmax);
                    int sl2 = -1;
                    for (int s = 0; s < nd; ++s)
                        if (sr[s] == row) sl2 = s;
                    if (sl2 >= 0) {
                        double2 y = sp[sl2][lane];
                        for (int s = sl2 + 1; s < nd; ++s) {
                            const double f = M[mq(row, s)];
                            const double2 pv = sp[s][lane];
                            y = make_double2(fma(-f, pv.x, y.x), fma(-f, pv.y, y.y));
                        }
                        x[k] = y;
                    }
                }
            }
            const __amdgpu_buffer_rsrc_t ro = buf_rsrc(Tos + rb * ld);
#pragma unroll
            for (int k = 0; k < RW; ++k)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, x[k]), ro, lob, min(k, kmax) * ldb, SA);
        }
    };
    // block b: strip b % nstrips of row run b / nstrips -- consecutive blocks,
    // dealt round-robin over the XCDs, update the same rows at the same time,
    // so each run's multipliers are fetched about once per XCD (equal spans
    // of the strip-major (strip, row) space instead, one per resident
    // workgroup, re-fetched them per strip: 119 -> 174 us at cfg3)
    const int strip = (int)(blockIdx.x % (unsigned)nstrips);
    const long long r0 = (long long)(blockIdx.x / (unsigned)nstrips) * run;
    piece(strip, r0, min(rows, r0 + run));
    // tail > 0: the grid covers strips [0, nstrips) only and the last strip
    // (the one past them: column n and the row pitch's padding) is dealt out
    // `tail` rows to every block -- a whole block per run of that thin strip
    // would leave about one resident slot in nine empty (nstrips + 1 = 65
    // strips over 512 slots: 7 runs x 65 = 455 blocks)
    if (tail > 0) {
        const long long t0 = (long long)blockIdx.x * tail;
        if (t0 < rows) {                         // block-uniform
            __syncthreads();                     // every wave is done with sp
            piece(nstrips, t0, min(rows, t0 + tail));
        }
    }
}

// ---------------------------------------------------------------------------
// The register-operand FMA block of k_sweep_rl (below): 16 FMAs of pivots 2c,
// 2c + 1 on a batch's 8 rows, one column per lane, the pivot-row values in
// plain VGPRs and the multiplier read with a row_newbcast DPP operand from
// lane 8h + k of the lane's 16-lane row:
//     v_fmac_f64_dpp x[k], -m[c], p[2c + h] row_newbcast:(8h + k)
// ---------------------------------------------------------------------------
#define RGF(XK, P, L) "v_fmac_f64_dpp %" #XK ", -%8, %" #P " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
#define RG_OUTS(x) "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
// pivots 2c, 2c + 1 on the batch's 8 rows
__device__ __forceinline__ void rg_pair(double (&x)[8], double m, double pa, double pb)
{
    asm("s_nop 1\n" RGF(0, 9, 0) RGF(1, 9, 1) RGF(2, 9, 2) RGF(3, 9, 3) RGF(4, 9, 4) RGF(5, 9, 5) RGF(6, 9, 6)
            RGF(7, 9, 7) RGF(0, 10, 8) RGF(1, 10, 9) RGF(2, 10, 10) RGF(3, 10, 11) RGF(4, 10, 12) RGF(5, 10, 13)
                RGF(6, 10, 14) RGF(7, 10, 15)
        : RG_OUTS(x) : "v"(m), "v"(pa), "v"(pb));
}
// four pairs (pivots 8q .. 8q + 7) in one block: one hazard wait for the
// four multiplier registers instead of one per pair (SWEEP_RGQ)
#define RGQ(XK, M, P, L) "v_fmac_f64_dpp %" #XK ", -%" #M ", %" #P " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
__device__ __forceinline__ void rg_quad(double (&x)[8], double m0, double m1, double m2, double m3,
                                        const double *p)
{
    asm("s_nop 1\n" RGQ(0, 8, 12, 0) RGQ(1, 8, 12, 1) RGQ(2, 8, 12, 2) RGQ(3, 8, 12, 3) RGQ(4, 8, 12, 4) RGQ(5, 8, 12, 5) RGQ(6, 8, 12, 6) RGQ(7, 8, 12, 7) RGQ(0, 8, 13, 8) RGQ(1, 8, 13, 9) RGQ(2, 8, 13, 10) RGQ(3, 8, 13, 11) RGQ(4, 8, 13, 12) RGQ(5, 8, 13, 13) RGQ(6, 8, 13, 14) RGQ(7, 8, 13, 15)
        RGQ(0, 9, 14, 0) RGQ(1, 9, 14, 1) RGQ(2, 9, 14, 2) RGQ(3, 9, 14, 3) RGQ(4, 9, 14, 4) RGQ(5, 9, 14, 5) RGQ(6, 9, 14, 6) RGQ(7, 9, 14, 7) RGQ(0, 9, 15, 8) RGQ(1, 9, 15, 9) RGQ(2, 9, 15, 10) RGQ(3, 9, 15, 11) RGQ(4, 9, 15, 12) RGQ(5, 9, 15, 13) RGQ(6, 9, 15, 14) RGQ(7, 9, 15, 15)
        RGQ(0, 10, 16, 0) RGQ(1, 10, 16, 1) RGQ(2, 10, 16, 2) RGQ(3, 10, 16, 3) RGQ(4, 10, 16, 4) RGQ(5, 10, 16, 5) RGQ(6, 10, 16, 6) RGQ(7, 10, 16, 7) RGQ(0, 10, 17, 8) RGQ(1, 10, 17, 9) RGQ(2, 10, 17, 10) RGQ(3, 10, 17, 11) RGQ(4, 10, 17, 12) RGQ(5, 10, 17, 13) RGQ(6, 10, 17, 14) RGQ(7, 10, 17, 15)
        RGQ(0, 11, 18, 0) RGQ(1, 11, 18, 1) RGQ(2, 11, 18, 2) RGQ(3, 11, 18, 3) RGQ(4, 11, 18, 4) RGQ(5, 11, 18, 5) RGQ(6, 11, 18, 6) RGQ(7, 11, 18, 7) RGQ(0, 11, 19, 8) RGQ(1, 11, 19, 9) RGQ(2, 11, 19, 10) RGQ(3, 11, 19, 11) RGQ(4, 11, 19, 12) RGQ(5, 11, 19, 13) RGQ(6, 11, 19, 14) RGQ(7, 11, 19, 15)
        : RG_OUTS(x)
        : "v"(m0), "v"(m1), "v"(m2), "v"(m3), "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]),
          "v"(p[6]), "v"(p[7]));
}
#undef RGQ
#undef RG_OUTS
#undef RGF

// ---------------------------------------------------------------------------
// K3 (registers + LDS streaming): k_sweep_rl -- THE sweep of every group of
//   49..64 pivots (launch_sweep: the automatic depth is 64 for cfg3 and cfg4,
//   so this is the bench's update kernel; k_sweep_dp2 serves 17..48 and the
//   per-pivot path's 32).  The DPP sweeps above read P from LDS for every
//   pivot of every batch (16 bytes per lane per 8 FMAs: more LDS bandwidth per
//   FMA than a CU has at full FMA rate).  Here the pivot rows stay in
//   registers and no operand of an FMA comes from LDS: the tableau rows and
//   the multipliers travel HBM -> LDS with global_load_lds_dwordx4 (no VGPRs),
//   D batches deep, and each batch is read into registers once:
//     * a workgroup of W waves owns a strip of 64 W columns (one per lane) of a
//       run of rows; all W waves take the SAME 8-row batch, each on its own 64
//       columns, so the batch's multipliers (two MQ quads, 4 KB) are copied
//       once per workgroup -- one dwordx4 per wave;
//     * each wave keeps P[0..NB) of its column in registers (2 NB VGPRs);
//     * per batch: wait for its copies (vmcnt, one workgroup barrier), start the
//       copies of batch i + D - 1 into the slot batch i - 1 used, read x (8
//       rows) and the multipliers' DPP registers from LDS, the FMAs, store x.
//   A group the host knows to be short (49..63 pivots) runs the same pass
//   with the missing pivots' rows of P and multipliers zeroed by the host
//   (exact no-ops); shorter ones take k_sweep_dp2 at their own depth
//   (launch_sweep).  Every element gets exactly
//   upd()'s float64 operations in pivot order: bit-identical to
//   oracle/lp_f64.c.  cfg4 (W = 8, D = 4, 243 VGPRs, one workgroup per CU,
//   out of place: T -> the handle's other buffer, lpgpu.cpp, non-temporal
//   stores): ~775 us per 64-pivot launch = 0.70 of the HBM spec (in place
//   842 us); cfg3 (W = 4, D = 2, in place): 109 us = 0.62
//   (profiles/r04/README.md).
// ---------------------------------------------------------------------------
// LDS byte offset of a __shared__ location (for LDS accesses written in asm)
__device__ __forceinline__ unsigned lds_off(const double *p)
{
    return (unsigned)(unsigned long)(const __attribute__((address_space(3))) double *)p;
}
__device__ __forceinline__ unsigned lds_off(const int *p)
{
    return (unsigned)(unsigned long)(const __attribute__((address_space(3))) int *)p;
}
// k_sweep_rl's rows: x[k] = LDS[a + 512 k]
template <int RW>
__device__ __forceinline__ void lds_rows(double (&x)[RW], unsigned a)
{
    static_assert(RW == 8, "lds_rows");
    asm volatile("ds_read_b64 %0, %8\n ds_read_b64 %1, %8 offset:512\n ds_read_b64 %2, %8 offset:1024\n"
                 "ds_read_b64 %3, %8 offset:1536\n ds_read_b64 %4, %8 offset:2048\n ds_read_b64 %5, %8 offset:2560\n"
                 "ds_read_b64 %6, %8 offset:3072\n ds_read_b64 %7, %8 offset:3584"
                 : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7])
                 : "v"(a));
}
// k_sweep_rl's multiplier registers: m[c] = LDS[a + 64 c]
template <int C>
__device__ __forceinline__ void lds_mult_one(double &m, unsigned a)
{
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(m) : "v"(a), "n"(64 * C));
}
template <int NC, int C = 0>
__device__ __forceinline__ void lds_mult(double (&m)[NC], unsigned a)
{
    if constexpr (C < NC) {
        lds_mult_one<C>(m[C], a);
        lds_mult<NC, C + 1>(m, a);
    }
}
// m[C .. N)
template <int N, int NC, int C = 0>
__device__ __forceinline__ void lds_mult_first(double (&m)[NC], unsigned a)
{
    if constexpr (C < N && C < NC) {
        lds_mult_one<C>(m[C], a);
        lds_mult_first<N, NC, C + 1>(m, a);
    }
}
// pair c of a batch with the reads pipelined (k_sweep_rl, SWEEP_LDSPIPE):
// the read of m[c + 8] goes out, then the wait for m[c] -- in issue order
// m[c] is read 8 + c, so 8 reads may still be in flight (fewer over the last
// 8 pairs: the count field holds at most 15) -- then pair c's 16 FMAs
// (Q = 4: four pairs per step, rg_quad's one DPP hazard wait per block: the
// reads of m[c + 8 .. c + 11] out, then the wait for m[c + 3])
// (SWEEP_AHEAD = A registers read ahead: m[0 .. A) before the first pair,
// m[C + A .. C + A + Q) at step C; in issue order m[j] is read 8 + j, so
// after step C's reads A of them may still be in flight)
#ifndef SWEEP_AHEAD
#define SWEEP_AHEAD 8
#endif
template <int NC, int Q, int C = 0>
__device__ __forceinline__ void sweep_pairs(double (&x)[8], double (&m)[NC], const double (&p)[2 * NC], unsigned a)
{
    constexpr int A = SWEEP_AHEAD;
    static_assert(A % Q == 0 && A <= 15, "sweep_pairs: read-ahead");
    if constexpr (C < NC) {
        if constexpr (C + A < NC) lds_mult_one<C + A>(m[C + A], a);
        if constexpr (Q == 4 && C + A + 1 < NC) lds_mult_one<C + A + 1>(m[C + A + 1], a);
        if constexpr (Q == 4 && C + A + 2 < NC) lds_mult_one<C + A + 2>(m[C + A + 2], a);
        if constexpr (Q == 4 && C + A + 3 < NC) lds_mult_one<C + A + 3>(m[C + A + 3], a);
        constexpr int L = C + Q - 1;                  // the last register this step reads
        constexpr int K = L + A + 1 <= NC ? A : NC - 1 - L;
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(m[L]) : "n"(K) : "memory");
        if constexpr (Q == 4) {
            asm volatile("" : "+v"(m[C]), "+v"(m[C + 1]), "+v"(m[C + 2]));
            rg_quad(x, m[C], m[C + 1], m[C + 2], m[C + 3], &p[2 * C]);
        } else {
            rg_pair(x, m[C], p[2 * C], p[2 * C + 1]);
        }
        __builtin_amdgcn_sched_barrier(0);
        sweep_pairs<NC, Q, C + Q>(x, m, p, a);
    }
}

// pivots 16 K + j0 .. 16 K + j1 - 1 of a pivot-row chain: y <- fma(-m[lane
// 16 K + j of the 16-lane row], p[16 K + j], y), the multiplier broadcast by
// DPP (lane l of mk holds pivot 16 K + (l & 15)'s multiplier of the row)
template <int J>
__device__ __forceinline__ void fix1(double &y, double mk, double pj)
{
    asm("s_nop 4\n v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(y)
        : "v"(mk), "v"(pj), "n"(J));
}
#define FXF(L, P) "v_fmac_f64_dpp %0, -%1, %" #P " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
template <int K, int NB>
__device__ __forceinline__ void fix16(double &y, double mk, const double (&p)[NB])
{
    asm("s_nop 4\n" FXF(0, 2) FXF(1, 3) FXF(2, 4) FXF(3, 5) FXF(4, 6) FXF(5, 7) FXF(6, 8) FXF(7, 9) FXF(8, 10)
            FXF(9, 11) FXF(10, 12) FXF(11, 13) FXF(12, 14) FXF(13, 15) FXF(14, 16) FXF(15, 17)
        : "+v"(y)
        : "v"(mk), "v"(p[16 * K]), "v"(p[16 * K + 1]), "v"(p[16 * K + 2]), "v"(p[16 * K + 3]),
          "v"(p[16 * K + 4]), "v"(p[16 * K + 5]), "v"(p[16 * K + 6]), "v"(p[16 * K + 7]), "v"(p[16 * K + 8]),
          "v"(p[16 * K + 9]), "v"(p[16 * K + 10]), "v"(p[16 * K + 11]), "v"(p[16 * K + 12]),
          "v"(p[16 * K + 13]), "v"(p[16 * K + 14]), "v"(p[16 * K + 15]));
}
#undef FXF
template <int K, int NB, int J = 0>
__device__ __forceinline__ void fix16_after(double &y, double mk, const double (&p)[NB], int s0)
{
    if constexpr (J < 16) {
        if (16 * K + J > s0) fix1<J>(y, mk, p[16 * K + J]);      // uniform
        fix16_after<K, NB, J + 1>(y, mk, p, s0);
    }
}
template <int NB, int K = 0>
__device__ __forceinline__ void fix_chain_dpp(double &y, const double (&mk)[NB / 16], const double (&p)[NB], int s0)
{
    if constexpr (K < NB / 16) {
        if (16 * K > s0) fix16<K, NB>(y, mk[K], p);            // uniform: every pivot after s0
        else if (16 * K + 15 > s0) fix16_after<K, NB>(y, mk[K], p, s0);
        fix_chain_dpp<NB, K + 1>(y, mk, p, s0);
    }
}
// The group's pivot rows among local rows [ra, rz), on this lane's column
// col: a pivot row s0 holds P[s0] after pivot s0 and takes only the later
// pivots (upd()).  Rewritten after the pass (every store of the pass has
// landed: vmcnt(0) before), two rows per round trip: lane l loads the row's
// multipliers of pivots 16 k + (l & 15), k = 0..3 (MQ), and P[s0] at its
// column; then each row's chain runs from registers with the multiplier
// broadcast by DPP.  (fmod > 0: only the rows of the 8-row batches fsel,
// fsel + fmod, ... from ra -- the tail piece's batches of one wave)
// the next pivot row of the lanes h (the lowest lane's row) and the LAST
// pivot of the group on that row (a row pivoted twice in the group ends as
// the later pivot's row plus the pivots after it: the earlier chain is
// dead); clears every lane of that row from h
__device__ __forceinline__ int next_pivot_row(u64 &h, long long mysr, int &row)
{
    row = __builtin_amdgcn_readlane((int)(unsigned)mysr, __builtin_ctzll(h));
    const u64 same = __ballot((int)(unsigned)mysr == row) & h;
    h &= ~same;
    return 63 - __builtin_clzll(same);
}
// lane l's double, wave-uniform
__device__ __forceinline__ double readlane_f64(double v, int l)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// p[s0] for a wave-uniform s0: a tree of uniform branches (no per-element
// selects)
template <int L, int N, int NB>
__device__ __forceinline__ double pick_p(const double (&p)[NB], int s0)
{
    if constexpr (N == 1) {
        double v = p[L];
        asm volatile("" : "+v"(v));              // opaque: no select-of-loads fold (p to scratch)
        return v;
    } else {
        if (s0 < L + N / 2) return pick_p<L, N / 2, NB>(p, s0);
        return pick_p<L + N / 2, N - N / 2, NB>(p, s0);
    }
}
// LDS moves written in asm (k_sweep_rl: a compiler-visible LDS access makes
// the compiler wait for every LDS-DMA copy in flight first)
__device__ __forceinline__ double lds_ld64(unsigned a)
{
    double v;
    asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return v;
}
__device__ __forceinline__ void lds_st64(unsigned a, double v)
{
    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st32(unsigned a, int v)
{
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}

template <int NB>
__device__ __forceinline__ void fix_rows(const double *__restrict__ P, const double *__restrict__ M,
                                         double *Tout, long long ld, long long col, bool ok,
                                         const double (&p)[NB], long long mysr, long long ra, long long rz,
                                         int fmod = 0, int fsel = 0, u64 only = ~0ull)
{
    static_assert(NB % 16 == 0, "fix_rows: pivots in 16s");
    constexpr int NK = NB / 16;
    const int lane = threadIdx.x & 63;
    u64 h = __ballot(mysr >= ra && mysr < rz && (fmod == 0 || (int)((mysr - ra) >> 3) % fmod == fsel)) & only;
    while (h) {
        int ra32, rb32;
        const int sa = next_pivot_row(h, mysr, ra32);
        const bool two = h != 0;
        const int sb = two ? next_pivot_row(h, mysr, rb32) : sa;
        if (!two) rb32 = ra32;
        const long long ra_ = ra32, rb_ = rb32;
        double ma[NK], mb[NK];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            ma[k] = M[mq(ra_, 16 * k + (lane & 15))];
            mb[k] = M[mq(rb_, 16 * k + (lane & 15))];
        }
        double ya = P[(long long)sa * ld + col], yb = P[(long long)sb * ld + col];
        fix_chain_dpp<NB>(ya, ma, p, sa);
        if (ok) Tout[ra_ * ld + col] = ya;
        if (two) {
            fix_chain_dpp<NB>(yb, mb, p, sb);
            if (ok) Tout[rb_ * ld + col] = yb;
        }
    }
}

#ifndef SWEEP_LA
#define SWEEP_LA 0
#endif
#ifndef SWEEP_LA_T
#define SWEEP_LA_T SWEEP_LA    // (A/B) the tableau rows' load policy alone
#endif
#ifndef SWEEP_LA_OOP
#define SWEEP_LA_OOP 2         // ... out of place (SA & 2: a tableau far beyond the Infinity Cache,
#endif                         // its stores non-temporal): the row loads non-temporal too
#ifndef SWEEP_UBASE
#define SWEEP_UBASE 1          // k_sweep_rl, 4 waves: whole batches' row loads from a wave-uniform base
#endif                         // (1: buffer loads, 2: global loads, 0: per-lane clamped addresses)
#ifndef SWEEP_RGQ
#define SWEEP_RGQ 1            // k_sweep_rl, 4 waves: the FMAs in blocks of four pivot pairs (one DPP hazard
#endif                         // wait each; cfg3 sweep 106.7-107.9 -> 104.1-104.6 us; 8 waves: no gain seen)
#ifndef SWEEP_LDSPIPE
#define SWEEP_LDSPIPE 1        // k_sweep_rl: a batch's LDS reads pipelined with its FMAs (sweep_pairs)
#endif
template <int W, int NB, int D, int SA>
__global__ void __launch_bounds__(64 * W)
k_sweep_rl(const double *T, double *Tout, const double *__restrict__ P, const double *__restrict__ M,
           const long long *__restrict__ dR, const Ctl *__restrict__ ctl, long long ld, long long rows, int grp,
           int nstrips, long long run, long long tail, long long tcol, long long tend, int nexp,
           unsigned *dflips, unsigned flipseq, unsigned long long *clk, unsigned lseq, long long runb, int na)
{
    // tail > 0: the grid covers strips [0, nstrips) of the columns and the 64
    // columns from tcol (the tableau's last columns: n + 1 is rarely a
    // multiple of 64 W; the pitch's padding columns are 0 and stay 0, never
    // swept; tend: one past the last column) are dealt out `tail` rows to
    // every block -- a strip of its own would give those few columns a whole
    // block per row run (cfg4: 30 of 510 resident slots)
    constexpr int RW = 8;                        // rows per batch
    constexpr int NC = NB / 2;                   // multiplier registers (2 pivots x 8 rows each)
    constexpr int XS = W * RW * 64;              // doubles of a slot's rows (W waves x 8 rows x 64 columns)
    // the tableau rows' load policy: out of place (cfg4: 2.2 GB, far beyond
    // the Infinity Cache) non-temporal like the stores -- sweep 789-806 ->
    // 773-785 us, the next selection 6.53-6.55 -> 6.48-6.50 us per pivot;
    // in place (cfg3) the default, which keeps the tableau in the cache for
    // the selection (non-temporal there: 102.4-102.6 -> 104.9-106.7 us)
    constexpr int LAT = (SA & 2) ? SWEEP_LA_OOP : SWEEP_LA_T;
    // a slot's multipliers: two MQ quads, the second QP doubles further on.
    // The multiplier registers of 16 lanes read rows 0-3 of quad 0 and rows
    // 4-7 of quad 1 at the same offsets: 2 KB apart they share LDS banks (a
    // 2-way conflict on every read, SQ_LDS_BANK_CONFLICT 43 % of the LDS
    // cycles at cfg3); 16 doubles further on they do not.
#ifndef SWEEP_QP
#define SWEEP_QP 16
#endif
    constexpr int QP = (D * (XS + 2 * 4 * BMAX + SWEEP_QP) * 8 + 8 * NB <= 80 * 1024 || W > 4) ? SWEEP_QP : 0;
    constexpr int MS = 2 * 4 * BMAX + QP;        // doubles of a slot's multipliers
    static_assert(NB % 2 == 0 && NB <= BMAX && D >= 2 && W >= 4, "k_sweep_rl");
    __shared__ __attribute__((aligned(16))) double xs[D][XS];
    __shared__ __attribute__((aligned(16))) double ms[D][MS];
    __shared__ long long sr[NB];
    // the group's pivot rows met in the pass: their multipliers (pivot l at
    // [f][l]) copied out of the batch's slot, and (local row << 8 | last
    // pivot on it), for the fix-up after the pass -- NF rows: 64 where the
    // LDS allows (4-wave, 2 deep: 2 workgroups per CU still fit), else 16
    // (the rest re-read from memory)
    constexpr int LDS_BASE = D * (XS + MS) * 8 + NB * 8;
    constexpr int NF = (W <= 4 && LDS_BASE + 64 * (NB * 8 + 4) <= 80 * 1024) ? 64 : 16;
    __shared__ __attribute__((aligned(16))) double fixm[NF][NB];
    __shared__ int fmeta[NF];
    const int nd = (int)ctl->ndef[grp];
    if (nd == 0 || ctl->bar_timeout) return;     // nothing deferred / group redone by the host
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // out of place (Tout != T): this sweep ran -- the host's record of which
    // buffer holds the tableau (every block takes the same branch above)
    if (dflips && blockIdx.x == 0 && threadIdx.x == 0) *dflips = flipseq;
    // block 0's clocks over its pass (Args::sweep_clk): the shader clock of
    // the launch = cycles / 100 MHz ticks (every block is resident from the
    // start and the runs finish together, so block 0 spans the launch)
    const unsigned long long clk_c0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x < NB) sr[threadIdx.x] = (int)threadIdx.x < nd ? dR[threadIdx.x] : -2;
    auto srow = [&](int s) -> long long { return sr[s]; };
    const int strip = (int)(blockIdx.x % (unsigned)nstrips);
    // row run ri of the strip: runs 0 .. na - 1 of `run` rows, the rest of
    // runb (two workgroups per CU: the grid's first half, dispatched first,
    // takes the longer runs -- see launch_sweep)
    const long long ri = (long long)(blockIdx.x / (unsigned)nstrips);
    const long long r0 = ri < na ? ri * run : (long long)na * run + (ri - na) * runb;
    const long long r1 = min(rows, r0 + (ri < na ? run : runb));
    // this lane's column.  Lanes past the pitch (the last strip of a pitch
    // that is not a multiple of 64 W: whole waves) load from column ld - 2 /
    // ld - 1 and their stores are dropped (below), so every wave issues the
    // same instructions (the waits count them)
    const long long colw = (long long)strip * 64 * W + 64 * wave;
    const long long col = min(colw + (lane & ~1), ld - 2) + (lane & 1);
    const bool cok = colw + lane < ld;
    // the tail piece of this block: rows [t0, t1), column tc of each lane
    const long long t0 = (long long)blockIdx.x * tail, t1 = tail > 0 ? min(rows, t0 + tail) : 0;
    const long long tc = min(tcol + lane, ld - 1);
    const bool tok = tcol + lane < ld;
    if (nd != nexp) {
        // a group that stopped early (the solve ended inside it: once per
        // call) -- pivot by pivot from memory.  A group the host knows to be
        // short of NB (nexp < NB: a call's last, a depth of 49..63) runs the
        // full pass: the host zeroed its pivot rows and multipliers past nexp
        // (launch_sweep), so those pivots are exact no-ops, fma(-0, 0, x) == x
        __syncthreads();
        auto one = [&](long long row, long long c, bool ok) {
            double x = T[row * ld + c];
            for (int s = 0; s < nd; ++s) {
                if (srow(s) == row) x = P[(long long)s * ld + c];      // the pivot row becomes P[s]
                else x = fma(-M[mq(row, s)], P[(long long)s * ld + c], x);
            }
            if (ok) Tout[row * ld + c] = x;
        };
        for (long long row = r0; row < r1; ++row) one(row, col, cok);
        for (long long row = t0 + wave; row < t1; row += W) one(row, tc, tok);
        return;
    }
    double p[NB];
#pragma unroll
    for (int s = 0; s < NB; ++s) p[s] = P[(long long)s * ld + col];
    const long long nbat = (r1 - r0 + RW - 1) / RW;
    const long long nquad = (rows + 3) >> 2;
    // copies of batch i into slot i % D: lane l of a wave brings 16 bytes --
    // rows: row 2 q + (l >> 5) of the wave's 8, columns 2 (l & 31) .. +1 of
    // its 64, for q = 0..3 (4 instructions); multipliers: quad (wave >> 1) of
    // the batch, bytes 1 KB x (wave & 1) + 16 l of it (one instruction)
    // (a whole batch: the batch's first row as a wave-uniform base and each
    // lane's byte offset from it, fixed for the pass -- the per-lane 64-bit
    // row x pitch products of the clamped form were ~30 VALU instructions per
    // batch, a dozen of them quarter-rate multiplies, beside 512 FMAs)
    unsigned loff[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        loff[q] = (unsigned)(((2 * q + (lane >> 5)) * ld + min(colw + 2 * (lane & 31), ld - 2)) * 8);
    auto issue = [&](long long i, int slot) {
        const long long rb = r0 + i * RW;
        const long long last = r1 - 1;
        constexpr int UB = SWEEP_UBASE;
        if (UB == 1 && rb + RW - 1 <= last) {
            // buffer loads into LDS: the batch's row as the resource base
            // (scalar), the lane's offset a 32-bit VGPR
            const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<double *>(T + rb * ld), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rt, (__attribute__((address_space(3))) void *)&xs[slot][(wave * RW + 2 * q) * 64], 16,
                    (int)loff[q], 0, 0, LAT);
        } else if (UB == 2 && rb + RW - 1 <= last) {
            const char *tb = reinterpret_cast<const char *>(T + rb * ld);   // wave-uniform
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const double *>(tb + loff[q]),
                                                 (__attribute__((address_space(3))) void *)&xs[slot][(wave * RW + 2 * q) * 64],
                                                 16, 0, LAT);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const long long row = min(rb + 2 * q + (lane >> 5), last);
                const long long cc = min(colw + 2 * (lane & 31), ld - 2);
                __builtin_amdgcn_global_load_lds(T + row * ld + cc,
                                                 (__attribute__((address_space(3))) void *)&xs[slot][(wave * RW + 2 * q) * 64],
                                                 16, 0, LAT);
            }
        }
        // (W >= 4: quads 0, 1 x halves 0, 1 by waves 0..3; more waves re-copy)
        const int w4 = wave & 3;
        const long long qd = min((rb >> 2) + (w4 >> 1), nquad - 1);
        __builtin_amdgcn_global_load_lds(M + qd * (4 * BMAX) + (w4 & 1) * 128 + 2 * lane,
                                         (__attribute__((address_space(3))) void *)&ms[slot][(w4 >> 1) * (4 * BMAX + QP) + (w4 & 1) * 128],
                                         16, 0, SWEEP_LA);
    };
    // vector-memory instructions a wave issues per batch after the copies of
    // batch i: the copies of the next batches (5 each) and the stores (8 each)
    constexpr int PER = 5 + RW;
    __syncthreads();                             // sr staged
    // lane s: pivot s's local row (-2: none / another rank's).  From LDS,
    // before the first copies: a VGPR loaded from global memory and read in
    // the pass made the compiler wait vmcnt(0) at the pass's barrier
    const long long mysr = lane < NB ? sr[lane] : -2;
    const u64 runpiv = __ballot(mysr >= r0 && mysr < r1);     // the run holds a pivot row
#pragma unroll 1
    for (int i = 0; i < D - 1; ++i) issue(i, i);
    // P's registers read here, after the first copies: the compiler's wait
    // for their loads (vmcnt of the copies issued since) lands before the
    // pass, not at a barrier inside it (a vmcnt(0) every batch otherwise)
#pragma unroll
    for (int s = 0; s < NB; ++s) asm volatile("" ::"v"(p[s]));
    int slot = 0;                                // batch i's slot, i % D
    const int vh = (lane & 15) >> 3, vk = lane & 7;
    int nf = 0;                                  // pivot rows captured (wave-uniform)
    u64 ovf = 0;                                 // pivot lanes past NF captured rows
    // batch j's copies are the oldest outstanding but for the D - 2 later
    // batches' copies and stores issued since (the copies of the last
    // batches are issued anyway, re-reading the last one)
    // (the first D - 1 batches: fewer issued since -- the prologue's
    // copies have no stores between them)
    auto wait_copies = [&](long long j) {
        static_assert(D <= 4, "k_sweep_rl: waits written for D <= 4");
        if (j >= D - 1) {
            if constexpr (D == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if constexpr (D == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + PER) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + 2 * PER) : "memory");
        } else if (j == 0) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * 5) : "memory");
        } else if (j == 1) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D == 3 ? PER : 5 + PER) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");   // D == 4, j == 2
        }
    };
#pragma unroll 1
    for (long long i = 0; i < nbat; ++i) {
        wait_copies(i);
        __syncthreads();                         // every wave's copies of batch i are in LDS
        issue(min(i + D - 1, nbat - 1), slot == 0 ? D - 1 : slot - 1);   // the slot batch i - 1 used
        const long long rb = r0 + i * RW;
        const int kmax = (int)min((long long)RW - 1, r1 - 1 - rb);
        double x[RW], m[NC];
        // multiplier of pivot 2c + h, batch row k (past kmax: row kmax's)
        const int kr = min(vk, kmax);
        if (SWEEP_LDSPIPE && kmax == RW - 1) {
            // the batch's LDS reads pipelined with its FMAs: the rows and the
            // first 8 multiplier registers, then pair c's FMAs issue as soon
            // as m[c] has landed while m[c + 8]'s read is in flight (all 40
            // reads up front behind one lgkmcnt(0): the SIMD's two waves idled
            // through every batch's LDS round trip, the 8 waves of a CU
            // contending for the LDS right after the barrier)
            const unsigned xa = lds_off(&xs[slot][wave * RW * 64 + lane]);
            const unsigned ma = lds_off(&ms[slot][(kr >> 2) * (4 * BMAX + QP) + (kr & 3) + vh * 4]);
            lds_rows<RW>(x, xa);
            lds_mult_first<SWEEP_AHEAD, NC>(m, ma);
            // (x's reads are older than the multipliers': the first pair's
            // wait covers them)
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                         "+v"(x[7]));
            sweep_pairs<NC, (SWEEP_RGQ && NC % 4 == 0) ? 4 : 1>(x, m, p, ma);
        } else if (kmax == RW - 1) {
            // the LDS reads in asm: a compiler-visible read of LDS the copies
            // write made it wait for every copy in flight (vmcnt(0)) first;
            // the wait above already covers this batch's
            const unsigned xa = lds_off(&xs[slot][wave * RW * 64 + lane]);
            const unsigned ma = lds_off(&ms[slot][(kr >> 2) * (4 * BMAX + QP) + (kr & 3) + vh * 4]);
            lds_rows<RW>(x, xa);
            lds_mult<NC>(m, ma);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // the loaded registers as outputs of asm ordered after the wait:
            // nothing that reads them (FMAs, the padding select) moves above it
#pragma unroll
            for (int k = 0; k < RW; ++k) asm volatile("" : "+v"(x[k]));
#pragma unroll
            for (int c = 0; c < NC; ++c) asm volatile("" : "+v"(m[c]));
        } else {
#pragma unroll
            for (int k = 0; k < RW; ++k) x[k] = xs[slot][(wave * RW + min(k, kmax)) * 64 + lane];
            const double *mrow = &ms[slot][(kr >> 2) * (4 * BMAX + QP) + (kr & 3)];
#pragma unroll
            for (int c = 0; c < NC; ++c) m[c] = mrow[(2 * c + vh) * 4];
        }
        if (SWEEP_LDSPIPE && kmax == RW - 1) {
            // (the FMAs ran with the reads above)
        } else if constexpr (SWEEP_RGQ && NC % 4 == 0) {
#pragma unroll
            for (int c = 0; c < NC; c += 4) rg_quad(x, m[c], m[c + 1], m[c + 2], m[c + 3], &p[2 * c]);
        } else {
#pragma unroll
            for (int c = 0; c < NC; ++c) rg_pair(x, m[c], p[2 * c], p[2 * c + 1]);
        }
        // a pivot row s0 of the group in this batch (about one batch in eight
        // at cfg3): it holds P[s0] after pivot s0 and takes only the later
        // pivots -- recomputed here from P (registers) and its multipliers
        // (this batch's LDS slot), not re-read from memory after the pass
        // the group's pivot rows in this batch (about one batch in five at
        // cfg3, one in sixty at cfg4): their multipliers, in this slot until
        // the next iteration's copies, set aside in fixm -- one wave per row,
        // lane l pivot l's -- so the fix-up after the pass needs no memory
        // round trip
        for (u64 hit = runpiv ? __ballot(mysr >= rb && mysr <= rb + kmax) : 0; hit;) {
            int row;
            const int sl = next_pivot_row(hit, mysr, row);
            if (nf < NF) {
                if (wave == nf % W) {
                    const int k = row - (int)rb;
                    const double v = lds_ld64(lds_off(&ms[slot][(k >> 2) * (4 * BMAX + QP) + (k & 3) + 4 * lane]));
                    lds_st64(lds_off(&fixm[nf][lane]), v);
                    if (lane == 0) lds_st32(lds_off(&fmeta[nf]), ((row - (int)r0) << 8) | sl);
                }
                ++nf;
            } else {
                ovf |= __ballot((int)(unsigned)mysr == row);
            }
        }
        {
            // write-through stores (SA), as the DPP sweeps'.  A wave whose 64
            // columns lie past the pitch (ld is a multiple of 64, so a wave is
            // wholly inside or wholly past it) stores through a resource of 0
            // records: the hardware drops every one of its stores, and the
            // wave still issues them (its vmcnt waits count them)
            const bool wok = __builtin_amdgcn_readfirstlane((int)cok) != 0;
            const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
                Tout + rb * ld + colw, (short)0, wok ? 0x7fffffff : 0, 0x00020000);
            const int voff = lane * 8, ldb = (int)(ld * 8);
#pragma unroll
            for (int k = 0; k < RW; ++k)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, x[k]), ro, voff, min(k, kmax) * ldb, SA);
        }
        slot = slot + 1 == D ? 0 : slot + 1;
    }
    // the group's pivot rows in this run, rewritten from registers and LDS
    // (pivot row s0: P[s0], then the pivots after s0 -- upd()): every store
    // of the pass has landed and every wave's fixm copies are in
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    constexpr int NK = NB / 16;
    for (int f = 0; f < nf; ++f) {
        int meta;
        double mk[NK];
        // plain LDS reads (the pass's copies have all landed: vmcnt(0)
        // above): the row's meta word and its 4 multiplier registers in one
        // round trip, not five
        meta = __builtin_amdgcn_readfirstlane(fmeta[f]);
#pragma unroll
        for (int k = 0; k < NK; ++k) mk[k] = fixm[f][16 * k + (lane & 15)];
        const int s0 = meta & 255;
        double y = pick_p<0, NB, NB>(p, s0);
        fix_chain_dpp<NB>(y, mk, p, s0);
        if (cok) Tout[(r0 + (meta >> 8)) * ld + col] = y;
    }
    if (ovf) fix_rows<NB>(P, M, Tout, ld, col, cok, p, mysr, r0, r1, 0, 0, ovf);
    if (clk && threadIdx.x == 0) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
        if (blockIdx.x == 0) {
            unsigned long long *e = clk + (lseq % SWEEP_CLK_RING) * 4;
            e[1] = c1 - clk_c0;
            e[2] = rt1 - clk_r0;
            e[3] = clk_r0;
            e[0] = lseq;
        }
        if (blockIdx.x < SWEEP_BLK_MAX) {         // every block's pass, the latest launch
            unsigned long long *e = clk + SWEEP_CLK_RING * 4 + blockIdx.x * 4;
            e[0] = lseq;
            e[1] = clk_r0;
            e[2] = rt1;
            e[3] = c1 - clk_c0;
        }
    }
    if (t0 >= t1) return;                        // block-uniform: no tail piece
    // (rows across lanes only where the block's W waves cover its tail in
    // one pass; a longer tail -- tall tableaux on few blocks -- takes the
    // columns-across-lanes loop below, ADVICE r4.  A loop here instead cost
    // the whole kernel scalar registers: cfg3 108 -> 110 us.)
    if (tend - tcol <= 4 && t1 - t0 <= 64LL * W) {
        // ---- the tail piece of a few columns [tcol, tend) (cfg3, cfg4: one),
        //      rows across lanes: lane l of wave w takes row t0 + 64 w + l,
        //      its 64 multipliers and P[s] at the column (a per-pivot scalar,
        //      broadcast by readlane) -- one memory round trip, then upd()'s
        //      chain in pivot order with the pivot rows' P[s] taken in it
        //      (the chain of one(); no fix-up after).  (Columns across lanes,
        //      below: 1 useful lane in 64 and a round trip per 8 rows, plus
        //      the pivot rows' -- 10 us of the cfg4 launch)
        if (64 * wave < t1 - t0) {               // wave-uniform
            const long long rw = t0 + 64 * wave + lane;
            const bool rok = rw < t1;
            const long long rr = rok ? rw : t1 - 1;
            const int rri = (int)rr;
            double m[NB];
#pragma unroll
            for (int s = 0; s < NB; ++s) m[s] = M[mq(rr, s)];
            // (no pivot row of the group among the tail's rows -- nearly
            // always -- the chain without the per-pivot row check)
            const bool tpiv = __ballot(mysr >= t0 && mysr < t1) != 0;
            for (long long c = tcol; c < tend; ++c) {
                double x = T[rr * ld + c];
                const double pv = lane < NB ? P[(long long)lane * ld + c] : 0.0;
                if (tpiv) {
#pragma unroll
                    for (int s = 0; s < NB; ++s) {
                        const double ps = readlane_f64(pv, s);
                        x = rri == __builtin_amdgcn_readlane((int)(unsigned)mysr, s) ? ps : fma(-m[s], ps, x);
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < NB; ++s) x = fma(-m[s], readlane_f64(pv, s), x);
                }
                if (rok) Tout[rr * ld + c] = x;
            }
        }
        return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ---- the tail piece: the 64 columns from tcol (one per lane) of rows
    //      [t0, t1), wave w on batches t0 + 8 w, t0 + 8 (w + W), ...: the same
    //      register FMAs with every operand loaded from memory (a few batches
    //      per block)
#pragma unroll
    for (int s = 0; s < NB; ++s) p[s] = P[(long long)s * ld + tc];
    for (long long rb = t0 + RW * wave; rb < t1; rb += RW * W) {
        const int kmax = (int)min((long long)RW - 1, t1 - 1 - rb);
        const int kr = min(vk, kmax);
        double x[RW], m[NC];
#pragma unroll
        for (int k = 0; k < RW; ++k) x[k] = T[(rb + min(k, kmax)) * ld + tc];
#pragma unroll
        for (int c = 0; c < NC; ++c) m[c] = M[mq(rb + kr, 2 * c + vh)];
#pragma unroll
        for (int c = 0; c < NC; ++c) rg_pair(x, m[c], p[2 * c], p[2 * c + 1]);
        if (tok) {
#pragma unroll
            for (int k = 0; k < RW; ++k) Tout[(rb + min(k, kmax)) * ld + tc] = x[k];
        }
    }
    // the tail's pivot rows, by the wave that stored them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    static_assert(RW == 8, "fix_rows: 8-row batches");
    fix_rows<NB>(P, M, Tout, ld, tc, tok, p, mysr, t0, t1, W, wave);
}

// peer exchange check (row-sharded setup): lane p writes this rank's granule
// into rank p's summary slot, then every lane waits for rank p's granule in
// the local buffer (bounded)
// (every rank also sends its flag bits; *ok = 1 | OR of the ranks' flags << 1
// when all arrived, 0 otherwise)
__global__ void k_peer_ping(Args A, unsigned tag, unsigned flags, int *ok)
{
    const int N = A.nranks, p = threadIdx.x;
    if (p < N) st_sys(&(*gp(A.peer + p))[A.rank * 8], ((u64)tag << 32) | (flags << 8) | (unsigned)A.rank);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool got = p >= N;
    unsigned f = 0;
    while (!got) {
        const u64 v = ld_sys(&A.xbuf[p * 8]);
        got = (unsigned)(v >> 32) == tag && ((unsigned)v & 0xffu) == (unsigned)p;
        f = ((unsigned)v >> 8) & 0xffffu;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;   // 2 s
        __builtin_amdgcn_s_sleep(2);
    }
    const bool all = __all(got);
    // OR of the flags over the lanes (ranks)
    for (int o = 32; o >= 1; o >>= 1) f |= (unsigned)__shfl_xor((int)f, o);
    if (threadIdx.x == 0) *ok = all ? (int)(1u | (f << 1)) : 0;
}

// ---------------------------------------------------------------------------
// Column scans (findPivotMaxIncrease / findPivotAll, simplex.py:286-360) and
// form checks (tableau.py:466-521): per column of the local constraint rows,
// one pass over the (current) tableau.  Block = 64 columns x 4 waves of rows,
// rows read coalesced across the lanes.
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256) k_colstat(Args A, ColStat *out)
{
    __shared__ ColStat part[4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long j = (long long)blockIdx.x * 64 + lane;
    ColStat c;
    c.gmin = INFINITY;
    c.npos = c.npos0 = c.nnz = c.none = c.nneg = 0;
    c.one_row = NONE;
    c.pad = 0;
    if (j < A.ld)
        for (long long li = 1 + wave; li < A.rows; li += 4) {
            const double x = A.T[li * A.ld + j];
            bool ok;
            const double q = row_ratio(x, A.T[li * A.ld], A.tol, ok);
            if (ok) {
                c.npos += 1;
                c.gmin = fmin(c.gmin, q);
            }
            c.npos0 += x > 0.0;
            c.nnz += x != 0.0;
            c.nneg += x < 0.0;
            if (x == 1.0) {
                c.none += 1;
                if (c.one_row == NONE) c.one_row = li - 1 + A.rb;
            }
        }
    part[wave][lane] = c;
    __syncthreads();
    if (wave == 0 && j < A.ld) {
        for (int w = 1; w < 4; ++w) {
            const ColStat &d = part[w][lane];
            c.gmin = fmin(c.gmin, d.gmin);
            c.npos += d.npos;
            c.npos0 += d.npos0;
            c.nnz += d.nnz;
            c.nneg += d.nneg;
            c.none += d.none;
            c.one_row = d.one_row < c.one_row ? d.one_row : c.one_row;
        }
        out[j] = c;
    }
}

// rows inside each column's ratio band (thr[j] = INFINITY: none), in row
// order: first[j] = the first (global index), count[j]; with pairs != nullptr
// the (row, variable) pairs of column j go to pairs[2 * (offs[j] + k)]
__global__ void __launch_bounds__(64) k_colband(Args A, const double *thr, long long *first,
                                               long long *count, const long long *offs,
                                               long long *pairs)
{
    const long long j = (long long)blockIdx.x * 64 + threadIdx.x;
    if (j >= A.ld) return;
    const double th = thr[j];
    long long f = NONE, k = 0;
    if (th < INFINITY)
        for (long long li = 1; li < A.rows; ++li) {
            bool ok;
            const double q = row_ratio(A.T[li * A.ld + j], A.T[li * A.ld], A.tol, ok);
            if (ok && q <= th) {
                const long long rg = li - 1 + A.rb;
                if (f == NONE) f = rg;
                if (pairs) {
                    pairs[2 * (offs[j] + k)] = rg;
                    pairs[2 * (offs[j] + k) + 1] = j - 1;
                }
                ++k;
            }
        }
    first[j] = f;
    count[j] = k;
}

// per local constraint row: b_i > 0 and every a_ij <= 0 (isInfeasible,
// tableau.py:510-514)
__global__ void __launch_bounds__(256) k_rowpos(Args A, int *rowpos)
{
    __shared__ int any;
    const long long li = 1 + blockIdx.x;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    int mine = 0;
    for (long long j = 1 + threadIdx.x; j <= A.n; j += blockDim.x)
        mine |= A.T[li * A.ld + j] > 0.0;
    if (mine) any = 1;
    __syncthreads();
    if (threadIdx.x == 0) rowpos[li - 1] = (A.T[li * A.ld] > 0.0 && !any) ? 1 : 0;
}

hipError_t launch_colstat(hipStream_t s, const Args &A, ColStat *out)
{
    hipLaunchKernelGGL(k_colstat, dim3((unsigned)((A.ld + 63) / 64)), dim3(256), 0, s, A, out);
    return hipGetLastError();
}

hipError_t launch_colband(hipStream_t s, const Args &A, const double *thr, long long *first,
                          long long *count, const long long *offs, long long *pairs)
{
    hipLaunchKernelGGL(k_colband, dim3((unsigned)((A.ld + 63) / 64)), dim3(64), 0, s, A, thr, first,
                       count, offs, pairs);
    return hipGetLastError();
}

hipError_t launch_rowpos(hipStream_t s, const Args &A, int *rowpos)
{
    if (A.rc < 1) return hipSuccess;
    hipLaunchKernelGGL(k_rowpos, dim3((unsigned)A.rc), dim3(256), 0, s, A, rowpos);
    return hipGetLastError();
}

__global__ void k_resume(Ctl *ctl)
{
    ctl->status = LP_PIVOTED;
    ctl->ndef[0] = 0;
    ctl->ndef[1] = 0;
}

// in-process shard group: allreduce-min of one double across n device buffers
__global__ void k_group_min(double *const *ptrs, int n)
{
    double g = INFINITY;
    for (int k = 0; k < n; ++k) g = fmin(g, *ptrs[k]);
    for (int k = 0; k < n; ++k) *ptrs[k] = g;
}

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------


// compile-time bound of the deferred-pivot count: 0, 1, 2, 4, 8, 16, 32
static int bound_of(int t)
{
    return t <= 0 ? 0 : t <= 1 ? 1 : t <= 2 ? 2 : t <= 4 ? 4 : t <= 8 ? 8 : t <= 16 ? 16 : t <= 32 ? 32 : 64;
}

#define TP_DISPATCH(t, KERNEL, ...)                                                           \
    switch (bound_of(t)) {                                                                     \
    case 0: hipLaunchKernelGGL(KERNEL<0>, __VA_ARGS__); break;                                 \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                                 \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                                 \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                                 \
    case 8: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;                                 \
    case 16: hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__); break;                               \
    case 32: hipLaunchKernelGGL(KERNEL<32>, __VA_ARGS__); break;                               \
    default: hipLaunchKernelGGL(KERNEL<64>, __VA_ARGS__); break;                               \
    }

hipError_t launch_reset(hipStream_t s, const Args &A, int mode, int rule, int chain, long long cap,
                        long long r, long long c)
{
    hipLaunchKernelGGL(k_reset, dim3(1), dim3(1), 0, s, A, mode, rule, chain, cap, r, c);
    return hipGetLastError();
}

hipError_t launch_load_eager(hipStream_t s, const Args &A)
{
    const long long w = A.ld > A.rows ? A.ld : A.rows;
    const long long g = (w + 255) / 256;
    hipLaunchKernelGGL(k_load_eager, dim3((unsigned)(g < 1024 ? g : 1024)), dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_enter(hipStream_t s, const Args &A)
{
    hipLaunchKernelGGL(k_enter, dim3(1), dim3(ENTER_THREADS), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_ratio(hipStream_t s, const Args &A, int t, int grp, int mode, int from_erec,
                        long long check_local_row)
{
    const int g = ratio_blocks(A.rows);
    if (g <= 0 || t < 0 || t >= BMAX) return hipErrorInvalidValue;
    TP_DISPATCH(t, k_ratio, dim3(g), dim3(RATIO_THREADS), 0, s, A, t, grp, mode, from_erec,
                check_local_row)
    return hipGetLastError();
}

hipError_t launch_pick(hipStream_t s, const Args &A, int t, int mode)
{
    if (t < 0 || t >= BMAX) return hipErrorInvalidValue;
    TP_DISPATCH(t, k_pick, dim3(prow_blocks(A.ld)), dim3(256), 0, s, A, t, mode)
    return hipGetLastError();
}

hipError_t launch_gather(hipStream_t s, const Args &A, int t)
{
    const long long g = (A.rows + 255) / 256;
    hipLaunchKernelGGL(k_gather, dim3((unsigned)(g < 1024 ? g : 1024)), dim3(256), 0, s, A, t);
    return hipGetLastError();
}

hipError_t launch_prow(hipStream_t s, const Args &A, int t, int grp, int rsrc, int peek)
{
    if (t < 0 || t >= BMAX) return hipErrorInvalidValue;
    TP_DISPATCH(t, k_prow, dim3(prow_blocks(A.ld)), dim3(PROW_THREADS), 0, s, A, t, grp, rsrc,
                peek)
    return hipGetLastError();
}

// compute units of the current device (cached per process)
static int sweep_cus()
{
    static int ncu = 0;
    if (ncu == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            ncu = n;
        else
            ncu = 256;
    }
    return ncu;
}

// resident sweep workgroups per CU: the runtime's occupancy answer for the
// compiled kernel (cached per kernel)
// the CUs a sweep grid is sized for: all of them (tests: LPGPU_SWEEP_CUS
// sizes it for fewer -- longer row runs and tail pieces per block than any
// real device gives at test sizes)
static int sweep_grid_cus()
{
    static int ncu = 0;
    if (ncu == 0) {
        ncu = sweep_cus();
        if (const char *v = std::getenv("LPGPU_SWEEP_CUS"))
            if (std::atoi(v) > 0) ncu = std::min(ncu, std::atoi(v));
    }
    return ncu;
}
static int sweep_blocks_per_cu(const void *fn, int threads)
{
    static std::mutex mu;
    static std::map<const void *, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(fn);
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, threads, 0) != hipSuccess || n < 1) {
        (void)hipGetLastError();
        n = 1;
    }
    cache[fn] = n;
    return n;
}

// The sweep launch: k_sweep_rl for groups of 49..64 pivots (the automatic
// depth of cfg3 and cfg4 is 64, so it is the bench's kernel), k_sweep_dp2 for
// up to 48 (and every tableau narrower than two 64-column strips).  Stores are
// write-through (sc1): the tableau lines leave the L2 as they are written
// instead of in the writeback at the kernel's end (profiles/r01/README.md).
hipError_t launch_sweep(hipStream_t s, const Args &A, int grp, int nd_max, int cnt, hipEvent_t e0, hipEvent_t e1,
                        bool *flipped)
{
    if (flipped) *flipped = false;
    // the kernel's depth: the group's known pivot count when the host knows it
    // (a call's last group, explicit pivots), else the handle's depth
    if (cnt > 0 && cnt < nd_max) nd_max = cnt;
    constexpr int RW = 4, SA = 16;
    // (tests: LPGPU_SWEEP_TAIL=0 -- the last partial strip as a strip of its
    // own instead of dealt out to every block; 2 -- k_sweep_dp2's tail at any
    // run length)
    static const int tail_env = [] {
        const char *v = std::getenv("LPGPU_SWEEP_TAIL");
        return v ? std::atoi(v) : 1;
    }();
    const int nb = nd_max <= 16 ? 16 : nd_max <= 32 ? 32 : nd_max <= 48 ? 48 : 64;
    if (nb == 64 && A.ld % 64 == 0 && A.ld >= 128) {
        // k_sweep_rl: strips of 64 W columns, pivot rows in registers, rows
        // and multipliers streamed into LDS; W = 4 waves, two batches in
        // flight, two workgroups per CU, row runs split by workgroup age
        // (below).  (Until late in round 6 runs of 16384+ rows -- cfg4 --
        // took one 8-wave, 4-deep workgroup per CU; with the split the 4-wave
        // pass is faster there too: cfg4 785-817 -> 759-779 us per launch on
        // two boxes, the 16384-row rank equal, profiles/r06/ab_r06_sweep_w4.txt).
        // Ranks sharing one GPU (tests and rehearsals: A.share > 1) with
        // 16384+ rows keep the 8-wave pass, one workgroup per CU: each rank's
        // XCD-shard selection is persistent and holds a wave on the CUs'
        // SIMDs while the other rank still sweeps, and the 4-wave pass's
        // 512 workgroups could then not all be placed (a co-located 2-GPU
        // rank pair timed out, tests/test_gpu_r4_procs.py)
        const bool w8 = A.share > 1 && A.rows >= 16384;
        const int WL = w8 ? 8 : 4;
        // out of place into the handle's other buffer when it has one (the
        // host then takes Tout as the tableau; see Args::dflips), with
        // non-temporal loads and stores (SA | 2): a tableau that large is far
        // beyond the Infinity Cache, and the pass then does not evict what the
        // selection keeps there -- cfg4 sweep 787-806 -> 775-781 us, selection
        // 7.12-7.15 -> 6.84-6.93 us per pivot (same box); at cfg3 (in place)
        // they cost the selection its cached tableau (4.50 -> 4.65 us)
        double *To = (A.Tout && A.Tout != A.T) ? A.Tout : A.T;
        const bool oop = To != A.T;
        const void *fn = w8 ? (oop ? (const void *)&k_sweep_rl<8, 64, 4, SA | 2> : (const void *)&k_sweep_rl<8, 64, 4, SA>)
                            : (oop ? (const void *)&k_sweep_rl<4, 64, 2, SA | 2> : (const void *)&k_sweep_rl<4, 64, 2, SA>);
        // a group of nexp = 49..63 pivots: the pivot rows and multipliers
        // past it zeroed (stale rows of an earlier group otherwise; rows of
        // P and entries of MQ that no selection of this group writes), so
        // the pass treats them as exact no-ops
        int nexp = nd_max < nb ? nd_max : nb;
        if (nexp < nb) {
            hipError_t e = hipMemsetAsync(A.P + (long long)nexp * A.ld, 0, (size_t)(nb - nexp) * A.ld * 8, s);
            if (e == hipSuccess)
                e = hipMemset2DAsync(A.MQ + nexp * 4, 4 * BMAX * 8, 0, (size_t)(nb - nexp) * 4 * 8,
                                     (size_t)((A.rows + 3) / 4), s);
            if (e != hipSuccess) return e;
        }
        const int bpc = sweep_blocks_per_cu(fn, 64 * WL);
        // the columns swept: 0..n (the padding past them is 0 and stays 0).
        // Whole strips of 64 WL columns; a last partial strip of <= 64
        // columns is dealt out to every block (tail)
        const long long ncol = A.n + 1, nfull = ncol / (64 * WL), rest = ncol - nfull * 64 * WL;
        const bool spread = tail_env != 0 && nfull >= 1 && rest > 0 && rest <= 64;
        const long long nsg = spread ? nfull : (ncol + 64 * WL - 1) / (64 * WL);
        const long long slots = (long long)sweep_grid_cus() * bpc;
        long long nrun = slots / nsg;
        if (nrun < 1) nrun = 1;
        long long run = (A.rows + nrun - 1) / nrun;
        run = (run + 7) / 8 * 8;                 // whole 8-row batches (the multipliers' quads)
        nrun = (A.rows + run - 1) / run;
        // Two workgroups per CU (the 4-wave pass): the grid's first half of
        // runs -- dispatched first, each CU's older workgroup, which the
        // CU's wave-age issue priority runs ahead -- takes SWEEP_SPLIT of the
        // rows, the second half the rest.  Equal runs ended bimodally (the
        // older workgroups at 66-78 us, the younger, then alone on the CU at
        // one wave per SIMD, at 93-102 us: profiles/r06/sweep_blocks_r06_cfg3.txt);
        // cfg3 sweep 104-106 -> 98-100 us (profiles/r06/ab_r06_sweep_split.txt).
        // LPGPU_SWEEP_SPLIT=f overrides (0: equal runs)
#ifndef SWEEP_SPLIT
#define SWEEP_SPLIT 0.62
#endif
        static const double split_env = [] {
            const char *v = std::getenv("LPGPU_SWEEP_SPLIT");
            return v ? std::atof(v) : SWEEP_SPLIT;
        }();
        long long runb = run;
        int na = (int)nrun;
        if (split_env > 0.0 && split_env < 1.0 && bpc == 2 && nrun >= 2 && nrun % 2 == 0) {
            const long long h = nrun / 2;
            long long ra = ((long long)(split_env * (double)A.rows) / h + 7) / 8 * 8;
            long long rb = ((A.rows - h * ra + h - 1) / h + 7) / 8 * 8;
            // (every run starts inside the tableau and the runs cover it)
            if (ra > 0 && rb > 0 && h * ra + h * rb >= A.rows && h * ra + (h - 1) * rb < A.rows) {
                run = ra;
                runb = rb;
                na = (int)h;
            }
        }
        const dim3 grid((unsigned)(nrun * nsg));
        long long tail = spread ? ((A.rows + nrun * nsg - 1) / (nrun * nsg) + 7) / 8 * 8 : 0;
        long long tcol = nfull * 64 * WL;
        const double *T = A.T, *Pp = A.P, *Mp = A.MQ;
        unsigned *dfl = oop ? A.dflips : nullptr;
        unsigned fseq = A.flipseq;
        const long long *dRp = A.dR;
        const Ctl *ctlp = A.ctl;
        long long ld = A.ld, rows = A.rows;
        int grpv = grp, nsv = (int)nsg;
        long long tend = ncol;
        unsigned long long *clk = A.sweep_clk;
        unsigned lseq = A.sweep_lseq;
        void *args[] = {&T, &To, &Pp, &Mp, &dRp, &ctlp, &ld, &rows, &grpv, &nsv, &run, &tail, &tcol, &tend, &nexp,
                        &dfl, &fseq, &clk, &lseq, &runb, &na};
        const hipError_t err = hipExtLaunchKernel(fn, grid, dim3(64 * WL), args, 0, s, e0, e1, 0);
        if (err == hipSuccess && flipped) *flipped = oop;
        return err != hipSuccess ? err : hipGetLastError();
    }
    // k_sweep_dp2 (in place), 10-wave workgroups on 128-column strips
    constexpr int WV = 10;
    const long long ns = (A.ld + 127) / 128;
    const void *fn = nb == 16 ? (const void *)&k_sweep_dp2<WV, 16, SA>
                   : nb == 32 ? (const void *)&k_sweep_dp2<WV, 32, SA>
                   : nb == 48 ? (const void *)&k_sweep_dp2<WV, 48, SA>
                              : (const void *)&k_sweep_dp2<WV, 64, SA>;
    const int bpc = sweep_blocks_per_cu(fn, 64 * WV);
    // the last strip (column n and the pitch's padding) spread over all
    // blocks where the runs are long (>= 2048 rows per block: the grid then
    // fills every resident slot); at short runs the extra piece (a P restage
    // + one batch) costs more than the slots give back
    const long long slots = (long long)sweep_grid_cus() * bpc;
    const bool tailed = ns >= 2 && (tail_env == 2 || (tail_env == 1 && A.rows * (ns - 1) >= 2048 * slots));
    const long long nsg = tailed ? ns - 1 : ns;   // strips with blocks of their own
    long long nrun = slots / nsg;
    if (nrun < 1) nrun = 1;
    long long run = (A.rows + nrun - 1) / nrun;
    run = (run + RW - 1) / RW * RW;
    nrun = (A.rows + run - 1) / run;
    const dim3 grid((unsigned)(nrun * nsg));
    // tail rows per block: a multiple of the batch (the multipliers' 4-row quads)
    long long tail = tailed ? ((A.rows + nrun * nsg - 1) / (nrun * nsg) + RW - 1) / RW * RW : 0;
    const double *T = A.T, *Pp = A.P, *Mp = A.MQ;   // the sweep reads the quad copy
    double *To = A.T;
    const long long *dRp = A.dR;
    const Ctl *ctlp = A.ctl;
    long long ld = A.ld, rows = A.rows;
    int grpv = grp, nsv = (int)nsg;
    void *args[] = {&T, &To, &Pp, &Mp, &dRp, &ctlp, &ld, &rows, &grpv, &nsv, &run, &tail};
    const hipError_t err = hipExtLaunchKernel(fn, grid, dim3(64 * WV), args, 0, s, e0, e1, 0);
    return err != hipSuccess ? err : hipGetLastError();
}

// ---- k_group geometry and launch ------------------------------------------
// compiled variants (summaries per lane, columns per lane, rows per lane)
#define GROUP_VARIANTS(X) \
    X(1, 2, 1) X(2, 2, 1) X(4, 2, 1) X(1, 3, 1) X(2, 3, 1) X(1, 4, 1) X(2, 4, 1) X(4, 4, 1) X(4, 2, 2) X(4, 4, 2) \
        X(4, 2, 4) X(4, 4, 4)

static const void *group_kernel(int nr, int ipl, int rpl, bool xr, bool hk = false)
{
#define X(NRV, IPLV, RPLV)                                                                     \
    if (nr == NRV && ipl == IPLV && rpl == RPLV)                                               \
        return xr ? reinterpret_cast<const void *>(&k_group<NRV, IPLV, RPLV, true>)            \
             : hk ? reinterpret_cast<const void *>(&k_group<NRV, IPLV, RPLV, false, true>)     \
                  : reinterpret_cast<const void *>(&k_group<NRV, IPLV, RPLV, false>);
    GROUP_VARIANTS(X)
#undef X
    return nullptr;
}

// resident k_group blocks per CU the launch may rely on: the runtime's
// occupancy answer for the compiled kernel (its VGPRs, SGPRs, static and
// dynamic LDS), capped by the LDS a CU holds when every block's share is
// rounded up to 2 KB (allocation granule and slack: the runtime admitted 3
// blocks of 53 KB per CU, of which the hardware did not keep the last ones
// resident -- 8 in-process cfg4 shards timed out, round 2), one less unless
// that LDS cap is what limits it
// (MI355X_MICROARCH, residency: the API can admit one block per CU more than
// the hardware does at some SGPR counts)
static int group_per_cu(const void *fn, size_t lds)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, GROUP_THREADS, lds) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    hipFuncAttributes at{};
    size_t stat = 0;
    if (hipFuncGetAttributes(&at, fn) == hipSuccess) stat = at.sharedSizeBytes;
    (void)hipGetLastError();
    const long long per = ((long long)(lds + stat) + 2047) / 2048 * 2048;
    const long long lds_cap = (long long)(160 * 1024) / per;
    if (n >= lds_cap) return (int)lds_cap;
    return n - 1;
}

static GroupGeom group_geom_uncached(long long rc, long long ld, long long n, int bmax, int xr, int nshard,
                                     int share, bool xs_ok)
{
    GroupGeom G;
    if (rc < 1 || ld < 1 || ld >= 0x7fffffffLL || rc >= 0x7fffffffLL || bmax < 1 || bmax > BMAX ||
        nshard < 1 || share < 1)
        return G;   // indices travel as 31 bits
    static int xcd_on = -1;
    if (xcd_on < 0) {
        const char *v = std::getenv("LPGPU_SEL_XCD");
        xcd_on = v ? std::atoi(v) : 1;
    }
    // the one-XCD selection k_sel (select.hip) where the shape fits it
    // (ranks sharing a GPU: only the XR variant that may use one XCD, which
    // then sizes for the co-located ranks itself)
    if (xcd_on && xr != 1 && nshard == 1 && (share == 1 || xr == 2)) {
        const GroupGeom S = sel_geom(rc, n, bmax, sweep_cus() / 8, xr != 0, xs_ok && xr != 1, share);
        if (S.g > 0) return S;
    }
    static long long gmin_env = -1;
    if (gmin_env < 0) {
        const char *v = std::getenv("LPGPU_SEL_BLOCKS");
        gmin_env = v ? std::atoll(v) : 0;
    }
    const int cus = sweep_cus(), xcd_cus = cus / 8;
    // candidate block counts, preferred first: at least one own row per
    // lane-slot, every lane at most 4 columns; with a few extra blocks every
    // lane down to 2 columns ("wide"), or not ("narrow", fewer blocks: fits
    // where the wide one does not); more blocks where one's LDS would exceed
    // GROUP_LDS_MAX
    struct Cand {
        long long g;
        int rpl;
    };
    Cand cand[2 * GROUP_MAXRPL];
    int nc = 0;
    for (int rpl = 1; rpl <= GROUP_MAXRPL; rpl *= 2)   // compiled: 1, 2, 4 rows per lane
        for (int wide = 1; wide >= 0; --wide) {
            long long g = (rc + 64LL * rpl - 1) / (64LL * rpl);
            if (g < GROUP_MINBLOCKS) g = GROUP_MINBLOCKS;
            if (gmin_env > g) g = gmin_env;   // A/B: more blocks than rows need
            const long long g2 = (ld + 2 * GROUP_THREADS - 1) / (2 * GROUP_THREADS);
            const long long g4 = (ld + 4 * GROUP_THREADS - 1) / (4 * GROUP_THREADS);
            if (wide && g2 > g && g2 <= g + g / 8) g = g2;
            if (g4 > g) g = g4;
            while (g < GROUP_MAXBLOCKS && group_lds(rc, ld, g, bmax) > GROUP_LDS_MAX) g *= 2;
            if (g > GROUP_MAXBLOCKS) g = GROUP_MAXBLOCKS;
            bool dup = false;
            for (int k = 0; k < nc; ++k) dup = dup || (cand[k].g == g && cand[k].rpl == rpl);
            if (!dup) cand[nc++] = Cand{g, rpl};
        }
    // every block of every launch that waits on this one must be resident at
    // the same time.  Workgroups are dealt round-robin over the 8 XCDs, so
    // each XCD must hold its eighth: one XCD (L2-resident hand-offs, xmode)
    // where the blocks fit there, else the whole device
    // blocks spread over the XCDs: a multiple of 8 of them, so that k_group's
    // two-level exchange applies (G / 8 blocks per XCD; LPGPU_HIER=0: flat)
    static int hier_env = -1;
    if (hier_env < 0) {
        const char *v = std::getenv("LPGPU_HIER");
        hier_env = v ? std::atoi(v) : 1;
    }
    for (int pass = 0; pass < 2; ++pass)
        for (int k = 0; k < nc; ++k) {
            long long g = cand[k].g;
            if (pass == 1 && hier_env && !xr && nshard == 1 && g >= 64)
                g = std::min<long long>((g + 7) / 8 * 8, GROUP_MAXBLOCKS);
            const int rpl = cand[k].rpl;
            const long long cpb = (ld + g - 1) / g, rpb = (rc + g - 1) / g;
            const long long lds = group_lds(rc, ld, g, bmax);
            if (cpb > 4 * GROUP_THREADS || rpb > (long long)rpl * GROUP_THREADS || lds > GROUP_LDS_MAX)
                continue;
            int nr = (int)((g + GROUP_THREADS - 1) / GROUP_THREADS);
            nr = nr <= 1 ? 1 : nr <= 2 ? 2 : 4;
            int ipl = (int)((cpb + GROUP_THREADS - 1) / GROUP_THREADS);
            ipl = ipl <= 2 ? 2 : (ipl == 3 && nr <= 2) ? 3 : 4;
            if (rpl >= 2) {
                nr = 4;
                ipl = ipl <= 2 ? 2 : 4;
            }
            // spread single-device groups: the variant with the two-level exchange
            const bool hk = pass == 1 && hier_env && !xr && nshard == 1 && g % 8 == 0 && g >= 64;
            const void *fn = group_kernel(nr, ipl, rpl, xr != 0, hk);
            if (!fn) continue;
            const int per_cu = group_per_cu(fn, (size_t)lds);
            if (per_cu < 1) continue;
            const bool one = pass == 0;
            if (one && !(xcd_on && xr != 1 && nshard == 1 && share == 1 && g <= (long long)per_cu * xcd_cus))
                continue;
            // ranks sharing a GPU launch their groups unsynchronised, so another
            // rank's sweep or set-up kernel can hold a slot while this group must
            // be resident: there, one block slot per CU stays free (4 ranks of
            // cfg4 on one GPU filled 2 of 2 slots per CU and timed out, round 2)
            const int per_cu_job = share > 1 ? per_cu - 1 : per_cu;
            if (!one && (g * nshard * share + 7) / 8 > (long long)per_cu_job * xcd_cus) continue;
            G.g = g;
            G.nr = nr;
            G.ipl = ipl;
            G.rpl = rpl;
            G.lds = (size_t)lds;
            G.per_cu = per_cu;
            G.xmode = one ? 1 : 0;
            G.hk = hk ? 1 : 0;
            return G;
        }
    return GroupGeom{};
}

GroupGeom group_geom(long long rc, long long ld, long long n, int bmax, int xr, int nshard, int share, bool xs_ok)
{
    static std::mutex mu;
    static std::map<std::array<long long, 9>, GroupGeom> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const std::array<long long, 9> key{rc, ld, n, bmax, xr, nshard, share, dev, xs_ok ? 1 : 0};
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    const GroupGeom G = group_geom_uncached(rc, ld, n, bmax, xr, nshard, share, xs_ok);
    cache[key] = G;
    return G;
}

hipError_t launch_group(hipStream_t s, const Args &A, const GroupGeom &geo, int grp, int count,
                        int from_erec, unsigned seq, int bmax, int xr, const Args *As, int nshard,
                        int first, int fmode, int frule, long long fcap, hipEvent_t e0, hipEvent_t e1)
{
    if (geo.g == 0 || count < 1 || count > bmax || bmax > BMAX) return hipErrorInvalidValue;
    if (xr && (A.nranks > NRANK_MAX || !A.xbuf || !A.peer)) return hipErrorInvalidValue;
    if (geo.sel) {
        if (As) return hipErrorInvalidValue;
        return launch_sel(s, A, geo, grp, count, from_erec, seq, xr, first, fmode, frule, fcap, e0, e1);
    }
    const void *fn = group_kernel(geo.nr, geo.ipl, geo.rpl, xr != 0, geo.hk != 0);
    if (!fn) return hipErrorInvalidValue;
    const int xmode = (geo.xmode && !As) ? 1 : 0;
    const dim3 grid((unsigned)(geo.g * (As ? nshard : 1) * (xmode ? 8 : 1)));
    Args a0 = A;
    const Args *as = As;
    int gper = (int)geo.g;
    void *args[] = {&a0, &as, &gper, &grp, &count, &from_erec, &seq, &bmax,
                    const_cast<int *>(&xmode), &first, &fmode, &frule, &fcap};
    return launch_persistent(fn, grid, args, geo.lds, s, e0, e1);
}

// A persistent selection launch (k_group, k_sel): its blocks wait on each
// other, so all must be resident at once -- sized from the compiled kernel's
// occupancy (group_geom / sel_geom), with every exchange bounded (a group
// that is not resident times out and is redone on the per-pivot kernels).
// LPGPU_COOP=1: a cooperative launch instead, which the runtime admits only
// if every block fits at once (hipErrorCooperativeLaunchTooLarge otherwise);
// tests/test_gpu_r3.py runs the suite's persistent geometries that way to
// check the sizing against the runtime's admission.  Not the default: same
// speed on the bench (cfg4 46.3-46.6k against 46.6-46.7k pivots/s) but 25-35
// us more per call on small LPs (cfg1 41-54 -> 77-83 us).
hipError_t launch_persistent(const void *fn, dim3 grid, void **args, size_t lds, hipStream_t s, hipEvent_t e0,
                             hipEvent_t e1)
{
    static int coop = -1;
    if (coop < 0) {
        const char *v = std::getenv("LPGPU_COOP");
        coop = v ? std::atoi(v) : 0;
    }
    if (!coop) return hipExtLaunchKernel(fn, grid, dim3(GROUP_THREADS), args, lds, s, e0, e1, 0);
    hipError_t err = e0 ? hipEventRecord(e0, s) : hipSuccess;
    if (err == hipSuccess) err = hipLaunchCooperativeKernel(fn, grid, dim3(GROUP_THREADS), args, lds, s);
    if (err == hipSuccess && e1) err = hipEventRecord(e1, s);
    return err;
}

hipError_t launch_resume(hipStream_t s, const Args &A)
{
    hipLaunchKernelGGL(k_resume, dim3(1), dim3(1), 0, s, A.ctl);
    return hipGetLastError();
}

hipError_t launch_peer_ping(hipStream_t s, const Args &A, unsigned tag, unsigned flags, int *ok_dev)
{
    if (A.nranks > NRANK_MAX || !A.xbuf || !A.peer || flags > 0xffffu) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_peer_ping, dim3(1), dim3(64), 0, s, A, tag, flags, ok_dev);
    return hipGetLastError();
}

hipError_t launch_group_min(hipStream_t s, double *const *ptrs, int n)
{
    hipLaunchKernelGGL(k_group_min, dim3(1), dim3(1), 0, s, ptrs, n);
    return hipGetLastError();
}

}  // namespace lpk
