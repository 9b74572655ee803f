// Device kernels of the dense simplex pivot engine (gfx950 / CDNA4).
//
// One pivot, single device = four launches, all decisions on device:
//   k_enter   entering-column scan of row 0          simplex.py:228-232 / :262-267
//   k_ratio   min-ratio test + multiplier snapshot    simplex.py:235-246 / :270-281
//   k_prow    normalised pivot row P                  tableau.py:302 (rowDiv)
//   k_update  rank-1 elimination of every other row  tableau.py:303-308 -> :269-289
// Row-sharded (one rank per GPU) inserts the exchange:
//   k_enter, k_ratio(LOCAL) -> allreduce-min(g) -> k_pick -> allgather(slots)
//   -> k_prow_sharded -> k_update
// Float semantics are fixed in oracle/lp_f64.c's header and must stay
// bit-identical to it (tests/test_gpu_parity.py compares whole tableaux).
//
// Local storage: row 0 (objective, replicated on every rank) + this rank's
// constraint rows, row-major, leading dimension ld (a multiple of 64 doubles
// = 512 B, so every row starts on a cache-line boundary and 16-byte vector
// accesses are aligned).
#include "engine.h"

namespace lpk {

__device__ __forceinline__ double wave_min(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ long long wave_min_ll(long long v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const long long w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

// block-wide minima; every thread gets the result.  scratch >= 16 entries.
__device__ double block_min(double v, double *scratch)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    v = wave_min(v);
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    double r = scratch[0];
    for (int w = 1; w < nw; ++w) r = fmin(r, scratch[w]);
    return r;
}

__device__ long long block_min_ll(long long v, long long *scratch)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    v = wave_min_ll(v);
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    long long r = scratch[0];
    for (int w = 1; w < nw; ++w) r = scratch[w] < r ? scratch[w] : r;
    return r;
}

__device__ __forceinline__ double tie_band(double g, double tie) { return g + tie * fabs(g); }

// ratio of one constraint row for the entering column; ok=false if a <= tol.pivot
__device__ __forceinline__ double row_ratio(double a, double b, const lp_tol &tol, bool &ok)
{
    ok = a > tol.pivot;
    const double num = fabs(b) <= tol.zero ? 0.0 : b;
    return ok ? num / a : 0.0;
}

// local row of global constraint r, or -1 if another rank holds it
__device__ __forceinline__ long long local_of(const Args &A, long long r)
{
    return (r >= A.rb && r < A.rb + A.rc) ? r - A.rb + 1 : -1;
}

__device__ __forceinline__ long long as_ll(double d) { return __double_as_longlong(d); }
__device__ __forceinline__ double as_d(long long v) { return __longlong_as_double(v); }

// ---------------------------------------------------------------------------
// control
// ---------------------------------------------------------------------------

__global__ void k_reset(Ctl *ctl, int mode, int rule, long long cap, long long r, long long c,
                        const double *T)
{
    ctl->status = LP_PIVOTED;
    ctl->mode = mode;
    ctl->rule = rule;
    ctl->cap = cap;
    ctl->r = r;
    ctl->c = c;
    ctl->npiv = 0;
    ctl->nstd = 0;
    ctl->stuck = 0;
    ctl->z0 = -T[0];
    ctl->ticket = 0;
}

// ---------------------------------------------------------------------------
// K1: entering column (one workgroup of 1024 threads over row 0)
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(ENTER_THREADS) k_enter(Args A)
{
    __shared__ double sd[16];
    __shared__ long long sl[16];
    __shared__ int s_rule, s_go;
    Ctl *ctl = A.ctl;
    if (threadIdx.x == 0) {
        int go = ctl->status == LP_PIVOTED;
        int rule = ctl->rule;
        if (go && ctl->mode == MODE_SOLVE) {
            // stall bookkeeping for the pivot just done (simplex.py:132-137)
            if (ctl->npiv > 0 && rule == LP_RULE_STANDARD) {
                const double z = -A.T[0];
                const double z0 = ctl->z0;
                if (fabs(z - z0) <= A.tol.stall * fmax(1.0, fabs(z0))) ctl->stuck += 1;
                else ctl->stuck = 0;
            }
            // switch to the min-index rule once stuck (simplex.py:123,138)
            if (rule == LP_RULE_STANDARD && ctl->stuck >= A.m + A.n) {
                rule = LP_RULE_MIN_INDEX;
                ctl->rule = rule;
            }
        }
        if (go && ctl->cap >= 0 && ctl->npiv >= ctl->cap) {
            ctl->status = LP_CAP_REACHED;
            go = 0;
        }
        s_rule = rule;
        s_go = go;
    }
    __syncthreads();
    if (!s_go) return;
    const double *c0 = A.T;
    const long long n = A.n;
    long long j = NONE;
    if (s_rule == LP_RULE_MIN_INDEX) {
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

// ---------------------------------------------------------------------------
// K2: ratio test over this rank's constraint rows + multiplier snapshot.
//   Each block owns RATIO_CHUNK consecutive rows and publishes
//   (local min l_b, first row within the tie band of l_b, its ratio).  The
//   last block to arrive combines them in row order.  Because every earlier
//   row of a block has a ratio above tie_band(l_b) >= tie_band(g), the first
//   block with l_b <= tie_band(g) holds the answer: its own candidate if that
//   is inside the global band, otherwise a rescan of that block alone.  The
//   result equals the two-pass scan of oracle/lp_f64.c for any scheduling.
// ---------------------------------------------------------------------------

// first local row in [li0, li1) with ratio <= thr (block-wide), NONE if none
__device__ long long rescan_rows(const Args &A, long long C, long long li0, long long li1,
                                 double thr, long long *scratch)
{
    long long best = NONE;
    for (long long li = li0 + threadIdx.x; li < li1; li += blockDim.x) {
        bool ok;
        const double *t = A.T + li * A.ld;
        const double q = row_ratio(t[C], t[0], A.tol, ok);
        if (ok && q <= thr) { best = li; break; }
    }
    return block_min_ll(best, scratch);
}

// first local row within tie_band(g) using the block records (block-wide)
__device__ long long pick_from_records(const Args &A, long long C, double g, long long *scratch)
{
    const double thr = tie_band(g, A.tol.ratio_tie);
    const unsigned nb = (unsigned)((A.rc + RATIO_CHUNK - 1) / RATIO_CHUNK);
    long long bsel = NONE;
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) {
        const double l = __hip_atomic_load(&A.rec[b].l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (l <= thr) { bsel = b; break; }
    }
    bsel = block_min_ll(bsel, scratch);
    if (bsel == NONE) return NONE;
    const double qb = __hip_atomic_load(&A.rec[bsel].q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long ib = __hip_atomic_load(&A.rec[bsel].i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (qb <= thr) return ib;
    const long long b0 = 1 + bsel * RATIO_CHUNK;
    return rescan_rows(A, C, b0, min(b0 + RATIO_CHUNK, A.rows), thr, scratch);
}

__global__ void __launch_bounds__(RATIO_THREADS) k_ratio(Args A, int mode, long long check_row)
{
    __shared__ double sd[16];
    __shared__ long long sl[16];
    __shared__ double s_q;
    __shared__ int s_last;
    Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) {
        if (mode == RATIO_LOCAL && blockIdx.x == 0 && threadIdx.x == 0) *A.xg = INFINITY;
        return;
    }
    const long long C = ctl->c + 1;
    const long long li0 = 1 + (long long)blockIdx.x * RATIO_CHUNK;
    const long long li1 = min(li0 + RATIO_CHUNK, A.rows);
    if (blockIdx.x == 0 && threadIdx.x == 0) A.mult[0] = A.T[C];

    // one row per thread (RATIO_CHUNK == blockDim.x)
    const long long li = li0 + threadIdx.x;
    bool ok = false;
    double q = 0.0;
    if (li < li1) {
        const double *t = A.T + li * A.ld;
        const double a = t[C];
        A.mult[li] = a;
        q = row_ratio(a, t[0], A.tol, ok);
    }
    const double lb = block_min(ok ? q : INFINITY, sd);
    long long ib = NONE;
    if (lb < INFINITY) ib = block_min_ll(ok && q <= tie_band(lb, A.tol.ratio_tie) ? li : NONE, sl);
    if (threadIdx.x == 0) s_q = 0.0;
    __syncthreads();
    if (ib != NONE && li == ib) s_q = q;
    __syncthreads();
    // publish: one lane stores the record, releases it, then takes a ticket
    // (agent-scope release/acquire, cdna_hip_programming.md Guideline 16)
    if (threadIdx.x == 0) {
        A.rec[blockIdx.x].l = lb;
        A.rec[blockIdx.x].i = ib;
        A.rec[blockIdx.x].q = s_q;
        __threadfence();
        const unsigned t = atomicAdd(&ctl->ticket, 1u);
        s_last = (t == gridDim.x - 1);
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();  // acquire the other blocks' records

    double g = INFINITY;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x)
        g = fmin(g, __hip_atomic_load(&A.rec[b].l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    g = block_min(g, sd);

    if (mode == RATIO_LOCAL) {
        if (threadIdx.x == 0) { *A.xg = g; ctl->ticket = 0; }
        return;
    }
    if (mode == RATIO_CHECK) {
        // Simplex.pivot(r, c): row r must attain the minimum ratio (simplex.py:204-215)
        if (threadIdx.x == 0) {
            const double *t = A.T + check_row * A.ld;
            bool okr;
            const double qr = row_ratio(t[C], t[0], A.tol, okr);
            if (t[C] == 0.0) ctl->status = LP_ZERO_PIVOT;
            else if (!(g < INFINITY) || !okr || !(qr <= tie_band(g, A.tol.ratio_tie)))
                ctl->status = LP_BAD_PIVOT;
            ctl->ticket = 0;
        }
        return;
    }
    if (!(g < INFINITY)) {
        if (threadIdx.x == 0) { ctl->status = LP_UNBOUNDED; ctl->ticket = 0; }
        return;
    }
    const long long win = pick_from_records(A, C, g, sl);
    if (threadIdx.x == 0) {
        ctl->r = win - 1 + A.rb;
        ctl->ticket = 0;
    }
}

// ---------------------------------------------------------------------------
// K2s (sharded): after allreduce-min of the ratio, each rank offers its first
// row within the global tie band (or the requested row) in its exchange slot.
// Every block recomputes the (cheap) candidate and copies a slice of the row.
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256) k_pick(Args A, int mode)
{
    __shared__ long long sl[16];
    Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) return;
    const long long C = ctl->c + 1;
    long long li = -1;
    long long code = 0;
    if (mode == PICK_RATIO) {
        const double g = *A.xg;
        if (!(g < INFINITY)) {
            // every rank sees the same global minimum: unbounded everywhere
            if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_UNBOUNDED;
            return;
        }
        const long long w = pick_from_records(A, C, g, sl);
        li = (w == NONE) ? -1 : w;
    } else {
        li = local_of(A, ctl->r);
        if (li >= 0 && mode == PICK_CHECK) {
            const double *t = A.T + li * A.ld;
            bool okr;
            const double g = *A.xg;
            const double qr = row_ratio(t[C], t[0], A.tol, okr);
            if (t[C] == 0.0) code = LP_ZERO_PIVOT;
            else if (!(g < INFINITY) || !okr || !(qr <= tie_band(g, A.tol.ratio_tie)))
                code = LP_BAD_PIVOT;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.xs[0] = as_d(li < 0 ? NONE : li - 1 + A.rb);
        A.xs[1] = as_d(code);
    }
    if (li < 0) return;
    const double *src = A.T + li * A.ld;
    for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < A.ld;
         j += (long long)gridDim.x * blockDim.x)
        A.xs[SLOT_HDR + j] = src[j];
}

// ---------------------------------------------------------------------------
// K2': explicit pivot (Tableau.pivot): multiplier snapshot only
// ---------------------------------------------------------------------------

__global__ void k_gather(Args A)
{
    Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) return;
    const long long C = ctl->c + 1;
    for (long long li = blockIdx.x * (long long)blockDim.x + threadIdx.x; li < A.rows;
         li += (long long)gridDim.x * blockDim.x)
        A.mult[li] = A.T[li * A.ld + C];
}

// ---------------------------------------------------------------------------
// K3: normalised pivot row P = T[R] / a_RC, P[C] = 1   (tableau.py:300-302)
// ---------------------------------------------------------------------------

__device__ void finish_pivot_bookkeeping(const Args &A, Ctl *ctl)
{
    const long long k = ctl->npiv;
    if (k < A.logcap) {
        A.log[2 * k] = ctl->r;
        A.log[2 * k + 1] = ctl->c;
    }
    ctl->npiv = k + 1;
    if (ctl->mode == MODE_SOLVE && ctl->rule == LP_RULE_STANDARD) ctl->nstd += 1;
}

__global__ void k_prow(Args A)
{
    Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) return;
    const long long R = local_of(A, ctl->r);
    const long long C = ctl->c + 1;
    const double *t = A.T + R * A.ld;
    const double a = t[C];
    if (a == 0.0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_ZERO_PIVOT;
        return;
    }
    for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < A.ld;
         j += (long long)gridDim.x * blockDim.x)
        A.P[j] = (j == C) ? 1.0 : t[j] / a;
    if (blockIdx.x == 0 && threadIdx.x == 0) finish_pivot_bookkeeping(A, ctl);
}

// sharded: choose the lowest offered row among the gathered slots, normalise it
__global__ void k_prow_sharded(Args A)
{
    Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) return;
    const long long slot = SLOT_HDR + A.ld;
    long long best = NONE;
    int who = -1;
    long long code = 0;
    for (int k = 0; k < A.nranks; ++k) {
        const long long idx = as_ll(A.xr[k * slot]);
        const long long cd = as_ll(A.xr[k * slot + 1]);
        if (cd != 0) code = cd;
        if (idx < best) { best = idx; who = k; }
    }
    if (code != 0 || best == NONE) {
        if (blockIdx.x == 0 && threadIdx.x == 0)
            ctl->status = code != 0 ? (int)code : LP_UNBOUNDED;
        return;
    }
    const long long C = ctl->c + 1;
    const double *t = A.xr + who * slot + SLOT_HDR;
    const double a = t[C];
    if (a == 0.0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) ctl->status = LP_ZERO_PIVOT;
        return;
    }
    for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < A.ld;
         j += (long long)gridDim.x * blockDim.x)
        A.P[j] = (j == C) ? 1.0 : t[j] / a;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctl->r = best;
        finish_pivot_bookkeeping(A, ctl);
    }
}

// ---------------------------------------------------------------------------
// K4: rank-1 elimination, in place.
//   Tile = 128 columns (one wave: 64 lanes x 16 B) x UPD_ROWS rows; the four
//   waves of a block take interleaved rows of the tile.  Each lane keeps its
//   two P values in registers for all its rows; per row the multiplier is a
//   wave-uniform scalar load.  Rows with a zero multiplier are skipped
//   (tableau.py:272), the pivot row is overwritten with P, the pivot column
//   becomes the exact unit vector.
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256) k_update(Args A)
{
    const Ctl *ctl = A.ctl;
    if (ctl->status != LP_PIVOTED) return;
    const long long R = local_of(A, ctl->r);   // -1 on a non-owner rank
    const long long C = ctl->c + 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long j0 = (long long)blockIdx.x * 128 + lane * 2;
    if (j0 >= A.ld) return;
    const double2 p = *reinterpret_cast<const double2 *>(A.P + j0);
    const bool c0 = (j0 == C), c1 = (j0 + 1 == C);
    const long long rbeg = (long long)blockIdx.y * UPD_ROWS + wave;
    const long long rend = min((long long)(blockIdx.y + 1) * UPD_ROWS, A.rows);
    double *base = A.T + j0;
    for (long long i = rbeg; i < rend; i += 4 * UPD_UNROLL) {
        double2 x[UPD_UNROLL];
        double f[UPD_UNROLL];
#pragma unroll
        for (int u = 0; u < UPD_UNROLL; ++u) {
            const long long ii = i + 4 * u;
            f[u] = (ii < rend) ? A.mult[ii] : 0.0;
            if (ii < rend && ii != R && f[u] != 0.0)
                x[u] = *reinterpret_cast<const double2 *>(base + ii * A.ld);
        }
#pragma unroll
        for (int u = 0; u < UPD_UNROLL; ++u) {
            const long long ii = i + 4 * u;
            if (ii >= rend) continue;
            double2 *dst = reinterpret_cast<double2 *>(base + ii * A.ld);
            if (ii == R) {
                *dst = p;
            } else if (f[u] != 0.0) {
                double2 y;
                y.x = c0 ? 0.0 : fma(-f[u], p.x, x[u].x);
                y.y = c1 ? 0.0 : fma(-f[u], p.y, x[u].y);
                *dst = y;
            }
        }
    }
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

int ratio_blocks(long long rows) { return (int)((rows - 1 + RATIO_CHUNK - 1) / RATIO_CHUNK); }

hipError_t launch_reset(hipStream_t s, Ctl *ctl, int mode, int rule, long long cap, long long r,
                        long long c, const double *T)
{
    hipLaunchKernelGGL(k_reset, dim3(1), dim3(1), 0, s, ctl, mode, rule, cap, r, c, T);
    return hipGetLastError();
}

hipError_t launch_enter(hipStream_t s, const Args &A)
{
    hipLaunchKernelGGL(k_enter, dim3(1), dim3(ENTER_THREADS), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_ratio(hipStream_t s, const Args &A, int mode, long long check_local_row)
{
    const int g = ratio_blocks(A.rows);
    if (g <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ratio, dim3(g), dim3(RATIO_THREADS), 0, s, A, mode, check_local_row);
    return hipGetLastError();
}

static unsigned row_blocks(long long ld) { return (unsigned)((ld + 255) / 256); }

hipError_t launch_pick(hipStream_t s, const Args &A, int mode)
{
    hipLaunchKernelGGL(k_pick, dim3(row_blocks(A.ld)), dim3(256), 0, s, A, mode);
    return hipGetLastError();
}

hipError_t launch_gather(hipStream_t s, const Args &A)
{
    const long long g = (A.rows + 255) / 256;
    hipLaunchKernelGGL(k_gather, dim3((unsigned)(g < 1024 ? g : 1024)), dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_prow(hipStream_t s, const Args &A)
{
    hipLaunchKernelGGL(k_prow, dim3(row_blocks(A.ld)), dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_prow_sharded(hipStream_t s, const Args &A)
{
    hipLaunchKernelGGL(k_prow_sharded, dim3(row_blocks(A.ld)), dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_update(hipStream_t s, const Args &A)
{
    const dim3 grid((unsigned)((A.ld + 127) / 128), (unsigned)((A.rows + UPD_ROWS - 1) / UPD_ROWS));
    hipLaunchKernelGGL(k_update, grid, dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_group_min(hipStream_t s, double *const *ptrs, int n)
{
    hipLaunchKernelGGL(k_group_min, dim3(1), dim3(1), 0, s, ptrs, n);
    return hipGetLastError();
}

}  // namespace lpk
