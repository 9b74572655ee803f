// Device helpers shared by the engine's kernels (kernels.hip) and the
// one-XCD persistent selection (select.hip): reductions, global-memory views,
// hand-off stores and loads, the float64 contract's numerics, and the tagged
// granule exchange of the persistent selections.  Internal linkage: each
// translation unit gets its own copy.
#pragma once

#include "engine.h"

namespace lpk {
namespace {

// ---------------------------------------------------------------------------
// reductions
// ---------------------------------------------------------------------------

// Wave-wide minimum in registers: DPP moves (no LDS round trips): two quad
// permutes and two row rotates reduce each row of 16 lanes, two row
// broadcasts fold the four rows into lane 63, a readlane makes the result
// wave-uniform.  Must be called with all 64 lanes active.
template <int CTRL, int ROWS>
__device__ __forceinline__ long long dpp64(long long v)
{
    const int lo = __builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(v >> 32), (int)(v >> 32), CTRL, ROWS, 0xf, false);
    return ((long long)hi << 32) | (unsigned)lo;
}

template <typename Op>
__device__ __forceinline__ long long wave_reduce64(long long v, Op op)
{
    v = op(v, dpp64<0xB1, 0xf>(v));    // quad_perm [1,0,3,2]
    v = op(v, dpp64<0x4E, 0xf>(v));    // quad_perm [2,3,0,1]
    v = op(v, dpp64<0x124, 0xf>(v));   // row_ror:4
    v = op(v, dpp64<0x128, 0xf>(v));   // row_ror:8   (row of 16 reduced)
    v = op(v, dpp64<0x142, 0xa>(v));   // row_bcast:15 into rows 1, 3
    v = op(v, dpp64<0x143, 0xc>(v));   // row_bcast:31 into rows 2, 3
    const int lo = __builtin_amdgcn_readlane((int)v, 63);
    const int hi = __builtin_amdgcn_readlane((int)(v >> 32), 63);
    return ((long long)hi << 32) | (unsigned)lo;
}

__device__ __forceinline__ double wave_min(double v)
{
    return __longlong_as_double(wave_reduce64(__double_as_longlong(v), [](long long a, long long b) {
        return __double_as_longlong(fmin(__longlong_as_double(a), __longlong_as_double(b)));
    }));
}

__device__ __forceinline__ long long wave_min_ll(long long v)
{
    return wave_reduce64(v, [](long long a, long long b) { return b < a ? b : a; });
}

// block-wide minima; every thread gets the result.  scratch >= 16 entries.
// A single-wave block reduces in registers only.
[[maybe_unused]] __device__ double block_min(double v, double *scratch)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    v = wave_min(v);
    if (nw == 1) return v;
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    double r = scratch[0];
    for (int w = 1; w < nw; ++w) r = fmin(r, scratch[w]);
    return r;
}

[[maybe_unused]] __device__ long long block_min_ll(long long v, long long *scratch)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    v = wave_min_ll(v);
    if (nw == 1) return v;
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    long long r = scratch[0];
    for (int w = 1; w < nw; ++w) r = scratch[w] < r ? scratch[w] : r;
    return r;
}

// ---------------------------------------------------------------------------
// cross-block hand-off (only k_ratio's LOCAL / CHECK modes): payload stored
// write-through (sc1), every storing wave drains, one lane per block takes an
// agent-scope ticket; the last arriver reads with sc1 loads
// (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH "Valid forms" row 1).
// ---------------------------------------------------------------------------

// Global-address-space views of device pointers: accesses through them are
// global_* instructions.  A flat_* access (what a generic pointer loaded from
// memory compiles to) also counts in lgkmcnt, so every later LDS wait would
// wait for it too.  Only for pointers into device memory (never LDS).
#define GAS __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ GAS T *gp(T *p)
{
    return (GAS T *)p;
}
template <typename T>
__device__ __forceinline__ const GAS T *gp(const T *p)
{
    return (const GAS T *)p;
}

template <typename T>
__device__ __forceinline__ void st_sc1(T *p, T v)
{
    __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T>
__device__ __forceinline__ T ld_sc1(const T *p)
{
    return __hip_atomic_load(gp(const_cast<T *>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// every thread calls; returns true in the last block to arrive
[[maybe_unused]] __device__ bool arrive_last(unsigned *ticket, int *s_flag)
{
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        *s_flag = (t == gridDim.x - 1);
    }
    __syncthreads();
    return *s_flag != 0;
}

// ---------------------------------------------------------------------------
// numerics shared by every kernel
// ---------------------------------------------------------------------------

// g + tie |g|, clamped to the largest double: a band that overflows holds
// every finite value (as oracle/lp_f64.c's +inf band does for its finite
// candidates) but never +inf, the "no candidate" marker of every summary, so
// a ballot of `x <= band` can only name a lane that has a candidate (ADVICE
// r5: a finite g near DBL_MAX made +inf pass and a speculative row load
// index NONE)
__device__ __forceinline__ double tie_band(double g, double tie)
{
    const double r = g + tie * fabs(g);
    return r <= 1.7976931348623157e308 ? r : 1.7976931348623157e308;
}

// ratio of one constraint row; ok=false if a <= tol.pivot   (simplex.py:273-276)
__device__ __forceinline__ double row_ratio(double a, double b, const lp_tol &tol, bool &ok)
{
    ok = a > tol.pivot;
    const double num = fabs(b) <= tol.zero ? 0.0 : b;
    return ok ? num / a : 0.0;
}

// one pivot applied to one element (row li, value x before the pivot):
// the pivot row becomes P, every other row gets fma(-f, P[j], x).  In the
// pivot column x == f and P == 1, so the result is exactly +0 (the unit
// column).  A zero multiplier leaves x unchanged (tableau.py:272 skips such
// rows; in float64 only the sign of a zero x could differ, which nothing
// downstream can observe), so no branch is needed.
__device__ __forceinline__ double upd(long long li, long long R, double f, double p, double x)
{
    return li == R ? p : fma(-f, p, x);
}

// current value of (li, j): stored value x with deferred pivots 0..t-1
// (generic form, used on rare paths)
[[maybe_unused]] __device__ double current(const Args &A, int t, long long li, long long j, double x)
{
    for (int s = 0; s < t; ++s)
        x = upd(li, A.dR[s], A.M[mi(A.rows, li, s)], A.P[s * A.ld + j], x);
    return x;
}

// current value of (li, C) for the thread's own row: the multipliers of the
// row are loaded as one contiguous run; dR[s] and P[s][C] come staged in LDS
template <int TP>
__device__ __forceinline__ double current_col(const Args &A, int t, long long li, double x,
                                              const long long *sR, const double *sPc)
{
    if constexpr (TP > 0) {
        double mv[TP];
#pragma unroll
        for (int s = 0; s < TP; ++s) mv[s] = A.M[mi(A.rows, li, s)];
#pragma unroll
        for (int s = 0; s < TP; ++s)
            if (s < t) x = upd(li, sR[s], mv[s], sPc[s], x);
    }
    return x;
}

// current value of (R, j) for the thread's own column of one row R: the TP
// pivot-row values are independent coalesced loads issued together
template <int TP>
__device__ __forceinline__ double current_row(const Args &A, int t, long long R, long long j,
                                              double x)
{
    if constexpr (TP > 0) {
        double pv[TP];
#pragma unroll
        for (int s = 0; s < TP; ++s) pv[s] = A.P[s * A.ld + j];
#pragma unroll
        for (int s = 0; s < TP; ++s)
            if (s < t) x = upd(R, A.dR[s], A.M[mi(A.rows, R, s)], pv[s], x);
    }
    return x;
}

__device__ __forceinline__ long long local_of(const Args &A, long long r)
{
    return (r >= A.rb && r < A.rb + A.rc) ? r - A.rb + 1 : -1;
}

__device__ __forceinline__ long long as_ll(double d) { return __double_as_longlong(d); }
__device__ __forceinline__ double as_d(long long v) { return __longlong_as_double(v); }


// diagnostic build only (-DLPK_STAMPS, `make variant NAME=stamps
// DEFS=-DLPK_STAMPS`, run with LPGPU_STAMPS=1): block 0 / lane 0 records the
// 100 MHz real-time clock at phase points of pivot t.  Compiled out of the
// product build: a stamp's store, even behind a runtime test, made the
// compiler wait for every outstanding store (s_waitcnt vmcnt(0)) before its
// registers were reused, in the middle of the pivot-row phase.
#ifdef LPK_STAMPS
constexpr bool STAMPS = true;
__device__ __forceinline__ void stamp(const Args &A, unsigned b, int t, int k)
{
    if (A.stamps && b == 0 && threadIdx.x == 0 && t < BMAX)
        *gp(A.stamps + t * 16 + k) = (long long)__builtin_amdgcn_s_memrealtime();
}
// every block: when it published its ratio (k = 0) / row-0 (k = 1) summary,
// knew the entering column (k = 2), had its column elements (k = 3)
__device__ __forceinline__ void bstamp(const Args &A, unsigned b, int t, int k)
{
    if (A.stamps && threadIdx.x == 0 && t < BMAX)
        *gp(A.stamps + BMAX * 16 + (b * BMAX + t) * 4 + k) = (long long)__builtin_amdgcn_s_memrealtime();
}
#else
constexpr bool STAMPS = false;
__device__ __forceinline__ void stamp(const Args &, unsigned, int, int) {}
__device__ __forceinline__ void bstamp(const Args &, unsigned, int, int) {}
#endif

typedef unsigned long long u64;
constexpr int NRMAX = (GROUP_MAXBLOCKS + GROUP_THREADS - 1) / GROUP_THREADS;
constexpr int NGR = 5;   // ratio summary: l (2), q (2), i
constexpr int NGE = 8;   // row-0 summary: l (2), q (2), i, fneg | rule << 31, P[t][0] (2)

__device__ __forceinline__ unsigned lo32(double d) { return (unsigned)as_ll(d); }
__device__ __forceinline__ unsigned hi32(double d) { return (unsigned)((u64)as_ll(d) >> 32); }
__device__ __forceinline__ double mk_d(unsigned lo, unsigned hi)
{
    return as_d((long long)(((u64)hi << 32) | lo));
}
__device__ __forceinline__ unsigned idx32(long long i) { return i == NONE ? 0x7fffffffu : (unsigned)i; }
__device__ __forceinline__ long long un_idx(unsigned w) { return w == 0x7fffffffu ? NONE : (long long)w; }

// the summary of pivot t, phase ph of launch seq: 0 ratio, 1 row 0 (this
// device); XR: 2 rank summary, 3 pivot-row slice, 4 / 5 straddle rescan;
// 7 is the setup ping (never a pivot's tag)
__device__ __forceinline__ unsigned gtag(unsigned seq, int t, int ph)
{
    return seq * (8 * BMAX) + 8 * t + ph;     // seq < 2^23 (the host wraps it)
}

// hand-off store of k_group.  fast: every block of the launch runs on ONE XCD
// (checked at launch start), so the XCD's L2 is the coherence point for all
// of them: a plain store (write-through L1 -> L2, line kept in L2) acked by
// the drain is visible to the others' sc1 loads (L1 bypassed, L2-served)
// without a trip to memory.  Otherwise an sc1 (write-through) store.
template <typename T>
__device__ __forceinline__ void st_x(T *p, T v, bool fast)
{
    if (fast) __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else st_sc1(p, v);
}

// Summary regions are granule-major: granule g of block b at [g * GROUP_MAXBLOCKS + b],
// so one poll instruction (granule g of 64 consecutive blocks) reads 512
// contiguous bytes -- 4 cache lines instead of 32-64 with block-major slots.
// Every block polls every summary until all have arrived, so the poll
// traffic is G x lines per instruction x NG per round: block-major, 64
// blocks polling 8-granule summaries asked an XCD's L2 for several times
// the lines its 16 channels serve per cycle, and every other access of the
// selection (the publications themselves, the column and row loads) queued
// behind the polls.
// That layout is for blocks on ONE XCD (xs = 0).  Blocks spread over the XCDs
// (xs = 1) keep block-major 64-byte slots (two consecutive blocks, on two
// XCDs, per line): there the stores matter -- write-through partial-line
// stores from several XCDs into one line serialise (granule-major: selection
// 14.4 -> 16.3 us per pivot at cfg4; granule rows grouped by XCD: 18.7), and
// so does pairing two blocks of one XCD in a line (16.0-17.0) or giving each
// block a whole line (more lines per poll: 16.9-18.7) (profiles/r02/README.md).
constexpr int GSLOT = 8;    // granules per block slot, block-major
__device__ __forceinline__ unsigned gslot(int g, unsigned b, int xs)
{
    return xs ? b * GSLOT + g : g * GROUP_MAXBLOCKS + b;
}
// lanes 0..n-1 store word[lane] of block b's summary (after the drain)
__device__ __forceinline__ void publish(u64 *region, unsigned b, unsigned tag, unsigned w, int n, bool fast,
                                        int xs)
{
    drain_stores();
    if ((int)threadIdx.x < n) st_x(&region[gslot(threadIdx.x, b, xs)], ((u64)tag << 32) | w, fast);
}

// every block's summary, lane l holding blocks l + 64k; polls until every
// granule carries `tag`.  Bounded by spin_max polls (a never-expected
// timeout flags the ctl; the host then redoes the group, lpgpu.cpp).
// (Keeping a second poll in flight was measured: the gather ends sooner but
// the leftover loads delay the next phase's loads by as much -- vmcnt retires
// in order.)
template <int NR, int NG, bool GMAJ = true>
__device__ bool gather(const u64 *base, unsigned G, unsigned tag, unsigned (&w)[NR][NG],
                       unsigned *timeout_flag, unsigned spin_max, int xs = 0)
{
    for (unsigned spins = 0;; ++spins) {
        // every load is issued before any is waited for: lanes past the last
        // block re-read block G-1 (in bounds, already tagged) and ignore it
        bool ok = true;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            const unsigned bb = min(threadIdx.x + k * GROUP_THREADS, G - 1);
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const u64 v = ld_sc1(GMAJ ? &base[gslot(g, bb, xs)] : &base[bb * 8 + g]);
                w[k][g] = (unsigned)v;
                ok = ok && (unsigned)(v >> 32) == tag;
            }
        }
        if (__all(ok)) return true;
        if (spins > spin_max) {          // seconds by default: never expected
            st_sc1(timeout_flag, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// lane f's value (f uniform)
__device__ __forceinline__ unsigned rl32(unsigned v, int f) { return __builtin_amdgcn_readlane(v, f); }
__device__ __forceinline__ double rl_d(unsigned lo, unsigned hi, int f)
{
    return mk_d(rl32(lo, f), rl32(hi, f));
}

// first summary (b = lane + 64k order) with l <= thr: returns k * 64 + lane, or -1
template <int NR>
__device__ __forceinline__ int first_in_band(const double (&l)[NR], unsigned G, double thr)
{
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const unsigned b = threadIdx.x + k * GROUP_THREADS;
        const u64 mask = __ballot(b < G && l[k] <= thr);
        if (mask) return k * GROUP_THREADS + __builtin_ctzll(mask);
    }
    return -1;
}

// combine of G per-block summaries held in registers (summary b = lane + 64k):
// two-pass semantics of the oracle.  The first summary inside the band is the
// lowest lane of the first k whose ballot is non-empty.  Returns the winning
// summary's candidate, or -1 - b when summary b is the first inside the band
// but its own candidate is not (rare: rescan b's slice).
template <int NR>
__device__ long long combine_loaded(const double (&l)[NR], const long long (&i)[NR],
                                    const double (&q)[NR], unsigned G, double thr)
{
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const unsigned b = threadIdx.x + k * GROUP_THREADS;
        const u64 mask = __ballot(b < G && l[k] <= thr);
        if (mask) {
            const int f = __builtin_ctzll(mask);
            const long long bsel = (long long)k * GROUP_THREADS + f;
            const double qs = mk_d(__builtin_amdgcn_readlane(lo32(q[k]), f),
                                   __builtin_amdgcn_readlane(hi32(q[k]), f));
            const long long is = ((long long)(unsigned)__builtin_amdgcn_readlane((int)(i[k] >> 32), f) << 32) |
                                 (unsigned)__builtin_amdgcn_readlane((int)i[k], f);
            return qs <= thr ? is : -1 - bsel;
        }
    }
    return NONE;
}

#ifndef LPK_CH
#define LPK_CH 8
#endif
constexpr int CH = LPK_CH;    // deferred pivots applied per chunk (loads issued together)

// ---- row-sharded persistent selection (XR): device-side exchange between
// ranks through each rank's exchange buffer (xbuf), written by its peers over
// xGMI with system-scope stores and polled locally (tagged 8-byte granules,
// as inside a device).  Layout in granules:
//   [XS_SUM]   2 parities x (NRANK_MAX + 1) slots x 8: the ranks' leaving-row
//              summaries (slot NRANK_MAX: a straddle resolution)
//   [XS_PROW]  2 parities x nranks source ranks x GROUP_MAXBLOCKS x 512: each
//              rank's candidate pivot row, block b's columns as {lo, tag},
//              {hi, tag} granule pairs (parities: a rank may run one pivot
//              ahead of a slow reader, never two)
//   then       GROUP_MAXBLOCKS x 8: this rank's per-block straddle rescans
template <typename T>
__device__ __forceinline__ void st_sys(T *p, T v)
{
    __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T ld_sys(const T *p)
{
    return __hip_atomic_load(gp(const_cast<T *>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// a cross-rank wait is bounded by wall-clock time (the ranks' launches are
// enqueued by different processes): Args::xwait_ms of the 100 MHz real-time
// counter (30 s by default)

// NG granules of each of n slots (slot p = lane p, p < n <= 64) at stride 8
template <int NG>
__device__ bool gather_x(const u64 *slots, int n, unsigned tag, unsigned (&w)[NG],
                         unsigned *timeout_flag, unsigned long long xticks)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int p = min((int)threadIdx.x, n - 1);
    for (;;) {
        bool ok = true;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const u64 v = ld_sys(&slots[p * 8 + g]);
            w[g] = (unsigned)v;
            ok = ok && (unsigned)(v >> 32) == tag;
        }
        if (__all(ok)) return true;
        if (__builtin_amdgcn_s_memrealtime() - t0 > xticks) {
            st_sc1(timeout_flag, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Two-level exchange, level 1 -> 2 (k_group, blocks spread over the XCDs):
// the last block of XCD group x gathers the group's G8 summaries (logical
// slots x G8 .. x G8 + G8 - 1, granule-major, L2-resident) and publishes ONE
// summary of the same format to slot x of the level-2 region (block-major,
// write-through): l = the group minimum; q, i = the candidate of the group's
// first member within the band of l, or q = INFINITY (rescan the group) when
// that member's own candidate lies outside it.  Entering summaries (row 0)
// also carry fneg = the group's first column with c_j < -cost, and member 0's
// flag bits and words 6, 7 (block 0's rule / stop flag / P[t][0] travel in
// group 0's summary).
template <int NG>
__device__ bool hier_combine(const u64 *lvl1, u64 *lvl2, unsigned x, unsigned G8, unsigned tag, double tie,
                             bool entering, unsigned *tflag, unsigned spin_max)
{
    unsigned w[1][NG];
    if (!gather<1, NG>(lvl1 + x * G8, G8, tag, w, tflag, spin_max)) return false;
    const bool in = threadIdx.x < G8;
    const double l = in ? mk_d(w[0][0], w[0][1]) : INFINITY;
    const double lx = wave_min(l);
    unsigned o[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) o[g] = rl32(w[0][g], 0);   // member 0's words
    o[0] = lo32(lx);
    o[1] = hi32(lx);
    if (lx < INFINITY) {
        const double thr = tie_band(lx, tie);
        const int f = __builtin_ctzll(__ballot(in && l <= thr));
        double q = rl_d(w[0][2], w[0][3], f);
        const unsigned i = rl32(w[0][4], f);
        if (!(q <= thr)) q = INFINITY;
        o[2] = lo32(q);
        o[3] = hi32(q);
        o[4] = entering ? (i & 0x7fffffffu) | (o[4] & 0x80000000u) : i;
    }
    if constexpr (NG > 5) {                      // word 5 exists in entering summaries only
        if (entering) {
            const long long fn = in ? (long long)(w[0][5] & 0x7fffffffu) : 0x7fffffffLL;
            o[5] = (unsigned)wave_min_ll(fn) | (o[5] & 0x80000000u);
        }
    }
    unsigned wv = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g)
        if ((int)threadIdx.x == g) wv = o[g];
    publish(lvl2, x, tag, wv, NG, false, 1);
    return true;
}

// row-0 summary of a block's own columns from per-lane values (columns
// j = jc0 + lane + 64k; vv = INFINITY where j is not a variable column):
// slice minimum el, first column within the tie band of el (ei, its value
// eq), first column with c_j < -tol.cost (efn).  The first column with a
// property is the lowest lane of the first k whose ballot is non-empty.
template <int IPL>
__device__ __forceinline__ void row0_summary(const double (&vv)[IPL], double vmin, long long jc0,
                                             const lp_tol &tol, double &el, long long &ei, double &eq,
                                             long long &efn)
{
    constexpr int nth = GROUP_THREADS;
    el = wave_min(vmin);
    efn = NONE;
    ei = NONE;
    eq = 0.0;
    const double ethr = tie_band(el, tol.cost_tie);
#pragma unroll
    for (int k = 0; k < IPL; ++k) {
        const u64 mn = __ballot(vv[k] < -tol.cost);
        if (mn && efn == NONE) efn = jc0 + k * nth + __builtin_ctzll(mn);
        const u64 mb = __ballot(el < INFINITY && vv[k] <= ethr);
        if (mb && ei == NONE) {
            const int f = __builtin_ctzll(mb);
            ei = jc0 + k * nth + f;
            eq = rl_d(lo32(vv[k]), hi32(vv[k]), f);
        }
    }
}

}  // namespace
}  // namespace lpk
