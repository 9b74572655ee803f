// One-XCD persistent pivot selection (k_sel): every selection of a group of
// chained pivots in ONE launch whose G <= 64 single-wave workgroups share one
// XCD -- the cfg3 tableau (4096 x 8192) on one GPU, and each rank's 4096-row
// shard of cfg4 across eight (BASELINE.json north_star).  k_sel<XS>: a
// tableau of up to 8 x 4096 rows (cfg4 on one GPU, or one rank of 2 / 4 GPUs
// with XR) as 8 such row shards in one launch, one per XCD (sel_body).
//
// Same contract as k_group (kernels.hip), rebuilt around what bounds a pivot
// there -- a chain of dependent latencies (two block exchanges, two dependent
// memory round trips, two deferred-pivot chains) -- with the per-pivot work
// on that chain cut down:
//   * the deferred-pivot chains run from registers: a lane's multipliers of
//     its own row (M, pivot s of this launch in mreg[s]) stay in VGPRs, and
//     the other operand of each FMA (P[s][C] for the column, M[R][s] for the
//     pivot row) is broadcast from lane s % 16 of the lane's 16-lane row by
//     the FMA itself (v_fmac_f64_dpp row_newbcast) -- no LDS round trip per
//     pivot on the column side, one 16-byte LDS read per two pivots and
//     column on the row side (P[s][own column], software-pipelined);
//   * no select in the chains: a row that was an earlier pivot row s* of the
//     launch starts from P[s*] and its multipliers of pivots <= s* are zero
//     (fma(-p, 0, x) == x for finite p), the operations of upd() exactly;
//   * column 0 (b) is computed by every block: the ratio summary carries the
//     candidate's pivot element and current b, so every block forms
//     P[t][0] = b / a itself -- no owner of column 0, the pivot row's
//     columns 1..n split evenly (cfg3: 64 blocks x 128 columns, two per lane),
//     and the stall bookkeeping (simplex.py:123-137) runs in every block from
//     the same values, so the rule and stop flag need no broadcast;
//   * a block publishes its ratio summary without draining its stores: the
//     summary carries everything the pivot row needs (the multipliers of
//     earlier pivots were drained at earlier row-0 publications), and a near
//     tie that straddles the band is answered by the block that holds it (one
//     more hand-off) instead of rescans of its stored values;
//   * the multipliers' sweep copy (MQ) and column 0 are stored once at the
//     end of the launch, from registers.
// Every element still gets the float64 operations of oracle/lp_f64.c in the
// same order (bit-identical tableaux); simplex.py:218-284 (selection),
// tableau.py:295-308 (pivot), simplex.py:110-148 (solve loop).
#include "engine.h"
#include "device.h"

#include <hip/hip_ext.h>

#include <array>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

namespace lpk {
namespace {

// diagnostic build only (-DLPK_STAMPS, LPGPU_STAMPS=1): per-phase shader-
// cycle sums kept in scalar registers for the whole launch and stored once
// at its end (scripts/sel_clocks.py) -- no memory traffic in the loop
#ifdef LPK_STAMPS
// (the sums are 32-bit and kept in VGPRs -- in SGPRs they pushed the kernel
// into spilling scalar registers, which distorted what they measured)
#define SEL_CLK_DECL unsigned clk_[24] = {}; unsigned long long clk_t = __builtin_amdgcn_s_memtime(), clk_r0 = 0;
#define SEL_CLK(k)                                                                \
    do {                                                                          \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();               \
        clk_[k] = vgpr(clk_[k] + (unsigned)(n_ - clk_t));                         \
        clk_t = n_;                                                               \
    } while (0)
#define SEL_DONE(x)                                                               \
    do {                                                                          \
        const int z_ = __builtin_amdgcn_readfirstlane((int)__double_as_longlong(x)); \
        asm volatile("s_nop 0" ::"s"(z_));                                        \
    } while (0)
// per pivot t < 48 and block: 100 MHz real-time stamps of phase points
// (scripts/sel_clocks.py --events): 0 pivot start, 1 column arrived, 2 ratio
// summary published, 3 every ratio summary seen, 4 row-0 summary published,
// 5 every row-0 summary seen
#define SEL_EV(k)                                                                                   \
    do {                                                                                            \
        if (A.stamps && lane == 0 && t < 48 && shard == 0 && b < 64)                                \
            *gp(A.stamps + BMAX * 16 + 4096 + ((long long)t * 64 + b) * 8 + (k)) =                  \
                (long long)__builtin_amdgcn_s_memrealtime();                                        \
    } while (0)
#else
#define SEL_CLK_DECL
#define SEL_CLK(k) do {} while (0)
#define SEL_DONE(x) do {} while (0)
#define SEL_EV(k) do {} while (0)
#endif

typedef double d16 __attribute__((ext_vector_type(16)));

// ---- deferred-pivot chains --------------------------------------------------
// x <- fma(-v[lane L of this lane's 16-lane row], m, x): the DPP operand is the
// broadcast one.  fma(-v, m, x) == fma(-m, v, x) bit for bit (the product is
// exact before the single rounding), so either operand order is upd()'s.
// Each block starts with s_nop: the DPP source must not be written by a VALU
// instruction in the two (five after an EXEC write) cycles before.
#define SEL_F(L, M) "v_fmac_f64_dpp %0, -%1, %" #M " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
#define SEL_COL8(L0, L1, L2, L3, L4, L5, L6, L7)                                                      \
    asm("s_nop 4\n" SEL_F(L0, 2) SEL_F(L1, 3) SEL_F(L2, 4) SEL_F(L3, 5) SEL_F(L4, 6) SEL_F(L5, 7)     \
            SEL_F(L6, 8) SEL_F(L7, 9)                                                                 \
        : "+v"(a)                                                                                     \
        : "v"(v), "v"(mk[o]), "v"(mk[o + 1]), "v"(mk[o + 2]), "v"(mk[o + 3]), "v"(mk[o + 4]),          \
          "v"(mk[o + 5]), "v"(mk[o + 6]), "v"(mk[o + 7]))

// column chain: a (this lane's row, column C) <- pivots 0..t-1, whole chunks
// of 8 (pivots t.. of the last chunk: v = 0 and m = 0, exact no-ops)
template <int NK, int C>
__device__ __forceinline__ void col_chunk(double &a, double v, const d16 &mk)
{
    constexpr int o = 8 * (C & 1);
    if constexpr (C & 1) SEL_COL8(8, 9, 10, 11, 12, 13, 14, 15);
    else SEL_COL8(0, 1, 2, 3, 4, 5, 6, 7);
}
template <int NK>
__device__ __forceinline__ void col_chain(double &a, const double (&pk)[NK], const d16 &m0, const d16 &m1,
                                          const d16 &m2, const d16 &m3, int t)
{
    // (the first chunk past t ends the chain: one taken branch, not one per
    // remaining chunk)
    if (t <= 0) return;
    col_chunk<NK, 0>(a, pk[0], m0);
    if (t <= 8) return;
    col_chunk<NK, 1>(a, pk[0], m0);
    if (t <= 16) return;
    col_chunk<NK, 2>(a, pk[1], m1);
    if (t <= 24) return;
    col_chunk<NK, 3>(a, pk[1], m1);
    if constexpr (NK > 2) {
        if (t <= 32) return;
        col_chunk<NK, 4>(a, pk[2], m2);
        if (t <= 40) return;
        col_chunk<NK, 5>(a, pk[2], m2);
        if (t <= 48) return;
        col_chunk<NK, 6>(a, pk[3], m3);
        if (t <= 56) return;
        col_chunk<NK, 7>(a, pk[3], m3);
    }
}
#undef SEL_COL8

// row chain, pivots 2h, 2h + 1 on the lane's IPL columns: x[k] <- fma(-mr[L], p[k], x[k])
template <int IPL>
struct RowPair;
#define SEL_RF(XI, MI, PI, L) "v_fmac_f64_dpp %" #XI ", -%" #MI ", %" #PI " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n"
template <>
struct RowPair<1> {
    template <int L0, int L1, bool NOP>
    static __device__ __forceinline__ void run(double (&x)[1], double mr, const double2 (&p)[1]);
};
template <>
struct RowPair<2> {
    template <int L0, int L1, bool NOP>
    static __device__ __forceinline__ void run(double (&x)[2], double mr, const double2 (&p)[2]);
};
template <>
struct RowPair<4> {
    template <int L0, int L1, bool NOP>
    static __device__ __forceinline__ void run(double (&x)[4], double mr, const double2 (&p)[4]);
};
// (NOP: the chain's first pair waits out the DPP hazard of the broadcast
// operands' VALU writes; later pairs read the same, unchanged registers)
#define SEL_PAIR_DEF1(L0, L1, NOP, PRE)                                                                    \
    template <>                                                                                           \
    __device__ __forceinline__ void RowPair<1>::run<L0, L1, NOP>(double (&x)[1], double mr,                \
                                                                 const double2 (&p)[1])                   \
    {                                                                                                     \
        asm(PRE SEL_RF(0, 1, 2, L0) SEL_RF(0, 1, 3, L1) : "+v"(x[0]) : "v"(mr), "v"(p[0].x), "v"(p[0].y));  \
    }                                                                                                     \
    template <>                                                                                           \
    __device__ __forceinline__ void RowPair<2>::run<L0, L1, NOP>(double (&x)[2], double mr,                \
                                                                 const double2 (&p)[2])                   \
    {                                                                                                     \
        asm(PRE SEL_RF(0, 2, 3, L0) SEL_RF(1, 2, 5, L0) SEL_RF(0, 2, 4, L1) SEL_RF(1, 2, 6, L1)            \
            : "+v"(x[0]), "+v"(x[1])                                                                      \
            : "v"(mr), "v"(p[0].x), "v"(p[0].y), "v"(p[1].x), "v"(p[1].y));                                \
    }                                                                                                     \
    template <>                                                                                           \
    __device__ __forceinline__ void RowPair<4>::run<L0, L1, NOP>(double (&x)[4], double mr,                \
                                                                 const double2 (&p)[4])                   \
    {                                                                                                     \
        asm(PRE SEL_RF(0, 4, 5, L0) SEL_RF(1, 4, 7, L0) SEL_RF(2, 4, 9, L0) SEL_RF(3, 4, 11, L0)           \
                SEL_RF(0, 4, 6, L1) SEL_RF(1, 4, 8, L1) SEL_RF(2, 4, 10, L1) SEL_RF(3, 4, 12, L1)           \
            : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3])                                              \
            : "v"(mr), "v"(p[0].x), "v"(p[0].y), "v"(p[1].x), "v"(p[1].y), "v"(p[2].x), "v"(p[2].y),      \
              "v"(p[3].x), "v"(p[3].y));                                                                  \
    }
#define SEL_PAIR_DEF(L0, L1) SEL_PAIR_DEF1(L0, L1, true, "s_nop 4\n") SEL_PAIR_DEF1(L0, L1, false, "")
SEL_PAIR_DEF(0, 1)
SEL_PAIR_DEF(2, 3)
SEL_PAIR_DEF(4, 5)
SEL_PAIR_DEF(6, 7)
SEL_PAIR_DEF(8, 9)
SEL_PAIR_DEF(10, 11)
SEL_PAIR_DEF(12, 13)
SEL_PAIR_DEF(14, 15)
#undef SEL_PAIR_DEF
#undef SEL_PAIR_DEF1
#undef SEL_RF
#undef SEL_F

// row chain: x (pivot row, own columns) <- pivots 0..t-1 in pairs; the pivot
// values P[s][own column] come from LDS (16 bytes = two pivots per read),
// three pairs ahead of the FMAs in a ring of four (pivots past t: mr = 0 and
// P = 0; reads past the last pair land in the slack after lP, unused).
// Unrolled by template recursion: the ring slots and broadcast lanes are
// compile-time constants.
template <int IPL, int NB>
__device__ __forceinline__ void lds_pair(double2 (&r)[IPL], const double *lP, const int (&kc)[IPL], int h)
{
#pragma unroll
    for (int k = 0; k < IPL; ++k) r[k] = *reinterpret_cast<const double2 *>(&lP[kc[k] * (NB + 2) + 2 * h]);
}
template <int IPL, int NB, int H>
__device__ __forceinline__ void row_steps(double (&x)[IPL], const double (&mr)[NB / 16], const double *lP,
                                          const int (&kc)[IPL], int t, double2 (&ring)[4][IPL])
{
    // t checked every second pair: the pivots of a pair past t have m = 0 and
    // P = 0 (LDS zeroed at launch start), exact no-ops
    if constexpr ((H & 1) == 0) {
        if (2 * H >= t) return;
    }
    lds_pair<IPL, NB>(ring[(H + 3) & 3], lP, kc, H + 3);
    // keep the read-ahead: without the barrier the scheduler sinks each read
    // to its FMAs and every pair waits out a full LDS latency
    __builtin_amdgcn_sched_barrier(0);
    RowPair<IPL>::template run<2 * (H & 7), 2 * (H & 7) + 1, H == 0>(x, mr[H >> 3], ring[H & 3]);
    if constexpr (H + 1 < NB / 2) row_steps<IPL, NB, H + 1>(x, mr, lP, kc, t, ring);
}
template <int IPL, int NB>
__device__ __forceinline__ void row_chain(double (&x)[IPL], const double (&mr)[NB / 16], const double *lP,
                                          const int (&kc)[IPL], int t)
{
    if (t <= 0) return;
    double2 ring[4][IPL];
    lds_pair<IPL, NB>(ring[0], lP, kc, 0);
    lds_pair<IPL, NB>(ring[1], lP, kc, 1);
    lds_pair<IPL, NB>(ring[2], lP, kc, 2);
    __builtin_amdgcn_sched_barrier(0);
    row_steps<IPL, NB, 0>(x, mr, lP, kc, t, ring);
}

// Summary regions of k_sel: granule g of block b at [g * 64 + b] (G <= 64):
// one poll instruction reads granule g of every block (512 contiguous bytes,
// 4 cache lines), and every granule's address is one register plus an
// immediate offset (the per-granule addresses of the general layout, kept
// live across the pivot loop, cost k_sel about 70 VGPRs).
constexpr int SEL_SLOT = 64;
constexpr int SEL_SLEEP = 1;   // s_sleep between the polls of an exchange (64 clocks per unit; 0 and 2: no change)
// a loop-invariant operand moved into a VGPR (the asm makes it look
// divergent, so it stays there): k_sel keeps most of its kernel arguments,
// per-block constants and tolerances in VGPRs -- in SGPRs the compiler ran
// out (106) and spilled about 70 of them into VGPR lanes, a v_readlane per use
template <typename T>
__device__ __forceinline__ T vgpr(T x)
{
    asm("" : "+v"(x));
    return x;
}

// row r of a row-major array of ldb-byte rows: one 32 x 32 + 64-bit
// multiply-add (a 64-bit row index times a 64-bit pitch costs four VALU ops
// on the leaving row's critical path)
template <typename T>
__device__ __forceinline__ T *rowp(T *base, long long r, unsigned ldb)
{
    return reinterpret_cast<T *>(reinterpret_cast<char *>(base) + (unsigned long long)(unsigned)r * ldb);
}
template <typename T>
__device__ __forceinline__ const T *rowp(const T *base, long long r, unsigned ldb)
{
    return reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + (unsigned long long)(unsigned)r * ldb);
}
// all N values materialised at this point (and none sunk into a branch)
template <int N>
__device__ __forceinline__ void keep_all(double (&v)[N])
{
    if constexpr (N == 1) asm("" : "+v"(v[0]));
    else if constexpr (N == 2) asm("" : "+v"(v[0]), "+v"(v[1]));
    else asm("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}
// a wave's ballot of a condition: the lane mask straight from the compare
// (HIP's __ballot takes an int, which costs a select and a second compare)
__device__ __forceinline__ u64 bal(bool c) { return __builtin_amdgcn_ballot_w64(c); }
// every active lane: the same, against EXEC
__device__ __forceinline__ bool wall(bool c) { return __builtin_amdgcn_ballot_w64(c) == __builtin_amdgcn_read_exec(); }

// p + byte offset: with p wave-uniform and a 32-bit per-lane offset the
// access is one global instruction with a scalar base (no per-lane 64-bit
// address arithmetic)
template <typename T>
__device__ __forceinline__ T *at(T *p, unsigned off)
{
    return reinterpret_cast<T *>(reinterpret_cast<char *>(p) + off);
}
template <typename T>
__device__ __forceinline__ const T *at(const T *p, unsigned off)
{
    return reinterpret_cast<const T *>(reinterpret_cast<const char *>(p) + off);
}

// hand-off store: FAST (every block on one XCD, checked at launch start) is a
// plain store that stays in the XCD's L2, else write-through (device.h st_x)
template <bool FAST, typename T>
__device__ __forceinline__ void stx(T *p, T v)
{
    if constexpr (FAST) __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else st_sc1(p, v);
}

// minimum of two doubles as v_min_f64 computes it, without the NaN
// canonicalisation fmin() adds (no operand here is a NaN).  (The compiler
// puts the two wait states a DPP read of the result needs after it.)
__device__ __forceinline__ double vmin(double a, double b)
{
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
template <int CTRL, int RM>
__device__ __forceinline__ double dppd(double v)
{
    const u64 x = (u64)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)x, CTRL, RM, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(x >> 32), CTRL, RM, 0xf, false);
    return mk_d(lo, hi);
}
// wave minimum (all 64 lanes active), wave-uniform: two quad permutes and two
// row rotates reduce each row of 16, two row broadcasts fold the rows into
// lane 63 (the other lanes end with partial or undefined values)
__device__ __forceinline__ double wmin(double v)
{
    v = vmin(v, dppd<0xB1, 0xf>(v));
    v = vmin(v, dppd<0x4E, 0xf>(v));
    v = vmin(v, dppd<0x124, 0xf>(v));
    v = vmin(v, dppd<0x128, 0xf>(v));
    v = vmin(v, dppd<0x142, 0xa>(v));
    v = vmin(v, dppd<0x143, 0xc>(v));
    return rl_d(lo32(v), hi32(v), 63);
}
// lane l's word of a summary assembled from wave-uniform values: v_writelane
// per word (a select chain on the lane index compiled to a branch per word)
template <int L>
__device__ __forceinline__ unsigned wl_(unsigned w, unsigned v)
{
    asm("v_writelane_b32 %0, %1, %2" : "+v"(w) : "s"(__builtin_amdgcn_readfirstlane(v)), "n"(L));
    return w;
}
#define wl(W, V, L) wl_<L>((W), (V))

// the words of a summary: lane g (< n) stores word g of block b
template <bool FAST, int SLOT = SEL_SLOT>
__device__ __forceinline__ void sel_put(u64 *region, unsigned b, unsigned tag, unsigned w, int n)
{
    if ((int)threadIdx.x < n) stx<FAST>(&region[threadIdx.x * SLOT + b], ((u64)tag << 32) | w);
}
// every block's summary (lane l: block min(l, G - 1)); polls until every
// granule carries `tag`, bounded by spin_max polls (the host then redoes the
// group on the per-pivot kernels)
// (STRIDE: granules between granule g and g + 1 of a slot)
template <int NG, int STRIDE = SEL_SLOT>
__device__ bool sel_gather(const u64 *base, unsigned G, unsigned tag, unsigned (&w)[NG], unsigned *timeout_flag,
                           unsigned spin_max)
{
    const u64 *p = base + min((unsigned)threadIdx.x, G - 1);
    for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const u64 v = ld_sc1(p + g * STRIDE);
            w[g] = (unsigned)v;
            ok = ok && (unsigned)(v >> 32) == tag;
        }
        if (wall(ok)) return true;
        if (spins > spin_max) {
            st_sc1(timeout_flag, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(SEL_SLEEP);
    }
}


// row-0 summary of a block's own columns (columns j = jc0 + lane + 64 k; vv =
// INFINITY where j is not one of them): slice minimum el, first column within
// the tie band of el (ei, its value eq, and P[t][ei] = epc from pv), first
// column with c_j < -tol.cost (efn)
template <int IPL>
__device__ __forceinline__ void sel_summary(const double (&vv)[IPL], const double (&pv)[IPL], double vmin_,
                                            long long jc0, const lp_tol &tol, double &el, long long &ei,
                                            double &eq, double &epc, long long &efn)
{
    // (branch-free: every ballot, then the first k with a hit picked by
    // scalar selects; the readlanes of each k issue together)
    u64 mn[IPL];
#pragma unroll
    for (int k = 0; k < IPL; ++k) mn[k] = bal(vv[k] < -tol.cost);   // independent of the minimum
    el = wmin(vmin_);
    const double ethr = tie_band(el, tol.cost_tie);
    efn = NONE;
#pragma unroll
    for (int k = IPL - 1; k >= 0; --k)
        if (mn[k]) efn = jc0 + k * 64 + __builtin_ctzll(mn[k]);
    ei = NONE;
    eq = 0.0;
    epc = 0.0;
    if (el < INFINITY) {
        u64 mb[IPL];
#pragma unroll
        for (int k = 0; k < IPL; ++k) mb[k] = bal(vv[k] <= ethr);   // (direct compares: no select + recompare)
        int kf = IPL, f = 0;
#pragma unroll
        for (int k = IPL - 1; k >= 0; --k)
            if (mb[k]) {
                kf = k;
                f = __builtin_ctzll(mb[k]);
            }
        if (kf < IPL) {
            ei = jc0 + kf * 64 + f;
            double q1 = 0.0, p1 = 0.0;
#pragma unroll
            for (int k = 0; k < IPL; ++k) {
                const double qk = rl_d(lo32(vv[k]), hi32(vv[k]), f), pk = rl_d(lo32(pv[k]), hi32(pv[k]), f);
                q1 = k == kf ? qk : q1;
                p1 = k == kf ? pk : p1;
            }
            eq = q1;
            epc = p1;
        }
    }
}
// the words of a row-0 summary: l (2), q (2), i, fneg, P[t][i] (2)
__device__ __forceinline__ unsigned esum_words(double el, double eq, long long ei, long long efn, double epc)
{
    unsigned w = idx32(ei);
    w = wl(w, lo32(el), 0);
    w = wl(w, hi32(el), 1);
    w = wl(w, lo32(eq), 2);
    w = wl(w, hi32(eq), 3);
    w = wl(w, idx32(efn), 5);
    w = wl(w, lo32(epc), 6);
    w = wl(w, hi32(epc), 7);
    return w;
}
// sel_gather split in two: issue() sends the first polls, finish() checks them
// (and polls on); work placed between the two runs while the polls are in
// flight (the scheduling barriers keep the loads ahead of it)
template <int NG, int STRIDE = SEL_SLOT>
struct SelPoll {
    const u64 *p;
    u64 v[NG];
    __device__ __forceinline__ void load(u64 (&d)[NG])
    {
#pragma unroll
        for (int g = 0; g < NG; ++g) d[g] = ld_sc1(p + g * STRIDE);
    }
    __device__ __forceinline__ bool take(unsigned tag, const u64 (&d)[NG], unsigned (&w)[NG])
    {
        bool ok = true;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            w[g] = (unsigned)d[g];
            ok = ok && (unsigned)(d[g] >> 32) == tag;
        }
        return wall(ok);
    }
    __device__ __forceinline__ void issue(const u64 *base, unsigned G)
    {
        p = base + min((unsigned)threadIdx.x, G - 1);
        load(v);
        __builtin_amdgcn_sched_barrier(0);
    }
    __device__ __forceinline__ bool finish(unsigned tag, unsigned (&w)[NG], unsigned *timeout_flag,
                                           unsigned spin_max)
    {
        __builtin_amdgcn_sched_barrier(0);
        for (unsigned spins = 0;; ++spins) {
            if (take(tag, v, w)) return true;
            if (spins > spin_max) {
                st_sc1(timeout_flag, 1u);
                return false;
            }
            __builtin_amdgcn_s_sleep(SEL_SLEEP);
            load(v);
        }
    }
};

constexpr int SEL_NGR = 9;   // ratio summary: l (2), i, a (2), b (2), q of the candidate (2)
constexpr int SEL_NGE = 8;   // row-0 summary: l (2), q (2), i, fneg, P[t][i] (2)
constexpr int SEL_NGS = 5;   // rescan / straddle answer: i, a (2), b (2)
constexpr int SEL_NGX = 7;   // XR rank summary: l (2), global row, a (2), b (2)
// XS: the shards' summaries are written to one replica per reading shard
// (one copy that all 512 blocks poll: cfg4 selection 7.2-7.4 -> 8.1 us per pivot)
constexpr int XS_NREP = XS_SHARDS;
#define XS_RD(s) (s)

// pivot TQ's deferred register work (sel_body): its multiplier into m<TQ / 16>
// [TQ % 16] -- every vector takes a select at the index, in place (a branch
// per vector made the compiler copy all four) -- and to M; the multipliers of
// its leaving row zeroed (fma(-p, 0, x) == x: that row is P[TQ] from then on)
#define SEL_SETTLE(TQ)                                                                              \
    do {                                                                                            \
        const int tq_ = (TQ), u_ = tq_ & 15, kq_ = tq_ >> 4;                                        \
        m0[u_] = kq_ == 0 ? apend : m0[u_];                                                         \
        m1[u_] = kq_ == 1 ? apend : m1[u_];                                                         \
        if constexpr (NK > 2) m2[u_] = kq_ == 2 ? apend : m2[u_];                                   \
        if constexpr (NK > 3) m3[u_] = kq_ == 3 ? apend : m3[u_];                                   \
        if (own) stx<FAST && !XS>(at(Mb + (long long)tq_ * rowsv, moff), apend);                    \
        if (zpend) {                                                                                \
            m0 = (d16)0.0;                                                                          \
            if (tq_ >= 16) m1 = (d16)0.0;                                                           \
            if (NK > 2 && tq_ >= 32) m2 = (d16)0.0;                                                 \
            if (NK > 3 && tq_ >= 48) m3 = (d16)0.0;                                                 \
        }                                                                                           \
    } while (0)

// The pivot loop of k_sel.  NB: most pivots of a launch (register
// multipliers); IPL: own columns per lane (cpb <= 64 IPL); XR: one rank of a
// row-sharded job (leaving row and pivot row exchanged between ranks through
// the peers' exchange buffers, as in k_group); FAST: every block on one XCD.
// XS: shard `shard` of XS_SHARDS row shards of ONE tableau, one per XCD, in
// one launch: the shard's G blocks own rows [1 + shard rps, 1 + shard rps +
// rps) and, like every shard, all the variable columns; the shards exchange
// their leaving-row candidates through the common region of Args::gran, and
// every shard forms the winner's pivot row itself from the shared tableau (the
// multipliers are stored write-through for that) -- no row travels.
// first: as k_group's (call start: reset / eager / enter).
template <int IPL, int NB, bool XR, bool FAST, bool XS>
__device__ __forceinline__ void sel_body(const Args &A, const unsigned b, const unsigned G, int grp, int count,
                                         int from_erec, unsigned seq, int first, int fmode, long long fcap,
                                         double *lP, long long npiv, long long nstd, long long stuck, int rule,
                                         const unsigned shard)
{
    constexpr int CS = NB + 2;             // LDS stride of a column's pivot values (16-B reads, no conflicts)
    constexpr int NK = NB / 16;            // broadcast registers
    const int lane = threadIdx.x;
    Ctl *ctl = A.ctl;
    const bool reset = (first & 1) != 0, eager = (first & 2) != 0, enter = (first & 4) != 0;
    const long long cap = reset ? fcap : *gp(&ctl->cap);
    const int mode = reset ? fmode : *gp(&ctl->mode);
    // the tableau, pivot rows and multipliers stay scalar bases (one global
    // instruction per access with a per-lane 32-bit offset); the other
    // loop-invariant operands live in VGPRs (vgpr())
    double *const Tb = A.T;
    double *const Pb = A.P;
    double *const Mb = A.M;
    const long long ld = vgpr(A.ld);
    const unsigned ldb = vgpr((unsigned)(A.ld * 8));       // bytes per row (host: ld * 8 < 2^32)
    double *const MQv = vgpr(A.MQ);
    double *const row0v = vgpr(A.row0);
    double *const col0v = vgpr(A.col0);
    const long long rowsv = vgpr(A.rows);
    const long long nv = vgpr(A.n);
    lp_tol tol;
    tol.cost = vgpr(A.tol.cost);
    tol.cost_tie = vgpr(A.tol.cost_tie);
    tol.pivot = vgpr(A.tol.pivot);
    tol.zero = vgpr(A.tol.zero);
    tol.ratio_tie = vgpr(A.tol.ratio_tie);
    tol.stall = vgpr(A.tol.stall);
    // own rows: lane l holds row lr0 + l; own columns: j = jc0 + l + 64 k, a
    // block's share of the variable columns 1..n (column 0 is every block's)
    const long long rps = XS ? (A.rc + XS_SHARDS - 1) / XS_SHARDS : A.rc;   // rows of a shard
    const long long rs0 = XS ? (long long)shard * rps : 0;                   // its first (0-based)
    const long long rpb = (rps + G - 1) / G;
    const long long lr0 = vgpr(1 + rs0 + (long long)b * rpb),
                    lr1 = vgpr(min(1 + rs0 + min((long long)b * rpb + rpb, rps), A.rows));
    const long long li = lr0 + lane;
    const bool own = li < lr1;
    const long long cpb = (A.n + G - 1) / G;
    const long long jc0 = vgpr(1 + (long long)b * cpb), jc1 = vgpr(min(1 + (long long)b * cpb + cpb, A.n + 1));
    int jk[IPL];
    bool cok[IPL];
    int kc[IPL];
    unsigned xoff[IPL];                    // byte offsets: own column in a row (clamped to the row)
#pragma unroll
    for (int k = 0; k < IPL; ++k) {
        jk[k] = (int)jc0 + lane + 64 * k;
        cok[k] = jk[k] < jc1;
        kc[k] = (int)min((long long)lane + 64 * k, cpb - 1);
        xoff[k] = vgpr((unsigned)min((long long)jk[k], nv) * 8u);
    }
    // byte offsets of the broadcast operands: P[16 k + lane % 16][.] and
    // M[16 k + lane % 16][.] (every row of P and M exists: NB <= BMAX)
    unsigned pkoff[NK], mroff[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const unsigned s = 16u * k + (lane & 15);
        pkoff[k] = vgpr(s * (unsigned)ld * 8u);
        mroff[k] = vgpr(s * (unsigned)rowsv * 8u);
    }
    const unsigned moff = vgpr((unsigned)li * 8u);
    // the row the lane's column element comes from: its tableau row, or the
    // pivot row P[s*] once the lane's row was pivot row s* of this launch
    const double *arow = vgpr(Tb + (own ? li : 0) * ld);
    // current row 0 on own columns, row0[0], column 0 of the own row: the
    // eager copies, or (first launch after an upload) the stored tableau's
    double l0v[IPL];
#pragma unroll
    for (int k = 0; k < IPL; ++k) l0v[k] = cok[k] ? (eager ? *gp(Tb + jk[k]) : *gp(row0v + jk[k])) : 0.0;
    double v0 = eager ? *gp(Tb) : *gp(row0v);
    double lcv = own ? (eager ? *gp(Tb + li * ld) : *gp(col0v + li)) : 0.0;
    if (eager) {
        // the other blocks read row0[C] (a pivot's row-0 multiplier); the
        // entering-column exchange below drains these first
#pragma unroll
        for (int k = 0; k < IPL; ++k)
            if (cok[k]) st_sc1(&row0v[jk[k]], l0v[k]);
    }
    // LDS pivot values start at zero: the chains' padding pivots multiply them by 0
    for (long long e = lane; e < (cpb * CS + 8) / 2; e += GROUP_THREADS)
        reinterpret_cast<double2 *>(lP)[e] = make_double2(0.0, 0.0);
    // summary regions: ratio, row 0, XCD check, rescan answers (XS: the
    // shard's own set; xsum: the shards' common region)
    u64 *const gset = A.gran + (XS ? (long long)shard * GRAN_SHARD : 0);
    u64 *const grR = vgpr(gset);
    u64 *const grE = vgpr(gset + GROUP_MAXBLOCKS * GSLOT);
    u64 *const grS = vgpr(gset + 3 * GROUP_MAXBLOCKS * GSLOT);
    u64 *const xsum = vgpr(A.gran + XS_SHARDS * GRAN_SHARD);   // + reader shard x XS_READER_STRIDE
    ERec *const erecv = vgpr(A.erec);
    long long *const logv = vgpr(A.log);
    long long *const dRv = vgpr(A.dR);
    long long *const dCv = vgpr(A.dC);
    const long long logcapv = vgpr(A.logcap);
    const unsigned spin = A.spin_max;
    Ctl *const ctlv = vgpr(ctl);            // the loop's hand-off flags and records
    u64 *const xbufv = vgpr(A.xbuf);        // XR: this rank's exchange buffer, the peers'
    unsigned long long *const *const peerv = vgpr(A.peer);
    // XR: lane p (< nranks) holds peer p's exchange buffer address (a load
    // per peer and pivot was a dependent memory round trip ahead of the sends)
    u64 peerl = 0;
    if constexpr (XR) peerl = lane < A.nranks ? (u64)*gp(peerv + lane) : 0ull;
    auto peer = [&](int p) -> u64 * {
        return reinterpret_cast<u64 *>(((u64)__builtin_amdgcn_readlane((unsigned)(peerl >> 32), p) << 32) |
                                       (u64)(unsigned)__builtin_amdgcn_readlane((unsigned)peerl, p));
    };
    const long long rbv = vgpr(A.rb);
    double z0 = 0.0;
    if (reset) {
        z0 = -v0;                              // obj_val at the start (simplex.py:118)
        if (b == 0 && lane == 0) {
            stx<FAST>(&ctl->status, (int)LP_PIVOTED);
            stx<FAST>(&ctl->mode, mode);
            stx<FAST>(&ctl->rule, rule);
            stx<FAST>(&ctl->chain, 1);
            stx<FAST>(&ctl->cap, cap);
            stx<FAST>(&ctl->r, -1LL);
            stx<FAST>(&ctl->c, -1LL);
            stx<FAST>(&ctl->npiv, 0LL);
            stx<FAST>(&ctl->nstd, 0LL);
            stx<FAST>(&ctl->stuck, 0LL);
            stx<FAST>(&ctl->z0, z0);
            stx<FAST>(&ctl->ndef[grp ^ 1], 0LL);
            st_sc1(&ctl->bar_timeout, 0u);
        }
    } else {
        z0 = *gp(&ctl->z0);
    }
    // this lane's row: the multiplier of pivot s in m<s / 16>[s % 16]
    d16 m0 = (d16)0.0, m1 = (d16)0.0, m2 = (d16)0.0, m3 = (d16)0.0;
    int pstar = -1;                             // the latest pivot of the launch whose row was the lane's
    // the previous pivot's register work, done while the next column travels:
    // its multiplier of the lane's row (apend) into m and to M, and -- in the
    // lane holding its leaving row (zpend) -- that row's multipliers zeroed
    double apend = 0.0;
    bool zpend = false;
    long long sRv = -1;                         // lane s: pivot s's local row (-1: another rank's)
    int status = LP_PIVOTED;
    int stop = 0;                               // the objective increased (simplex.py:133)
    int ndone = 0;
    unsigned long long xwait = 0;              // XR: block 0's cross-rank waits (Ctl::xwait_ticks)
    SEL_CLK_DECL
    // ---- the first pivot's entering column (call start: every block's
    //      summary of its row-0 slice; later launches: the previous launch's
    //      records; or given).  Row 0 in memory is current here (kernel
    //      boundary, or stored write-through above), so f0 and rare rescans
    //      read it directly.
    long long C = NONE;
    double f0 = 0.0, pcw = 0.0;               // row 0 at C; P[t - 1][C] (t > 0, from the summaries)
    {
        const bool capped = cap >= 0 && npiv >= cap;
        if (!from_erec && !enter) {
            C = ld_sc1(&ctl->c) + 1;
        } else {
            double el[1] = {INFINITY}, eq[1] = {0.0};
            long long ei[1] = {NONE}, ef[1] = {NONE};
            if (from_erec) {
                if ((unsigned)lane < G) {
                    el[0] = ld_sc1(&erecv[lane].l);
                    ei[0] = ld_sc1(&erecv[lane].i);
                    eq[0] = ld_sc1(&erecv[lane].q);
                    ef[0] = ld_sc1(&erecv[lane].fneg);
                }
            } else {
                double vv[IPL], vmn = INFINITY, pz[IPL];
#pragma unroll
                for (int k = 0; k < IPL; ++k) {
                    vv[k] = cok[k] ? l0v[k] : INFINITY;
                    vmn = vmin(vmn, vv[k]);
                    pz[k] = 0.0;
                }
                double sel_, seq_, spc_;
                long long sei_, sfn_;
                sel_summary<IPL>(vv, pz, vmn, jc0, tol, sel_, sei_, seq_, spc_, sfn_);
                const unsigned etag = gtag(seq, 0, 0);
                drain_stores();
                sel_put<FAST>(grE, b, etag, esum_words(sel_, seq_, sei_, sfn_, spc_), SEL_NGE);
                unsigned w[SEL_NGE];
                if (!sel_gather<SEL_NGE>(grE, G, etag, w, &ctlv->bar_timeout, spin)) status = LP_DEVICE_ERROR;
                if ((unsigned)lane < G) {
                    el[0] = mk_d(w[0], w[1]);
                    eq[0] = mk_d(w[2], w[3]);
                    ei[0] = un_idx(w[4]);
                    ef[0] = un_idx(w[5]);
                }
            }
            if (capped) {
                C = NONE;
            } else if (rule == LP_RULE_MIN_INDEX) {
                C = wave_min_ll(ef[0]);
            } else {
                const double g = wmin(el[0]);
                if (g < -tol.cost) {
                    const double ethr = tie_band(g, tol.cost_tie);
                    C = combine_loaded<1>(el, ei, eq, G, ethr);
                    if (C < 0) {                // rare: rescan that block's slice of row 0
                        const long long k0 = 1 + (-1 - C) * cpb, k1 = min(k0 + cpb, A.n + 1);
                        long long best = NONE;
                        for (long long k = k0 + lane; k < k1; k += GROUP_THREADS)
                            if (ld_sc1(&row0v[k]) <= ethr) { best = k; break; }
                        C = wave_min_ll(best);
                    }
                }
            }
            if (C == NONE && status == LP_PIVOTED) status = capped ? LP_CAP_REACHED : LP_OPTIMAL;
        }
        if (C != NONE) f0 = ld_sc1(&row0v[C]);
    }
    for (int tv = 0; tv < count && status == LP_PIVOTED; ++tv) {
        const int t = __builtin_amdgcn_readfirstlane(tv);
        if (t == 0) {
            SEL_CLK(15);                      // the launch's start, not a pivot's phase
#ifdef LPK_STAMPS
            clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif
        }
        SEL_EV(0);
        // ---- one round trip: the own rows' elements of column C (a pivot row
        //      of this launch: P[pstar][C]) and P[s][C] of the earlier pivots
        //      for the broadcasts; P[t - 1][C] came with the summaries
        // (every load unconditional and the selects after the last one: a
        // select right after its load made the compiler wait for each load
        // in turn -- four round trips instead of one)
        const double *const cP = Pb + C;      // wave-uniform
        double a = ld_sc1(arow + C);
        double pk[NK];
        // rows past t - 2 read row t - 2 instead (discarded below): a row of
        // this launch, in L2 -- a stale row of an earlier launch is an HBM miss
        const unsigned pkc = (unsigned)max(t - 2, 0) * (unsigned)ld * 8u;
#pragma unroll
        for (int k = 0; k < NK; ++k) pk[k] = ld_sc1(at(cP, 16 * k + (lane & 15) <= t - 2 ? pkoff[k] : pkc));
        if (t > 0) SEL_SETTLE(t - 1);
        const bool apcw = pstar >= 0 && pstar == t - 1;
        a = own ? (apcw ? pcw : a) : 0.0;
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int sk = 16 * k + (lane & 15);
            pk[k] = sk < t - 1 ? pk[k] : sk == t - 1 ? pcw : 0.0;
        }
        SEL_CLK(1);
        if (STAMPS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // diagnostic: the column has arrived
        SEL_CLK(2);
        SEL_EV(1);
        col_chain<NK>(a, pk, m0, m1, m2, m3, t);
        SEL_DONE(a);
        SEL_CLK(3);
        // ---- ratio test over the own rows; the block's candidate: the first
        //      row inside the band of the block minimum
        bool okq;
        const double q = row_ratio(a, lcv, tol, okq);
        okq = okq && own;
        const double qq = okq ? q : INFINITY;
        const double lb = wmin(qq);
        long long ib = NONE;
        double ab = 0.0, bb = 0.0, qb = 0.0;
        if (lb < INFINITY) {
            const u64 mask = bal(qq <= tie_band(lb, tol.ratio_tie));   // (the band is at most DBL_MAX)
            const int f = __builtin_ctzll(mask);
            ib = lr0 + f;
            ab = rl_d(lo32(a), hi32(a), f);
            bb = rl_d(lo32(lcv), hi32(lcv), f);
            qb = rl_d(lo32(q), hi32(q), f);
        }
        SEL_DONE(lb);
        SEL_CLK(4);
        // the drain makes the previous pivot's P stores visible with this
        // summary (read from pivot t + 1 on); this pivot's multipliers are
        // stored after it and drained with the next one
        drain_stores();
        // (fault injection (tests): block 1 (0) never publishes)
        if (!(A.fault == t + 1 && b == min(1u, G - 1) && shard == 0)) {
            unsigned wv = idx32(ib);
            wv = wl(wv, lo32(lb), 0);
            wv = wl(wv, hi32(lb), 1);
            wv = wl(wv, lo32(ab), 3);
            wv = wl(wv, hi32(ab), 4);
            wv = wl(wv, lo32(bb), 5);
            wv = wl(wv, hi32(bb), 6);
            wv = wl(wv, lo32(qb), 7);
            wv = wl(wv, hi32(qb), 8);
            sel_put<FAST>(grR, b, gtag(seq, t, 0), wv, SEL_NGR);
        }
        SEL_EV(2);
        SEL_CLK(5);
        // ---- leaving row: the polls go out first, then (while the summaries
        //      travel) the multiplier into its register and to memory
        unsigned w[SEL_NGR];
        SelPoll<SEL_NGR> pr;
        pr.issue(grR, G);
        apend = a;
        if (b == 0 && lane == 0) {            // read after the launch only (after the publication:
            *gp(&ctlv->c) = C - 1;            // stores pending at a drain delay the summary)
            *gp(&Mb[mi(rowsv, 0, t)]) = f0;   // row 0's multiplier (+ the sweep's copy)
            *gp(&MQv[mq(0, t)]) = f0;
        }
        if (!pr.finish(gtag(seq, t, 0), w, &ctlv->bar_timeout, spin)) {
            status = LP_DEVICE_ERROR;
            break;
        }
        SEL_CLK(6);
        SEL_EV(3);
        // ---- pivot row on the own columns: prow(Rl, av) = current values of
        //      local row Rl (stored row, or P[s*] if it was pivot row s* of
        //      this launch, + the later pivots of the launch) / av.  In two
        //      halves: prow_issue(Rl) sends the loads, prow_finish(av) runs
        //      the chain (the plain path issues them as soon as the leaving
        //      row is known, before the rest of the decision)
        long long R = NONE;                   // this device's leaving row (XR: its candidate)
        double aR = 0.0, bR = 0.0;
        double pv[IPL];
        double p0 = 0.0;
        double px[IPL], pmr[NK];
        int psst = -1;
        auto prow_issue = [&](long long Rl) {
            const u64 rp = bal(sRv == Rl);                          // (lanes >= t hold -1)
            psst = rp ? 63 - __builtin_clzll(rp) : -1;             // uniform
            // every load issued before any select (see the column's)
            const double *const xr = rowp(Tb, Rl, ldb);            // wave-uniform
            const double *const mrp = Mb + Rl;
#pragma unroll
            for (int k = 0; k < IPL; ++k) px[k] = *gp(at(xr, xoff[k]));
#pragma unroll
            for (int k = 0; k < NK; ++k) pmr[k] = ld_sc1(at(mrp, mroff[k]));
            __builtin_amdgcn_sched_barrier(0);
        };
        auto prow_finish = [&](double avv) {
            const int sst = psst;
            double x[IPL], mr[NK];
            // while the row travels: column 0's pivot value (every block),
            // computed here (the compiler would sink it to its first use, on
            // the way to the row-0 summary)
            if constexpr (!XR) {
                p0 = bR / aR;
                asm volatile("" : "+v"(p0));
            }
#pragma unroll
            for (int k = 0; k < IPL; ++k) x[k] = sst >= 0 ? lP[kc[k] * CS + sst] : (cok[k] ? px[k] : 0.0);
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int s = 16 * k + (lane & 15);
                mr[k] = (s < t && s > sst) ? pmr[k] : 0.0;
            }
            if (STAMPS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // diagnostic: the row has arrived
            SEL_CLK(8);
            row_chain<IPL, NB>(x, mr, lP, kc, t);
            SEL_DONE(x[IPL - 1]);
            SEL_CLK(9);
            // every lane divides, then selects: one barrier over all IPL
            // quotients, so that their division sequences interleave (a
            // branch around each, or a barrier per quotient, ran them one
            // after another)
            double qd[IPL];
#pragma unroll
            for (int k = 0; k < IPL; ++k) qd[k] = x[k] / avv;
            keep_all<IPL>(qd);
#pragma unroll
            for (int k = 0; k < IPL; ++k) pv[k] = (jk[k] == C) ? 1.0 : qd[k];
            SEL_DONE(pv[IPL - 1]);
            SEL_CLK(10);
        };
        auto prow = [&](long long Rl, double avv) {
            prow_issue(Rl);
            prow_finish(avv);
        };
        const double rl = (unsigned)lane < G ? mk_d(w[0], w[1]) : INFINITY;
        const double g = wmin(rl);
        SEL_DONE(g);
        SEL_CLK(20);
        if (g < INFINITY) {
            const double thr = tie_band(g, tol.ratio_tie);
            const int bs = __builtin_ctzll(bal(rl <= thr));         // (rl = inf: no candidate, never inside the clamped band)
            // (block bs has a candidate: its minimum is finite)
            const long long Rc = un_idx(rl32(w[2], bs));
            if constexpr (!XS) prow_issue(Rc);
            aR = rl_d(w[3], w[4], bs);
            bR = rl_d(w[5], w[6], bs);
            const double qR = rl_d(w[7], w[8], bs);
            if (qR <= thr) {                  // block bs's candidate lies inside the global band
                R = Rc;
            } else {
                // rare: block bs's first row inside the global band is not its
                // candidate; it answers with that row (one more hand-off)
                const unsigned stag = gtag(seq, t, 4);
                if (b == (unsigned)bs) {
                    const int f = __builtin_ctzll(bal(okq && q <= thr));
                    const double af = rl_d(lo32(a), hi32(a), f), bf = rl_d(lo32(lcv), hi32(lcv), f);
                    unsigned wv = (unsigned)(lr0 + f);
                    wv = wl(wv, lo32(af), 1);
                    wv = wl(wv, hi32(af), 2);
                    wv = wl(wv, lo32(bf), 3);
                    wv = wl(wv, hi32(bf), 4);
                    sel_put<FAST>(grS, 0, stag, wv, SEL_NGS);
                }
                unsigned y[SEL_NGS];
                if (!sel_gather<SEL_NGS>(grS, 1, stag, y, &ctlv->bar_timeout, spin)) {
                    status = LP_DEVICE_ERROR;
                    break;
                }
                R = (long long)rl32(y[0], 0);
                aR = rl_d(y[1], y[2], 0);
                bR = rl_d(y[3], y[4], 0);
                if constexpr (!XS) prow_issue(R);
            }
        } else if (!XR && !XS) {
            status = LP_UNBOUNDED;
            break;
        }
        SEL_CLK(7);
        double gR = g;                        // the device's minimum (XS: over its shards)
        double lps = INFINITY;                // XS: lane x < 8 holds shard x's minimum
        bool win = true;                      // this rank holds the leaving row
        long long rglob = R == NONE ? -1 : R - 1 + rbv;
        if constexpr (XS) {
            // ---- leaving row across the XCD shards: block 0 of every shard
            //      publishes (shard minimum, row, pivot element, b), write-
            //      through, granule-major (one poll instruction reads granule
            //      g of all shards: 64 bytes); every block takes the first
            //      shard inside the global band (rows are shard-ordered, so
            //      that is the reference's first row)
            const int par = t & 1;
            u64 *const xsl = xsum + XS_RD(shard) * XS_READER_STRIDE + par * 128;   // this shard's replica
            if (b == 0 && lane < SEL_NGX) {
                unsigned wv = R == NONE ? 0xffffffffu : (unsigned)(R - 1);
                wv = wl(wv, lo32(g), 0);
                wv = wl(wv, hi32(g), 1);
                wv = wl(wv, lo32(aR), 3);
                wv = wl(wv, hi32(aR), 4);
                wv = wl(wv, lo32(bR), 5);
                wv = wl(wv, hi32(bR), 6);
                const u64 v = ((u64)gtag(seq, t, 2) << 32) | wv;
#pragma unroll
                for (int r = 0; r < XS_NREP; ++r)
                    st_sc1(&xsum[r * XS_READER_STRIDE + par * 128 + lane * XS_SHARDS + shard], v);
            }
            // while the shards' summaries travel: the loads of this shard's
            // candidate row (used as they are if it wins; otherwise they have
            // brought that row into the Infinity Cache, where the winning
            // shard's own loads make the other shards' reads of ITS row hits)
            long long Rpre = NONE;
            if constexpr (!XR) {
                if (R != NONE) {
                    prow_issue(R);
                    Rpre = R;
                }
            }
            unsigned x[SEL_NGX];
            const unsigned long long xw0 = __builtin_amdgcn_s_memrealtime();
            if (!sel_gather<SEL_NGX, XS_SHARDS>(xsl, XS_SHARDS, gtag(seq, t, 2), x, &ctlv->bar_timeout, spin)) {
                status = LP_DEVICE_ERROR;
                break;
            }
            SEL_CLK(14);
            const double lp = lane < XS_SHARDS ? mk_d(x[0], x[1]) : INFINITY;
            const double gg = wmin(lp);
            lps = lane < XS_SHARDS ? lp : INFINITY;
            if (!(gg < INFINITY)) {
                if constexpr (!XR) {
                    status = LP_UNBOUNDED;
                    break;
                }
            }
            const double thr = tie_band(gg, tol.ratio_tie);
            if (gg < INFINITY) {
            const int ps = __builtin_ctzll(bal(lp <= thr));         // (lanes >= XS_SHARDS, shards without a candidate: inf)
            double as = rl_d(x[3], x[4], ps), bs = rl_d(x[5], x[6], ps);
            bool okp;
            const double qs = row_ratio(as, bs, tol, okp);
            long long rg;
            if (okp && qs <= thr) {
                rg = (long long)rl32(x[2], ps);
            } else {
                // rare: a near-tie straddles the band across shards.  Shard
                // ps's blocks each offer their first own row inside it (its
                // rescan slots), its block 0 publishes the lowest to all
                u64 *const xst = xsum + XS_RD(shard) * XS_READER_STRIDE + 256 + par * 8;
                if ((int)shard == ps) {
                    const u64 mk = bal(okq && q <= thr);
                    const int fr = mk ? __builtin_ctzll(mk) : 0;
                    const double ar = rl_d(lo32(a), hi32(a), fr), br = rl_d(lo32(lcv), hi32(lcv), fr);
                    u64 *const loc = grS + 1024;
                    if (lane < SEL_NGS) {
                        unsigned wv = mk ? (unsigned)(lr0 + fr) : 0x7fffffffu;
                        wv = wl(wv, lo32(ar), 1);
                        wv = wl(wv, hi32(ar), 2);
                        wv = wl(wv, lo32(br), 3);
                        wv = wl(wv, hi32(br), 4);
                        st_sc1(&loc[b * 8 + lane], ((u64)gtag(seq, t, 4) << 32) | wv);
                    }
                    unsigned wlo[1][SEL_NGS];
                    if (!gather<1, SEL_NGS, false>(loc, G, gtag(seq, t, 4), wlo, &ctlv->bar_timeout, spin)) {
                        status = LP_DEVICE_ERROR;
                        break;
                    }
                    const int bf = __builtin_ctzll(bal((unsigned)lane < G && wlo[0][0] != 0x7fffffffu));
                    if (b == 0 && lane < SEL_NGS) {
                        unsigned wv = rl32(wlo[0][0], bf) - 1u;
                        wv = wl(wv, rl32(wlo[0][1], bf), 1);
                        wv = wl(wv, rl32(wlo[0][2], bf), 2);
                        wv = wl(wv, rl32(wlo[0][3], bf), 3);
                        wv = wl(wv, rl32(wlo[0][4], bf), 4);
                        const u64 v = ((u64)gtag(seq, t, 5) << 32) | wv;
#pragma unroll
                        for (int r = 0; r < XS_NREP; ++r)
                            st_sc1(&xsum[r * XS_READER_STRIDE + 256 + par * 8 + lane], v);
                    }
                }
                unsigned y[SEL_NGS];
                if (!sel_gather<SEL_NGS, 1>(xst, 1, gtag(seq, t, 5), y, &ctlv->bar_timeout, spin)) {
                    status = LP_DEVICE_ERROR;
                    break;
                }
                rg = (long long)__builtin_amdgcn_readfirstlane(y[0]);
                as = mk_d(__builtin_amdgcn_readfirstlane(y[1]), __builtin_amdgcn_readfirstlane(y[2]));
                bs = mk_d(__builtin_amdgcn_readfirstlane(y[3]), __builtin_amdgcn_readfirstlane(y[4]));
            }
            rglob = rg + rbv;
            R = rg + 1;
            aR = as;
            bR = bs;
            gR = gg;
            } else {
                R = NONE;                     // XR: no candidate on this device
                gR = INFINITY;
            }
            if (status != LP_PIVOTED) break;
            if constexpr (!XR) xwait = vgpr(xwait + (__builtin_amdgcn_s_memrealtime() - xw0));
            // every shard: the pivot row on its blocks' columns from the
            // stored row and the leaving row's multipliers (write-through);
            // XR: the device's candidate, computed in the cross-rank step
            if constexpr (!XR) {
                if (R != Rpre) prow_issue(R);
                prow_finish(aR);
            }
        }
        if constexpr (XR) {
            // ---- leaving row across ranks (as k_group): every rank sends
            //      (local minimum, global row, pivot element, b) to all ranks
            //      and, without waiting for the verdict, its candidate's
            //      normalised row on every block's columns
            const int par = t & 1;
            const int N = A.nranks;                 // (a uniform loop bound: kept scalar)
            const unsigned long long xticks = (unsigned long long)A.xwait_ms * 100000ull;
            // (XS: the rank's candidate is its shards' (above); the summaries
            // go to one replica per XCD shard of every rank, and each peer's
            // copy of the pivot row is sent by one of the shards)
            constexpr int NREP = XS ? XS_SHARDS : 1;
            u64 *xsl = xbufv + (XS ? (long long)shard * XS_XREP : 0) + par * XS_SUM_PAR;
            if (b == 0 && lane < SEL_NGX && shard == 0) {
                const unsigned long long tg = (u64)gtag(seq, t, 2) << 32;
                unsigned wv = R == NONE ? 0xffffffffu : (unsigned)rglob;
                wv = wl(wv, lo32(gR), 0);
                wv = wl(wv, hi32(gR), 1);
                wv = wl(wv, lo32(aR), 3);
                wv = wl(wv, hi32(aR), 4);
                wv = wl(wv, lo32(bR), 5);
                wv = wl(wv, hi32(bR), 6);
                for (int p = 0; p < N; ++p)
#pragma unroll
                    for (int r = 0; r < NREP; ++r)
                        st_sys(&peer(p)[r * XS_XREP + par * XS_SUM_PAR + A.rank * 8 + lane], tg | wv);
            }
            auto send_row = [&](int ph) {
                const unsigned long long tg = (u64)gtag(seq, t, ph) << 32;
                for (int p = 0; p < N; ++p) {
                    if (p == A.rank) continue;
                    if (XS && ((p - A.rank + N) % N - 1) % XS_SHARDS != (int)shard) continue;
                    u64 *dst = peer(p) + XS_PROW + (long long)(par * N + A.rank) * XS_PROW_RANK +
                               (long long)b * XS_PROW_BLOCK;
#pragma unroll
                    for (int k = 0; k < IPL; ++k) {
                        const int kk = lane + 64 * k;
                        if (cok[k]) {
                            st_sys(&dst[2 * kk], tg | lo32(pv[k]));
                            st_sys(&dst[2 * kk + 1], tg | hi32(pv[k]));
                        }
                    }
                }
            };
            if (R != NONE) {
                // (one XCD: the loads were issued at the rank's decision)
                if constexpr (XS) prow(R, aR);
                else prow_finish(aR);
                send_row(3);
            }
            SEL_CLK(16);
            unsigned x[SEL_NGX];
            const unsigned long long xw0 = __builtin_amdgcn_s_memrealtime();
            if (!gather_x<SEL_NGX>(xsl, N, gtag(seq, t, 2), x, &ctlv->bar_timeout, xticks)) {
                status = LP_DEVICE_ERROR;
                break;
            }
            SEL_CLK(14);
            const double lp = lane < N ? mk_d(x[0], x[1]) : INFINITY;
            const double gg = wmin(lp);
            if (!(gg < INFINITY)) {
                status = LP_UNBOUNDED;
                break;
            }
            const double thr = tie_band(gg, tol.ratio_tie);
            const int ps = __builtin_ctzll(bal(lp <= thr));         // (lanes >= N, ranks without a candidate: inf)
            double as = rl_d(x[3], x[4], ps), bs = rl_d(x[5], x[6], ps);
            bool okp;
            const double qs = row_ratio(as, bs, tol, okp);
            long long rg;
            int ph = 3;                       // the tag of the winner's row slices
            if (okp && qs <= thr) {
                rg = (long long)rl32(x[2], ps);
            } else {
                // rare: a near-tie straddles the band across ranks.  Rank ps
                // finds its first row inside it (each block offers its first
                // own row, block 0 sends the lowest to every rank) and ships
                // that row's normalised values instead of its candidate's
                // (XS: the rank's first shard whose minimum lies inside the
                // band holds that row: its blocks offer, its block 0 sends)
                const int sfirst = XS ? __builtin_ctzll(bal(lane < XS_SHARDS && lps <= thr) | (1ull << 63)) : 0;
                if (A.rank == ps && (int)shard == sfirst) {
                    const u64 mk = bal(okq && q <= thr);
                    const int fr = mk ? __builtin_ctzll(mk) : 0;
                    const double ar = rl_d(lo32(a), hi32(a), fr), br = rl_d(lo32(lcv), hi32(lcv), fr);
                    u64 *loc = XS ? grS + 1536 : xbufv + XS_PROW + 2LL * N * XS_PROW_RANK;
                    if (lane < SEL_NGS) {
                        unsigned wv = mk ? (unsigned)(lr0 + fr) : 0x7fffffffu;
                        wv = wl(wv, lo32(ar), 1);
                        wv = wl(wv, hi32(ar), 2);
                        wv = wl(wv, lo32(br), 3);
                        wv = wl(wv, hi32(br), 4);
                        st_sc1(&loc[b * 8 + lane], ((u64)gtag(seq, t, 4) << 32) | wv);
                    }
                    unsigned wlo[1][SEL_NGS];
                    if (!gather<1, SEL_NGS, false>(loc, G, gtag(seq, t, 4), wlo, &ctlv->bar_timeout, spin)) {
                        status = LP_DEVICE_ERROR;
                        break;
                    }
                    const int bf = __builtin_ctzll(bal((unsigned)lane < G && wlo[0][0] != 0x7fffffffu));
                    const unsigned r0w = rl32(wlo[0][0], bf), a0 = rl32(wlo[0][1], bf), a1 = rl32(wlo[0][2], bf),
                                   b0 = rl32(wlo[0][3], bf), b1 = rl32(wlo[0][4], bf);
                    if (b == 0 && lane < SEL_NGS) {
                        unsigned wv = (unsigned)((long long)r0w - 1 + rbv);
                        wv = wl(wv, a0, 1);
                        wv = wl(wv, a1, 2);
                        wv = wl(wv, b0, 3);
                        wv = wl(wv, b1, 4);
                        for (int p = 0; p < N; ++p)
#pragma unroll
                            for (int r = 0; r < NREP; ++r)
                                st_sys(&peer(p)[r * XS_XREP + par * XS_SUM_PAR + NRANK_MAX * 8 + lane],
                                       ((u64)gtag(seq, t, 5) << 32) | wv);
                    }
                }
                unsigned y[SEL_NGS];
                if (!gather_x<SEL_NGS>(xsl + NRANK_MAX * 8, 1, gtag(seq, t, 5), y, &ctlv->bar_timeout, xticks)) {
                    status = LP_DEVICE_ERROR;
                    break;
                }
                rg = (long long)__builtin_amdgcn_readfirstlane(y[0]);
                as = mk_d(__builtin_amdgcn_readfirstlane(y[1]), __builtin_amdgcn_readfirstlane(y[2]));
                bs = mk_d(__builtin_amdgcn_readfirstlane(y[3]), __builtin_amdgcn_readfirstlane(y[4]));
                ph = 6;
                if (A.rank == ps) {
                    prow(rg - rbv + 1, as);
                    send_row(6);
                }
            }
            win = A.rank == ps;
            rglob = rg;
            R = win ? rg - rbv + 1 : -1;
            aR = as;
            bR = bs;
            // column 0's pivot value now, while the winner's row travels
            p0 = bR / aR;
            asm volatile("" : "+v"(p0));
            if (!win) {
                // the winning rank's block b sent these columns
                const u64 *src = xbufv + XS_PROW + (long long)(par * N + ps) * XS_PROW_RANK +
                                 (long long)b * XS_PROW_BLOCK;
                const unsigned tg = gtag(seq, t, ph);
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    bool ok = true;
#pragma unroll
                    for (int k = 0; k < IPL; ++k) {
                        const int kk = kc[k];
                        const u64 lo = ld_sys(&src[2 * kk]), hi = ld_sys(&src[2 * kk + 1]);
                        pv[k] = mk_d((unsigned)lo, (unsigned)hi);
                        ok = ok && (!cok[k] || ((unsigned)(lo >> 32) == tg && (unsigned)(hi >> 32) == tg));
                    }
                    if (wall(ok)) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > xticks) {
                        st_sc1(&ctlv->bar_timeout, 1u);
                        status = LP_DEVICE_ERROR;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(SEL_SLEEP);
                }
                if (status != LP_PIVOTED) break;
            }
            SEL_CLK(17);
            xwait = vgpr(xwait + (__builtin_amdgcn_s_memrealtime() - xw0));
        } else if constexpr (!XS) {
            prow_finish(aR);                  // (loads issued at the decision)
        }
        // ---- P[t], row 0 and column 0 (every block: p0 = b / a).  P[t] is
        //      read from pivot t + 2 on (drained with pivot t + 1's ratio
        //      summary; pivot t + 1 gets P[t][C] with the row-0 summaries);
        //      row 0 is stored once, at the end of the launch
        {
            double *const pt = rowp(Pb, t, ldb);               // wave-uniform
#pragma unroll
            for (int k = 0; k < IPL; ++k)
                if (cok[k]) stx<FAST>(at(pt, xoff[k]), pv[k]);
            if (b == 0 && lane == 0) *gp(pt) = p0;          // read after the launch (sweep)
        }
        double vn[IPL], vv[IPL], vmn = INFINITY;
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            vn[k] = upd(0, -1, f0, pv[k], l0v[k]);
            vv[k] = cok[k] ? vn[k] : INFINITY;
            vmn = vmin(vmn, vv[k]);
        }
        v0 = upd(0, -1, f0, p0, v0);
        double el, eq, epc;
        long long ei, efn;
        sel_summary<IPL>(vv, pv, vmn, jc0, tol, el, ei, eq, epc, efn);
        SEL_DONE(epc);
        SEL_CLK(21);
        const bool more = t + 1 < count;
        const unsigned etag = gtag(seq, t, 1);
        if (more) sel_put<FAST>(grE, b, etag, esum_words(el, eq, ei, efn, epc), SEL_NGE);
        SEL_EV(4);
        SEL_CLK(11);
        // ---- while the summaries travel: the pivot-row values into LDS,
        //      column 0 of the own rows (this pivot's multiplier is a), the
        //      pivot row's register state, the stall bookkeeping, records
        SelPoll<SEL_NGE> pe;
        if (more) pe.issue(grE, G);
#pragma unroll
        for (int k = 0; k < IPL; ++k) {
            if (cok[k]) lP[kc[k] * CS + t] = pv[k];
            l0v[k] = vn[k];
        }
        if (own) lcv = (li == R) ? p0 : fma(-a, p0, lcv);
        zpend = li == R;                      // that lane only: its row is P[t] from now on
        if (zpend) {
            pstar = t;
            arow = rowp(Pb, t, ldb);
        }
        if (lane == t) sRv = R;
        // stall bookkeeping (simplex.py:132-137), min-index switch
        // (:123,138) and the objective check (:133): every block, from
        // the same values
        if (mode == MODE_SOLVE && rule == LP_RULE_STANDARD) {
            nstd += 1;
            const double z = -v0;
            const double band = tol.stall * fmax(1.0, fabs(z0));
            if (z - z0 > band) stop = 1;
            if (fabs(z - z0) <= band) stuck += 1;
            else stuck = 0;
            if (stuck >= A.m + A.n) rule = LP_RULE_MIN_INDEX;
        }
        if (b == G - 1 && lane < 7) {
            long long *adr = &dRv[t];
            long long val = R;
            if (lane == 1) { adr = &dCv[t]; val = C; }
            else if (lane == 2) { adr = &ctlv->r; val = rglob; }
            else if (lane == 3) { adr = &ctlv->npiv; val = npiv + 1; }
            else if (lane == 4) { adr = &ctlv->ndef[grp]; val = t + 1; }
            else if (lane == 5) { adr = logv + 2 * min(npiv, logcapv - 1); val = rglob; }
            else if (lane == 6) { adr = logv + 2 * min(npiv, logcapv - 1) + 1; val = C - 1; }
            if (lane < 5 || npiv < logcapv) *gp(adr) = val;
        }
        if (b == 0 && lane == 0 && mode == MODE_SOLVE) {
            *gp(&ctlv->nstd) = nstd;
            *gp(&ctlv->stuck) = stuck;
            *gp(&ctlv->rule) = rule;
        }
        ++npiv;
        ++ndone;
        if (!more) {
            if (lane == 0) {                  // the next launch reads plain summaries
                *gp(&erecv[b].l) = el;
                *gp(&erecv[b].i) = ei;
                *gp(&erecv[b].q) = eq;
                *gp(&erecv[b].fneg) = efn;
            }
            break;
        }
        // ---- the next pivot's entering column
        SEL_CLK(12);
        unsigned we[SEL_NGE];
        if (!pe.finish(etag, we, &ctlv->bar_timeout, spin)) {
            status = LP_DEVICE_ERROR;
            break;
        }
        SEL_CLK(13);
        SEL_EV(5);
        {
            // the standard rule's minimum first, unconditionally: the loop's
            // bookkeeping below fills its dependency gaps (behind the rule and
            // stop branches it ran after them)
            const bool in = (unsigned)lane < G;
            const double el2 = in ? mk_d(we[0], we[1]) : INFINITY;
            const double g2 = wmin(el2);
            SEL_DONE(g2);
            SEL_CLK(18);
            rule = __builtin_amdgcn_readfirstlane(rule);
            stop = __builtin_amdgcn_readfirstlane(stop);
            const long long ef2 = in ? un_idx(we[5]) : NONE;
            const bool capped = cap >= 0 && npiv >= cap;
            long long Cn = NONE;
            int owner = -1;                   // the block that answers (rescan / min-index)
            double ethr = 0.0;
            if (stop || capped) {
                Cn = NONE;
            } else if (rule == LP_RULE_MIN_INDEX) {
                Cn = wave_min_ll(ef2);
                if (Cn != NONE) owner = (int)((Cn - 1) / cpb);
            } else {
                if (g2 < -tol.cost) {
                    ethr = tie_band(g2, tol.cost_tie);
                    // (lanes >= G: inf, never inside the clamped band)
                    const int bs = __builtin_ctzll(bal(el2 <= ethr));
                    // (every readlane at once, then the check)
                    const double qs = rl_d(we[2], we[3], bs);
                    const long long cb = un_idx(rl32(we[4], bs));
                    const double pb = rl_d(we[6], we[7], bs);
                    if (qs <= ethr) {
                        Cn = cb;
                        f0 = qs;
                        pcw = pb;
                    } else {
                        owner = bs;           // rare: the first column of its slice inside the band
                    }
                }
            }
            if (owner >= 0) {
                // the owning block answers: the column, its row-0 value and
                // P[t][column] from its registers (one more hand-off)
                const unsigned atag = gtag(seq, t + 1, 6);
                if (b == (unsigned)owner) {
                    long long cc = Cn;
                    int kf = 0, lf = 0;
                    if (cc == NONE) {
                        bool found = false;
#pragma unroll
                        for (int k = 0; k < IPL; ++k) {
                            const u64 mk = bal(cok[k] && vn[k] <= ethr);
                            if (!found && mk) {
                                found = true;
                                kf = k;
                                lf = __builtin_ctzll(mk);
                            }
                        }
                        cc = jc0 + 64 * kf + lf;
                    } else {
                        kf = (int)((cc - jc0) >> 6);
                        lf = (int)((cc - jc0) & 63);
                    }
                    double fv = 0.0, pvv = 0.0;
#pragma unroll
                    for (int k = 0; k < IPL; ++k)
                        if (k == kf) {
                            fv = rl_d(lo32(vn[k]), hi32(vn[k]), lf);
                            pvv = rl_d(lo32(pv[k]), hi32(pv[k]), lf);
                        }
                    unsigned wv = (unsigned)cc;
                    wv = wl(wv, lo32(fv), 1);
                    wv = wl(wv, hi32(fv), 2);
                    wv = wl(wv, lo32(pvv), 3);
                    wv = wl(wv, hi32(pvv), 4);
                    sel_put<FAST>(grS + 8, 0, atag, wv, SEL_NGS);
                }
                unsigned y[SEL_NGS];
                if (!sel_gather<SEL_NGS>(grS + 8, 1, atag, y, &ctlv->bar_timeout, spin)) {
                    status = LP_DEVICE_ERROR;
                    break;
                }
                Cn = (long long)rl32(y[0], 0);
                f0 = rl_d(y[1], y[2], 0);
                pcw = rl_d(y[3], y[4], 0);
            }
            C = Cn;
            SEL_DONE(pcw);
            SEL_CLK(19);
            if (C == NONE) status = stop ? LP_OBJ_INCREASED : capped ? LP_CAP_REACHED : LP_OPTIMAL;
        }
        SEL_CLK(0);
    }
#ifdef LPK_STAMPS
    if (A.stamps && lane == 0 && shard == 0) {
        long long *o = A.stamps + BMAX * 16 + (long long)b * 32;
        for (int k = 0; k < 16; ++k) o[k] = (long long)clk_[k];
        for (int k = 16; k < 24; ++k) o[20 + k - 16] = (long long)clk_[k];   // XR, sub-phases
        o[16] = ndone;
        o[17] = (long long)(__builtin_amdgcn_s_memrealtime() - clk_r0);   // 100 MHz ticks of the pivots
        o[18] = (long long)(clk_t - 0);
    }
#endif
    // the sweep's copy of the launch's multipliers (MQ, 4-row quads), column 0
    // of the own rows, row 0 on the own columns and its corner: read after
    // the launch
    {
        const int nds = __builtin_amdgcn_readfirstlane(ndone);
        if (nds > 0) SEL_SETTLE(nds - 1);
#pragma unroll
        for (int s = 0; s < NB; ++s)
            if (s < nds && own) {
                const d16 &mk = (s >> 4) == 0 ? m0 : (s >> 4) == 1 ? m1 : (s >> 4) == 2 ? m2 : m3;
                *gp(&MQv[mq(li, s)]) = mk[s & 15];
            }
        if (own) *gp(&col0v[li]) = lcv;
#pragma unroll
        for (int k = 0; k < IPL; ++k)
            if (cok[k]) *gp(&row0v[jk[k]]) = l0v[k];
        if (b == 0 && lane == 0) {
            *gp(&row0v[0]) = v0;
            *gp(&col0v[0]) = v0;
        }
    }
    if ((XR || XS) && b == 0 && lane == 0 && shard == 0) {
        *gp(&ctl->xwait_ticks) += xwait;
        *gp(&ctl->xwait_pivots) += ndone;
    }
    if (b == 0 && lane == 0) {
        // an increase at the launch's last pivot: nothing read the flag yet
        if (stop && status == LP_PIVOTED) status = LP_OBJ_INCREASED;
        if (status != LP_PIVOTED) st_sc1(&ctl->status, status);
    }
}

}  // namespace

template <int IPL, int NB, bool XR, bool XS>
__global__ void __launch_bounds__(GROUP_THREADS)
k_sel(Args A, int gper, int grp, int count, int from_erec, unsigned seq, int first, int fmode, int frule,
      long long fcap)
{
    static_assert(NB % 16 == 0 && NB <= BMAX, "k_sel: pivots per launch");
    // the grid is 8 x G.  One XCD: only blocks 0, 8, 16, ... work -- they share
    // one XCD under the round-robin dealing of workgroups (checked below).
    // XS: every block works, block 8 b + x being block b of shard x (so each
    // shard's blocks share one XCD, checked below, and each XCD holds one shard)
    // (A.xtarget >= 0: the blocks that land on XCD xtarget work instead -- the
    // same G blocks b = blockIdx.x / 8 under the round-robin dealing, on an
    // XCD the host chose: ranks sharing one GPU take different ones)
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    if (!XS && (A.xtarget < 0 ? (blockIdx.x & 7u) != 0u : xcc != (unsigned)A.xtarget)) return;
    extern __shared__ __attribute__((aligned(16))) double lP[];   // [cpb][NB + 2]: P[s][own column]
    const unsigned b = blockIdx.x >> 3, G = (unsigned)gper;
    const unsigned shard = XS ? (blockIdx.x & 7u) : 0u;
    const int lane = threadIdx.x;
    Ctl *const ctl = A.ctl;
    const bool reset = (first & 1) != 0;
    if (b == 0 && lane == 0 && shard == 0) *gp(&ctl->ndef[grp]) = 0;
    if (!reset && (ld_sc1(&ctl->status) != LP_PIVOTED || ld_sc1(&ctl->bar_timeout) != 0u)) return;
    long long npiv = reset ? 0 : ld_sc1(&ctl->npiv);
    int rule = reset ? frule : ld_sc1(&ctl->rule);
    long long nstd = 0, stuck = 0;
    if (!reset) {
        nstd = ld_sc1(&ctl->nstd);
        stuck = ld_sc1(&ctl->stuck);
    }
    rule = __builtin_amdgcn_readfirstlane(rule);
    if (lane == 0 && shard == 0) {
        // the loop state before this group: what a timed-out group is redone from
        st_sc1(&ctl->g_npiv, npiv);
        st_sc1(&ctl->g_nstd, nstd);
        st_sc1(&ctl->g_stuck, stuck);
        st_sc1(&ctl->g_rule, rule);
        st_sc1(&ctl->g_seq, seq);
    }
    {
        // every block publishes its XCD.  The hand-offs are plain stores that
        // stay in the XCD's L2, correct only if every block (of the shard)
        // runs there: if not (never seen), the group is abandoned like a
        // timed-out one and the host redoes it on the per-pivot kernels
        // (lpgpu.cpp recover_timeout).  (The eager row-0 copies of a call's
        // first launch are drained by its entering-column exchange, not by
        // this one.)
        // (what is compared: the XCD and the block's residue mod 8, so that
        // under XCD targeting the G working blocks are also one residue class,
        // i.e. b = 0 .. G - 1 each exactly once)
        unsigned me = xcc | ((blockIdx.x & 7u) << 8);
        if (A.fault_xcc && b == min(1u, G - 1) && shard == 0) me ^= 1u;   // tests: a misplaced block
        u64 *const grX = A.gran + (XS ? (long long)shard * GRAN_SHARD : 0) + 2 * GROUP_MAXBLOCKS * GSLOT;
        drain_stores();
        if (lane == 0) st_sc1(&grX[b], ((u64)gtag(seq, 0, 7) << 32) | me);
        unsigned wx[1];
        if (!sel_gather<1>(grX, min(G, 64u), gtag(seq, 0, 7), wx, &ctl->bar_timeout, A.spin_max)) {
            if (b == 0 && lane == 0) st_sc1(&ctl->status, (int)LP_DEVICE_ERROR);
            return;
        }
        bool same = !((unsigned)lane < G) || wx[0] == me;
        if (!wall(same)) {
            if (b == 0 && lane == 0) {
                *gp(&ctl->sel_flags) = 8u | 4u;
                st_sc1(&ctl->bar_timeout, 1u);
            }
            return;
        }
    }
    // diagnostics: 1 one XCD, 4 k_sel, 16 XCD shards
    if (b == 0 && lane == 0 && shard == 0) *gp(&ctl->sel_flags) = XS ? (16u | 4u) : (1u | 4u);
    sel_body<IPL, NB, XR, true, XS>(A, b, G, grp, count, from_erec, seq, first, fmode, fcap, lP, npiv, nstd, stuck,
                                    rule, shard);
}

// ---- geometry and launch ----------------------------------------------------
namespace {

const void *sel_kernel(int ipl, int nb, bool xr, bool xs)
{
#define SEL_K(I, N) (xr ? reinterpret_cast<const void *>(&k_sel<I, N, true, false>) \
                        : reinterpret_cast<const void *>(&k_sel<I, N, false, false>))
#define SEL_XS(I) reinterpret_cast<const void *>(&k_sel<I, 64, false, true>)
#define SEL_XR_XS(I) reinterpret_cast<const void *>(&k_sel<I, 64, true, true>)
    if (xs && xr) return nb != 64 ? nullptr : ipl == 1 ? SEL_XR_XS(1) : ipl == 2 ? SEL_XR_XS(2) : SEL_XR_XS(4);
    if (xs) return nb != 64 ? nullptr : ipl == 1 ? SEL_XS(1) : ipl == 2 ? SEL_XS(2) : SEL_XS(4);
    if (nb == 32) return ipl == 1 ? SEL_K(1, 32) : ipl == 2 ? SEL_K(2, 32) : SEL_K(4, 32);
    return ipl == 1 ? SEL_K(1, 64) : ipl == 2 ? SEL_K(2, 64) : SEL_K(4, 64);
#undef SEL_XR_XS
#undef SEL_XS
#undef SEL_K
}

int sel_per_cu(const void *fn, size_t lds)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, GROUP_THREADS, lds) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    // every block's LDS rounded up to 2 KB (allocation granule and slack),
    // one block less than the runtime's answer unless LDS is the limit
    // (kernels.hip group_per_cu)
    const long long per = ((long long)lds + 2047) / 2048 * 2048;
    const long long lds_cap = (long long)(160 * 1024) / per;
    if (n >= lds_cap) return (int)lds_cap;
    return n - 1;
}

}  // namespace

GroupGeom sel_geom(long long rc, long long n, int bmax, int xcd_cus, bool xr, bool xs_ok, int share)
{
    GroupGeom G;
    static const int on = [] {
        const char *v = std::getenv("LPGPU_SEL");   // A/B: 0 = k_group only
        return v ? std::atoi(v) : 1;
    }();
    if (!on || rc < 1 || n < 1 || bmax < 1 || bmax > BMAX) return G;
    // one XCD, or (too tall for one: more than 64 x 64 rows) XS_SHARDS row
    // shards of rps rows, one per XCD, each shard's blocks over all columns
    int xs = 0;
    long long rps = rc;
    if ((rc + 63) / 64 > 64) {
        if (!xs_ok || bmax <= 32) return G;
        xs = XS_SHARDS;
        rps = (rc + XS_SHARDS - 1) / XS_SHARDS;
    }
    // the fewest blocks (g) with every lane at most 4 columns, or more where
    // a block's LDS (the pivot values of its columns) leaves too few blocks
    // per CU for g on one XCD
    const long long g0 = std::max((rps + 63) / 64, (n + 255) / 256);
    const int nb = bmax <= 32 ? 32 : 64;
    long long g = 0, cpb = 0;
    int ipl = 0, per_cu = 0;
    size_t lds = 0;
    bool bad = false;
    auto fits = [&](long long gc) {
        cpb = (n + gc - 1) / gc;
        ipl = (int)((cpb + 63) / 64);
        if (ipl == 3) ipl = 4;
        if (ipl > 4) return false;
        lds = ((size_t)cpb * (nb + 2) + 8) * sizeof(double);   // + the row chain's read-ahead slack
        const void *fn = sel_kernel(ipl, nb, xr, xs > 0);
        if (!fn) {
            bad = true;
            return false;
        }
        per_cu = sel_per_cu(fn, lds);
        if (std::getenv("LPGPU_GEOM_DEBUG"))
            fprintf(stderr, "sel_geom rc %lld n %lld bmax %d xs %d g %lld ipl %d lds %zu per_cu %d xcd_cus %d\n", rc,
                    n, bmax, xs, gc, ipl, lds, per_cu, xcd_cus);
        // blocks this launch and the co-located ranks' need on one XCD at once.
        // XCD shards: every block works, share x gc per XCD.  One XCD (each
        // co-located rank on its own, Args::xtarget): gc, plus one free slot --
        // the other ranks' grids deal 7 of every 8 blocks to XCDs they do not
        // work on, and those idle blocks (exiting at once) still need a slot
        // to pass through in dispatch order: with the XCD full, the other
        // rank's launch stalls there and never reaches its own XCD
        const long long need = xs ? gc * std::max(share, 1) : share > 1 ? gc + 1 : gc;
        return per_cu >= 1 && need <= (long long)per_cu * xcd_cus;
    };
    // XCD shards: 64 blocks first where they fit -- the shard's rows are few
    // (2/4-GPU ranks of cfg4: 1024 / 2048 per XCD), the columns are what a
    // lane's chain walks, and two columns per lane beat four: 8192 x 8192
    // 102.9k -> 109.4k, 16384 x 8192 77.7k -> 80.9k pivots/s (round 5,
    // scripts/geo_probe.py xs)
    if (xs && g0 < 64 && fits(64)) g = 64;
    for (long long gc = g0; g == 0 && !bad && gc <= 64; gc = gc < 64 && gc + 8 > 64 ? 64 : gc + 8)
        if (fits(gc)) g = gc;
    if (g == 0) return G;
    G.g = g;
    G.nr = 1;
    G.ipl = ipl;
    G.rpl = 1;
    G.xmode = 1;
    G.sel = nb;
    G.xs = xs;
    G.lds = lds;
    G.per_cu = per_cu;
    return G;
}

hipError_t launch_sel(hipStream_t s, const Args &A, const GroupGeom &geo, int grp, int count, int from_erec,
                      unsigned seq, int xr, int first, int fmode, int frule, long long fcap, hipEvent_t e0,
                      hipEvent_t e1)
{
    if (geo.g == 0 || geo.sel == 0 || count < 1 || count > geo.sel) return hipErrorInvalidValue;
    if (xr && (A.nranks > NRANK_MAX || !A.xbuf || !A.peer)) return hipErrorInvalidValue;
    if (geo.xs && geo.xs != XS_SHARDS) return hipErrorInvalidValue;
    if (A.rc > 64 * geo.g * (geo.xs ? XS_SHARDS : 1) || A.n > 64LL * geo.ipl * geo.g) return hipErrorInvalidValue;
    if (geo.nr != 1) return hipErrorInvalidValue;
    const void *fn = sel_kernel(geo.ipl, geo.sel, xr != 0, geo.xs > 0);
    if (!fn) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(geo.g * 8));
    Args a0 = A;
    int gper = (int)geo.g;
    void *args[] = {&a0, &gper, &grp, &count, &from_erec, &seq, &first, &fmode, &frule, &fcap};
    return launch_persistent(fn, grid, args, geo.lds, s, e0, e1);
}

}  // namespace lpk
