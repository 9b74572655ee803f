// Shared definitions of the HIP engine (device control block, kernel
// arguments, launch wrappers).  Not part of the public C-ABI (include/lpgpu.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lpgpu.h"

namespace lpk {

constexpr int MODE_RUN = 0;    // fixed rule, no stall logic (findPivot*, lp_run)
constexpr int MODE_SOLVE = 1;  // Simplex.solve semantics (simplex.py:110-148)

// k_ratio modes
constexpr int RATIO_FULL = 0;   // single device: publish per-block candidates
constexpr int RATIO_LOCAL = 1;  // sharded: also reduce this rank's minimum ratio
constexpr int RATIO_CHECK = 2;  // validate a given row (Simplex.pivot)

// where k_prow finds the leaving row
constexpr int RSRC_RECORDS = 0;  // combine k_ratio's per-block records
constexpr int RSRC_GIVEN = 1;    // dR[t] set by the caller (Tableau.pivot / Simplex.pivot)
constexpr int RSRC_SLOTS = 2;    // sharded: lowest row index offered in the gathered slots
constexpr int RSRC_BAND = 3;     // sharded, one exchange: band test on the slots' (l, q)

// internal status (never returned through the C-ABI): the one-exchange
// protocol met a near-tie straddling the tie band; the host redoes that
// pivot with the two-exchange protocol (oracle/sharded_model.py step 4)
constexpr int ST_STRADDLE = 3;

// k_pick modes (sharded)
constexpr int PICK_RATIO = 0;     // first local row within the tie band of the global min
constexpr int PICK_CHECK = 1;     // owner validates the requested row (Simplex.pivot)
constexpr int PICK_EXPLICIT = 2;  // owner contributes the requested row (Tableau.pivot)
constexpr int PICK_LOCAL = 3;     // first local row within the LOCAL band + (l, q)

constexpr int BMAX = 64;           // most pivots deferred into one sweep
constexpr int RATIO_THREADS = 256;
constexpr int RATIO_CHUNK = 256;   // rows per ratio block (one per thread)
constexpr int PROW_THREADS = 256;  // columns per pivot-row block (one per thread)

constexpr int ENTER_THREADS = 1024;
constexpr int SLOT_HDR = 8;        // doubles of header in front of an exchanged row

constexpr long long NONE = 0x7fffffffffffffffLL;

// multipliers are stored pivot-major: M[s * rows + li] is the value of
// (local row li, dC[s]) just before pivot s, so one pivot's multipliers of
// consecutive rows are contiguous (coalesced stores, wide scalar loads)
__host__ __device__ inline long long mi(long long rows, long long li, long long s)
{
    return s * rows + li;
}
constexpr int M_PAD = 64;          // doubles after each parity's M (wide loads past the last row)

// Device-resident control block: the pivot loop's whole state lives here so
// batches of pivots are enqueued without host round trips.
struct Ctl {
    int status;          // lp_status of the current step; LP_PIVOTED = keep going
    int mode;            // MODE_RUN / MODE_SOLVE
    int rule;            // lp_rule for the next selection
    int chain;           // 1: pivots follow each other in one call
    long long r, c;      // current pivot (global constraint index, variable index)
    long long npiv;      // pivots performed since the last reset
    long long nstd;      // of which with the standard rule (solve mode)
    long long stuck;     // steps_stuck (simplex.py:119)
    long long cap;       // pivot cap (< 0: none)
    long long ndef[2];   // pivots of the current group (by group parity) not yet swept
    double z0;           // obj_val at the start of solve (simplex.py:118)
    unsigned ticket;     // last-block ticket of k_ratio (LOCAL / CHECK modes)
    unsigned pad;
    unsigned bar[2];     // grid-barrier counters of k_group (by group parity)
    unsigned bar_timeout;// set if a k_group barrier gave up (never expected)
    unsigned sel_xcc;    // XCD of the last one-XCD k_group launch (0xff: spread); a
                         // pipelined sweep beside the next selection keeps off it
    unsigned long long tiles[2];  // pipelined sweep: next tile (by group parity; k_group zeroes it)
};

// Per-block ratio-test summary.
struct Rec {
    double l;            // block minimum ratio (INFINITY if no eligible row)
    long long i;         // first local row within the tie band of l
    double q;            // its ratio
    double pad;
};

// Per-block entering-column summary over a slice of row 0.
struct ERec {
    double l;            // slice minimum of c_j
    long long i;         // first column within the tie band of l
    double q;            // its value
    long long fneg;      // first column with c_j < -tol.cost
    long long rule;      // k_group: block 0 publishes the rule for the next pivot here
    long long pad[3];
};

// Deferred pivots: pivot s (0 <= s < ndef) of the current group is
//   (dR[s] local row or -1, dC[s] tableau column), multipliers M[i*BMAX + s]
//   = value of (i, dC[s]) just before pivot s, normalised row P[s*ld + j].
// The current value of any element is its stored value with pivots 0..t-1
// applied in order by upd() (kernels.hip) -- the sweep writes exactly that.
struct Args {
    double *T;           // local tableau: row 0 + local constraint rows
    double *row0;        // current row 0 (ld doubles)
    double *col0;        // current column 0 of the local rows (rows doubles)
    double *M;           // BMAX x rows multipliers, pivot-major (mi())
    double *P;           // BMAX x ld normalised pivot rows
    long long *dR;       // BMAX local pivot rows (-1: another rank's row)
    long long *dC;       // BMAX pivot columns (tableau index)
    Ctl *ctl;
    long long *log;      // (r, c) per pivot
    Rec *rec;
    ERec *erec;
    double *xg;          // sharded: this rank's / the global minimum ratio (1 double)
    double *xs;          // sharded: send slot (SLOT_HDR + ld)
    double *xr;          // sharded: gathered slots (nranks x (SLOT_HDR + ld))
    long long logcap;
    long long m, n;      // GLOBAL problem size
    long long ld;        // leading dimension of T, P, row0 (doubles)
    long long rows;      // local rows incl. row 0
    long long rb;        // first global constraint row of this rank
    long long rc;        // local constraint rows
    int nranks;
    int pad;
    lp_tol tol;
    long long *stamps;   // diagnostic build only (LPGPU_STAMPS=1): k_group phase clocks
    unsigned long long *gran;  // k_group summaries: 3 phases (ratio, row 0, XCD check) x GROUP_MAXBLOCKS x 8 tagged granules
    // pipelined groups (k_group only): the previous group's pivots are not yet
    // in T (its sweep runs concurrently); lag = 1 applies them on the fly first
    const double *Pp;    // previous group's P (BMAX x ld)
    const double *Mp;    // previous group's M
    const long long *dRp;// previous group's local pivot rows
    int lag;
    int rank;            // this rank (row-sharded jobs)
    // row-sharded persistent selection: this rank's exchange buffer and every
    // rank's (peer[rank] == xbuf), written by the peers over xGMI
    unsigned long long *xbuf;
    unsigned long long *const *peer;
};

// exchange buffer layout (granules of 8 bytes), see kernels.hip (XR)
constexpr int NRANK_MAX = 64;
constexpr long long XS_SUM_PAR = (NRANK_MAX + 1) * 8;            // per parity
constexpr long long XS_PROW = 2 * XS_SUM_PAR;
constexpr long long XS_PROW_BLOCK = 2 * 4 * 64;                   // 2 granules x 4 columns x 64 lanes
constexpr long long XS_PROW_RANK = 256 * XS_PROW_BLOCK;           // GROUP_MAXBLOCKS blocks per source rank
// + 2 parities x nranks x XS_PROW_RANK of pivot-row slices, then the local
// straddle slots
__host__ __device__ inline long long xs_granules(int nranks)
{
    return XS_PROW + 2LL * nranks * XS_PROW_RANK + 256 * 8;
}

// launch wrappers (kernels.hip).  t = index of the pivot within its group
// (known to the host, which enqueues the groups); grp = group parity.
hipError_t launch_reset(hipStream_t s, const Args &A, int mode, int rule, int chain, long long cap,
                        long long r, long long c);
hipError_t launch_load_eager(hipStream_t s, const Args &A);
hipError_t launch_enter(hipStream_t s, const Args &A);
hipError_t launch_ratio(hipStream_t s, const Args &A, int t, int grp, int mode, int from_erec,
                        long long check_local_row);
hipError_t launch_pick(hipStream_t s, const Args &A, int t, int mode);
hipError_t launch_gather(hipStream_t s, const Args &A, int t);
hipError_t launch_prow(hipStream_t s, const Args &A, int t, int grp, int rsrc, int peek);
// T_out <- A.T with the group's pivots (T_out == A.T: in place); nd_max >= ndef
// (e0, e1: events recorded at the kernel's start and end, for lp_profile)
hipError_t launch_sweep(hipStream_t s, const Args &A, int grp, int nd_max, double *T_out,
                        hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
// one persistent launch selecting up to `count` chained pivots of a group;
// seq numbers the launches of a handle (1 .. 2^24-1, then wraps to 1): it tags
// the launch's summaries so no stale granule can match
// xr: one rank of a row-sharded job (2: its selection may run on one XCD).
// As (device array of nshard Args): the
// in-process shards of one device, all in this one launch
hipError_t launch_group(hipStream_t s, const Args &A, int grp, int count, int from_erec,
                        unsigned seq, int bmax, int lag_layout, int xr = 0,
                        const Args *As = nullptr, int nshard = 1, hipEvent_t e0 = nullptr,
                        hipEvent_t e1 = nullptr);
// row-sharded: every rank writes a tagged granule to every rank's buffer and
// waits (bounded) for all of them; *ok = 1 if all arrived (peer exchange works)
hipError_t launch_peer_ping(hipStream_t s, const Args &A, unsigned tag, unsigned flags, int *ok_dev);
int group_fits(const Args &A, int bmax, int lag_layout, int xr, int nshard);
#ifndef LPK_GROUP_BLOCKS
#define LPK_GROUP_BLOCKS 64
#endif
#ifndef LPK_GROUP_ROWS
#define LPK_GROUP_ROWS 64
#endif
constexpr int GROUP_BLOCKS = LPK_GROUP_BLOCKS;   // co-resident workgroups of k_group (<= CUs) ...
constexpr int GROUP_MAXBLOCKS = 256;
constexpr int GROUP_ROWS = LPK_GROUP_ROWS;       // ... raised so a block owns at most this many rows
constexpr int GROUP_THREADS = 64;  // one wave: block reductions stay in registers
constexpr long long GROUP_LDS_MAX = 96 * 1024;
// dynamic LDS of one k_group block: per own row / own column the pivots'
// values at stride count + 1 (multipliers, pivot-row values; twice with a
// lagging previous group of up to `count` pivots) + row 0 / column 0 slices
__host__ __device__ inline long long group_lds(long long rc, long long ld, long long g, int count,
                                               int lag)
{
    const long long rpb = (rc + g - 1) / g, cpb = (ld + g - 1) / g;
    return ((rpb + cpb) * (count + 1) * (lag ? 2 : 1) + cpb + rpb + 8) * 8;   // + a chunk of slack
}
// workgroups of k_group for this shape, 0 if it does not fit (the per-pivot
// kernels are used instead): a block owns at most GROUP_ROWS rows (one per
// lane) and at most 4 columns per lane; a few extra blocks are taken when
// that brings every lane down to 2 columns
__host__ __device__ inline long long group_blocks(long long rc, long long ld, int count, int lag)
{
    if (ld >= 0x7fffffffLL || rc >= 0x7fffffffLL) return 0;   // indices travel as 31 bits
    long long g = (rc + GROUP_ROWS - 1) / GROUP_ROWS;
    if (g < GROUP_BLOCKS) g = GROUP_BLOCKS;
    const long long g2 = (ld + 2 * GROUP_THREADS - 1) / (2 * GROUP_THREADS);
    const long long g4 = (ld + 4 * GROUP_THREADS - 1) / (4 * GROUP_THREADS);
    if (g2 > g && g2 <= g + g / 8) g = g2;
    if (g4 > g) g = g4;
    while (g < GROUP_MAXBLOCKS && group_lds(rc, ld, g, count, lag) > GROUP_LDS_MAX) g *= 2;
    if (g > GROUP_MAXBLOCKS) g = GROUP_MAXBLOCKS;
    if ((ld + g - 1) / g > 4 * GROUP_THREADS) return 0;   // more than 4 columns per lane
    if ((rc + g - 1) / g > GROUP_ROWS) return 0;          // more than one row per lane
    return group_lds(rc, ld, g, count, lag) > GROUP_LDS_MAX ? 0 : g;
}
// k_group workgroups when they are all to run on ONE XCD (cus = its CUs; on
// unless LPGPU_SEL_XCD=0): at most GROUP_ROWS rows per block, at most 4
// columns per lane, and every block co-resident on those CUs (LDS-bound).
// 0 when the mode is off or the shape does not fit.
inline long long group_blocks_xcd(long long rc, long long ld, int count, int cus, int lag = 0)
{
    static int on = -1;
    if (on < 0) {
        const char *v = std::getenv("LPGPU_SEL_XCD");
        on = v ? std::atoi(v) : 1;
    }
    if (!on || cus <= 0 || ld >= 0x7fffffffLL || rc >= 0x7fffffffLL) return 0;
    long long g = (rc + GROUP_ROWS - 1) / GROUP_ROWS;
    const long long g4 = (ld + 4 * GROUP_THREADS - 1) / (4 * GROUP_THREADS);
    if (g4 > g) g = g4;
    if (g < 1) g = 1;
    if (g > GROUP_MAXBLOCKS) return 0;
    // blocks per CU: LDS-bound, and at most one single-wave block per SIMD
    // (k_group takes up to 256 VGPRs: one wave per SIMD is all that is sure)
    long long per_cu = 160 * 1024 / (group_lds(rc, ld, g, count, lag) + 4096);   // + static LDS
    if (per_cu > 4) per_cu = 4;
    return per_cu >= 1 && g <= per_cu * cus ? g : 0;
}
// group_blocks_xcd for this device (0: the shape does not fit one XCD)
long long group_blocks_xcd_here(long long rc, long long ld, int count, int lag);
// can the pipelined mode's lagging selection share the device with the sweep?
int pipeline_fits(long long rc, long long ld, int count);
hipError_t launch_group_min(hipStream_t s, double *const *ptrs, int n);

// per-column statistics of the local constraint rows (row 0 excluded)
struct ColStat {
    double gmin;         // minimum ratio over rows with a > tol.pivot (INFINITY: none)
    long long npos;      // rows with a > tol.pivot
    long long npos0;     // rows with a > 0
    long long nnz;       // rows with a != 0
    long long none;      // rows with a == 1
    long long one_row;   // first such row (global constraint index) or NONE
    long long nneg;      // rows with a < 0
    long long pad;
};
hipError_t launch_colstat(hipStream_t s, const Args &A, ColStat *out);   // out[ld]
hipError_t launch_colband(hipStream_t s, const Args &A, const double *thr, long long *first,
                          long long *count, const long long *offs, long long *pairs);
hipError_t launch_rowpos(hipStream_t s, const Args &A, int *rowpos);     // rowpos[rc]
hipError_t launch_resume(hipStream_t s, const Args &A);
__host__ __device__ inline int ratio_blocks(long long rows)
{
    return (int)((rows - 1 + RATIO_CHUNK - 1) / RATIO_CHUNK);
}
__host__ __device__ inline int prow_blocks(long long ld)
{
    return (int)((ld + PROW_THREADS - 1) / PROW_THREADS);
}

}  // namespace lpk
