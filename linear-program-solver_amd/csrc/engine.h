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

// multipliers: M[mi(rows, li, s)] is the value of (local row li, dC[s]) just
// before pivot s, pivot-major: one pivot's multipliers of consecutive rows are
// contiguous (the selection stores a pivot's column with one coalesced store
// per 64 rows).
__host__ __device__ inline long long mi(long long rows, long long li, long long s)
{
    return s * rows + li;
}
// The sweep's copy MQ (written by the selection at the end of each group, from
// the multipliers it keeps in LDS): 4-row quads, quad q = rows 4q..4q+3 holds
// its BMAX pivots x 4 rows contiguously, pivot-major inside (s * 4 + row % 4),
// so a sweep batch (4 rows, aligned) finds a 4-pivot chunk of its multipliers
// in ONE 128-byte line (cfg4 sweep 1106 -> 1046 us per 64-pivot launch,
// scripts/sweep_probe.hip: 1088-1100 -> 1031-1039).  Selection stores in this
// layout per pivot (64 rows -> 16 lines) cost 0.6 us per pivot at cfg4.
__host__ __device__ inline long long mq(long long li, long long s)
{
    return (li >> 2) * (4LL * BMAX) + s * 4 + (li & 3);
}
// doubles of MQ: whole quads (a batch's loads past the last row stay inside
// its quad)
__host__ __device__ inline long long mq_len(long long rows) { return (rows + 3) / 4 * 4 * BMAX; }
constexpr int M_PAD = 64;          // doubles after each parity's M

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
    unsigned bar[2];     // unused (kept zero)
    unsigned bar_timeout;// set if a k_group exchange gave up (never expected)
    unsigned sel_flags;  // the last persistent selection launch (block 0): 1 every block on one XCD,
                         // 2 the two-level exchange engaged (k_group), 4 the one-XCD kernel k_sel ran,
                         // 8 k_sel found its blocks on several XCDs (group abandoned, redone by the host)
    // k_group: the loop state at the start of the launch (every block writes
    // the same values before any pivot of the group: a timeout is only seen
    // by a block that ran, so the snapshot is always the failing launch's,
    // and later launches of the batch return at once); after it the host
    // restores it and redoes the group on the per-pivot kernels (the sweep
    // of a timed-out group is skipped, so T still holds the group's start)
    long long g_npiv, g_nstd, g_stuck;
    int g_rule;
    unsigned g_seq;      // the launch (seq) the snapshot belongs to; 0: none
    // row-sharded persistent selection (XR): block 0's time from sending its
    // summary to holding the winner's pivot row, summed over the handle's
    // pivots (100 MHz real-time ticks), and those pivots (lp_xwait)
    unsigned long long xwait_ticks;
    long long xwait_pivots;
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
    double *MQ;          // the sweep's copy of M in 4-row quads (mq())
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
    int gmaj;            // k_group: granule-major summaries when on one XCD (1, default) or never (0)
    lp_tol tol;
    long long *stamps;   // diagnostic build only (LPGPU_STAMPS=1): k_group phase clocks
    // persistent selections' summaries: GRAN_REGIONS regions of GROUP_MAXBLOCKS x GSLOT (8)
    // tagged granules -- ratio, row 0, XCD check, and the fourth: k_group's
    // two-level exchange (8 ratio + 8 row-0 level-2 slots) / k_sel's rescan
    // and owner answers
    unsigned long long *gran;   // GRAN_TOTAL granules (below)
    unsigned spin_max;   // k_group: polls of one exchange before it gives up (timeout)
    unsigned xwait_ms;   // k_group (XR): wall-clock bound of a cross-rank wait
    int fault;           // tests only (LPGPU_FAULT): t + 1 -> block 1 withholds pivot t's ratio summary
    int hier;            // k_group: two-level exchange when the blocks are spread over the XCDs (1) or flat (0)
    int rank;            // this rank (row-sharded jobs)
    // one-XCD k_sel (not XS): -1 the blocks 0, 8, 16, ... work (whichever XCD
    // block 0 lands on); 0..7 the blocks that find themselves on XCD xtarget
    // work -- ranks sharing one GPU each take their own XCD (lpgpu.cpp)
    int xtarget;
    // ranks of this job sharing this rank's GPU (tests, rehearsals; 1 in a
    // real multi-GPU job): launch_sweep keeps the 8-wave pass there
    int share;
    int fault_xcc;       // tests only (LPGPU_FAULT_XCC): block 1 (shard 0) reports another XCD
    // row-sharded persistent selection: this rank's exchange buffer and every
    // rank's (peer[rank] == xbuf), written by the peers over xGMI
    unsigned long long *xbuf;
    unsigned long long *const *peer;
    // out-of-place sweep (k_sweep_rl, LPGPU_SWEEP_OOP): the pass reads T and
    // writes Tout (the handle's other tableau buffer; Tout == T: in place), and
    // block 0 of a sweep that ran stores flipseq into *dflips -- the host's
    // record of which buffer holds the tableau after a batch (a sweep skipped
    // because the solve ended or a group timed out leaves the previous one)
    double *Tout;
    unsigned *dflips;
    unsigned flipseq;
    // per-launch clocks of the sweep (k_sweep_rl, block 0): launch lseq writes
    // entry lseq % SWEEP_CLK_RING = {lseq, shader cycles, 100 MHz ticks, start
    // tick} of its block 0's pass -- the shader clock during each launch
    // (lpdiag_sweep_clocks, bench.py, scripts/sweep_clock.py)
    unsigned long long *sweep_clk;
    unsigned sweep_lseq;
};
constexpr int SWEEP_CLK_RING = 1024;
// after the ring: per block of the latest launch {lseq, start tick, pass-end
// tick, shader cycles of the pass} (lpdiag_sweep_block_clocks)
constexpr int SWEEP_BLK_MAX = 8192;

// exchange buffer layout (granules of 8 bytes), see kernels.hip (XR)
constexpr int NRANK_MAX = 64;
constexpr long long XS_SUM_PAR = (NRANK_MAX + 1) * 8;            // per parity
// the summary slots in XS_SHARDS replicas, one per XCD shard of a rank that
// runs k_sel<XR, XS> (every other selection kernel uses replica 0)
constexpr long long XS_XREP = 2 * XS_SUM_PAR;
constexpr long long XS_PROW = 8 * XS_XREP;
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
// T <- T with the group's pivots (k_sweep_rl with A.Tout != A.T: into Tout,
// *flipped = true; every other sweep in place); nd_max >= ndef: the handle's
// pivots per sweep; cnt (> 0): the most pivots this group can hold, when the
// host knows it (a call's last group, an explicit pivot) -- a shallower
// kernel then, or the padded k_sweep_rl (e0, e1: events recorded at the
// kernel's start and end, for lp_profile)
hipError_t launch_sweep(hipStream_t s, const Args &A, int grp, int nd_max, int cnt = -1, hipEvent_t e0 = nullptr,
                        hipEvent_t e1 = nullptr, bool *flipped = nullptr);

constexpr int GROUP_MAXBLOCKS = 256;
constexpr int GRAN_REGIONS = 4;       // regions of Args::gran (see there)
// Args::gran: one set of GRAN_REGIONS regions of GROUP_MAXBLOCKS x 8 granules
// per XCD shard of the XCD-sharded selection (k_sel<XS>, select.hip; every
// other persistent selection uses set 0), then the shards' common region
// (their leaving-row summaries and straddle answers)
constexpr int XS_SHARDS = 8;          // XCD shards of one device (MI355X: 8 XCDs)
constexpr long long GRAN_SHARD = (long long)GRAN_REGIONS * GROUP_MAXBLOCKS * 8;
// common region: one replica per reading shard, XS_READER_STRIDE apart (a
// summary polled by 64 blocks per line instead of 512 all on one line)
constexpr long long XS_READER_STRIDE = 1032;
constexpr long long GRAN_TOTAL = (XS_SHARDS + 2) * GRAN_SHARD;
constexpr int GROUP_MINBLOCKS = 64;    // a small tableau still spreads its columns over 64 blocks
constexpr int GROUP_THREADS = 64;      // one wave: block reductions stay in registers
constexpr int GROUP_MAXRPL = 4;        // own rows per lane (<= 64 x 256 x 4 = 65536 rows per device, as LDS allows)
constexpr long long GROUP_LDS_MAX = 96 * 1024;
// dynamic LDS of one k_group block: per own row / own column the pivots'
// values at stride count + 1 (multipliers, pivot-row values) + row 0 /
// column 0 slices
__host__ __device__ inline long long group_lds(long long rc, long long ld, long long g, int count)
{
    const long long rpb = (rc + g - 1) / g, cpb = (ld + g - 1) / g;
    return ((rpb + cpb) * (count + 1) + cpb + rpb + 8) * 8;   // + a chunk of slack
}

// Geometry of one persistent selection launch (k_group), decided on the host
// from the compiled kernel's occupancy (group_geom, kernels.hip).  g == 0:
// the shape does not fit (the per-pivot kernels are used instead).
struct GroupGeom {
    long long g = 0;     // workgroups (one wave each) per shard
    int nr = 1;          // summaries per lane (g <= 64 nr)
    int ipl = 2;         // own columns per lane (cpb <= 64 ipl)
    int rpl = 1;         // own rows per lane (rpb <= 64 rpl)
    int xmode = 0;       // 1: every block on ONE XCD (grid 8 g, blocks 0, 8, 16, ...)
    int hk = 0;          // 1: blocks spread over the XCDs, the k_group variant with the two-level exchange
    size_t lds = 0;      // dynamic LDS per block
    int per_cu = 0;      // resident blocks per CU the launch relies on
    int sel = 0;         // > 0: the one-XCD selection k_sel (select.hip) for up to `sel` pivots per launch
    int xs = 0;          // > 0: k_sel split into `xs` row shards, one per XCD, in one launch (g blocks each)
};
// rc: local constraint rows (the largest shard's for a sharded job); bmax:
// pivots per group; xr: 0 single device, 1 row-sharded rank, 2 row-sharded
// rank that may use one XCD; nshard: in-process shards in one launch; share:
// processes whose launches must be resident on this device at the same time;
// xs_ok: a single-device tableau too tall for one XCD may take k_sel's XCD
// shards (else k_group).
GroupGeom group_geom(long long rc, long long ld, long long n, int bmax, int xr, int nshard, int share,
                     bool xs_ok = true);
// the one-XCD selection (select.hip): g <= 64 blocks, one own row per lane,
// the variable columns 1..n split evenly; g == 0 if the shape does not fit.
// xs_ok (single device): a tableau too tall for one XCD may run as XS_SHARDS
// row shards of <= 64 g rows, one per XCD, in one launch (geo.xs)
// share: ranks of a job on this GPU whose launches must be resident together
// (XR; the one-XCD kernel puts each on its own XCD, Args::xtarget, the XCD
// shards need share x g blocks on every XCD)
GroupGeom sel_geom(long long rc, long long n, int bmax, int xcd_cus, bool xr, bool xs_ok, int share = 1);
hipError_t launch_sel(hipStream_t s, const Args &A, const GroupGeom &geo, int grp, int count, int from_erec,
                      unsigned seq, int xr, int first, int fmode, int frule, long long fcap, hipEvent_t e0,
                      hipEvent_t e1);
// one persistent launch selecting up to `count` chained pivots of a group;
// seq numbers the launches of a handle (1 .. 2^23-1, then wraps to 1): it tags
// the launch's summaries so no stale granule can match.  xr: one rank of a
// row-sharded job.  As (device array of nshard Args): the in-process shards
// of one device, all in this one launch.  first: see k_group (call start).
hipError_t launch_group(hipStream_t s, const Args &A, const GroupGeom &geo, int grp, int count,
                        int from_erec, unsigned seq, int bmax, int xr, const Args *As, int nshard,
                        int first, int fmode, int frule, long long fcap, hipEvent_t e0 = nullptr,
                        hipEvent_t e1 = nullptr);
// a persistent selection launch (cooperative unless LPGPU_COOP=0)
hipError_t launch_persistent(const void *fn, dim3 grid, void **args, size_t lds, hipStream_t s, hipEvent_t e0,
                             hipEvent_t e1);
// row-sharded: every rank writes a tagged granule to every rank's buffer and
// waits (bounded) for all of them; *ok = 1 | flags OR << 1 if all arrived
hipError_t launch_peer_ping(hipStream_t s, const Args &A, unsigned tag, unsigned flags, int *ok_dev);
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
