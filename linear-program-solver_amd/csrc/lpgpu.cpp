// liblpgpu.so: host side of the C-ABI declared in include/lpgpu.h.
//
// Owns device memory, the HIP stream and the device-resident pivot loop.  A
// pivot never round-trips to the host: the host enqueues batches of pivot
// launches and reads only the control block back between batches.
//
// Row sharding: a handle may be one shard of a row-partitioned tableau.  The
// shards exchange two messages per pivot through a Comm:
//   allreduce-min of the local minimum ratio (8 B)   -> every rank knows g
//   allgather of one slot per rank (header + row)    -> every rank knows the
//                                                       leaving row and P
// Comm has two transports: RCCL (one process per GPU, production) and an
// in-process group of shards on one device (the test-suite uses it to prove
// that the pivot sequence does not depend on the shard count).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "engine.h"
#include "../../include/lpgpu_diag.h"

using lpk::Args;
using lpk::Ctl;
using lpk::Rec;

struct Comm;

struct lp_handle {
    int dev = 0;
    hipStream_t s = nullptr;
    bool own_stream = true;
    int64_t m = 0, n = 0, ld = 0;   // global problem
    int64_t rb = 0, rc = 0;         // local constraint block [rb, rb+rc)
    int64_t rows = 0;               // local rows = rc + 1
    double *T = nullptr, *P = nullptr, *M = nullptr, *MQ = nullptr, *row0 = nullptr, *col0 = nullptr;
    // out-of-place sweeps (LPGPU_SWEEP_OOP): two tableau buffers, T is the
    // current one -- Tb[flips & 1] after `flips` sweeps that wrote the other
    // (dflips: the device's record of the last one that ran, read at each sync)
    double *Tb[2] = {nullptr, nullptr};
    unsigned *dflips = nullptr;
    unsigned flips = 0, hflips = 0;
    unsigned long long *sweep_clk = nullptr;   // lpk::SWEEP_CLK_RING x 4 (Args::sweep_clk)
    unsigned sweep_lseq = 0;                // k_sweep_rl launches so far
    bool oop = false;
    long long *dR = nullptr, *dC = nullptr;
    lpk::ERec *erec = nullptr;
    int block = 0;                  // pivots deferred into one sweep (1..BMAX; 0 = auto)
    int block_auto = 0;             // the auto choice for this handle's shape (0: not yet made)
    bool persistent = true;         // one k_group launch per group where the shape fits
    int fallbacks = 0;              // timed-out persistent groups redone on the per-pivot kernels
    long long *stamps = nullptr;    // diagnostic phase clocks (LPGPU_STAMPS=1)
    unsigned long long *gran = nullptr;  // k_group summaries (tagged granules)
    unsigned gseq = 0;              // k_group launches so far (tags their summaries)
    unsigned spin_max = 1u << 22;   // polls of one k_group exchange before it gives up
    unsigned xwait_ms = 30000;      // bound of a cross-rank wait (XR)
    int fault_launch = 0, fault_t = 0;   // tests: LPGPU_FAULT=<launch>:<pivot>
    int fault_xcc = 0;              // tests: LPGPU_FAULT_XCC=<launch> (a block of k_sel reports another XCD)
    bool strict = false;            // LPGPU_STRICT=1 (tests): a timed-out group is an error
    bool xs_ok = true;              // a tall single-device tableau may take k_sel's XCD shards
                                    // (LPGPU_SEL_XS=0 / lpdiag_set_xcd_shards: k_group instead)
    // row-sharded persistent selection: device-side exchange between ranks
    unsigned long long *xbuf = nullptr;     // this rank's exchange buffer (peers write it)
    unsigned long long **dpeer = nullptr;   // device table: every rank's buffer
    std::vector<void *> ipc_open;           // peer buffers opened from IPC handles
    bool peer_ok = false;                   // the exchange is set up and validated
    bool xbuf_fine = false;                 // the exchange buffer is fine-grained device memory
    bool xr_xcd = false;                    // every rank on its own GPU: one-XCD selection
    int xtarget = -1;                       // k_sel's XCD when ranks share a GPU (Args::xtarget)
    int share = 1;                          // most ranks of the job on one GPU (from the ping)
    bool peer_enable = true;                // LPGPU_PEER=0 keeps the RCCL per-pivot path
    int last_path = 0;                      // lp_exchange_path of the last pivot loop
    hipStream_t sx = nullptr;               // in-process shards: own stream for the persistent launch
    // column scans / form checks (allocated on first use)
    lpk::ColStat *cstat = nullptr;
    double *cthr = nullptr;
    long long *cfirst = nullptr, *ccount = nullptr, *coffs = nullptr;
    int *rowflag = nullptr;
    bool eager_ok = false;          // row0/col0 mirror the stored tableau
    Ctl *ctl = nullptr;
    Ctl *hctl = nullptr;            // pinned mirror
    long long *log = nullptr;
    int64_t logcap = 0;
    Rec *rec = nullptr;
    double *xg = nullptr, *xs = nullptr, *xr = nullptr;   // sharded exchange buffers
    lp_tol tol{};
    bool prof = false;
    int prof_every = 1;             // time every prof_every-th launch of each kind
    int64_t prof_seen[2] = {0, 0};  // launches of each kind since lp_profile
    std::vector<hipEvent_t> ev;     // pairs (start, end) of update launches
    size_t evused = 0;
    std::vector<int> evkind;        // per pair: 0 sweep, 1 selection (k_group)
    double prof_ms = 0.0;
    int64_t prof_n = 0;
    double sel_ms = 0.0;            // k_group launches
    int64_t sel_n = 0;
    int rank = 0, nranks = 1;
    std::shared_ptr<Comm> comm;     // null: single device, no exchange
    std::string err;
};

static std::string g_create_err;

#define HCHK(h, expr)                                                              \
    do {                                                                           \
        hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess) {                                                    \
            (h)->err = std::string(#expr) + ": " + hipGetErrorString(e_);          \
            return LP_DEVICE_ERROR;                                                \
        }                                                                          \
    } while (0)

#define NCHK(h, expr)                                                              \
    do {                                                                           \
        ncclResult_t e_ = (expr);                                                  \
        if (e_ != ncclSuccess) {                                                   \
            (h)->err = std::string(#expr) + ": " + ncclGetErrorString(e_);         \
            return LP_DEVICE_ERROR;                                                \
        }                                                                          \
    } while (0)

#define CALL(expr)                                                                 \
    do {                                                                           \
        const int st_ = (expr);                                                    \
        if (st_ != LP_PIVOTED) return st_;                                         \
    } while (0)

static int fail(lp_handle *h, int code, const std::string &msg)
{
    h->err = msg;
    return code;
}

static int64_t slot_len(const lp_handle *h) { return lpk::SLOT_HDR + h->ld; }

// ---------------------------------------------------------------------------
// transports
// ---------------------------------------------------------------------------

using Members = std::vector<lp_handle *>;

struct Comm {
    virtual ~Comm() {}
    // the handles whose pivot loops this process drives in lock-step
    virtual Members members(lp_handle *h) = 0;
    virtual int allreduce_min(const Members &M) = 0;   // xg, one double, in place
    virtual int allgather(const Members &M) = 0;       // xs -> xr
};

// One process per rank.  The per-pivot exchanges use the RCCL communicator
// when there is one; a handle created without a unique id (or whose peers
// share a GPU, which RCCL refuses) can instead be given the host's own
// all-gather (lp_set_host_allgather: gloo, MPI, ...), which the per-pivot
// path then calls synchronously through pinned staging buffers.
struct RcclComm : Comm {
    ncclComm_t comm = nullptr;      // null: peer exchange / host collective only
    lp_allgather_fn host_fn = nullptr;
    void *host_ctx = nullptr;
    std::vector<unsigned char> hs, hr;   // staging for host_fn
    ~RcclComm() override
    {
        if (comm) ncclCommDestroy(comm);
    }
    Members members(lp_handle *h) override { return Members{h}; }
    // all-gather of `bytes` host bytes per rank into recv (rank order)
    int gather_host(lp_handle *h, const void *send, void *recv, size_t bytes)
    {
        if (host_fn) {
            if (host_fn(host_ctx, send, recv, (int64_t)bytes) != 0)
                return fail(h, LP_DEVICE_ERROR, "host all-gather failed");
            return LP_PIVOTED;
        }
        if (!comm) return fail(h, LP_DEVICE_ERROR, "no RCCL communicator and no host all-gather");
        unsigned char *d = nullptr;
        HCHK(h, hipMalloc(&d, bytes * (h->nranks + 1)));
        int st = LP_PIVOTED;
        if (hipMemcpyAsync(d, send, bytes, hipMemcpyHostToDevice, h->s) != hipSuccess ||
            ncclAllGather(d, d + bytes, bytes, ncclUint8, comm, h->s) != ncclSuccess ||
            hipMemcpyAsync(recv, d + bytes, bytes * h->nranks, hipMemcpyDeviceToHost, h->s) != hipSuccess ||
            hipStreamSynchronize(h->s) != hipSuccess)
            st = fail(h, LP_DEVICE_ERROR, "RCCL all-gather of column statistics failed");
        (void)hipFree(d);
        return st;
    }
    int allreduce_min(const Members &M) override
    {
        lp_handle *h = M[0];
        if (comm) {
            NCHK(h, ncclAllReduce(h->xg, h->xg, 1, ncclFloat64, ncclMin, comm, h->s));
            return LP_PIVOTED;
        }
        if (!host_fn) return fail(h, LP_DEVICE_ERROR, "no RCCL communicator and no host all-gather");
        double v = 0.0;
        std::vector<double> all(h->nranks);
        HCHK(h, hipMemcpyAsync(&v, h->xg, sizeof(double), hipMemcpyDeviceToHost, h->s));
        HCHK(h, hipStreamSynchronize(h->s));
        CALL(gather_host(h, &v, all.data(), sizeof(double)));
        for (double x : all) v = std::min(v, x);
        HCHK(h, hipMemcpyAsync(h->xg, &v, sizeof(double), hipMemcpyHostToDevice, h->s));
        HCHK(h, hipStreamSynchronize(h->s));
        return LP_PIVOTED;
    }
    int allgather(const Members &M) override
    {
        lp_handle *h = M[0];
        const size_t bytes = (size_t)slot_len(h) * sizeof(double);
        if (comm) {
            NCHK(h, ncclAllGather(h->xs, h->xr, (size_t)slot_len(h), ncclFloat64, comm, h->s));
            return LP_PIVOTED;
        }
        if (!host_fn) return fail(h, LP_DEVICE_ERROR, "no RCCL communicator and no host all-gather");
        hs.resize(bytes);
        hr.resize(bytes * h->nranks);
        HCHK(h, hipMemcpyAsync(hs.data(), h->xs, bytes, hipMemcpyDeviceToHost, h->s));
        HCHK(h, hipStreamSynchronize(h->s));
        CALL(gather_host(h, hs.data(), hr.data(), bytes));
        HCHK(h, hipMemcpyAsync(h->xr, hr.data(), hr.size(), hipMemcpyHostToDevice, h->s));
        HCHK(h, hipStreamSynchronize(h->s));
        return LP_PIVOTED;
    }
};

struct GroupComm : Comm {
    Members all;                   // every shard, rank order
    double **dptrs = nullptr;      // device array of the shards' xg pointers
    // the shards' kernel arguments, two slots by group parity (out-of-place
    // sweeps change them from group to group): a device array each, staged
    // from pinned host memory, and the event of each slot's last copy -- a
    // slot is rewritten only after that copy has run
    Args *dargs = nullptr;
    Args *hargs = nullptr;
    hipEvent_t staged[2] = {nullptr, nullptr};
    hipStream_t s = nullptr;       // shared by all shards, released with the last one
    ~GroupComm() override
    {
        if (dptrs) (void)hipFree(dptrs);
        if (dargs) (void)hipFree(dargs);
        if (hargs) (void)hipHostFree(hargs);
        for (hipEvent_t e : staged)
            if (e) (void)hipEventDestroy(e);
        if (s) (void)hipStreamDestroy(s);
    }
    // the shards' arguments for a one-launch persistent selection of a group
    // of parity grp; returns the device array through *out
    int stage_args(lp_handle *h, const std::vector<Args> &A, int grp, Args **out)
    {
        const size_t n = all.size();
        if (A.size() != n) return fail(h, LP_DEVICE_ERROR, "shard arguments: member count");
        if (!dargs) HCHK(h, hipMalloc(&dargs, 2 * n * sizeof(Args)));
        if (!hargs) HCHK(h, hipHostMalloc(&hargs, 2 * n * sizeof(Args), hipHostMallocDefault));
        const int k = grp & 1;
        if (!staged[k]) HCHK(h, hipEventCreateWithFlags(&staged[k], hipEventDisableTiming));
        else HCHK(h, hipEventSynchronize(staged[k]));
        std::copy(A.begin(), A.end(), hargs + k * n);
        HCHK(h, hipMemcpyAsync(dargs + k * n, hargs + k * n, n * sizeof(Args), hipMemcpyHostToDevice, s));
        HCHK(h, hipEventRecord(staged[k], s));
        *out = dargs + k * n;
        return LP_PIVOTED;
    }
    Members members(lp_handle *) override { return all; }
    int allreduce_min(const Members &M) override
    {
        lp_handle *h = M[0];
        HCHK(h, lpk::launch_group_min(h->s, dptrs, (int)M.size()));
        return LP_PIVOTED;
    }
    int allgather(const Members &M) override
    {
        const size_t bytes = (size_t)slot_len(M[0]) * sizeof(double);
        for (lp_handle *dst : M)
            for (size_t k = 0; k < M.size(); ++k)
                HCHK(dst, hipMemcpyAsync(dst->xr + k * slot_len(dst), M[k]->xs, bytes,
                                         hipMemcpyDeviceToDevice, dst->s));
        return LP_PIVOTED;
    }
};

static Members members_of(lp_handle *h) { return h->comm ? h->comm->members(h) : Members{h}; }
static int block_of(lp_handle *h);

// a multi-process shard: the scans combine every rank's per-column results
// through an all-gather (RcclComm::gather_host)
static RcclComm *multi_process(lp_handle *h)
{
    if (!h->comm || h->nranks <= 1) return nullptr;
    return dynamic_cast<RcclComm *>(h->comm.get());
}


// ---------------------------------------------------------------------------
// creation
// ---------------------------------------------------------------------------

static Args args_of(const lp_handle *h)
{
    Args A;
    A.T = h->T;
    A.Tout = h->oop ? h->Tb[(h->flips + 1) & 1] : h->T;
    A.dflips = h->dflips;
    A.flipseq = h->flips + 1;
    A.sweep_clk = h->sweep_clk;
    A.sweep_lseq = h->sweep_lseq;
    A.row0 = h->row0;
    A.col0 = h->col0;
    A.M = h->M;
    A.MQ = h->MQ;
    A.P = h->P;
    A.dR = h->dR;
    A.dC = h->dC;
    A.ctl = h->ctl;
    A.log = h->log;
    A.rec = h->rec;
    A.erec = h->erec;
    A.xg = h->xg;
    A.xs = h->xs;
    A.xr = h->xr;
    A.logcap = h->logcap;
    A.m = h->m;
    A.n = h->n;
    A.ld = h->ld;
    static const int gmaj = [] {
        const char *v = std::getenv("LPGPU_GMAJ");   // A/B: 0 = block-major summaries always
        return v ? std::atoi(v) : 1;
    }();
    A.gmaj = gmaj;
    A.rows = h->rows;
    A.rb = h->rb;
    A.rc = h->rc;
    A.nranks = h->nranks;
    A.tol = h->tol;
    A.stamps = h->stamps;
    A.gran = h->gran;
    A.spin_max = h->spin_max;
    A.xwait_ms = h->xwait_ms;
    A.fault = 0;
    static const int hier = [] {
        const char *v = std::getenv("LPGPU_HIER");   // A/B: 0 = flat exchange for spread blocks
        return v ? std::atoi(v) : 1;
    }();
    A.hier = hier;
    A.rank = h->rank;
    A.xtarget = h->xtarget;
    A.share = h->share;
    A.fault_xcc = 0;
    A.xbuf = h->xbuf;
    A.peer = h->dpeer;
    return A;
}

extern "C" void lp_default_tol(lp_tol *t)
{
    t->cost = 1e-9;
    t->cost_tie = 1e-12;
    t->pivot = 1e-9;
    t->zero = 1e-9;
    t->ratio_tie = 1e-12;
    t->stall = 1e-12;
}

extern "C" int lp_device_count(int *count)
{
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return LP_PIVOTED;
}

// Row pitch of the tableau in doubles: a multiple of 64 (512 B: rows start
// on a cache line, 16-byte accesses stay aligned) that holds n + 1 columns
// and is not "aliased".  A pitch of p x 512 B where p x d lies within
// 1.5 min(k, 3) of k x 128 (k x 64 KiB) for some d = 1..4 sends the
// selection's column gather -- one element from each of 32768 rows -- to few
// HBM channels, at about twice the time of its neighbours
// (scripts/gather_probe.hip, profiles/r02/gather_pitch.json: 3.6 us against
// 1.7 us at p = 127/129 and 4.1 / 3.8 at 254 / 258; 2.2-2.6 at 43, 64, 86,
// 172).  cfg3 / cfg4 (n = 8192): p = 129 -> 130.  At most 16 steps up.
static bool pitch_aliased(int64_t p)
{
    for (int64_t d = 1; d <= 4; ++d) {
        const int64_t q = p * d, k = (q + 64) / 128;
        if (k < 1) continue;
        const int64_t dist = q > 128 * k ? q - 128 * k : 128 * k - q;
        if (2 * dist <= 3 * std::min<int64_t>(k, 3)) return true;
    }
    return false;
}

static int64_t row_pitch(int64_t n)
{
    const int64_t p0 = (n + 1 + 63) / 64;
    const char *raw = std::getenv("LPGPU_LD_RAW");   // A/B: the plain rounded pitch
    if ((raw && raw[0] == '1') || p0 < 16) return p0 * 64;
    for (int64_t p = p0; p < p0 + 16; ++p)
        if (!pitch_aliased(p)) return p * 64;
    return p0 * 64;
}

// The kernels address the multipliers (BMAX x local rows) and a row batch
// (a few rows x pitch) with 32-bit byte offsets.
static bool geometry_fits(int64_t m, int64_t n, int nranks)
{
    const int64_t rows = (m + nranks - 1) / nranks + 1;
    return (rows * lpk::BMAX + lpk::M_PAD) * 8 < (int64_t(1) << 31) && n < (int64_t(1) << 26);
}

static void init_geometry(lp_handle *h, int64_t m, int64_t n, int rank, int nranks)
{
    h->m = m;
    h->n = n;
    h->ld = row_pitch(n);
    h->rank = rank;
    h->nranks = nranks;
    h->rb = m * rank / nranks;
    h->rc = m * (rank + 1) / nranks - h->rb;
    h->rows = h->rc + 1;
}

static int alloc_handle(lp_handle *h)
{
    if (const char *sel = std::getenv("LPGPU_SELECT"))
        h->persistent = std::strcmp(sel, "kernels") != 0;
    if (const char *v = std::getenv("LPGPU_SPIN_MAX")) h->spin_max = (unsigned)std::strtoul(v, nullptr, 10);
    if (const char *v = std::getenv("LPGPU_XWAIT_MS")) h->xwait_ms = (unsigned)std::strtoul(v, nullptr, 10);
    if (const char *v = std::getenv("LPGPU_FAULT")) std::sscanf(v, "%d:%d", &h->fault_launch, &h->fault_t);
    if (const char *v = std::getenv("LPGPU_FAULT_XCC")) h->fault_xcc = std::atoi(v);
    if (const char *v = std::getenv("LPGPU_STRICT")) h->strict = v[0] == '1';
    if (const char *v = std::getenv("LPGPU_SEL_XS")) h->xs_ok = v[0] != '0';
    if (const char *pe = std::getenv("LPGPU_PEER")) h->peer_enable = pe[0] != '0';
    if (const char *st = std::getenv("LPGPU_STAMPS"))
        if (st[0] == '1') {
            const size_t sb = (lpk::BMAX * 16 + lpk::GROUP_MAXBLOCKS * lpk::BMAX * 4) * sizeof(long long);
            HCHK(h, hipMalloc(&h->stamps, sb));
            HCHK(h, hipMemset(h->stamps, 0, sb));
        }
    HCHK(h, hipSetDevice(h->dev));
    if (!h->s) HCHK(h, hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking));
    const size_t tbytes = (size_t)h->rows * (size_t)h->ld * sizeof(double);
    HCHK(h, hipMalloc(&h->T, tbytes));
    HCHK(h, hipMemsetAsync(h->T, 0, tbytes, h->s));
    h->Tb[0] = h->T;
    // LPGPU_SWEEP_OOP: 1 always, 0 never, unset: by size (> 512 MiB)
    static const int oop_env = [] {
        const char *v = std::getenv("LPGPU_SWEEP_OOP");
        return v ? std::atoi(v) : 2;
    }();
    {
        // out-of-place sweeps where the tableau is far beyond the 256 MB
        // Infinity Cache: cfg4 (2.2 GB) 842 -> 812 us per sweep (0.64 -> 0.66
        // of the HBM spec, same box); at cfg3's 273 MB the in-place pass keeps
        // the tableau in the cache for the selection's column reads (OOP:
        // selection 4.47 -> 4.67 us per pivot, 157k -> 152k pivots/s).
        h->oop = oop_env == 1 || (oop_env == 2 && tbytes > ((size_t)512 << 20));
        // by size, only where the second buffer fits with room to spare (the
        // group data below, other handles): a tableau of more than about half
        // the device stays in place rather than failing to open
        // (test knobs, tests/test_gpu_r6.py: LPGPU_OOP_ROOM_MB, the headroom
        // asked for beyond the second buffer, default 1 GiB; LPGPU_OOP_FAIL_ALLOC=1
        // fails the second buffer's allocation as a full device would)
        static const unsigned long long room_mb = [] {
            const char *v = std::getenv("LPGPU_OOP_ROOM_MB");
            return v ? std::strtoull(v, nullptr, 10) : 1024ull;
        }();
        if (h->oop && oop_env == 2) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
                (void)hipGetLastError();
                h->oop = false;
            } else if ((unsigned long long)fr < tbytes + tbytes / 8 + (room_mb << 20)) {
                h->oop = false;
            }
        }
    }
    static const bool fail_alloc = [] {
        const char *v = std::getenv("LPGPU_OOP_FAIL_ALLOC");
        return v && v[0] == '1';
    }();
    if (h->oop) {
        // the second buffer: its padding columns stay 0 like T's (no sweep
        // writes past column n).  Unforced, a failed allocation falls back to
        // in-place sweeps.
        if (fail_alloc || hipMalloc(&h->Tb[1], tbytes) != hipSuccess) {
            (void)hipGetLastError();
            h->Tb[1] = nullptr;
            if (oop_env == 1) HCHK(h, hipErrorOutOfMemory);
            h->oop = false;
        }
    }
    {
        const size_t cb = (size_t)(lpk::SWEEP_CLK_RING + lpk::SWEEP_BLK_MAX) * 4 * sizeof(unsigned long long);
        HCHK(h, hipMalloc(&h->sweep_clk, cb));
        HCHK(h, hipMemsetAsync(h->sweep_clk, 0xff, cb, h->s));
    }
    if (h->oop) {
        HCHK(h, hipMemsetAsync(h->Tb[1], 0, tbytes, h->s));
        HCHK(h, hipMalloc(&h->dflips, sizeof(unsigned)));
        HCHK(h, hipMemsetAsync(h->dflips, 0, sizeof(unsigned), h->s));
    }
    // two sets of group data (P, M, dR, dC) by group parity
    HCHK(h, hipMalloc(&h->P, 2 * (size_t)lpk::BMAX * h->ld * sizeof(double)));
    HCHK(h, hipMemsetAsync(h->P, 0, 2 * (size_t)lpk::BMAX * h->ld * sizeof(double), h->s));
    const size_t mbytes = 2 * ((size_t)lpk::BMAX * h->rows + lpk::M_PAD) * sizeof(double);
    const size_t mqbytes = ((size_t)lpk::mq_len(h->rows) + lpk::M_PAD) * sizeof(double);
    HCHK(h, hipMalloc(&h->MQ, mqbytes));
    HCHK(h, hipMemsetAsync(h->MQ, 0, mqbytes, h->s));
    HCHK(h, hipMalloc(&h->M, mbytes));
    HCHK(h, hipMemsetAsync(h->M, 0, mbytes, h->s));
    const size_t gbytes = (size_t)lpk::GRAN_TOTAL * sizeof(unsigned long long);
    HCHK(h, hipMalloc(&h->gran, gbytes));
    HCHK(h, hipMemsetAsync(h->gran, 0, gbytes, h->s));
    HCHK(h, hipMalloc(&h->row0, (size_t)h->ld * sizeof(double)));
    HCHK(h, hipMemsetAsync(h->row0, 0, (size_t)h->ld * sizeof(double), h->s));
    HCHK(h, hipMalloc(&h->col0, (size_t)h->rows * sizeof(double)));
    HCHK(h, hipMemsetAsync(h->col0, 0, (size_t)h->rows * sizeof(double), h->s));
    HCHK(h, hipMalloc(&h->dR, 2 * (size_t)lpk::BMAX * sizeof(long long)));
    HCHK(h, hipMalloc(&h->dC, 2 * (size_t)lpk::BMAX * sizeof(long long)));
    HCHK(h, hipMalloc(&h->erec, (size_t)std::max(lpk::GROUP_MAXBLOCKS, lpk::prow_blocks(h->ld)) *
                                     sizeof(lpk::ERec)));
    h->eager_ok = true;   // all zero
    HCHK(h, hipMalloc(&h->ctl, sizeof(Ctl)));
    HCHK(h, hipMemsetAsync(h->ctl, 0, sizeof(Ctl), h->s));
    HCHK(h, hipHostMalloc(&h->hctl, sizeof(Ctl), hipHostMallocDefault));
    std::memset(h->hctl, 0, sizeof(Ctl));
    h->logcap = 4096;
    HCHK(h, hipMalloc(&h->log, (size_t)h->logcap * 2 * sizeof(long long)));
    const int nrec = std::max(lpk::GROUP_MAXBLOCKS, lpk::ratio_blocks(h->rows));
    HCHK(h, hipMalloc(&h->rec, (size_t)nrec * sizeof(Rec)));
    HCHK(h, hipMemsetAsync(h->rec, 0, (size_t)nrec * sizeof(Rec), h->s));
    if (h->nranks > 1 || h->comm) {
        HCHK(h, hipMalloc(&h->xg, sizeof(double)));
        HCHK(h, hipMalloc(&h->xs, (size_t)slot_len(h) * sizeof(double)));
        HCHK(h, hipMalloc(&h->xr, (size_t)slot_len(h) * h->nranks * sizeof(double)));
        HCHK(h, hipMemsetAsync(h->xs, 0, (size_t)slot_len(h) * sizeof(double), h->s));
    }
    HCHK(h, hipStreamSynchronize(h->s));
    lp_default_tol(&h->tol);
    return LP_PIVOTED;
}

extern "C" int lp_create(int64_t m, int64_t n, int device, lp_handle **out)
{
    *out = nullptr;
    if (m <= 0 || n <= 0) {
        g_create_err = "need m > 0 and n > 0";
        return LP_BAD_ARG;
    }
    if (!geometry_fits(m, n, 1)) {
        g_create_err = "tableau too large for one device (at most 4194302 rows, 2^26 columns)";
        return LP_BAD_ARG;
    }
    lp_handle *h = new lp_handle;
    h->dev = device;
    init_geometry(h, m, n, 0, 1);
    const int st = alloc_handle(h);
    if (st != LP_PIVOTED) {
        g_create_err = h->err;
        lp_destroy(h);
        return st;
    }
    *out = h;
    return LP_PIVOTED;
}

extern "C" int lp_comm_unique_id(void *uid128)
{
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        g_create_err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return LP_DEVICE_ERROR;
    }
    std::memcpy(uid128, &id, sizeof(id));
    return LP_PIVOTED;
}

extern "C" int lp_create_sharded(int64_t m, int64_t n, int device, int rank, int nranks,
                                 const void *uid128, lp_handle **out)
{
    *out = nullptr;
    if (m <= 0 || n <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || m < nranks) {
        g_create_err = "need m >= nranks > 0, n > 0 and 0 <= rank < nranks";
        return LP_BAD_ARG;
    }
    if (!geometry_fits(m, n, nranks)) {
        g_create_err = "row block too large for one device (at most 4194302 rows, 2^26 columns)";
        return LP_BAD_ARG;
    }
    lp_handle *h = new lp_handle;
    h->dev = device;
    init_geometry(h, m, n, rank, nranks);
    auto comm = std::make_shared<RcclComm>();
    h->comm = comm;
    int st = alloc_handle(h);
    if (st == LP_PIVOTED && uid128) {
        ncclUniqueId id;
        std::memcpy(&id, uid128, sizeof(id));
        const ncclResult_t r = ncclCommInitRank(&comm->comm, nranks, id, rank);
        if (r != ncclSuccess) {
            h->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
            st = LP_DEVICE_ERROR;
        }
    }
    if (st != LP_PIVOTED) {
        g_create_err = h->err;
        lp_destroy(h);
        return st;
    }
    *out = h;
    return LP_PIVOTED;
}

extern "C" int lp_create_group(int64_t m, int64_t n, int device, int nshards, lp_handle **out)
{
    for (int k = 0; k < nshards; ++k) out[k] = nullptr;
    if (m <= 0 || n <= 0 || nshards <= 0 || m < nshards) {
        g_create_err = "need m >= nshards > 0 and n > 0";
        return LP_BAD_ARG;
    }
    if (!geometry_fits(m, n, nshards)) {
        g_create_err = "shard too large for one device (at most 4194302 rows, 2^26 columns)";
        return LP_BAD_ARG;
    }
    auto grp = std::make_shared<GroupComm>();
    hipStream_t s = nullptr;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        g_create_err = "stream creation failed";
        return LP_DEVICE_ERROR;
    }
    grp->s = s;
    int st = LP_PIVOTED;
    for (int k = 0; k < nshards && st == LP_PIVOTED; ++k) {
        lp_handle *h = new lp_handle;
        h->dev = device;
        h->s = s;
        h->own_stream = false;
        init_geometry(h, m, n, k, nshards);
        h->comm = grp;
        grp->all.push_back(h);
        out[k] = h;
        st = alloc_handle(h);
        if (st != LP_PIVOTED) g_create_err = h->err;
    }
    if (st == LP_PIVOTED) {
        // device-side exchange between the shards (same device: plain buffers)
        std::vector<unsigned long long *> xb;
        for (lp_handle *h : grp->all) {
            if (!h->peer_enable || nshards > lpk::NRANK_MAX) break;
            const size_t xbytes = lpk::xs_granules(h->nranks) * sizeof(unsigned long long);
            if (hipMalloc(&h->xbuf, xbytes) != hipSuccess || hipMemset(h->xbuf, 0, xbytes) != hipSuccess ||
                hipStreamCreateWithFlags(&h->sx, hipStreamNonBlocking) != hipSuccess) {
                g_create_err = "group exchange buffers";
                st = LP_DEVICE_ERROR;
                break;
            }
            xb.push_back(h->xbuf);
        }
        if (st == LP_PIVOTED && xb.size() == grp->all.size())
            for (lp_handle *h : grp->all) {
                if (hipMalloc(&h->dpeer, xb.size() * sizeof(void *)) != hipSuccess ||
                    hipMemcpy(h->dpeer, xb.data(), xb.size() * sizeof(void *), hipMemcpyHostToDevice) !=
                        hipSuccess) {
                    g_create_err = "group exchange table";
                    st = LP_DEVICE_ERROR;
                    break;
                }
                h->peer_ok = true;
            }
    }
    if (st == LP_PIVOTED) {
        std::vector<double *> p;
        for (lp_handle *h : grp->all) p.push_back(h->xg);
        if (hipMalloc(&grp->dptrs, p.size() * sizeof(double *)) != hipSuccess ||
            hipMemcpy(grp->dptrs, p.data(), p.size() * sizeof(double *), hipMemcpyHostToDevice) !=
                hipSuccess) {
            g_create_err = "group pointer table";
            st = LP_DEVICE_ERROR;
        }
    }
    if (st != LP_PIVOTED) {
        for (int k = nshards - 1; k >= 0; --k)
            if (out[k]) {
                lp_destroy(out[k]);
                out[k] = nullptr;
            }
        return st;
    }
    return LP_PIVOTED;
}

// ---------------------------------------------------------------------------
// device-side exchange between the ranks of a sharded job
// ---------------------------------------------------------------------------

extern "C" int lp_peer_handle(lp_handle *h, void *ipc64)
{
    if (!h || !h->comm || h->nranks > lpk::NRANK_MAX) return h ? fail(h, LP_BAD_ARG, "not a sharded handle") : LP_BAD_ARG;
    HCHK(h, hipSetDevice(h->dev));
    const size_t xbytes = lpk::xs_granules(h->nranks) * sizeof(unsigned long long);
    hipIpcMemHandle_t hd;
    if (!h->xbuf) {
        // fine-grained: peers' system-scope stores are visible to this device's
        // polling loads.  Plain device memory if that cannot be shared -- usable
        // only by ranks on this same GPU: lp_peer_open refuses the exchange
        // when such a buffer would be polled across devices, and
        // the job keeps its RCCL per-pivot path
        h->xbuf_fine = true;
        if (hipExtMallocWithFlags((void **)&h->xbuf, xbytes, hipDeviceMallocFinegrained) != hipSuccess ||
            hipIpcGetMemHandle(&hd, h->xbuf) != hipSuccess) {
            if (h->xbuf) (void)hipFree(h->xbuf);
            h->xbuf = nullptr;
            (void)hipGetLastError();
            HCHK(h, hipMalloc(&h->xbuf, xbytes));
            h->xbuf_fine = false;
        }
        HCHK(h, hipMemset(h->xbuf, 0, xbytes));
    }
    HCHK(h, hipIpcGetMemHandle(&hd, h->xbuf));
    static_assert(sizeof(hd) == LP_PEER_HANDLE_BYTES, "IPC handle size");
    std::memcpy(ipc64, &hd, sizeof(hd));
    return LP_PIVOTED;
}

extern "C" int lp_peer_open(lp_handle *h, const void *handles)
{
    if (!h || !h->comm || !h->xbuf) return h ? fail(h, LP_BAD_ARG, "lp_peer_handle first") : LP_BAD_ARG;
    HCHK(h, hipSetDevice(h->dev));
    std::vector<unsigned long long *> tab(h->nranks, nullptr);
    int here = 1;                           // ranks of the job on this rank's GPU
    const char *all = static_cast<const char *>(handles);
    for (int p = 0; p < h->nranks; ++p) {
        if (p == h->rank) {
            tab[p] = h->xbuf;
            continue;
        }
        hipIpcMemHandle_t hd;
        std::memcpy(&hd, all + (size_t)p * LP_PEER_HANDLE_BYTES, sizeof(hd));
        void *ptr = nullptr;
        HCHK(h, hipIpcOpenMemHandle(&ptr, hd, hipIpcMemLazyEnablePeerAccess));
        h->ipc_open.push_back(ptr);
        tab[p] = static_cast<unsigned long long *>(ptr);
        // a peer buffer on this very GPU: the two ranks share it (tests)
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, ptr) != hipSuccess || at.device == h->dev) ++here;
        (void)hipGetLastError();
    }
    if (!h->dpeer) HCHK(h, hipMalloc(&h->dpeer, lpk::NRANK_MAX * sizeof(void *)));
    HCHK(h, hipMemcpy(h->dpeer, tab.data(), tab.size() * sizeof(void *), hipMemcpyHostToDevice));
    // every rank pings every rank (collective: all ranks call this together)
    int *dok = nullptr, ok = 0;
    HCHK(h, hipMalloc(&dok, sizeof(int)));
    Args A = args_of(h);
    A.peer = h->dpeer;
    // the ping also carries, one-hot, how many ranks share this rank's GPU:
    // the OR over the ranks gives every rank the same maximum (their
    // persistent selections must then all be resident on that GPU at once)
    // (bit 8: this rank's exchange buffer is plain, coarse-grained memory)
    const unsigned flag = (1u << (std::min(here, 8) - 1)) | (h->xbuf_fine ? 0u : 0x100u);
    const hipError_t e = lpk::launch_peer_ping(h->s, A, 7u, flag, dok);
    if (e == hipSuccess) (void)hipMemcpyAsync(&ok, dok, sizeof(int), hipMemcpyDeviceToHost, h->s);
    const hipError_t e2 = hipStreamSynchronize(h->s);
    (void)hipFree(dok);
    if (e != hipSuccess || e2 != hipSuccess) return fail(h, LP_DEVICE_ERROR, "peer ping launch failed");
    // the ping used the summary slots: clear them for the pivots
    HCHK(h, hipMemset(h->xbuf, 0, lpk::xs_granules(h->nranks) * sizeof(unsigned long long)));
    HCHK(h, hipDeviceSynchronize());
    if (!ok) return fail(h, LP_DEVICE_ERROR, "peer exchange check timed out");
    h->peer_ok = true;
    h->block_auto = 0;                      // the exchange changes the selection's placement
    const unsigned bits = ((unsigned)ok >> 1) & 0xffu;
    h->share = 1;
    while (h->share < 8 && (bits >> h->share)) ++h->share;
    // a coarse-grained exchange buffer anywhere, with the ranks on more than
    // one GPU: polling loads of one device are not guaranteed to see another
    // device's stores into such memory, so no rank takes the device-side
    // exchange (every rank sees the same OR of the flags: a collective answer)
    if ((((unsigned)ok >> 1) & 0x100u) && h->share < h->nranks)
        return fail(h, LP_DEVICE_ERROR, "exchange buffer not fine-grained across devices");
    h->xr_xcd = h->share == 1;
    h->xtarget = -1;
    if (const char *v = std::getenv("LPGPU_XR_XCD")) {
        // A/B and tests: 0 off; 1 on even for ranks sharing a GPU (tests of
        // the one-XCD cross-rank selection k_sel<XR> on one box).  Ranks
        // sharing a GPU then each take their own XCD (Args::xtarget: rank % 8,
        // distinct for up to 8 ranks), so each rank's launch needs only its
        // own XCD's slots -- the same residency as one rank per GPU; more than
        // 8 ranks on one GPU keep the spread kernels
        if (v[0] == '0') h->xr_xcd = false;
        if (v[0] == '1') h->xr_xcd = h->share == 1 || h->nranks <= 8;
        if (h->xr_xcd && h->share > 1) h->xtarget = h->rank % 8;
    }
    return LP_PIVOTED;
}

extern "C" int lp_peer_enable(lp_handle *h, int enable)
{
    for (lp_handle *x : members_of(h))
        if (x) {
            if (enable && !x->dpeer) return fail(h, LP_BAD_ARG, "no peer exchange set up");
            x->peer_ok = enable != 0;
            x->block_auto = 0;
        }
    return LP_PIVOTED;
}

extern "C" int lp_set_host_allgather(lp_handle *h, lp_allgather_fn fn, void *ctx)
{
    RcclComm *rc = multi_process(h);
    if (!rc) return fail(h, LP_BAD_ARG, "not a multi-process sharded handle");
    rc->host_fn = fn;
    rc->host_ctx = ctx;
    return LP_PIVOTED;
}

extern "C" int lp_shard_rows(const lp_handle *h, int64_t *row_begin, int64_t *row_count)
{
    *row_begin = h->rb;
    *row_count = h->rc;
    return LP_PIVOTED;
}

extern "C" int lp_destroy(lp_handle *h)
{
    if (!h) return LP_PIVOTED;
    (void)hipSetDevice(h->dev);
    if (h->s) (void)hipStreamSynchronize(h->s);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->sx) (void)hipStreamSynchronize(h->sx);
    for (void *p : {(void *)h->cstat, (void *)h->cthr, (void *)h->cfirst, (void *)h->ccount,
                    (void *)h->coffs, (void *)h->rowflag})
        if (p) (void)hipFree(p);
    for (void *p : h->ipc_open) (void)hipIpcCloseMemHandle(p);
    if (h->dpeer) (void)hipFree(h->dpeer);
    if (h->xbuf) (void)hipFree(h->xbuf);
    if (h->sx) (void)hipStreamDestroy(h->sx);
    if (h->Tb[0]) (void)hipFree(h->Tb[0]);
    if (h->Tb[1]) (void)hipFree(h->Tb[1]);
    if (h->dflips) (void)hipFree(h->dflips);
    if (h->sweep_clk) (void)hipFree(h->sweep_clk);
    if (h->P) (void)hipFree(h->P);
    if (h->M) (void)hipFree(h->M);
    if (h->MQ) (void)hipFree(h->MQ);
    if (h->row0) (void)hipFree(h->row0);
    if (h->col0) (void)hipFree(h->col0);
    if (h->dR) (void)hipFree(h->dR);
    if (h->dC) (void)hipFree(h->dC);
    if (h->erec) (void)hipFree(h->erec);
    if (h->stamps) (void)hipFree(h->stamps);
    if (h->gran) (void)hipFree(h->gran);
    if (h->ctl) (void)hipFree(h->ctl);
    if (h->hctl) (void)hipHostFree(h->hctl);
    if (h->log) (void)hipFree(h->log);
    if (h->rec) (void)hipFree(h->rec);
    if (h->xg) (void)hipFree(h->xg);
    if (h->xs) (void)hipFree(h->xs);
    if (h->xr) (void)hipFree(h->xr);
    if (h->comm) {
        if (auto g = std::dynamic_pointer_cast<GroupComm>(h->comm)) {
            auto it = std::find(g->all.begin(), g->all.end(), h);
            if (it != g->all.end()) *it = nullptr;
        }
        h->comm.reset();
    }
    if (h->s && h->own_stream) (void)hipStreamDestroy(h->s);
    delete h;
    return LP_PIVOTED;
}

extern "C" int lp_set_tol(lp_handle *h, const lp_tol *tol)
{
    for (lp_handle *x : members_of(h))
        if (x) x->tol = *tol;
    return LP_PIVOTED;
}

extern "C" int lp_get_tol(const lp_handle *h, lp_tol *tol)
{
    *tol = h->tol;
    return LP_PIVOTED;
}

extern "C" const char *lp_last_error(const lp_handle *h)
{
    return h ? h->err.c_str() : g_create_err.c_str();
}

// ---------------------------------------------------------------------------
// row transfers
// ---------------------------------------------------------------------------

// global row -> local row, or -1 if this rank does not hold it
static int64_t local_row(const lp_handle *h, int64_t R)
{
    if (R == 0) return 0;
    if (R >= 1 + h->rb && R < 1 + h->rb + h->rc) return R - h->rb;
    return -1;
}

template <bool UP>
static int transfer_rows(lp_handle *h, int64_t row0, int64_t nrows, double *buf, int64_t ldh)
{
    if (row0 < 0 || nrows < 0 || row0 + nrows > h->m + 1 || ldh < h->n + 1)
        return fail(h, LP_BAD_ARG, "row range or leading dimension out of bounds");
    HCHK(h, hipSetDevice(h->dev));
    int64_t k = 0;
    while (k < nrows) {
        const int64_t R = row0 + k;
        const int64_t L = local_row(h, R);
        if (L < 0) return fail(h, LP_BAD_ARG, "row not held by this shard");
        int64_t run = 1;   // longest run of consecutive local rows
        if (R > 0)
            while (k + run < nrows && local_row(h, R + run) == L + run) ++run;
        double *dev = h->T + L * h->ld;
        double *host = buf + k * ldh;
        const size_t w = (size_t)(h->n + 1) * sizeof(double);
        if (UP)
            HCHK(h, hipMemcpy2DAsync(dev, h->ld * sizeof(double), host, ldh * sizeof(double), w,
                                     run, hipMemcpyHostToDevice, h->s));
        else
            HCHK(h, hipMemcpy2DAsync(host, ldh * sizeof(double), dev, h->ld * sizeof(double), w,
                                     run, hipMemcpyDeviceToHost, h->s));
        k += run;
    }
    HCHK(h, hipStreamSynchronize(h->s));
    return LP_PIVOTED;
}

extern "C" int lp_upload_rows(lp_handle *h, int64_t row0, int64_t nrows, const double *src,
                              int64_t ldh)
{
    h->eager_ok = false;
    return transfer_rows<true>(h, row0, nrows, const_cast<double *>(src), ldh);
}

extern "C" int lp_set_block(lp_handle *h, int pivots_per_sweep)
{
    if (pivots_per_sweep < 0 || pivots_per_sweep > lpk::BMAX)
        return fail(h, LP_BAD_ARG, "pivots_per_sweep must be in [1, 64], or 0 (auto)");
    for (lp_handle *x : members_of(h))
        if (x) x->block = pivots_per_sweep;
    return LP_PIVOTED;
}

extern "C" int lp_get_block(const lp_handle *h, int *pivots_per_sweep)
{
    *pivots_per_sweep = block_of(const_cast<lp_handle *>(h));
    return LP_PIVOTED;
}

extern "C" int lp_download_rows(lp_handle *h, int64_t row0, int64_t nrows, double *dst,
                                int64_t ldh)
{
    return transfer_rows<false>(h, row0, nrows, dst, ldh);
}

// ---------------------------------------------------------------------------
// pivot machinery
// ---------------------------------------------------------------------------

static int ensure_log(lp_handle *h, int64_t need)
{
    if (need <= h->logcap) return LP_PIVOTED;
    int64_t cap = h->logcap;
    while (cap < need) cap *= 2;
    long long *nl = nullptr;
    HCHK(h, hipMalloc(&nl, (size_t)cap * 2 * sizeof(long long)));
    HCHK(h, hipMemcpyAsync(nl, h->log, (size_t)h->logcap * 2 * sizeof(long long),
                           hipMemcpyDeviceToDevice, h->s));
    HCHK(h, hipStreamSynchronize(h->s));
    HCHK(h, hipFree(h->log));
    h->log = nl;
    h->logcap = cap;
    return LP_PIVOTED;
}

// event pair around a launch on stream st when profiling (kind 0 sweep, 1 selection)
// the next pair of profiling events, recorded by the launch itself at the
// kernel's start and end (hipExtLaunchKernelGGL): kernel time, no dispatch gap
static int prof_slot(lp_handle *h, hipEvent_t *e0, hipEvent_t *e1, int kind)
{
    *e0 = *e1 = nullptr;
    if (!h->prof) return LP_PIVOTED;
    if (h->prof_seen[kind]++ % h->prof_every != 0) return LP_PIVOTED;   // not sampled
    if (h->evused + 2 > h->ev.size()) {
        hipEvent_t a, b;
        HCHK(h, hipEventCreate(&a));
        HCHK(h, hipEventCreate(&b));
        h->ev.push_back(a);
        h->ev.push_back(b);
        h->evkind.push_back(0);
    }
    *e0 = h->ev[h->evused];
    *e1 = h->ev[h->evused + 1];
    h->evkind[h->evused / 2] = kind;
    h->evused += 2;
    return LP_PIVOTED;
}

// cnt: the most pivots the group can hold (the kernel's depth when below the
// handle's: a call's last group, an explicit pivot)
static int launch_sweep_timed(lp_handle *h, const Args &A, int grp, int cnt, bool *flipped)
{
    hipEvent_t e0, e1;
    CALL(prof_slot(h, &e0, &e1, 0));
    // the caller's Args live across a batch of launches: the clock record's
    // launch number is this launch's own
    Args a = A;
    a.sweep_lseq = h->sweep_lseq;
    HCHK(h, lpk::launch_sweep(h->s, a, grp, block_of(h), cnt, e0, e1, flipped));
    ++h->sweep_lseq;
    return LP_PIVOTED;
}

// call-start work folded into the first k_group launch of a call (k_group's
// `first` bits): reset of the loop state, eager row 0 / column 0 after an
// upload, the first entering column
struct CallStart {
    int first = 0;       // 0: not the first launch of the call
    int mode = 0, rule = 0;
    long long cap = -1;
};

static int launch_group_timed(lp_handle *h, const Args &A, const lpk::GroupGeom &geo, int grp, int cnt,
                              int from_erec, int xr, const Args *As, int nshard, const CallStart &cs)
{
    // every rank of a sharded job advances gseq identically (same calls, same order)
    h->gseq = h->gseq % ((1u << 23) - 1) + 1;   // gtag: seq * 8 * BMAX fits 32 bits
    hipEvent_t e0, e1;
    CALL(prof_slot(h, &e0, &e1, 1));
    Args a = A;
    if (h->fault_launch > 0 && (unsigned)h->fault_launch == h->gseq) a.fault = h->fault_t + 1;
    if (h->fault_xcc > 0 && (unsigned)h->fault_xcc == h->gseq) a.fault_xcc = 1;
    HCHK(h, lpk::launch_group(h->s, a, geo, grp, cnt, from_erec, h->gseq, block_of(h), xr, As, nshard,
                              cs.first, cs.mode, cs.rule, cs.cap, e0, e1));
    return LP_PIVOTED;
}

// Which pivot path a pivot loop of this handle takes (lp_exchange_path):
//   single device: one persistent k_group launch per group where its
//   geometry fits (occupancy of the compiled kernel), else per-pivot kernels;
//   row-sharded: the persistent cross-rank k_group (device-side peer
//   exchange) where the exchange is set up and every rank's launch fits on
//   its GPU at once -- at most 4 ranks per GPU (8 processes on one GPU have
//   more queues than the hardware scheduler keeps mapped at once, and a rank
//   whose queue is not mapped never answers: measured, round 1) -- else one
//   collective per pivot.  Every rank decides from the same values (global
//   sizes, the ping's shared-GPU count), so all take the same path.
static lpk::GroupGeom persistent_geom_b(lp_handle *h, size_t nmem, int *xr, int bmax)
{
    *xr = 0;
    lpk::GroupGeom none;
    if (!h->persistent) return none;
    if (!h->comm) return lpk::group_geom(h->rc, h->ld, h->n, bmax, 0, 1, 1, h->xs_ok);
    if (!h->peer_ok || h->share > 4) return none;
    const int64_t rcmax = (h->m + h->nranks - 1) / h->nranks;
    *xr = (nmem == 1 && h->xr_xcd) ? 2 : 1;
    return lpk::group_geom(rcmax, h->ld, h->n, bmax, *xr, (int)nmem, nmem == 1 ? h->share : 1, h->xs_ok);
}

// Pivots per sweep when the handle says auto (0).  More pivots per sweep cut
// the sweep's traffic per pivot, but each selection block keeps its rows'
// multipliers and its columns' pivot-row values in LDS, so past some depth
// the persistent selection may no longer fit on one XCD (its L2-resident
// hand-offs): the deepest of 64 / 48 / 32 whose selection still runs on one
// XCD (or as k_sel's XCD shards); 64 where none does (a tall shard spread over
// the device anyway); 32 on the per-pivot kernels.  Since round 3's k_sel,
// cfg3 (4096 x 8192) and cfg4 (32768 x 8192) both take 64 (cfg3: 146-148k
// pivots/s, profiles/r03/README.md).  Every rank of a sharded job decides
// from the same global sizes.
static int block_of(lp_handle *h)
{
    if (h->block > 0) return h->block;
    if (h->block_auto > 0) return h->block_auto;
    const size_t nmem = h->comm ? std::max<size_t>(members_of(h).size(), 1) : 1;
    int xr = 0, pick = 0;
    for (int b : {64, 48, 32}) {
        const lpk::GroupGeom g = persistent_geom_b(h, nmem, &xr, b);
        if (g.g > 0 && g.xmode) { pick = b; break; }
    }
    if (!pick) pick = persistent_geom_b(h, nmem, &xr, 64).g > 0 ? 64 : 32;
    h->block_auto = pick;
    return pick;
}

static lpk::GroupGeom persistent_geom(lp_handle *h, const Members &M, int *xr)
{
    return persistent_geom_b(h, M.size(), xr, block_of(h));
}

// one persistent selection launch per rank for a group of cnt pivots.  The
// in-process shards of one device go into ONE launch (their blocks wait on
// each other, so all of them must be resident together).
static int enqueue_group(const Members &M, const std::vector<Args> &A, const lpk::GroupGeom &geo, int xr,
                         int grp, int cnt, int from_erec, const CallStart &cs)
{
    if (M.size() == 1) return launch_group_timed(M[0], A[0], geo, grp, cnt, from_erec, xr, nullptr, 1, cs);
    lp_handle *h0 = M[0];
    auto g = std::dynamic_pointer_cast<GroupComm>(h0->comm);
    if (!g) return fail(h0, LP_DEVICE_ERROR, "multi-member launch without a shard group");
    std::vector<Args> As = A;
    const unsigned next = h0->gseq % ((1u << 23) - 1) + 1;   // the seq launch_group_timed takes
    for (size_t k = 0; k < M.size(); ++k)
        if (M[k]->fault_launch > 0 && (unsigned)M[k]->fault_launch == next) As[k].fault = M[k]->fault_t + 1;
    Args *dA = nullptr;
    CALL(g->stage_args(h0, As, grp, &dA));
    // the members' launch counters advance together (their tags must match)
    for (size_t k = 1; k < M.size(); ++k) M[k]->gseq = next;
    return launch_group_timed(h0, A[0], geo, grp, cnt, from_erec, xr, dA, (int)M.size(), cs);
}

// fold the recorded launches into the totals.  Called when the totals are
// read (lp_update_time / lp_select_time), not at every sync, so the event
// queries stay out of a timed pivot loop; the events of one call are all
// complete once it has returned (its last step is a stream sync)
static int collect_profile(lp_handle *h)
{
    for (size_t k = 0; k + 1 < h->evused; k += 2) {
        float ms = 0.f;
        HCHK(h, hipEventElapsedTime(&ms, h->ev[k], h->ev[k + 1]));
        if (h->evkind[k / 2] == 1) {
            h->sel_ms += ms;
            h->sel_n += 1;
        } else {
            h->prof_ms += ms;
            h->prof_n += 1;
        }
    }
    h->evused = 0;
    return LP_PIVOTED;
}

static int sync_ctl(const Members &M)
{
    for (lp_handle *h : M) {
        HCHK(h, hipSetDevice(h->dev));
        HCHK(h, hipMemcpyAsync(h->hctl, h->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, h->s));
        if (h->oop) HCHK(h, hipMemcpyAsync(&h->hflips, h->dflips, sizeof(unsigned), hipMemcpyDeviceToHost, h->s));
    }
    for (lp_handle *h : M) HCHK(h, hipStreamSynchronize(h->s));
    // out-of-place sweeps: the buffer the last sweep that RAN wrote (sweeps
    // after a stop or a timed-out group return at once and leave it)
    for (lp_handle *h : M)
        if (h->oop && h->hflips != h->flips) {
            h->flips = h->hflips;
            h->T = h->Tb[h->flips & 1];
        }
    return LP_PIVOTED;
}

static std::vector<Args> args_all(const Members &M)
{
    std::vector<Args> v;
    for (lp_handle *h : M) v.push_back(args_of(h));
    return v;
}

// Leaving-row choice + pivot row of pivot t of group grp.
// sel: 0 = ratio test, 1 = validated row (Simplex.pivot), 2 = explicit row
// (Tableau.pivot).  from_erec: the entering column comes from the previous
// pivot's row-0 summaries (chained pivots).  peek: stop once the leaving row
// is known (findPivot*(False)).
static int enqueue_select(const Members &M, const std::vector<Args> &A, int t, int grp, int sel,
                          int from_erec, bool peek, bool one_exchange = false)
{
    lp_handle *h0 = M[0];
    if (!h0->comm) {
        if (sel == 0) {
            HCHK(h0, lpk::launch_ratio(h0->s, A[0], t, grp, lpk::RATIO_FULL, from_erec, -1));
            HCHK(h0, lpk::launch_prow(h0->s, A[0], t, grp, lpk::RSRC_RECORDS, peek));
        } else {
            if (sel == 1)
                HCHK(h0, lpk::launch_ratio(h0->s, A[0], t, grp, lpk::RATIO_CHECK, 0,
                                           local_row(h0, h0->hctl->r + 1)));
            else HCHK(h0, lpk::launch_gather(h0->s, A[0], t));
            HCHK(h0, lpk::launch_prow(h0->s, A[0], t, grp, lpk::RSRC_GIVEN, 0));
        }
        return LP_PIVOTED;
    }
    if (sel == 0 && one_exchange && !peek) {
        // one allgather per pivot: (index, local min, ratio, current row) per
        // rank; a near-tie straddling the band stops with ST_STRADDLE
        for (size_t k = 0; k < M.size(); ++k)
            HCHK(M[k], lpk::launch_ratio(M[k]->s, A[k], t, grp, lpk::RATIO_FULL, from_erec, -1));
        for (size_t k = 0; k < M.size(); ++k)
            HCHK(M[k], lpk::launch_pick(M[k]->s, A[k], t, lpk::PICK_LOCAL));
        CALL(h0->comm->allgather(M));
        for (size_t k = 0; k < M.size(); ++k)
            HCHK(M[k], lpk::launch_prow(M[k]->s, A[k], t, grp, lpk::RSRC_BAND, 0));
        return LP_PIVOTED;
    }
    for (size_t k = 0; k < M.size(); ++k) {
        if (sel == 2) HCHK(M[k], lpk::launch_gather(M[k]->s, A[k], t));
        else HCHK(M[k], lpk::launch_ratio(M[k]->s, A[k], t, grp, lpk::RATIO_LOCAL, from_erec, -1));
    }
    if (sel != 2) CALL(h0->comm->allreduce_min(M));
    const int pm = sel == 0 ? lpk::PICK_RATIO : sel == 1 ? lpk::PICK_CHECK : lpk::PICK_EXPLICIT;
    for (size_t k = 0; k < M.size(); ++k) HCHK(M[k], lpk::launch_pick(M[k]->s, A[k], t, pm));
    CALL(h0->comm->allgather(M));
    for (size_t k = 0; k < M.size(); ++k)
        HCHK(M[k], lpk::launch_prow(M[k]->s, A[k], t, grp, lpk::RSRC_SLOTS, peek));
    return LP_PIVOTED;
}

// (out of place: a sweep that wrote the other buffer makes it the tableau of
// every later launch -- the handle's T and the members' Args)
static int enqueue_sweep(const Members &M, std::vector<Args> &A, int grp, int cnt)
{
    for (size_t k = 0; k < M.size(); ++k) {
        lp_handle *h = M[k];
        bool flipped = false;
        CALL(launch_sweep_timed(h, A[k], grp, cnt, &flipped));
        if (flipped) {
            h->flips += 1;
            h->T = h->Tb[h->flips & 1];
            A[k] = args_of(h);
        }
    }
    return LP_PIVOTED;
}

// every call starts here: eager row 0 / column 0 current, control reset
static int begin_call(const Members &M, const std::vector<Args> &A, int mode, int rule, int chain,
                      int64_t cap, int64_t r, int64_t c)
{
    for (size_t k = 0; k < M.size(); ++k) {
        lp_handle *h = M[k];
        HCHK(h, hipSetDevice(h->dev));
        if (!h->eager_ok) {
            HCHK(h, lpk::launch_load_eager(h->s, A[k]));
            h->eager_ok = true;
        }
        HCHK(h, lpk::launch_reset(h->s, A[k], mode, rule, chain, cap, r, c));
        h->hctl->r = r;
        h->hctl->c = c;
    }
    return LP_PIVOTED;
}

// ---------------------------------------------------------------------------
// the pivot loop
// ---------------------------------------------------------------------------

// A persistent group timed out: one of its exchanges never completed (every
// block of the launch must be resident at once -- the launch is sized from
// the compiled kernel's occupancy, so this is never expected; a fault-
// injection test covers it).  The failed group's sweep and every later launch
// of the batch were skipped, so each member's stored tableau holds the state
// at the start of the failed group.  Restore the loop state the group's
// prologue recorded (Ctl::g_*), reload the eager row 0 / column 0 from the
// tableau and go on with the per-pivot kernels: the same float64 operations,
// so the results are unchanged.
static int recover_timeout(const Members &M, const std::vector<Args> &A, int mode, int rule, int64_t cap,
                           unsigned first_seq)
{
    for (size_t k = 0; k < M.size(); ++k) {
        lp_handle *h = M[k];
        Ctl c = *h->hctl;
        // the handle stays on the per-pivot kernels from here on (a timeout
        // is never expected; lp_exchange_path reports it as a fallback), and
        // its automatic pivots per sweep is re-chosen for those kernels
        h->persistent = false;
        h->block_auto = 0;
        h->fallbacks += 1;
        h->eager_ok = false;
        HCHK(h, lpk::launch_load_eager(h->s, A[k]));
        h->eager_ok = true;
        if (c.g_seq == 0 || c.g_seq == first_seq) {
            // the call's first group: its prologue may not have run at all
            HCHK(h, lpk::launch_reset(h->s, A[k], mode, rule, 1, cap, -1, -1));
            c.npiv = 0;
            c.status = LP_PIVOTED;
        } else {
            c.status = LP_PIVOTED;
            c.npiv = c.g_npiv;
            c.nstd = c.g_nstd;
            c.stuck = c.g_stuck;
            c.rule = c.g_rule;
            c.bar_timeout = 0;
            c.ndef[0] = c.ndef[1] = 0;
            c.g_seq = 0;
            *h->hctl = c;
            HCHK(h, hipMemcpyAsync(h->ctl, h->hctl, sizeof(Ctl), hipMemcpyHostToDevice, h->s));
        }
        HCHK(h, hipStreamSynchronize(h->s));
        h->hctl->npiv = c.npiv;
        h->hctl->status = LP_PIVOTED;
        h->hctl->bar_timeout = 0;
        h->err = (c.sel_flags & 8u) ? "the one-XCD selection's blocks were not on one XCD; the group was redone on "
                                      "the per-pivot kernels"
                                    : "a persistent selection group timed out; it was redone on the per-pivot kernels";
    }
    return LP_PIVOTED;
}

// A multi-process job's ranks decide about a timed-out cross-rank group
// together: every rank all-gathers (timed out, the group it was in) at the end
// of each batch.  If they all timed out in the same group, each redoes it on
// the per-pivot kernels (recover_timeout) in lock-step.  If only some did --
// a rank that saw every summary of the last group finished it and swept its
// rows -- the ranks' tableaux are at different pivots and cannot be realigned:
// every rank returns LP_DEVICE_ERROR instead of running collectives that no
// longer pair up.  (In-process shard groups time out together: one launch.)
static int agree_on_timeout(lp_handle *h, bool &timed_out)
{
    auto *rc = dynamic_cast<RcclComm *>(h->comm.get());
    // no collective at all (peer exchange only): nothing to agree with
    if (!rc || h->nranks < 2 || (!rc->comm && !rc->host_fn)) return LP_PIVOTED;
    const long long mine[2] = {timed_out ? 1LL : 0LL, timed_out ? (long long)h->hctl->g_npiv : -1LL};
    std::vector<long long> all(2 * (size_t)h->nranks);
    CALL(rc->gather_host(h, mine, all.data(), sizeof(mine)));
    bool any = false, same = true;
    for (int r = 0; r < h->nranks; ++r) {
        any = any || all[2 * r] != 0;
        same = same && all[2 * r] == all[0] && all[2 * r + 1] == all[1];
    }
    if (any && !same)
        return fail(h, LP_DEVICE_ERROR,
                    "a cross-rank selection group timed out on some ranks only; the shards are no longer "
                    "at the same pivot");
    timed_out = any;
    return LP_PIVOTED;
}

// Runs pivots until the device reports a status other than LP_PIVOTED or
// `limit` pivots have been enqueued (limit < 0: unlimited).  Pivots are
// enqueued in groups of `block` followed by one sweep; the host knows each
// pivot's index t in its group and the group parity.  Batch sizes are a
// deterministic sequence, so every rank of a sharded job enqueues the same
// collectives in the same order.
static int pivot_loop(lp_handle *h, int mode, int rule, int64_t cap, int64_t limit)
{
    const Members M = members_of(h);
    std::vector<Args> A = args_all(M);
    int xr = 0;
    lpk::GroupGeom geo = persistent_geom(h, M, &xr);
    CallStart cs;
    for (lp_handle *x : M) HCHK(x, hipSetDevice(x->dev));
    if (geo.g > 0) {
        // reset, eager copies and the first entering column happen in the
        // first k_group launch (no k_reset / k_load_eager / k_enter launches)
        bool eager = true;
        for (lp_handle *x : M) eager = eager && x->eager_ok;
        cs.first = 1 | 4 | (eager ? 0 : 2);
        cs.mode = mode;
        cs.rule = rule;
        cs.cap = cap;
        for (lp_handle *x : M) {
            x->eager_ok = true;
            x->hctl->r = x->hctl->c = -1;
        }
    } else {
        CALL(begin_call(M, A, mode, rule, 1, cap, -1, -1));
        for (size_t k = 0; k < M.size(); ++k) HCHK(M[k], lpk::launch_enter(M[k]->s, A[k]));
    }
    // (re-read after a timeout recovery: the per-pivot kernels take their own
    // automatic depth, and the sweep launches ask block_of for theirs)
    int B = block_of(h);
    int64_t done = 0;      // pivots performed (device count)
    int64_t batch = 2 * B;   // open-ended solves: few launches for a short solve, then doubling
    int grp = 0;
    bool chained = false;  // the next pivot's entering column comes from the previous pivot
    unsigned first_seq = 0;
    for (;;) {
        // a known pivot count goes in one batch (launches after a stop exit
        // at once); open-ended solves grow their batches
        int64_t b = batch;
        if (limit >= 0) b = std::min<int64_t>(limit - done, std::max<int64_t>(batch, 1 << 15));
        for (lp_handle *x : M) CALL(ensure_log(x, done + b + 1));
        A = args_all(M);
        const int path = geo.g > 0 ? (h->comm ? LP_PATH_PEER : LP_PATH_PERSISTENT)
                                   : (h->comm ? LP_PATH_COLLECTIVE : LP_PATH_KERNELS);
        for (lp_handle *x : M) x->last_path = path;
        if (geo.g > 0) {
            // one persistent selection launch (per rank) + one in-place sweep per group
            for (int64_t k = 0; k < b; k += B) {
                const int cnt = (int)std::min<int64_t>(B, b - k);
                CALL(enqueue_group(M, A, geo, xr, grp, cnt, chained ? 1 : 0, cs));
                if (cs.first) first_seq = M[0]->gseq;
                cs.first = 0;
                CALL(enqueue_sweep(M, A, grp, cnt));
                grp ^= 1;
                chained = true;
            }
        } else {
            int t = 0;
            for (int64_t k = 0; k < b; ++k) {
                CALL(enqueue_select(M, A, t, grp, 0, chained ? 1 : 0, false, true));
                chained = true;
                if (++t == B || k + 1 == b) {
                    CALL(enqueue_sweep(M, A, grp, t));
                    grp ^= 1;
                    t = 0;
                }
            }
        }
        CALL(sync_ctl(M));
        A = args_all(M);                     // (out of place: the buffer the last sweep that ran wrote)
        bool timed_out = false;
        for (lp_handle *x : M) timed_out = timed_out || x->hctl->bar_timeout != 0;
        if (geo.g > 0 && xr) CALL(agree_on_timeout(h, timed_out));
        if (timed_out) {
            if (geo.g == 0) return fail(h, LP_DEVICE_ERROR, "exchange timed out on the per-pivot path");
            if (h->strict) return fail(h, LP_DEVICE_ERROR, "persistent selection group timed out (LPGPU_STRICT)");
            CALL(recover_timeout(M, A, mode, rule, cap, first_seq));
            geo = lpk::GroupGeom{};
            // groups of the depth the sweeps now take (recover_timeout re-chose
            // the automatic one for the per-pivot kernels): a group deeper than
            // the sweep kernel's compiled bound would drop pivots
            B = block_of(h);
            batch = std::min<int64_t>(batch, std::max<int64_t>(1024, 32 * B));
            for (size_t k = 0; k < M.size(); ++k) HCHK(M[k], lpk::launch_enter(M[k]->s, A[k]));
            chained = false;
            grp = 0;
            done = h->hctl->npiv;
            continue;
        }
        if (h->hctl->status == lpk::ST_STRADDLE) {
            // rare near-tie across ranks: the pivots before it are swept and
            // ctl->c holds its entering column; redo it with two exchanges
            for (size_t k = 0; k < M.size(); ++k) HCHK(M[k], lpk::launch_resume(M[k]->s, A[k]));
            CALL(enqueue_select(M, A, 0, grp, 0, 0, false, false));
            CALL(enqueue_sweep(M, A, grp, 1));
            grp ^= 1;
            CALL(sync_ctl(M));
        }
        done = h->hctl->npiv;
        if (h->hctl->status != LP_PIVOTED) return h->hctl->status;
        if (limit >= 0 && done >= limit) return LP_PIVOTED;
        batch = std::min<int64_t>(batch * 2, std::max<int64_t>(1024, 32 * B));
    }
}

extern "C" int lp_solve(lp_handle *h, int64_t max_pivots, int64_t *npiv, int64_t *nstd)
{
    const int st = pivot_loop(h, lpk::MODE_SOLVE, LP_RULE_STANDARD, max_pivots, -1);
    *npiv = h->hctl->npiv;
    *nstd = h->hctl->nstd;
    return st;
}

extern "C" int lp_run(lp_handle *h, int rule, int64_t k, int64_t *done)
{
    *done = 0;
    if (rule != LP_RULE_STANDARD && rule != LP_RULE_MIN_INDEX)
        return fail(h, LP_BAD_ARG, "unknown rule");
    if (k < 0) return fail(h, LP_BAD_ARG, "k < 0");
    const int st = pivot_loop(h, lpk::MODE_RUN, rule, -1, k);
    *done = h->hctl->npiv;
    return st;
}

extern "C" int lp_find_pivot(lp_handle *h, int rule, int do_pivot, int64_t *r, int64_t *c)
{
    *r = -1;
    *c = -1;
    if (rule != LP_RULE_STANDARD && rule != LP_RULE_MIN_INDEX)
        return fail(h, LP_BAD_ARG, "unknown rule");
    const Members M = members_of(h);
    std::vector<Args> A = args_all(M);
    CALL(begin_call(M, A, lpk::MODE_RUN, rule, 0, -1, -1, -1));
    for (size_t k = 0; k < M.size(); ++k) HCHK(M[k], lpk::launch_enter(M[k]->s, A[k]));
    CALL(enqueue_select(M, A, 0, 0, 0, 0, do_pivot == 0));
    if (do_pivot) CALL(enqueue_sweep(M, A, 0, 1));
    CALL(sync_ctl(M));
    if (h->hctl->status == LP_PIVOTED) {
        *r = h->hctl->r;
        *c = h->hctl->c;
    }
    return h->hctl->status;
}

static int explicit_pivot(lp_handle *h, int64_t r, int64_t c, bool checked)
{
    if (r < 0 || r >= h->m || c < 0 || c >= h->n)
        return fail(h, LP_BAD_ARG, "pivot index out of range");
    const Members M = members_of(h);
    std::vector<Args> A = args_all(M);
    CALL(begin_call(M, A, lpk::MODE_RUN, LP_RULE_STANDARD, 0, -1, r, c));
    CALL(enqueue_select(M, A, 0, 0, checked ? 1 : 2, 0, false));
    CALL(enqueue_sweep(M, A, 0, 1));
    CALL(sync_ctl(M));
    return h->hctl->status;
}

extern "C" int lp_pivot(lp_handle *h, int64_t r, int64_t c) { return explicit_pivot(h, r, c, false); }

extern "C" int lp_pivot_checked(lp_handle *h, int64_t r, int64_t c)
{
    return explicit_pivot(h, r, c, true);
}

// ---------------------------------------------------------------------------
// column scans: findPivotMaxIncrease, findPivotAll, form checks.  The stored
// tableau is current at every API boundary (each call sweeps its pending
// pivots).  Per-column results of every shard are combined on the host in
// rank order: the shards of one process directly, a multi-process job's
// through one all-gather per pass (RCCL, or the host's own collective).
// ---------------------------------------------------------------------------

static int scan_members(lp_handle *h, Members &M)
{
    M = members_of(h);
    for (lp_handle *x : M) {
        HCHK(x, hipSetDevice(x->dev));
        if (!x->eager_ok) {                  // row 0 / column 0 mirrors after an upload
            HCHK(x, lpk::launch_load_eager(x->s, args_of(x)));
            x->eager_ok = true;
        }
        if (!x->cstat) {
            HCHK(x, hipMalloc(&x->cstat, x->ld * sizeof(lpk::ColStat)));
            HCHK(x, hipMalloc(&x->cthr, x->ld * sizeof(double)));
            HCHK(x, hipMalloc(&x->cfirst, x->ld * sizeof(long long)));
            HCHK(x, hipMalloc(&x->ccount, x->ld * sizeof(long long)));
            HCHK(x, hipMalloc(&x->coffs, x->ld * sizeof(long long)));
            HCHK(x, hipMalloc(&x->rowflag, std::max<int64_t>(x->rc, 1) * sizeof(int)));
        }
    }
    return LP_PIVOTED;
}

// the scan results of every shard in rank order: the in-process members, or
// this process's shard and its peers' through the all-gather
template <class T>
static int gather_parts(lp_handle *h, const std::vector<T> &mine, std::vector<std::vector<T>> &parts)
{
    RcclComm *rc = multi_process(h);
    if (!rc) {
        parts.push_back(mine);
        return LP_PIVOTED;
    }
    std::vector<T> all(mine.size() * h->nranks);
    CALL(rc->gather_host(h, mine.data(), all.data(), mine.size() * sizeof(T)));
    parts.clear();
    for (int k = 0; k < h->nranks; ++k)
        parts.emplace_back(all.begin() + k * mine.size(), all.begin() + (k + 1) * mine.size());
    return LP_PIVOTED;
}

// per-column statistics over every shard, and the current row 0
static int column_stats(lp_handle *h, const Members &M, std::vector<lpk::ColStat> &cs,
                        std::vector<double> &row0)
{
    row0.assign(h->ld, 0.0);
    HCHK(h, hipMemcpyAsync(row0.data(), M[0]->row0, h->ld * sizeof(double), hipMemcpyDeviceToHost,
                           M[0]->s));
    std::vector<std::vector<lpk::ColStat>> parts;
    std::vector<lpk::ColStat> part(h->ld);
    for (lp_handle *x : M) {
        HCHK(x, lpk::launch_colstat(x->s, args_of(x), x->cstat));
        HCHK(x, hipMemcpyAsync(part.data(), x->cstat, x->ld * sizeof(lpk::ColStat),
                               hipMemcpyDeviceToHost, x->s));
        HCHK(x, hipStreamSynchronize(x->s));
        std::vector<std::vector<lpk::ColStat>> p;
        CALL(gather_parts(x, part, p));
        for (auto &q : p) parts.push_back(std::move(q));
    }
    cs = parts[0];
    for (size_t k = 1; k < parts.size(); ++k)
        for (int64_t j = 0; j < h->ld; ++j) {
            lpk::ColStat &c = cs[j];
            const lpk::ColStat &d = parts[k][j];
            c.gmin = std::min(c.gmin, d.gmin);
            c.npos += d.npos;
            c.npos0 += d.npos0;
            c.nnz += d.nnz;
            c.nneg += d.nneg;
            c.none += d.none;
            c.one_row = std::min(c.one_row, d.one_row);
        }
    return LP_PIVOTED;
}

// rows inside the band thr[j] of every shard: first[j] (global, first shard
// in rank order that has one) and per-shard counts (every shard of the job,
// rank order)
static int band_pass(lp_handle *h, const Members &M, const std::vector<double> &thr,
                     std::vector<long long> &first, std::vector<std::vector<long long>> &counts)
{
    first.assign(h->ld, lpk::NONE);
    counts.clear();
    std::vector<long long> fc(2 * h->ld);
    for (lp_handle *x : M) {
        HCHK(x, hipMemcpyAsync(x->cthr, thr.data(), x->ld * sizeof(double), hipMemcpyHostToDevice, x->s));
        HCHK(x, lpk::launch_colband(x->s, args_of(x), x->cthr, x->cfirst, x->ccount, nullptr, nullptr));
        HCHK(x, hipMemcpyAsync(fc.data(), x->cfirst, x->ld * sizeof(long long), hipMemcpyDeviceToHost, x->s));
        HCHK(x, hipMemcpyAsync(fc.data() + x->ld, x->ccount, x->ld * sizeof(long long),
                               hipMemcpyDeviceToHost, x->s));
        HCHK(x, hipStreamSynchronize(x->s));
        std::vector<std::vector<long long>> p;
        CALL(gather_parts(x, fc, p));
        for (auto &q : p) {
            for (int64_t j = 0; j < h->ld; ++j)
                if (first[j] == lpk::NONE) first[j] = q[j];
            counts.emplace_back(q.begin() + h->ld, q.end());
        }
    }
    return LP_PIVOTED;
}

static double band_of(double g, double tie) { return g + tie * std::fabs(g); }

extern "C" int lp_find_pivot_max_increase(lp_handle *h, int do_pivot, int64_t *r, int64_t *c)
{
    *r = -1;
    *c = -1;
    Members M;
    CALL(scan_members(h, M));
    std::vector<lpk::ColStat> cs;
    std::vector<double> row0;
    CALL(column_stats(h, M, cs, row0));
    const lp_tol &tol = h->tol;
    bool any_neg = false;
    double best = -INFINITY;
    std::vector<double> inc(h->n + 1, -INFINITY);
    for (int64_t j = 1; j <= h->n; ++j) {
        if (!(row0[j] < -tol.cost)) continue;
        any_neg = true;
        if (cs[j].npos == 0) return LP_UNBOUNDED;        // simplex.py:319-320
        inc[j] = -row0[j] * cs[j].gmin;
        best = std::max(best, inc[j]);
    }
    if (!any_neg) return LP_OPTIMAL;
    // first column within the tie band of the largest increase; a non-finite
    // largest increase (an overflowed -c_j * ratio) takes the first column
    // that attains it
    int64_t js = 0;
    if (std::isfinite(best)) {
        const double lim = best - tol.ratio_tie * std::fabs(best);
        for (int64_t j = 1; j <= h->n && js == 0; ++j)
            if (inc[j] >= lim) js = j;
    }
    for (int64_t j = 1; j <= h->n && js == 0; ++j)
        if (inc[j] == best) js = j;
    if (js == 0) return fail(h, LP_DEVICE_ERROR, "max-increase selection found no column");
    std::vector<double> thr(h->ld, INFINITY);
    thr[js] = band_of(cs[js].gmin, tol.ratio_tie);
    std::vector<long long> first;
    std::vector<std::vector<long long>> counts;
    CALL(band_pass(h, M, thr, first, counts));
    *r = first[js];
    *c = js - 1;
    if (do_pivot) {
        const int st = lp_pivot(h, *r, *c);
        if (st != LP_PIVOTED) return st;
    }
    return LP_PIVOTED;
}

extern "C" int lp_find_pivot_all(lp_handle *h, int64_t *rc, int64_t cap, int64_t *count)
{
    *count = 0;
    Members M;
    CALL(scan_members(h, M));
    std::vector<lpk::ColStat> cs;
    std::vector<double> row0;
    CALL(column_stats(h, M, cs, row0));
    std::vector<double> thr(h->ld, INFINITY);
    for (int64_t j = 1; j <= h->n; ++j)
        if (cs[j].npos > 0) thr[j] = band_of(cs[j].gmin, h->tol.ratio_tie);
    std::vector<long long> first;
    std::vector<std::vector<long long>> counts;
    CALL(band_pass(h, M, thr, first, counts));
    // column-major, shards (= rows) in order within a column
    const size_t S = counts.size();                 // shards of the whole job
    std::vector<std::vector<long long>> offs(S, std::vector<long long>(h->ld, 0));
    long long total = 0;
    for (int64_t j = 1; j <= h->n; ++j)
        for (size_t k = 0; k < S; ++k) {
            offs[k][j] = total;
            total += counts[k][j];
        }
    *count = total;
    if (total == 0 || cap <= 0) return LP_PIVOTED;
    long long *pairs = nullptr;
    HCHK(h, hipMalloc(&pairs, (size_t)total * 2 * sizeof(long long)));
    int st = LP_PIVOTED;
    RcclComm *mp = multi_process(h);
    for (size_t k = 0; k < M.size() && st == LP_PIVOTED; ++k) {
        lp_handle *x = M[k];
        const size_t ks = mp ? (size_t)x->rank : k;
        if (hipMemcpyAsync(x->cthr, thr.data(), x->ld * sizeof(double), hipMemcpyHostToDevice, x->s) !=
                hipSuccess ||
            hipMemcpyAsync(x->coffs, offs[ks].data(), x->ld * sizeof(long long), hipMemcpyHostToDevice,
                           x->s) != hipSuccess ||
            lpk::launch_colband(x->s, args_of(x), x->cthr, x->cfirst, x->ccount, x->coffs, pairs) !=
                hipSuccess ||
            hipStreamSynchronize(x->s) != hipSuccess)
            st = fail(h, LP_DEVICE_ERROR, "find-all pair pass failed");
    }
    std::vector<long long> mine((size_t)total * 2);
    if (st == LP_PIVOTED &&
        hipMemcpy(mine.data(), pairs, mine.size() * sizeof(long long), hipMemcpyDeviceToHost) != hipSuccess)
        st = fail(h, LP_DEVICE_ERROR, "find-all readback failed");
    (void)hipFree(pairs);
    if (st != LP_PIVOTED) return st;
    if (mp) {
        // every rank wrote only its own slots: take each slot from its owner
        std::vector<std::vector<long long>> p;
        CALL(gather_parts(h, mine, p));
        for (int64_t j = 1; j <= h->n; ++j)
            for (size_t k = 0; k < S; ++k)
                for (long long q = offs[k][j]; q < offs[k][j] + counts[k][j]; ++q) {
                    mine[2 * q] = p[k][2 * q];
                    mine[2 * q + 1] = p[k][2 * q + 1];
                }
    }
    const long long keep = std::min<long long>(total, cap);
    std::memcpy(rc, mine.data(), (size_t)keep * 2 * sizeof(long long));
    return LP_PIVOTED;
}

extern "C" int lp_form_checks(lp_handle *h, int32_t *flags, int64_t *bcols)
{
    Members M;
    CALL(scan_members(h, M));
    std::vector<lpk::ColStat> cs;
    std::vector<double> row0;
    CALL(column_stats(h, M, cs, row0));
    int infeasible = 0;
    std::vector<int> rf;
    for (lp_handle *x : M) {
        rf.assign(std::max<int64_t>(x->rc, 1), 0);
        HCHK(x, lpk::launch_rowpos(x->s, args_of(x), x->rowflag));
        HCHK(x, hipMemcpyAsync(rf.data(), x->rowflag, x->rc * sizeof(int), hipMemcpyDeviceToHost, x->s));
        HCHK(x, hipStreamSynchronize(x->s));
        int any = 0;
        for (int64_t i = 0; i < x->rc; ++i) any |= rf[i];
        std::vector<std::vector<int>> p;
        CALL(gather_parts(x, std::vector<int>{any}, p));
        for (auto &q : p) infeasible |= q[0];
    }
    // isCanonical (tableau.py:466-496): b >= 0, then per row the first column
    // with zero reduced cost that is a unit vector with its 1 there
    const bool ok_b = cs[0].nneg == 0;
    std::vector<int64_t> found(h->m, -1);
    if (ok_b)
        for (int64_t j = 1; j <= h->n; ++j)
            if (row0[j] == 0.0 && cs[j].nnz == 1 && cs[j].none == 1) {
                const long long i = cs[j].one_row;
                if (i >= 0 && i < h->m && found[i] == -1) found[i] = j - 1;
            }
    bool canonical = ok_b;
    for (int64_t i = 0; i < h->m && canonical; ++i) canonical = found[i] != -1;
    if (ok_b && bcols)                       // the reference leaves bcols alone when b < 0
        for (int64_t i = 0; i < h->m; ++i) bcols[i] = found[i];
    bool optimal = true, unbounded = false;
    for (int64_t j = 1; j <= h->n; ++j) {
        optimal = optimal && row0[j] >= 0.0;                          // tableau.py:500-502
        unbounded = unbounded || (row0[j] < 0.0 && cs[j].npos0 == 0);  // :504-508
    }
    flags[0] = canonical;
    flags[1] = optimal;
    flags[2] = unbounded;
    flags[3] = infeasible;                                  // :510-514
    flags[4] = cs[0].nnz < h->m;                            // :516-518: some b_i == 0
    return LP_PIVOTED;
}

extern "C" int lp_xwait(const lp_handle *h, int64_t *ticks, int64_t *pivots)
{
    *ticks = (int64_t)h->hctl->xwait_ticks;
    *pivots = h->hctl->xwait_pivots;
    return LP_PIVOTED;
}

extern "C" int lp_exchange_path(const lp_handle *h, int *path, int *fallbacks)
{
    *path = h->last_path;
    *fallbacks = h->fallbacks;
    return LP_PIVOTED;
}

extern "C" int lp_pivot_log(lp_handle *h, int64_t *rc, int64_t cap, int64_t *count)
{
    const int64_t n = h->hctl->npiv;
    *count = n;
    const int64_t k = std::min(std::min(n, cap), h->logcap);
    if (k > 0) {
        HCHK(h, hipSetDevice(h->dev));
        HCHK(h, hipMemcpyAsync(rc, h->log, (size_t)k * 2 * sizeof(long long),
                               hipMemcpyDeviceToHost, h->s));
        HCHK(h, hipStreamSynchronize(h->s));
    }
    return LP_PIVOTED;
}

extern "C" int lp_objective(lp_handle *h, double *z)
{
    double v = 0.0;
    HCHK(h, hipSetDevice(h->dev));
    HCHK(h, hipMemcpyAsync(&v, h->T, sizeof(double), hipMemcpyDeviceToHost, h->s));
    HCHK(h, hipStreamSynchronize(h->s));
    *z = -v;
    return LP_PIVOTED;
}

extern "C" int lp_profile(lp_handle *h, int enable)
{
    for (lp_handle *x : members_of(h)) {
        if (!x) continue;
        x->prof = enable != 0;
        x->prof_every = enable > 1 ? enable : 1;
        x->prof_seen[0] = x->prof_seen[1] = 0;
        x->prof_ms = 0.0;
        x->prof_n = 0;
        x->sel_ms = 0.0;
        x->sel_n = 0;
        x->evused = 0;
    }
    return LP_PIVOTED;
}

extern "C" int lp_select_time(lp_handle *h, double *ms, int64_t *launches)
{
    CALL(collect_profile(h));
    *ms = h->sel_ms;
    *launches = h->sel_n;
    return LP_PIVOTED;
}

extern "C" int lp_update_time(lp_handle *h, double *ms, int64_t *launches)
{
    CALL(collect_profile(h));
    *ms = h->prof_ms;
    *launches = h->prof_n;
    return LP_PIVOTED;
}

// diagnostic (not part of the C-ABI): k_group phase clocks of the last group
extern "C" int lpdiag_bstamps(lp_handle *h, long long *out)
{
    if (!h || !out || !h->stamps) return LP_BAD_ARG;
    HCHK(h, hipMemcpy(out, h->stamps + lpk::BMAX * 16,
                      lpk::GROUP_MAXBLOCKS * lpk::BMAX * 4 * sizeof(long long), hipMemcpyDeviceToHost));
    return LP_PIVOTED;
}

// diagnostics: the persistent selection this handle's pivot loops launch and
// what its last launch found on the device.  out[0..7] = blocks per shard,
// own columns per lane, own rows per lane, summaries per lane, one-XCD grid,
// k_group's two-level variant, k_sel's pivot capacity (0: k_group),
// Ctl::sel_flags of the last launch (1 one XCD, 2 two-level exchange engaged,
// 4 k_sel, 8 k_sel's blocks were not on one XCD, 16 k_sel as XCD shards), the
// XCD shards of the launch (out[8], 0: none); all 0 when the per-pivot kernels
// run
extern "C" int lpdiag_geometry(lp_handle *h, long long *out)
{
    if (!h || !out) return LP_BAD_ARG;
    const Members M = members_of(h);
    int xr = 0;
    const lpk::GroupGeom g = persistent_geom(h, M, &xr);
    out[0] = g.g;
    out[1] = g.ipl;
    out[2] = g.rpl;
    out[3] = g.nr;
    out[4] = g.xmode;
    out[5] = g.hk;
    out[6] = g.sel;
    out[7] = h->hctl->sel_flags;
    out[8] = g.xs;
    return LP_PIVOTED;
}

// diagnostics: the per-launch clock records of the 64-pivot sweep (Args::
// sweep_clk): up to `cap` of the latest, oldest first, 4 values each (launch
// number, shader cycles, 100 MHz ticks, start tick) -> *n records
extern "C" int lpdiag_sweep_clocks(lp_handle *h, unsigned long long *out, int cap, int *n)
{
    if (!h || !out || !n || cap < 0) return LP_BAD_ARG;
    HCHK(h, hipSetDevice(h->dev));
    HCHK(h, hipStreamSynchronize(h->s));
    std::vector<unsigned long long> ring((size_t)lpk::SWEEP_CLK_RING * 4);
    HCHK(h, hipMemcpy(ring.data(), h->sweep_clk, ring.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    const long long last = (long long)h->sweep_lseq;
    const long long first = std::max(0LL, last - std::min<long long>(cap, lpk::SWEEP_CLK_RING));
    int k = 0;
    for (long long q = first; q < last; ++q) {
        const unsigned long long *e = &ring[(size_t)(q % lpk::SWEEP_CLK_RING) * 4];
        if (e[0] != (unsigned long long)(unsigned)q) continue;   // a launch that returned early (no record)
        for (int j = 0; j < 4; ++j) out[4 * k + j] = e[j];
        ++k;
    }
    *n = k;
    return LP_PIVOTED;
}

// diagnostics: every block's pass in the latest 64-pivot sweep launch (4
// values each: block, start tick, pass-end tick, shader cycles; 100 MHz
// ticks of one device-wide clock) -> *n blocks
extern "C" int lpdiag_sweep_block_clocks(lp_handle *h, unsigned long long *out, int cap, int *n)
{
    if (!h || !out || !n || cap < 0) return LP_BAD_ARG;
    HCHK(h, hipSetDevice(h->dev));
    HCHK(h, hipStreamSynchronize(h->s));
    std::vector<unsigned long long> blk((size_t)lpk::SWEEP_BLK_MAX * 4);
    HCHK(h, hipMemcpy(blk.data(), h->sweep_clk + (size_t)lpk::SWEEP_CLK_RING * 4, blk.size() * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost));
    // the latest launch that ran (later ones of a batch may have returned at
    // once: the solve had stopped, or nothing was deferred)
    unsigned long long last = 0;
    bool any = false;
    for (int b = 0; b < lpk::SWEEP_BLK_MAX; ++b) {
        const unsigned long long v = blk[(size_t)b * 4];
        if (v == ~0ull) continue;
        if (!any || v > last) last = v;
        any = true;
    }
    int k = 0;
    for (int b = 0; any && b < lpk::SWEEP_BLK_MAX && k < cap; ++b) {
        const unsigned long long *e = &blk[(size_t)b * 4];
        if (e[0] != last) continue;
        out[4 * k] = (unsigned long long)b;
        out[4 * k + 1] = e[1];
        out[4 * k + 2] = e[2];
        out[4 * k + 3] = e[3];
        ++k;
    }
    *n = k;
    return LP_PIVOTED;
}

// diagnostics: the tableau buffers the sweeps use -- 2 out of place (the
// sweep reads one and writes the other), 1 in place
extern "C" int lpdiag_sweep_buffers(const lp_handle *h, int *nbuf)
{
    if (!h || !nbuf) return LP_BAD_ARG;
    *nbuf = h->oop ? 2 : 1;
    return LP_PIVOTED;
}

// diagnostics / A/B: whether a tall single-device tableau may run k_sel as XCD
// shards (1, default) or takes k_group (0); re-chooses the automatic pivots per
// sweep
extern "C" int lpdiag_set_xcd_shards(lp_handle *h, int on)
{
    if (!h) return LP_BAD_ARG;
    h->xs_ok = on != 0;
    h->block_auto = 0;
    return LP_PIVOTED;
}

extern "C" int lpdiag_stamps(lp_handle *h, long long *out)
{
    if (!h || !out || !h->stamps) return LP_BAD_ARG;
    HCHK(h, hipMemcpy(out, h->stamps, lpk::BMAX * 16 * sizeof(long long), hipMemcpyDeviceToHost));
    return LP_PIVOTED;
}
