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
constexpr int RATIO_FULL = 0;   // single device: pick the leaving row directly
constexpr int RATIO_LOCAL = 1;  // sharded: publish this rank's minimum ratio only
constexpr int RATIO_CHECK = 2;  // single device: validate a given row (Simplex.pivot)

// k_pick modes (sharded)
constexpr int PICK_RATIO = 0;     // first local row within the tie band of the global min
constexpr int PICK_CHECK = 1;     // owner validates the requested row (Simplex.pivot)
constexpr int PICK_EXPLICIT = 2;  // owner contributes the requested row (Tableau.pivot)

constexpr int RATIO_THREADS = 256;
constexpr int RATIO_CHUNK = 256;   // rows per ratio block (one per thread)
constexpr int UPD_ROWS = 64;       // rows per update block
constexpr int UPD_UNROLL = 4;      // rows in flight per wave
constexpr int ENTER_THREADS = 1024;
constexpr int SLOT_HDR = 8;        // doubles of header in front of an exchanged row

constexpr long long NONE = 0x7fffffffffffffffLL;

// Device-resident control block: the pivot loop's whole state lives here so
// a batch of pivots is enqueued without host round trips.
struct Ctl {
    int status;          // lp_status of the current step; LP_PIVOTED = keep going
    int mode;            // MODE_RUN / MODE_SOLVE
    int rule;            // lp_rule for the next selection
    int pad0;
    long long r, c;      // current pivot (global constraint index, variable index)
    long long npiv;      // pivots performed since the last reset
    long long nstd;      // of which with the standard rule (solve mode)
    long long stuck;     // steps_stuck (simplex.py:119)
    long long cap;       // pivot cap (< 0: none)
    double z0;           // obj_val at the start of solve (simplex.py:118)
    unsigned ticket;     // last-block ticket of k_ratio
    unsigned pad1;
};

// Per-block ratio-test summary.
struct Rec {
    double l;            // block minimum ratio (INFINITY if no eligible row)
    long long i;         // first local row within the tie band of l
    double q;            // its ratio
    double pad;
};

// Row-exchange slot: header + one raw tableau row (ld doubles).
//   hdr[0] = candidate global constraint index (NONE if none), as int64 bits
//   hdr[1] = code (0, LP_BAD_PIVOT or LP_ZERO_PIVOT), as int64 bits
struct Args {
    double *T;           // local tableau: row 0 + local constraint rows
    double *P;           // normalised pivot row (ld doubles)
    double *mult;        // column snapshot, one per local row
    Ctl *ctl;
    long long *log;      // (r, c) per pivot
    Rec *rec;
    double *xg;          // sharded: this rank's / the global minimum ratio (1 double)
    double *xs;          // sharded: send slot (SLOT_HDR + ld)
    double *xr;          // sharded: gathered slots (nranks x (SLOT_HDR + ld))
    long long logcap;
    long long m, n;      // GLOBAL problem size
    long long ld;        // leading dimension (doubles)
    long long rows;      // local rows incl. row 0
    long long rb;        // first global constraint row of this rank
    long long rc;        // local constraint rows
    int nranks;
    int pad;
    lp_tol tol;
};

// launch wrappers (kernels.hip)
hipError_t launch_reset(hipStream_t s, Ctl *ctl, int mode, int rule, long long cap, long long r,
                        long long c, const double *T);
hipError_t launch_enter(hipStream_t s, const Args &A);
hipError_t launch_ratio(hipStream_t s, const Args &A, int mode, long long check_local_row);
hipError_t launch_pick(hipStream_t s, const Args &A, int mode);
hipError_t launch_gather(hipStream_t s, const Args &A);
hipError_t launch_prow(hipStream_t s, const Args &A);
hipError_t launch_prow_sharded(hipStream_t s, const Args &A);
hipError_t launch_update(hipStream_t s, const Args &A);
hipError_t launch_group_min(hipStream_t s, double *const *ptrs, int n);
int ratio_blocks(long long rows);

}  // namespace lpk
