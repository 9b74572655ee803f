/*
 * lpgpu_diag.h -- diagnostics exported by liblpgpu.so beside the C-ABI of
 * lpgpu.h.  None of them is part of the reference's surface (lpsol has no
 * counterpart): they report how the engine laid a handle out on the device
 * and what its kernels measured, for bench.py, the tests and scripts/.  Every
 * call returns an lp_status (LP_BAD_ARG for a null handle or buffer).
 */
#ifndef LPGPU_DIAG_H
#define LPGPU_DIAG_H

#include "lpgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The persistent selection this handle's pivot loops launch, and what its
 * last launch found on the device: out[0..8] = blocks per shard, own columns
 * per lane, own rows per lane, summaries per lane, one-XCD grid, k_group's
 * two-level variant, k_sel's pivot capacity (0: k_group), the last launch's
 * flags (1 one XCD, 2 two-level exchange engaged, 4 k_sel, 8 k_sel's blocks
 * were not on one XCD, 16 k_sel as XCD shards), the XCD shards (0: none).
 * All 0 when the per-pivot kernels run.   */
int lpdiag_geometry(lp_handle *h, long long *out /* [9] */);

/* The tableau buffers the sweeps use: 2 out of place (the sweep reads one and
 * writes the other), 1 in place.  (LPGPU_SWEEP_OOP) */
int lpdiag_sweep_buffers(const lp_handle *h, int *nbuf);

/* Per 64-pivot sweep launch (k_sweep_rl), its block 0's clocks over the pass:
 * up to `cap` of the latest launches (at most 1024), oldest first, 4 values
 * each -- launch number, shader cycles (s_memtime), 100 MHz ticks
 * (s_memrealtime), start tick -> *n records.  cycles / (ticks / 1e8) is the
 * shader clock during that launch.   */
int lpdiag_sweep_clocks(lp_handle *h, unsigned long long *out /* [4 cap] */, int cap, int *n);

/* Every block's pass in the latest 64-pivot sweep launch: 4 values each --
 * block, start tick, pass-end tick (100 MHz, one device-wide clock), shader
 * cycles -> *n blocks (at most `cap`, at most 8192).  (scripts/sweep_blocks.py) */
int lpdiag_sweep_block_clocks(lp_handle *h, unsigned long long *out /* [4 cap] */, int cap, int *n);

/* A/B: whether a tall single-device tableau may run the selection as one row
 * shard per XCD (on != 0, the default) or takes k_group; re-chooses the
 * automatic pivots per sweep.   */
int lpdiag_set_xcd_shards(lp_handle *h, int on);

/* Phase stamps of a library built with LPK_STAMPS (scripts/sel_clocks.py,
 * scripts/diag_stamps.py); LP_BAD_ARG on the product build.
 * lpdiag_stamps: the per-pivot kernels' stamps, 64 x 16 values;
 * lpdiag_bstamps: the persistent selection's per-block phase clocks and
 * events, 256 x 64 x 4 values. */
int lpdiag_stamps(lp_handle *h, long long *out /* [1024] */);
int lpdiag_bstamps(lp_handle *h, long long *out /* [65536] */);

#ifdef __cplusplus
}
#endif

#endif /* LPGPU_DIAG_H */
