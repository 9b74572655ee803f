"""Round 4 ("Next round" 1): the per-rank selection kernels of the
2-, 4- and 8-GPU cfg4 jobs at their PRODUCT geometry, two processes on the one
GPU of the test box (tests/_peer_worker.py; no RCCL communicator -- RCCL
refuses two ranks on one device -- so the peer exchange is set up from IPC
handles all-gathered over gloo).

* 8 GPUs: every rank holds 4096 rows of cfg4 (32768 / 8) and runs the one-XCD
  cross-rank kernel k_sel<XR> (IPL = 2, 64 pivots) with G = 64 blocks, one row
  per lane, over 8,193 columns.  Here a tall tableau of 8192 rows is split in
  two, so each rank holds exactly 4096 rows and runs that kernel with G = 64.
  The two ranks' launches must be resident together: LPGPU_XR_XCD=1 puts each
  on its own XCD (Args::xtarget: rank % 8).  Residency arithmetic:
  at 8,193 columns a block's LDS (128 columns x 66 x 8 B = 67.6 KB) allows 2
  blocks per CU, so G = 64 fills its XCD's 64 slots -- and the other rank's
  grid, which deals 7 of every 8 (idle, exiting) blocks to XCDs it does not
  work on, finds no slot there and stalls in dispatch order (measured: a
  timeout).  At 6,144 columns (96 per block, 50.7 KB) 3 blocks fit per CU:
  G = 64 of 96 slots, the same kernel instantiation and block count as the
  8-GPU rank; sel_geom now demands that free slot for co-located ranks.
* 2 GPUs: every rank holds 16384 rows and runs k_sel<XR, XS> (the rank's rows
  as 8 XCD shards).  Two such launches on one GPU need 2 G blocks on every
  XCD: at 8,193 columns (G = 64 at two blocks per CU) they cannot share it, so
  the tests take 4,096 columns (G = 64 at one column per lane, 4 blocks per
  CU) and 4,500 (G = 64 at two columns per lane, the product's k_sel<2, 64,
  XR, XS>; 37.5 KB of LDS per block: 4 per CU, 128 per XCD for both ranks) --
  sel_geom sizes for the co-located ranks (share x G).

Each: >= 136 pivots at the automatic pivots per sweep (64: two full groups and
a partial one), LPGPU_STRICT=1 (a timed-out group fails the call), no fallback,
every rank's rows bit-identical to oracle/lp_f64.c.  Reference:
/root/reference/lpsol/simplex.py:251-284 (findPivotStandard), tableau.py:295-308.
"""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _two_ranks(args, extra_env, timeout=600):
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   WORLD_SIZE="2", LOCAL_RANK="0", LPGPU_STRICT="1", OMP_NUM_THREADS="8", **extra_env)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_peer_worker.py")] + args, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
    return outs


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_eight_gpu_rank_geometry_k_sel_xr():
    """one rank of cfg4 on 8 GPUs: 4096 rows, k_sel<XR> with G = 64 blocks
    and two columns per lane (6,144 columns: both ranks resident on the one
    GPU), automatic 64 pivots per sweep, 136 pivots bit-exact, no fallback"""
    outs = _two_ranks(["tall", "8192", "6144", "136", "0", "1e-12", "peer"],
                      {"LPGPU_XR_XCD": "1", "EXPECT_KERNEL": "k_sel", "EXPECT_GEOM": "64,2",
                       "EXPECT_BLOCK": "64"})
    for out in outs:
        assert "136 pivots" in out, out[-2000:]


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_two_gpu_rank_geometry_k_sel_xr_xs():
    """one rank of cfg4 on 2 GPUs: 16384 rows as 8 XCD shards (k_sel<XR, XS>),
    4,096 columns so that both ranks' shards fit every XCD together (G = 64,
    one column per lane: XCD shards take 64 blocks where they fit since
    round 5), automatic 64 pivots per sweep, 136 pivots bit-exact"""
    outs = _two_ranks(["tall", "32768", "4096", "136", "0", "1e-12", "peer"],
                      {"LPGPU_XR_XCD": "1", "EXPECT_KERNEL": "k_sel", "EXPECT_XS": "1", "EXPECT_GEOM": "64,1",
                       "EXPECT_BLOCK": "64"})
    for out in outs:
        assert "136 pivots" in out, out[-2000:]


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_two_gpu_rank_geometry_k_sel_xr_xs_two_columns_per_lane():
    """the 2-GPU rank's product instantiation k_sel<2, 64, XR, XS> (round 5:
    XCD shards take 64 blocks, two columns per lane at 8,193 columns): 16384
    rows per rank over 4,500 columns, 136 pivots bit-exact, no fallback"""
    outs = _two_ranks(["tall", "32768", "4500", "136", "0", "1e-12", "peer"],
                      {"LPGPU_XR_XCD": "1", "EXPECT_KERNEL": "k_sel", "EXPECT_XS": "1", "EXPECT_GEOM": "64,2",
                       "EXPECT_BLOCK": "64"})
    for out in outs:
        assert "136 pivots" in out, out[-2000:]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_eight_gpu_rank_geometry_wide_ties():
    """the 8-GPU rank kernel with a wide tie band (ratio_tie 0.25): near-ties
    straddle the band across the two ranks and inside a rank's blocks; the
    rescans keep the reference's first-row order, bit-exact"""
    _two_ranks(["tall", "8192", "6144", "80", "0", "0.25", "peer"],
               {"LPGPU_XR_XCD": "1", "EXPECT_KERNEL": "k_sel", "EXPECT_GEOM": "64,2"})


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_two_gpu_rank_geometry_wide_ties():
    """ties inside k_sel<XR, XS> -- straddles across the XCD shards
    of a rank (the rank's first shard inside the band answers) and across the
    ranks, automatic pivots per sweep, bit-exact"""
    _two_ranks(["tall", "32768", "4096", "80", "0", "0.5", "peer"],
               {"LPGPU_XR_XCD": "1", "EXPECT_KERNEL": "k_sel", "EXPECT_XS": "1"})
