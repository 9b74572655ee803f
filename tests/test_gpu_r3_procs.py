"""Round 3: the row-sharded multi-process job at the geometry that timed out
in round 2 (profiles/r02/README.md: four ranks of cfg4 sharing one GPU filled
every block slot of a CU and one persistent group timed out).  Each rank is a
process with an 8192-row (4 ranks) or 16384-row (2 ranks) shard of a tall
32768 x 8192 tableau, the automatic pivots per sweep, LPGPU_STRICT=1 (a timed-
out group fails the call instead of being redone), >= 70 pivots, every shard
bit-identical to oracle/lp_f64.c and no fallback (tests/_peer_worker.py)."""
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


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [4, 2])
def test_cfg4_shards_sharing_one_gpu(world):
    port = _free_port()
    procs = []
    for rank in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   WORLD_SIZE=str(world), LOCAL_RANK="0", LPGPU_STRICT="1",
                   OMP_NUM_THREADS=str(max(1, 16 // world)))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(HERE, "_peer_worker.py"), "tall", "32768", "8192", "72", "0", "1e-12",
             "peer"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=840)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
        assert "72 pivots" in out, out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,m,ns,k,block,tie", [
    ("mixed", 400, 100, 60, 8, 1e-12),
    ("mixed", 400, 100, 70, 0, 1e-12),           # auto pivots per sweep
    ("tall", 900, 40, 50, 32, 1e-12),
    ("mixed", 48, 32, 40, 4, 0.25),              # wide tie band: straddles across ranks
])
def test_one_xcd_cross_rank_selection(kind, m, ns, k, block, tie):
    """the selection kernel of one rank per GPU (k_sel<XR>: one XCD per rank,
    the leaving row and pivot row exchanged between ranks) on the one box:
    two processes forced onto it (LPGPU_XR_XCD=1; small tableaux, so both
    ranks' blocks are resident on the XCD together), bit-exact"""
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   WORLD_SIZE="2", LOCAL_RANK="0", LPGPU_XR_XCD="1", LPGPU_STRICT="1", EXPECT_KERNEL="k_sel")
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(HERE, "_peer_worker.py"), kind, str(m), str(ns), str(k), str(block),
             str(tie), "peer"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,m,ns,k,block,tie", [
    ("tall", 8400, 40, 90, 64, 1e-12),           # 4200 rows per rank: 8 shards of 525
    ("tall", 8400, 40, 70, 0, 1e-12),            # auto pivots per sweep
    ("tall", 9000, 60, 60, 64, 0.25),            # wide tie band: straddles across ranks and shards
])
def test_xcd_shards_cross_rank_selection(kind, m, ns, k, block, tie):
    """ranks taller than one XCD (2 and 4 GPUs of cfg4: 16384 / 8192 rows per
    rank): k_sel<XR, XS>, the rank's XCD shards exchange inside the device and
    the rank's candidate and pivot row go to the other ranks.  Two processes
    forced onto the one box (LPGPU_XR_XCD=1; narrow tableaux, so both ranks'
    launches are resident together), bit-exact against oracle/lp_f64.c"""
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   WORLD_SIZE="2", LOCAL_RANK="0", LPGPU_XR_XCD="1", LPGPU_STRICT="1", EXPECT_KERNEL="k_sel",
                   EXPECT_XS="1")
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(HERE, "_peer_worker.py"), kind, str(m), str(ns), str(k), str(block),
             str(tie), "peer"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
