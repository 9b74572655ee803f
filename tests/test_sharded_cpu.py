"""Row-sharded pivot protocol over torch.distributed (gloo, CPU).

oracle/sharded_model.py restates the engine's sharded exchange (one
allgather per pivot, rare two-step fallback) on the float64 oracle; here it
runs as 2 and 3 real processes and must reproduce the unsharded run exactly:
same pivot sequence, bit-identical rows.  A wide tie band forces the rare
fallback branch so both branches are exercised.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def straddle_tableau():
    """ratios in column x0: rank 0 rows 1.2, 1.0 | rank 1 rows 0.9, 2.0.
    With ratio_tie 0.25: g = 0.9, band(g) = 1.125; rank 0's own band is 1.25 so
    its first in-band row (1.2) lies outside the global band -> rare branch;
    the winner is rank 0's second row (1.0)."""
    T = np.zeros((5, 6))
    T[0, 1] = -1.0
    T[1:, 0] = [1.2, 1.0, 0.9, 2.0]
    T[1:, 1] = 1.0
    T[1:, 2:] = np.eye(4)
    return T


def _tableau(kind, m, ns):
    from lpsol_amd import generators as gen
    if kind == "straddle":
        return straddle_tableau()
    return gen.tableau(kind, m, ns, 17)


def _worker(rank, world, port, kind, m, ns, k, tol, out):
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    from lpsol_amd import generators as gen
    from oracle import sharded_model as sm
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    T = _tableau(kind, m, ns)
    st = sm.ShardState(T, rank, world, tol)

    def allgather(msg):
        x = torch.from_numpy(np.ascontiguousarray(msg, dtype=np.float64))
        bufs = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(bufs, x)
        return [b.numpy() for b in bufs]

    seq, end = sm.run(st, allgather, k)
    np.savez(os.path.join(out, f"r{rank}.npz"), seq=np.array(seq, dtype=np.int64).reshape(-1, 2),
             rows=st.rows, row0=st.row0, rb=st.rb, slow=st.slow_path, end=str(end))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind,m,ns,k,tol", [
    ("mixed", 30, 40, 60, None),
    ("tall", 45, 20, 40, None),
    ("mixed", 24, 24, 40, {"ratio_tie": 0.25}),     # wide band
    ("straddle", 4, 0, 1, {"ratio_tie": 0.25}),     # forces the rare branch
])
def test_sharded_protocol_matches_unsharded(tmp_path, world, kind, m, ns, k, tol):
    from oracle.f64 import F64Tableau
    port = _free_port()
    mp.spawn(_worker, args=(world, port, kind, m, ns, k, tol, str(tmp_path)), nprocs=world,
             join=True)
    T = _tableau(kind, m, ns)
    ref = F64Tableau(T, tol)
    _, log = ref.run(0, k)
    res = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    for r in res:
        assert r["seq"].tolist() == log.tolist()
        assert np.array_equal(r["row0"], ref.T[0])
        rb = int(r["rb"])
        assert np.array_equal(r["rows"], ref.T[1 + rb:1 + rb + len(r["rows"])])
    if kind == "straddle":
        assert log.tolist() == [[1, 0]]
        if world == 2:
            assert sum(int(r["slow"]) for r in res) == world, "rare branch not exercised"


def _cb_worker(rank, world, port, out):
    import ctypes as C
    import sys
    for p in (PKG, ROOT):
        if p not in sys.path:
            sys.path.insert(0, p)
    from lpsol_amd import _lib
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    cb = _lib.allgather_callback(_lib.gloo_allgather())
    send = bytes((rank * 17 + i) % 256 for i in range(40))      # one rank's 40-byte record
    sbuf = C.create_string_buffer(send, len(send))
    rbuf = C.create_string_buffer(len(send) * world)
    rc = cb(None, C.cast(sbuf, C.c_void_p), C.cast(rbuf, C.c_void_p), len(send))
    # a failing host collective reports 1 instead of raising through the C ABI
    bad = _lib.allgather_callback(lambda data: [data[:-1]])(None, C.cast(sbuf, C.c_void_p),
                                                           C.cast(rbuf, C.c_void_p), len(send))
    np.save(os.path.join(out, f"cb{rank}.npy"), np.frombuffer(rbuf.raw, dtype=np.uint8))
    with open(os.path.join(out, f"rc{rank}"), "w") as f:
        f.write(f"{rc} {bad}")
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_allgather_callback(tmp_path, world):
    """the lp_allgather_fn the engine calls for multi-process column scans
    (lp_set_host_allgather) over gloo: every rank's bytes, in rank order"""
    port = _free_port()
    mp.spawn(_cb_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    want = np.concatenate([np.array([(r * 17 + i) % 256 for i in range(40)], dtype=np.uint8)
                           for r in range(world)])
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"cb{r}.npy"), want)
        assert open(tmp_path / f"rc{r}").read() == "0 1"
