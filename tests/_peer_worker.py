"""One rank of a 2-process row-sharded job on ONE GPU (test_gpu_peer_procs.py):
no RCCL communicator (RCCL refuses two ranks on one device).  mode "peer":
the device-side peer exchange, set up from IPC handles all-gathered over
gloo; "scan": the same, then column scans and explicit pivots combined
through the host all-gather (gloo); "host": no peer exchange at all, every
per-pivot exchange through the host all-gather."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
sys.path.insert(0, ROOT)

import torch.distributed as dist  # noqa: E402

from lpsol_amd import Tableau, _lib, generators as gen  # noqa: E402
from oracle.f64 import F64Tableau  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    kind, m, ns, k, block, tie = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
        int(sys.argv[5]), float(sys.argv[6])
    mode = sys.argv[7] if len(sys.argv) > 7 else "peer"
    T = gen.tableau(kind, m, ns, 31)
    m, n = T.shape[0] - 1, T.shape[1] - 1
    e = _lib.create_sharded(m, n, rank, world, None, device=0)
    # the host all-gather carries the per-pivot exchanges where the
    # persistent cross-rank selection is not used (host mode; more than four
    # ranks on one GPU) and the column scans
    e.set_host_allgather(_lib.gloo_allgather())
    if mode != "host":
        hs = [None] * world
        dist.all_gather_object(hs, e.peer_handle())
        e.peer_open(b"".join(hs))
    e.upload(T)
    e.set_block(block)
    e.set_tol(ratio_tie=tie)
    st, done = e.run(_lib.RULE_STANDARD, k)
    o = F64Tableau(T, {"ratio_tie": tie})
    ost, olog = o.run(0, k)
    assert e.log().tolist() == olog.tolist(), (rank, e.log().tolist()[:5], olog.tolist()[:5])
    # which path ran: the persistent cross-rank selection with up to four
    # ranks on the one GPU, one collective per pivot beyond (lpgpu.cpp,
    # persistent_geom) or without the peer exchange
    path, fallbacks = e.exchange_path()
    if os.environ.get("EXPECT_KERNEL"):        # which selection kernel the persistent path ran
        geo = e.geometry()
        assert geo["kernel"] == os.environ["EXPECT_KERNEL"], (rank, geo)
        if os.environ.get("EXPECT_XS"):            # k_sel<XR> as XCD shards inside the rank
            assert geo["xcd_shards"] == 8 and geo["xcd_shards_engaged"], (rank, geo)
        else:
            assert geo["xcd_shards"] == 0 and geo["on_one_xcd"], (rank, geo)
        if os.environ.get("EXPECT_GEOM"):          # "blocks,ipl" of the launch the rank ran
            g, ipl = (int(x) for x in os.environ["EXPECT_GEOM"].split(","))
            assert (geo["blocks"], geo["ipl"]) == (g, ipl), (rank, geo)
    if os.environ.get("EXPECT_BLOCK"):            # the automatic pivots per sweep
        assert e.get_block() == int(os.environ["EXPECT_BLOCK"]), (rank, e.get_block())
    want = _lib.PATH_PEER if mode not in ("host", "fault") and world <= 4 else _lib.PATH_COLLECTIVE
    # "fault": rank 0's first persistent launch withholds a summary (LPGPU_FAULT);
    # every rank times out in that group, the ranks agree on it and all redo it
    # on the per-pivot kernels with one collective per pivot
    assert (path, fallbacks) == (want, 1 if mode == "fault" else 0), (rank, path, fallbacks)
    b, c = e.row_begin, e.row_count
    assert np.array_equal(e.rows(0, 1), o.T[:1])
    assert np.array_equal(e.rows(1 + b, c), o.T[1 + b:1 + b + c])
    if mode == "scan":
        scans(e, o)
    dist.barrier()
    e.close()
    dist.destroy_process_group()
    print(f"rank {rank} ok: {done} pivots")


def scans(e, o):
    """findPivotMaxIncrease / findPivotAll / form checks on the row shards of
    two processes == the f64 oracle on the whole tableau, along a walk of
    explicit max-increase pivots (each one collective)"""
    for _ in range(12):
        assert [list(p) for p in e.find_all()] == [list(p) for p in o.find_all()]
        f = e.form_checks()
        t = Tableau.fromArray(o.T)
        bc = [-2] * (o.T.shape[0] - 1)
        want = dict(canonical=t.isCanonical(bc), optimal=t.isOptimal(), unbounded=t.isUnbounded(),
                    infeasible=t.isInfeasible(), degenerate=t.isDegenerate())
        for key, v in want.items():
            assert f[key] == v, key
        assert (f["bcols"] or [-2] * len(bc)) == bc
        want = o.find_max_increase()
        got = e.find_max_increase(True)
        assert (list(got) if isinstance(got, tuple) else got) == \
            (list(want) if isinstance(want, tuple) else want)
        if isinstance(want, str):
            break
        o.pivot(*want)
    b, c = e.row_begin, e.row_count
    assert np.array_equal(e.rows(0, 1), o.T[:1])
    assert np.array_equal(e.rows(1 + b, c), o.T[1 + b:1 + b + c])


if __name__ == "__main__":
    main()
