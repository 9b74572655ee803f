"""Row-sharded job as two PROCESSES on one GPU with the device-side peer
exchange (IPC handles, peer stores, ping check): the multi-process plumbing
of the 8-GPU job, bit-identical to the f64 oracle."""
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
@pytest.mark.parametrize("kind,m,ns,k,block,tie,mode", [
    ("mixed", 200, 150, 60, 8, 1e-12, "peer"),
    ("tall", 300, 40, 50, 32, 1e-12, "peer"),
    ("mixed", 48, 32, 40, 4, 0.25, "peer"),       # wide tie band: straddles across ranks
    ("mixed", 120, 90, 20, 8, 1e-12, "scan"),     # + column scans, explicit pivots (host all-gather)
    ("pos", 64, 64, 10, 4, 1e-12, "scan"),
    ("mixed", 60, 50, 30, 8, 1e-12, "host"),      # every exchange through the host all-gather
])
def test_two_process_peer_exchange(kind, m, ns, k, block, tie, mode):
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                   WORLD_SIZE="2", LOCAL_RANK="0")
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(HERE, "_peer_worker.py"), kind, str(m), str(ns), str(k),
             str(block), str(tie), mode], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
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
