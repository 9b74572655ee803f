"""How often is the next entering column one the previous entering exchange
already named?  Design probe for the selection's speculative column loads.

k_sel's entering exchange at pivot t gives every block the 64 per-block row-0
summaries (block b: columns 1 + 128 b .. 128 b + 128 at cfg3), from which
C_{t+1} is decided.  The runners-up (the best columns of the next-best blocks)
are known at the same moment, one pivot before C_{t+2} is.  This runs the
float64 contract (oracle/lp_f64.c) on a workload and counts how often C_{t+2}
is among the K runners-up of the exchange that produced C_{t+1}.

    python scripts/spec_hit.py [kind m ns seed pivots blocks]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
from lpsol_amd import generators as gen  # noqa: E402
from oracle.f64 import F64Tableau  # noqa: E402

kind, m, ns, seed, npiv, G = (sys.argv[1], *map(int, sys.argv[2:7])) if len(sys.argv) > 6 else \
    ("mixed", 1024, 1024, 3, 400, 64)
T = gen.tableau(kind, m, ns, seed)
n = T.shape[1] - 1
o = F64Tableau(T)
cpb = -(-n // G)
KMAX = 8
hits = np.zeros(KMAX + 1, np.int64)
prev = None          # runner-up columns of the previous exchange, best first
total = 0
for t in range(npiv):
    r0 = o.T[0, 1:]
    pad = np.full(G * cpb, np.inf)
    pad[:n] = r0
    blk = pad.reshape(G, cpb)
    el = blk.min(axis=1)
    ei = np.argmin(blk, axis=1) + 1 + np.arange(G) * cpb      # (tie bands ignored: a probe)
    order = np.argsort(el, kind="stable")
    order = [b for b in order if el[b] < -1e-9]
    if not order:
        break
    C = int(ei[order[0]])
    if prev is not None:
        total += 1
        for k in range(1, KMAX + 1):
            if C in prev[:k]:
                hits[k] += 1
    prev = [int(ei[b]) for b in order[1:KMAX + 1]]
    f = o.find(0)
    if isinstance(f, str):
        break
    r, c = f
    assert c + 1 == C, (c, C)
    o.pivot(r, c)
print(f"{kind} {m}x{ns} seed {seed}: {total} exchanges, blocks {G}")
for k in range(1, KMAX + 1):
    print(f"  C(t+2) among the {k} runner(s)-up of exchange t+1: {hits[k] / max(total, 1):.3f}")
