"""Probe: one-GPU pivots/s of a tall tableau by selection form (one-XCD k_sel
with several rows per lane, or k_sel's 8 XCD shards): the per-rank row counts
of cfg4 on 2 / 4 GPUs (16384 / 8192 rows).  python scripts/geo_probe.py [xs]
(XCD shards take 64 blocks each where they fit -- two columns per lane
instead of four; LPGPU_SEL_XS64=0 for the fewest blocks, round 5's A/B)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
from lpsol_amd import _lib, generators as gen  # noqa: E402

XS_ONLY = len(sys.argv) > 1 and sys.argv[1] == "xs"
for m in (8192, 16384):
    T = gen.tableau("tall", m, 8192, 3)
    for xs in ((True,) if XS_ONLY else (True, False)):
        e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
        e.upload(T)
        e.set_xcd_shards(xs)
        e.run(_lib.RULE_STANDARD, 64 * 40)           # warm (device and engine)
        e.upload(T)
        e.run(_lib.RULE_STANDARD, 64 * 8)
        t0 = time.perf_counter()
        st, done = e.run(_lib.RULE_STANDARD, 64 * 64)
        dt = time.perf_counter() - t0
        print(m, "xs" if xs else "no-xs", e.geometry(), e.get_block(), f"{done / dt:.0f} pivots/s", e.exchange_path(), flush=True)
        e.close()
