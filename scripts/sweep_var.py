"""Probe: where the cfg4 sweep's run-to-run spread (790-870 us per launch
between processes on one box) comes from -- several engines in ONE process,
each with fresh buffers, each timed over several runs of 16 groups.

    python scripts/sweep_var.py [engines] [runs] [workload]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from bench import _lib  # noqa: E402

ne = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nr = int(sys.argv[2]) if len(sys.argv) > 2 else 3
wl = sys.argv[3] if len(sys.argv) > 3 else "cfg4"
kind, m, ns, n, _, _ = bench.workload(wl, 1, 0)
keep = []
for k in range(ne):
    e = _lib.Engine(m, n)
    e.set_block(64)
    bench.upload([e], kind, m, ns, [(0, m)])
    e.run(_lib.RULE_STANDARD, 5 * 64)
    out = []
    for r in range(nr):
        e.profile(True, every=1)
        e.run(_lib.RULE_STANDARD, 16 * 64)
        ms, cnt = e.update_time()
        sel_ms, sel_n = e.select_time()
        e.profile(False)
        out.append(f"{1e3 * ms / max(cnt, 1):.1f}/{1e3 * sel_ms / max(sel_n, 1) / 64:.2f}")
    print(f"engine {k}: sweep us / selection us per pivot per run:", " ".join(out), flush=True)
    if k % 2 == 0:
        keep.append(e)                           # alive: the next engine's buffers land elsewhere
    else:
        e.close()
for e in keep:
    e.close()
