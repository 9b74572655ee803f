"""Probe: are a leg's first sweep launches slower because of the data (the
tableau's first pivots) or because of the device (clocks, TLB, caches)?

One engine per workload; the same initial tableau is uploaded and 40 groups
(64 pivots each) run three times: A (first), B (immediately again: a warm
device, the same data), C (after 2 s idle).  Run under
`rocprofv3 --kernel-trace`; scripts/ramp_summary.py splits the sweep
launches into the passes.  Usage: python scripts/ramp_probe.py cfg3 [cfg4]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))

import bench  # noqa: E402
from lpsol_amd import _lib  # noqa: E402
from lpsol_amd import generators as gen  # noqa: E402

GROUPS = int(os.environ.get("RAMP_GROUPS", "40"))

for name in sys.argv[1:]:
    kind, m, ns, n, _, _ = bench.workload(name, 1, 0)
    T = gen.rows(kind, m, ns, bench.SEED, 0, m + 1)
    e = _lib.Engine(m, n, device=0)
    for tag, idle in (("A", 0.0), ("B", 0.0), ("C", 2.0)):
        time.sleep(idle)
        e.upload(T)
        t0 = time.perf_counter()
        st, done = e.run(_lib.RULE_STANDARD, 64 * GROUPS)
        print(f"{name} pass {tag}: {done} pivots in {time.perf_counter() - t0:.4f} s "
              f"(block {e.get_block()})", flush=True)
    e.close()
