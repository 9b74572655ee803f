"""Probe (follow-up of ramp_probe.py): data or device?  Per workload, three
passes of RAMP_GROUPS groups, each after an upload:
  A  the initial tableau (as ramp_probe's A);
  L  the tableau as it stands after A (late data) re-uploaded: slow first
     launches again => the device (idle gap), none => the data;
  W  the initial tableau again, but a second engine holding late data runs
     RAMP_GROUPS groups right before it (no idle gap): slow first launches
     => the data."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))

import bench  # noqa: E402
from lpsol_amd import _lib  # noqa: E402
from lpsol_amd import generators as gen  # noqa: E402

G = int(os.environ.get("RAMP_GROUPS", "40"))

for name in sys.argv[1:]:
    kind, m, ns, n, _, _ = bench.workload(name, 1, 0)
    T = gen.rows(kind, m, ns, bench.SEED, 0, m + 1)
    e = _lib.Engine(m, n, device=0)
    e2 = _lib.Engine(m, n, device=0)
    e.upload(T)
    e.run(_lib.RULE_STANDARD, 64 * G)
    print(f"{name} pass A", flush=True)
    late = e.download()
    e.upload(late)
    e.run(_lib.RULE_STANDARD, 64 * G)
    print(f"{name} pass L", flush=True)
    e2.upload(late)
    e.upload(T)
    e2.run(_lib.RULE_STANDARD, 64 * G)      # the warm-up pass (late data): pass index 2
    e.run(_lib.RULE_STANDARD, 64 * G)       # pass W: index 3
    print(f"{name} pass W", flush=True)
    e.close()
    e2.close()
    del late
