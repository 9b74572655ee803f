"""Probe: the cfg4 sweep's slow start after an idle gap (the upload; the
heater's close) -- the bench's sequence with different heaters, printing
the close time and each timed run's sweep average.

    python scripts/heat_probe.py <mode> [heat_ms]
      big    the bench's heater: a full-size scratch engine, closed before the warmup
      small  a heater of cfg3's shape (273 MB: freed in a few ms)
      keep   the full-size heater closed only after the timed runs
      none   no heater"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from bench import _lib  # noqa: E402

mode = sys.argv[1]
heat_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 150.0
kind, m, ns, n, _, _ = bench.workload("cfg4", 1, 0)
e = _lib.Engine(m, n)
e.set_block(64)
h = None
if mode in ("big", "keep"):
    h = _lib.Engine(m, n)
    h.set_block(64)
    bench.upload([e], kind, m, ns, [(0, m)], heaters=[h])
else:
    bench.upload([e], kind, m, ns, [(0, m)])
    if mode == "small":
        k3, m3, ns3, n3, _, _ = bench.workload("cfg3", 1, 0)
        h = _lib.Engine(m3, n3)
        h.set_block(64)
        bench.upload([h], k3, m3, ns3, [(0, m3)])
heat = bench.device_warmup(h, 64, heat_ms) if h is not None else {}
t0 = time.perf_counter()
if h is not None and mode != "keep":
    h.close()
close_ms = (time.perf_counter() - t0) * 1e3
e.run(_lib.RULE_STANDARD, 5 * 64)
out = []
for r in range(4):
    e.profile(True, every=1)
    e.run(_lib.RULE_STANDARD, 20 * 64)
    ms, cnt = e.update_time()
    e.profile(False)
    out.append(f"{1e3 * ms / max(cnt, 1):.0f}")
if mode == "keep":
    h.close()
print(f"{mode}: heat {heat} close {close_ms:.1f} ms; sweep us per 20-group run:", " ".join(out), flush=True)
e.close()
