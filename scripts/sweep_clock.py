"""Probe: the cfg4 sweep group by group after an upload,
with the shader clock of each launch from k_sweep_rl's own records
(Args::sweep_clk: block 0's shader cycles and 100 MHz ticks over its pass) --
a slow launch at a lower clock with the same cycles is a clock effect, more
cycles at the same clock a memory one.

    python scripts/sweep_clock.py [groups] [workload]

Prints, per repetition (upload, then `groups` 64-pivot groups in one call),
one line per launch: launch, block-0 us, GHz, kcycles; then summaries of the
first 10, launches 10-39 and the rest."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from bench import _lib  # noqa: E402


def report(tag, c):
    us = c[:, 2] / 100.0
    ghz = c[:, 1] / (c[:, 2] / 1e8) / 1e9
    kc = c[:, 1] / 1e3
    for i in range(len(c)):
        print(f"{tag} {i:3d} us {us[i]:7.1f} GHz {ghz[i]:5.3f} kcyc {kc[i]:7.1f}")
    for a, b in ((0, 10), (10, 40), (40, len(c))):
        if b > a:
            print(f"{tag} launches {a}-{b - 1}: us {us[a:b].mean():7.1f} GHz {ghz[a:b].mean():5.3f} "
                  f"kcyc {kc[a:b].mean():7.1f}  (GHz min {ghz[a:b].min():.3f} max {ghz[a:b].max():.3f})",
                  flush=True)


def main():
    ng = int(sys.argv[1]) if len(sys.argv) > 1 else 80
    wl = sys.argv[2] if len(sys.argv) > 2 else "cfg4"
    kind, m, ns, n, _, _ = bench.workload(wl, 1, 0)
    e = _lib.Engine(m, n)
    e.set_block(64)
    for rep in range(2):
        bench.upload([e], kind, m, ns, [(0, m)])
        t0 = time.perf_counter()
        st, done = e.run(_lib.RULE_STANDARD, ng * 64)
        dt = time.perf_counter() - t0
        print(f"rep {rep}: status {st} pivots {done} in {dt * 1e3:.1f} ms = {done / dt:.0f} pivots/s", flush=True)
        report(f"r{rep}", e.sweep_clocks(ng)[-ng:])
        time.sleep(0.5 if rep == 0 else 0)       # an idle gap like an upload's before the second
    e.close()


if __name__ == "__main__":
    main()
