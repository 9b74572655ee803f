"""Probe: how the blocks of one 64-pivot sweep launch share its time
(k_sweep_rl's per-block records, Args::sweep_clk: start and pass-end ticks of
every block, 100 MHz).  A launch lasts as long as its slowest block: the
spread of the blocks' pass ends against block 0's tells what the launch
waits for (strip, row run, XCD).

    python scripts/sweep_blocks.py [workload] [groups]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from bench import _lib  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    ng = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    kind, m, ns, n, _, _ = bench.workload(wl, 1, 0)
    e = _lib.Engine(m, n)
    e.set_block(64)
    bench.upload([e], kind, m, ns, [(0, m)])
    for rep in range(3):
        e.run(_lib.RULE_STANDARD, ng * 64)
        b = e.sweep_block_clocks()
        t0 = b[:, 1].min()
        start = (b[:, 1] - t0) / 100.0          # us
        end = (b[:, 2] - t0) / 100.0
        cyc = b[:, 3] / 1e3
        print(f"{wl} rep {rep}: {len(b)} blocks; start us: max {start.max():.1f}; pass end us: "
              f"min {end.min():.1f} median {np.median(end):.1f} p90 {np.percentile(end, 90):.1f} max {end.max():.1f}; "
              f"kcycles min {cyc.min():.1f} median {np.median(cyc):.1f} max {cyc.max():.1f}", flush=True)
        if rep == 2:
            nstr = None
            # per XCD (block % 8) and the slowest blocks
            for x in range(8):
                sel = b[:, 0] % 8 == x
                print(f"  XCD {x}: pass end median {np.median(end[sel]):.1f} max {end[sel].max():.1f} us", flush=True)
            order = np.argsort(-end)[:12]
            print("  slowest blocks (block, start, end us, kcycles):",
                  [(int(b[i, 0]), round(float(start[i]), 1), round(float(end[i]), 1), round(float(cyc[i]), 1))
                   for i in order], flush=True)
            h, edges = np.histogram(end, bins=12)
            print("  pass-end histogram:", list(zip([round(float(x), 1) for x in edges[:-1]], h.tolist())), flush=True)
    e.close()


if __name__ == "__main__":
    main()
