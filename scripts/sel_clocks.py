"""k_sel phase breakdown (diagnostic build, LPGPU_STAMPS=1): every block keeps
per-phase shader-cycle sums in registers for a whole launch and stores them
once at its end (select.hip SEL_CLK).  Prints, per phase, the mean over
blocks of cycles per pivot and the slowest block's, in cycles and in us at the
clock measured over the launch (shader cycles / 100 MHz real-time ticks).

    LPGPU_LIB=.../variants/stamps.so python scripts/sel_clocks.py [kind m ns block]
    python scripts/sel_clocks.py --file stamps_rank0.npz     (a bench rank's dump:
        LPGPU_LIB=.../stamps.so LPGPU_STAMPS=1 LPGPU_STAMPS_DUMP=dir bench.py ...)
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))

NAMES = {1: "issue", 2: "colload", 3: "colchain", 4: "ratio", 5: "rpub", 6: "rgather", 20: "leave:wmin",
         7: "leave:rest", 8: "rowload", 9: "rowchain", 10: "div", 16: "xsend", 14: "xshard/xgather", 17: "xrecv",
         21: "rowfin:summary", 11: "rowfin:rest+epub", 12: "tail", 13: "egather", 18: "decide:wmin",
         19: "decide:pick", 0: "decide:rest"}
ORDER = [1, 2, 3, 4, 5, 6, 20, 7, 8, 9, 10, 16, 14, 17, 21, 11, 12, 13, 18, 19, 0]


def clk(o, k):
    # select.hip: phases 0..15 at o[0..15], 16..23 at o[20..27]
    return o[k] if k < 16 else o[20 + k - 16]


def report(buf, G, blk):
    per = []
    ghz_s = []
    for b in range(G):
        o = buf[b * 32:b * 32 + 32]
        nd = o[16]
        if nd <= 1:
            continue
        # phase 0 and 12/13 run nd - 1 times (no next pivot after the last)
        per.append({k: clk(o, k) / (nd - 1 if k in (0, 12, 13, 18, 19) else nd) for k in ORDER})
        if o[17] > 0:
            ghz_s.append(sum(clk(o, k) for k in ORDER) / (o[17] * 10.0))   # cycles per ns -> GHz
    ghz = sorted(ghz_s)[len(ghz_s) // 2] if ghz_s else 2.1
    print(f"blocks {len(per)}, shader clock ~{ghz:.2f} GHz (cycles / real time over the launch)")
    tot = 0.0
    for k in ORDER:
        v = [p[k] for p in per]
        mean = sum(v) / len(v)
        if mean == 0 and k in (14, 16, 17, 18, 19, 20, 21):
            continue
        tot += mean
        print(f"{NAMES[k]:>14s}  mean {mean:7.0f} cyc {mean / ghz / 1000:5.2f} us   max {max(v):7.0f}   "
              f"min {min(v):7.0f}")
    print(f"{'sum':>14s}  mean {tot:7.0f} cyc {tot / ghz / 1000:5.2f} us per pivot")

    # ---- per-pivot events (100 MHz real-time, 10 ns ticks): where the exchange
    #      waits come from.  Per pivot: spread of the pivot starts over blocks,
    #      the slowest block's column arrival after its start, the spread of the
    #      ratio publications, and how long after the LAST publication each block
    #      saw all of them (the exchange's own latency); the same for row 0.
    EV = 4096
    npv = min(blk, 48)
    rows = []
    for t in range(1, npv - 1):
        ev = [[buf[EV + (t * 64 + b) * 8 + k] for k in range(6)] for b in range(G)]
        if any(e[0] == 0 or e[3] == 0 for e in ev):
            continue
        s0 = [e[0] for e in ev]
        col = [e[1] - e[0] for e in ev]
        p2 = [e[2] for e in ev]
        seen = [e[3] - max(p2) for e in ev]
        p4 = [e[4] for e in ev]
        seen_e = [e[5] - max(p4) for e in ev]
        rows.append((max(s0) - min(s0), sum(col) / G, max(col), max(p2) - min(p2), min(seen), sum(seen) / G,
                     max(seen), max(p4) - min(p4), sum(seen_e) / G, max(seen_e)))
    if rows:
        names_e = ["start spread", "col mean", "col max", "Rpub spread", "Rseen min", "Rseen mean", "Rseen max",
                   "Epub spread", "Eseen mean", "Eseen max"]
        print("per-pivot events (ns, mean over pivots 1..%d):" % (npv - 2))
        for i, nm in enumerate(names_e):
            v = [r[i] * 10.0 for r in rows]
            print(f"  {nm:>13s} {sum(v) / len(v):8.0f}   max {max(v):8.0f}")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--file":
        d = np.load(sys.argv[2])
        print("dump", sys.argv[2], "geometry", d["geometry"].tolist())
        report([int(x) for x in d["buf"]], int(d["blocks"]), int(d["block"]))
        return
    os.environ["LPGPU_STAMPS"] = "1"
    from lpsol_amd import _lib, generators as gen
    kind, m, ns, blk = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) \
        if len(sys.argv) > 4 else ("mixed", 4096, 4096, 48)
    mm, n = gen.shape(kind, m, ns)
    e = _lib.Engine(mm, n)
    for a in range(0, mm + 1, 2048):
        e.put_rows(a, gen.rows(kind, m, ns, 3, a, min(a + 2048, mm + 1)))
    e.set_block(blk)
    e.run(0, 4 * blk)
    e.run(0, blk)                      # the launch whose clocks are read
    geo = e.geometry()
    print("workload", kind, m, ns, "block", blk, "geometry", geo)
    assert geo["kernel"] == "k_sel", "not the one-XCD kernel"
    BMAX = 64
    buf = (C.c_longlong * (256 * BMAX * 4))()
    assert e.lib.lpdiag_bstamps(e.h, buf) == 0
    report(buf, geo["blocks"], blk)


if __name__ == "__main__":
    main()
