"""k_group phase breakdown (diagnostic build path: LPGPU_STAMPS=1)."""
import ctypes as C
import os
import sys

os.environ["LPGPU_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
from lpsol_amd import _lib, generators as gen  # noqa: E402

# python scripts/diag_stamps.py [kind m ns block]  (default: cfg3, 16 pivots a group)
kind, m, ns, blk = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) \
    if len(sys.argv) > 4 else ("mixed", 4096, 4096, 16)
mm, n = gen.shape(kind, m, ns)
e = _lib.Engine(mm, n)
for a in range(0, mm + 1, 2048):
    e.put_rows(a, gen.rows(kind, m, ns, 3, a, min(a + 2048, mm + 1)))
e.set_block(blk)
e.run(0, 4 * blk)
e.run(0, blk)
print("workload", kind, m, ns, "block", blk, "path", e.exchange_path())
BMAX = 64                      # lpk::BMAX: stamp rows per group
buf = (C.c_longlong * (BMAX * 16))()
assert e.lib.lpdiag_stamps(e.h, buf) == 0
# stamp k marks the END of segment names[k-1]; segment 13 runs to the next pivot's stamp 0
names = ["enter", "col0", "rload", "rcomp", "rpub", "gathR", "leave",
         "pload", "pcomp", "esum", "epub", "tail"]
rows = []
NT = min(blk, 32) - 1
for t in range(NT):
    st = [buf[t * 16 + k] for k in range(len(names))] + [buf[(t + 1) * 16]]
    d = [(st[k + 1] - st[k]) * 10 / 1000 for k in range(len(names))]   # 100 MHz ticks -> us
    rows.append(d)
    print(t, " ".join(f"{n}={x:4.2f}" for n, x in zip(names, d)))
avg = [sum(r[k] for r in rows[1:]) / (len(rows) - 1) for k in range(len(names))]
print("avg", " ".join(f"{n}={x:4.2f}" for n, x in zip(names, avg)), "sum", round(sum(avg), 2))
# pcomp split by stamps 12 (chain done) and 13 (division done): chain / div / store+row0
sub = [[(buf[t * 16 + 12] - buf[t * 16 + 8]) / 100, (buf[t * 16 + 13] - buf[t * 16 + 12]) / 100,
        (buf[t * 16 + 9] - buf[t * 16 + 13]) / 100] for t in range(1, NT)]
print("pcomp split: chain=%.2f div=%.2f store=%.2f" % tuple(sum(x[i] for x in sub) / len(sub) for i in range(3)))

# per-block event times (every block): C known (2), column loaded (3), ratio
# summary published (0), row-0 summary published (1); spread = last - first
bb = (C.c_longlong * (256 * BMAX * 4))()
assert e.lib.lpdiag_bstamps(e.h, bb) == 0
ev = {2: "C known", 3: "column loaded", 0: "ratio published", 1: "row0 published"}
sp = {k: [] for k in ev}
last = {}
rel = {k: [] for k in ev}   # mean time of the event after the pivot's earliest 'C known'
for t in range(1, NT):
    base = [bb[(b * BMAX + t) * 4 + 2] for b in range(256)]
    base = [x for x in base if x]
    if not base:
        continue
    t0 = min(base)
    for k in ev:
        v = [bb[(b * BMAX + t) * 4 + k] for b in range(256)]
        v = [x for x in v if x]
        if not v:
            continue
        sp[k].append((max(v) - min(v)) * 10 / 1000)
        rel[k].append(((sum(v) / len(v)) - t0) * 10 / 1000)
        if k == 0:
            order = sorted(range(len(v)), key=lambda i: v[i])
            for b in order[-3:]:
                last[b] = last.get(b, 0) + 1
for k in (2, 3, 0, 1):
    if sp[k]:
        print("%-16s spread avg %.2f max %.2f us | mean after first C-known %.2f us" % (
            ev[k], sum(sp[k]) / len(sp[k]), max(sp[k]), sum(rel[k]) / len(rel[k])))
print("most often among the last 3 ratio publishers:", sorted(last.items(), key=lambda kv: -kv[1])[:10])
