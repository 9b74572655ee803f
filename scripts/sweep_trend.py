"""Probe: the cfg4 sweep's duration group by group from the initial tableau,
twice on one engine (re-uploaded in between), to tell a device ramp from the
LP's progress (run under rocprofv3 --kernel-trace; scripts/sweep_trend.py
--report <dir> prints each k_sweep_rl launch's duration in order).

    python scripts/sweep_trend.py [groups] [workload]"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if len(sys.argv) > 2 and sys.argv[1] == "--report":
    rows = []
    for f in glob.glob(os.path.join(sys.argv[2], "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_sweep" in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    d = [(b - a) / 1e3 for a, b in rows]
    gaps = [(rows[i + 1][0] - rows[i][1]) / 1e6 for i in range(len(rows) - 1)]
    line = []
    for i, x in enumerate(d):
        if i and gaps[i - 1] > 20:               # > 20 ms between sweeps: a re-upload / the next engine
            print(" ".join(line))
            line = []
        line.append(f"{x:.0f}")
    print(" ".join(line))
    sys.exit(0)

import bench  # noqa: E402
from bench import _lib  # noqa: E402

ng = int(sys.argv[1]) if len(sys.argv) > 1 else 60
wl = sys.argv[2] if len(sys.argv) > 2 else "cfg4"
mode = sys.argv[3] if len(sys.argv) > 3 else "reupload"
kind, m, ns, n, _, _ = bench.workload(wl, 1, 0)
if mode == "reupload":
    e = _lib.Engine(m, n)
    e.set_block(64)
    for rep in range(2):
        bench.upload([e], kind, m, ns, [(0, m)])
        st, done = e.run(_lib.RULE_STANDARD, ng * 64)
        print("rep", rep, "status", st, "pivots", done, flush=True)
    e.close()
else:
    # "pair": two engines uploaded first, then run back to back -- the second
    # starts from the initial tableau on a device that has just run ng groups
    es = [_lib.Engine(m, n) for _ in range(2)]
    for e in es:
        e.set_block(64)
    bench.upload(es, kind, m, ns, [(0, m), (0, m)])
    for k, e in enumerate(es):
        st, done = e.run(_lib.RULE_STANDARD, ng * 64)
        print("engine", k, "status", st, "pivots", done, flush=True)
    for e in es:
        e.close()
