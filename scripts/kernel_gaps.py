"""Where a bench step's wall time goes between kernels: from a rocprofv3
--kernel-trace CSV (scripts/gpu.sh step `gaps`), the consecutive kernels of
the engine's stream in dispatch order, each kernel's duration and the idle
gap before it, averaged per kernel name over the last N steps.

    python scripts/kernel_gaps.py gpurun_out/kt [last_n_kernels]
"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if not files:
    raise SystemExit(f"no kernel_trace.csv under {d}")
rows = []
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                         r.get("Queue_Id", ""), r.get("Stream_Id", "")))
rows.sort()
# the engine's kernels: k_sel / k_group / k_sweep*
eng = [r for r in rows if any(k in r[2] for k in ("k_sel", "k_group", "k_sweep", "k_enter", "k_prow", "k_ratio"))]
eng = eng[-last:]
stat = {}
for prev, cur in zip(eng, eng[1:]):
    gap = (cur[0] - prev[1]) / 1e3
    dur = (cur[1] - cur[0]) / 1e3
    s = stat.setdefault(cur[2], {"gap": [], "dur": []})
    s["gap"].append(gap)
    s["dur"].append(dur)
span = (eng[-1][1] - eng[1][0]) / 1e3
busy = sum((r[1] - r[0]) for r in eng[1:]) / 1e3
print(f"{len(eng) - 1} kernels over {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us "
      f"({(span - busy) / span:.1%})")
for name, s in stat.items():
    print(f"  {name[:60]:60s} n {len(s['dur']):3d}  duration {statistics.mean(s['dur']):8.2f} us  "
          f"gap before {statistics.mean(s['gap']):6.2f} us (median {statistics.median(s['gap']):.2f}, "
          f"min {min(s['gap']):.2f}, max {max(s['gap']):.2f})")
# idle between kernels of one run (gaps over 100 us are the host between runs)
inner = [(c[0] - p[1]) / 1e3 for p, c in zip(eng, eng[1:]) if (c[0] - p[1]) / 1e3 < 100]
print(f"gaps under 100 us: {len(inner)}, total {sum(inner):.1f} us, mean {statistics.mean(inner):.2f} us")
