"""Split a ramp_probe kernel trace into passes: every sweep kernel's launches
in time order, in chunks of RAMP_GROUPS per pass; prints 8-launch means."""
import csv
import os
import sys

G = int(os.environ.get("RAMP_GROUPS", "40"))
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
kinds = sorted({r["Kernel_Name"].split("(")[0] for r in rows if "k_sweep" in r["Kernel_Name"]})
for k in kinds:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows
         if r["Kernel_Name"].startswith(k)]
    print(k, len(d), "launches")
    for p in range(0, len(d), G):
        s = d[p:p + G]
        print("  pass", p // G, [round(sum(s[i:i + 8]) / len(s[i:i + 8]), 1) for i in range(0, len(s), 8)])
