"""Mean PMC counter values per dispatch of the kernels matching a name, from
rocprofv3 --pmc output directories (scripts/gpu.sh step pmcx).

usage: python scripts/pmc_summary.py <dir> [<dir> ...] --kernel k_sweep_rl"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", action="append", default=[])
    a = ap.parse_args()
    res = {}
    for kern in a.kernel:
        vals = collections.defaultdict(dict)
        for d in a.dirs:
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if kern not in row.get("Kernel_Name", ""):
                            continue
                        key = f + ":" + row.get("Dispatch_Id", "")
                        c = row["Counter_Name"]
                        vals[c][key] = vals[c].get(key, 0.0) + float(row["Counter_Value"])
        res[kern] = {c: statistics.mean(v.values()) for c, v in sorted(vals.items())}
        res[kern]["dispatches"] = max((len(v) for v in vals.values()), default=0)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
