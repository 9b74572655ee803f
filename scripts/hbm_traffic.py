"""HBM bytes per sweep (k_sweep_dp) launch from two rocprofv3 --pmc passes.

FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950 (TCC slots), so
scripts/gpu.sh (step pmc) runs bench.py twice under rocprofv3, once per counter.
Both counters are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced streaming read, so it is doubled (MI355X_MICROARCH.md §HBM).

usage: python scripts/hbm_traffic.py FETCH_DIR WRITE_DIR OUT_JSON --block B --workload W

The result is stamped with the sha256 of the library's sources (bench.py
reports it as roofline.traffic only for builds of those sources, that
workload and block; hipcc output is not byte-reproducible, so not the .so's).
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


NAMES: set[str] = set()   # the matching kernels' names (demangled by rocprofv3)


def per_dispatch(d: str, counter: str, kernel: str) -> list[float]:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals: dict[str, float] = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                NAMES.add(row["Kernel_Name"].split("(")[0])
                if row.get("Counter_Name") != counter:
                    continue
                key = f + ":" + row.get("Dispatch_Id", str(len(vals)))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--block", type=int, default=16)
    ap.add_argument("--kernel", default="k_sweep_dp")
    ap.add_argument("--workload", default="cfg4")
    a = ap.parse_args()
    import bench
    fetch = per_dispatch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    write = per_dispatch(a.write_dir, "WRITE_SIZE", a.kernel)
    if not fetch or not write:
        raise SystemExit(f"no {a.kernel} dispatches with counters")
    f_kib, w_kib = statistics.mean(fetch), statistics.mean(write)
    hbm = (2.0 * f_kib + w_kib) * 1024.0
    _, m, _, n, _, _ = bench.workload(a.workload, 1, 0)
    alg = bench.sweep_bytes(m + 1, n, a.block)
    out = {
        "kernel": " / ".join(sorted(NAMES)) or f"{a.kernel}<{a.block}>",
        "workload": a.workload,
        "workload_desc": bench.WORKLOADS[a.workload][3] + " (bench.py, 1 GPU)",
        "src_sha256": bench.src_digest(),
        "lib_sha256": bench.lib_digest(),
        "block": a.block,
        "dispatches": [len(fetch), len(write)],
        "FETCH_SIZE_KiB_mean": f_kib,
        "WRITE_SIZE_KiB_mean": w_kib,
        "correction": "FETCH_SIZE x2 (gfx950 reports half of a wide coalesced read), KiB x1024",
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": hbm / alg,
    }
    # one entry per (workload, block, build): the file accumulates them
    entries = []
    if os.path.exists(a.out):
        with open(a.out) as fh:
            entries = json.load(fh).get("entries", [])
    entries = [e for e in entries if (e.get("workload"), e.get("block"), e.get("src_sha256")) !=
               (out["workload"], out["block"], out["src_sha256"])] + [out]
    with open(a.out, "w") as fh:
        json.dump({"entries": entries}, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
