"""bench.py's accounting, checked without a GPU: the algorithmic byte counts
behind `roofline.achieved`, the weak-scaling row split, and
the HBM traffic file it reports as `roofline.traffic`."""
import json
import os

import pytest

from conftest import ROOT

import bench


def test_pivot_bytes_matches_survey():
    # B = 8 * [2 (m+1)(n+1) + (n+1) + 2 (m+1)]; cfg3: 537,198,632 B
    assert bench.pivot_bytes(4096, 8192) == 537_198_632
    assert bench.pivot_bytes(512, 1024) == 8_429_608


def test_sweep_bytes_cfg3():
    # one 32-pivot sweep of cfg3: rows read + written, P and M read once
    rows, n = 4097, 8192
    assert bench.sweep_bytes(rows, n, 32) == 8 * (2 * rows * (n + 1) + 32 * (n + 1) + 32 * rows)
    assert bench.sweep_bytes(rows, n, 32) == 540_213_776


@pytest.mark.parametrize("nranks", [1, 2, 4, 8])
def test_workload_rows_partition(nranks):
    spans = [bench.workload(nranks, r) for r in range(nranks)]
    kind, m, ns, n, _, _ = spans[0]
    assert m == bench.ROWS_PER_GPU * nranks
    assert n == 8192
    assert [s[4] for s in spans] == [m * r // nranks for r in range(nranks)]
    assert spans[-1][5] == m
    for a, b in zip(spans, spans[1:]):
        assert a[5] == b[4]                                  # contiguous, no overlap


def test_traffic_file_is_for_this_workload():
    path = os.path.join(ROOT, "profiles", "r01", "hbm_traffic.json")
    d = json.load(open(path))
    assert d["kernel"].startswith(bench.SWEEP_KERNEL)
    assert d["algorithmic_bytes_per_launch"] == bench.sweep_bytes(4097, 8192, d["block"])
    assert bench.load_traffic(path, d["block"]) == d["hbm_bytes_per_launch"]
    assert bench.load_traffic(path, d["block"] + 1) is None
    assert 1.0 <= d["traffic_over_algorithmic"] < 1.2
