"""bench.py's accounting, checked without a GPU: the algorithmic byte counts
behind `roofline.achieved`, the strong-scaling row split,
the per-launch figures of a timed run, the traffic file's stamp and the
dense CPU baseline's pivot."""
import json

import numpy as np
import pytest

import bench
from lpsol_amd import generators as gen
from oracle import exact


def test_pivot_bytes_matches_survey():
    # B = 8 * [2 (m+1)(n+1) + (n+1) + 2 (m+1)]; cfg3: 537,198,632 B
    assert bench.pivot_bytes(4096, 8192) == 537_198_632
    assert bench.pivot_bytes(512, 1024) == 8_429_608
    assert bench.pivot_bytes(32768, 8192) == 4_296_212_520


def test_sweep_bytes_cfg3():
    # one 32-pivot sweep of cfg3: rows read + written, P and M read once
    rows, n = 4097, 8192
    assert bench.sweep_bytes(rows, n, 32) == 8 * (2 * rows * (n + 1) + 32 * (n + 1) + 32 * rows)
    assert bench.sweep_bytes(rows, n, 32) == 540_213_776


@pytest.mark.parametrize("name", ["cfg4", "cfg3"])
@pytest.mark.parametrize("nranks", [1, 2, 4, 8])
def test_strong_scaling_rows_partition(name, nranks):
    """the same tableau at every N, rows split like lp_create_sharded"""
    spans = [bench.workload(name, nranks, r) for r in range(nranks)]
    kind, m, ns, n, _, _ = spans[0]
    assert (m, n) == ((32768, 8192) if name == "cfg4" else (4096, 8192))
    assert [s[4] for s in spans] == [m * r // nranks for r in range(nranks)]
    assert spans[0][4] == 0 and spans[-1][5] == m
    for a, b in zip(spans, spans[1:]):
        assert a[5] == b[4]                                  # contiguous, no overlap


@pytest.mark.parametrize("steps,block", [(20, 32), (1, 32), (128, 16)])
def test_accounting_per_launch(steps, block):
    """every launch of a timed run carries exactly `block` pivots (one step =
    one group), so per-launch bytes and per-pivot selection time follow"""
    a = bench.accounting(steps, block, elapsed=0.5, sweep_avg_ms=0.1, sel_avg_ms=0.2,
                         local_rows=4097, n=8192)
    assert a["pivots"] == steps * block
    assert a["pivots_per_s"] == pytest.approx(steps * block / 0.5)
    assert a["ms_per_step"] == pytest.approx(500.0 / steps)
    assert a["sweep_bytes_per_launch"] == bench.sweep_bytes(4097, 8192, block)
    assert a["achieved_GBps"] == pytest.approx(bench.sweep_bytes(4097, 8192, block) / 1e-4 / 1e9)
    assert a["selection_us_per_pivot"] == pytest.approx(200.0 / block)
    assert a["sweep_time_share"] == pytest.approx(0.1 * steps / 500.0)


def test_traffic_needs_this_build(tmp_path):
    """roofline.traffic is reported only for builds of the sources, workload and
    block the PMC passes measured (scripts/hbm_traffic.py stamps them)"""
    p = tmp_path / "t.json"
    d = {"kernel": "k_sweep_dp<8, 32, 16, 1>", "block": 32, "workload": "cfg4", "src_sha256": "abc",
         "hbm_bytes_per_launch": 123.0}
    p.write_text(json.dumps(d))
    assert bench.load_traffic(str(p), 32, "cfg4", "abc") == 123.0
    assert bench.load_traffic(str(p), 32, "cfg4", "abd") is None
    assert bench.load_traffic(str(p), 32, "cfg3", "abc") is None
    assert bench.load_traffic(str(p), 16, "cfg4", "abc") is None
    p.write_text(json.dumps({"entries": [dict(d, workload="cfg3", hbm_bytes_per_launch=7.0), d]}))
    assert bench.load_traffic(str(p), 32, "cfg4", "abc") == 123.0
    assert bench.load_traffic(str(p), 32, "cfg3", "abc") == 7.0


def test_dense_pivot_is_the_reference_pivot():
    """pivot_dense (the CPU baseline's cost model: every column, as
    tableau.py:269-276) gives the same exact tableau as the oracle's pivot"""
    T = gen.tableau("mixed", 12, 10, 4)
    a, b = exact.from_array(T), exact.from_array(T)
    for _ in range(6):
        p = exact.find_standard(a)
        if isinstance(p, str):
            break
        exact.pivot(a, *p)
        exact.pivot_dense(b, *p)
        assert a == b


def test_cpu_baseline_sample_runs():
    """the bounded cpu_baseline leg on the cfg3 workload, a short sample"""
    r = bench.cpu_baseline("cfg3", seconds_target=0.5)
    assert r["cores"] == 1 and r["kind"] == "port" and r["value"] > 0
    assert "pivot_dense" in r["sample"]


def test_cpu_baseline_mid_run_sample():
    """the cpu_baseline's later-pivot point: the first pivots (here the
    reference's own cfg3 prefix, tests/golden/r3.json) replayed exactly on row
    0, the pivot rows and a sample, then pivot #(k+1) timed on the sample"""
    from conftest import load_golden
    seq = [tuple(p) for p in load_golden("r3.json")["standard_k"][0]["seq"]]
    r = bench.cpu_baseline("cfg3", seconds_target=0.5, seq=seq, k_mid=3)
    assert r["kind"] == "port" and r["cores"] == 1 and r["value"] > 0
    assert "seconds_per_pivot_at_1" in r and "seconds_per_pivot_at_4" in r
    assert r["seconds_per_pivot"] == r["seconds_per_pivot_at_4"]


class _FakeEngine:
    """records put_rows / run calls (bench's device warm-up and upload)"""

    def __init__(self, pivots_left=10 ** 9):
        self.puts, self.runs, self.left = [], [], pivots_left

    def put_rows(self, row0, rows):
        self.puts.append((row0, rows.shape[0], float(rows[0, 0])))

    def run(self, rule, k):
        done = min(k, self.left)
        self.left -= done
        self.runs.append(k)
        return 0, done


def test_device_warmup_runs_whole_groups_and_stops_when_the_lp_ends():
    assert bench.device_warmup(None, 64, 150.0) == {"ms": 0.0, "groups": 0}
    h = _FakeEngine(pivots_left=64 * 20)
    r = bench.device_warmup(h, 64, 1e6)
    assert r["groups"] == 20 and h.runs == [512, 512, 512]
    h = _FakeEngine()
    r = bench.device_warmup(h, 64, 0.0)
    assert r["groups"] == 0 and h.runs == []


def test_upload_feeds_the_heater_the_same_rows_locally_numbered():
    kind, m, ns, n, a0, a1 = bench.workload("cfg3", 2, 1)
    e, h = _FakeEngine(), _FakeEngine()
    bench.upload([e], kind, m, ns, [(a0, a1)], blk=1024, heaters=[h])
    assert [p[0] for p in e.puts] == [0] + [1 + a for a in range(a0, a1, 1024)]
    assert [p[0] for p in h.puts] == [0] + [1 + a - a0 for a in range(a0, a1, 1024)]
    assert [p[1:] for p in e.puts] == [p[1:] for p in h.puts]


def test_profile_every_for_times_every_long_sweep():
    """cfg4 on one GPU (a 2.1 GB local tableau): every sweep launch timed
    (VERDICT r5); cfg3 and the 8-GPU rank: every 4th / 8th; an explicit
    --profile-every wins"""
    assert bench.profile_every_for(32769, 8192, 20, 0) == 1
    assert bench.profile_every_for(4097, 8192, 20, 0) == 4
    assert bench.profile_every_for(4097, 8192, 64, 0) == 8
    assert bench.profile_every_for(32769, 8192, 20, 3) == 3


class _ClockEngine:
    """sweep_clocks() as lpdiag_sweep_clocks returns it: (launch, cycles,
    100 MHz ticks, start tick), oldest first"""

    def __init__(self, rows):
        self.rows = np.array(rows, dtype=np.int64)

    def sweep_clocks(self, cap):
        return self.rows[-cap:]


def test_sweep_clock_summary_reads_the_clock():
    # 1.6 M cycles over 80,000 ticks (800 us) = 2.0 GHz; 1.6 M over 72,727 = 2.2 GHz
    rows = [[0, 1_600_000, 80_000, 0], [1, 1_600_000, 72_727, 90_000], [2, 1_700_000, 85_000, 170_000]]
    s = bench.sweep_clock_summary(_ClockEngine(rows), 2)
    assert s["launches"] == 2
    assert s["ghz_per_launch"] == [2.2, 2.0]
    assert abs(s["kcycles_mean"] - 1650.0) < 1e-9
    assert abs(s["block0_us_mean"] - (727.27 + 850.0) / 2) < 1e-9
    assert abs(s["ghz_min"] - 2.0) < 1e-9 and abs(s["ghz_max"] - 2.2) < 1e-4
    assert bench.sweep_clock_summary(_ClockEngine(np.zeros((0, 4))), 4) == {"launches": 0}


def test_sweep_clock_summary_survives_a_failing_engine():
    class Bad:
        def sweep_clocks(self, cap):
            raise RuntimeError("no clocks")
    assert bench.sweep_clock_summary(Bad(), 4) == {"error": "no clocks"}
