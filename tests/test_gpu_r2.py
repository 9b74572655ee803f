"""Round-2 GPU tests (MI355X, through the C-ABI):

  * cfg4 -- the 32768 x 8192 G_tall tableau -- on one device (persistent
    selection with two rows per lane) and as 8 in-process row shards on one
    device, pivot sequence and every row bit-identical to oracle/lp_f64.c;
  * the timeout recovery of the persistent selection (fault injection: one
    block withholds a summary, the group is redone on the per-pivot kernels,
    results unchanged);
  * the reference's solve() assertions (simplex.py:133) and saveJson round
    trips through a device solve, pinned by tests/golden/r2.json.
"""
from fractions import Fraction

import numpy as np
import pytest

from conftest import fixture_input, load_golden

from lpsol_amd import Simplex, Tableau, _lib
from lpsol_amd import generators as gen
from oracle.f64 import F64Tableau

pytestmark = pytest.mark.gpu

R2 = load_golden("r2.json")
SMALL = load_golden("small.json")


@pytest.fixture(scope="module", autouse=True)
def gpu():
    _lib.load()
    assert _lib.device_count() > 0, "no GPU visible"


def _ids(fxs):
    return [fx["name"] for fx in fxs]


# ------------------------------------------------------------------ cfg4
CFG4 = ("tall", 32768, 8192, 3)


@pytest.fixture(scope="module")
def cfg4_oracle():
    """cfg4 after K standard pivots on the f64 oracle (one host core: ~0.3 s a pivot)"""
    kind, m, ns, seed = CFG4
    T = gen.tableau(kind, m, ns, seed)
    o = F64Tableau(T.copy())
    _, olog = o.run(0, 16)
    return T, o.T, olog


@pytest.mark.parametrize("block", [8, 32])
def test_cfg4_one_device_bit_exact(cfg4_oracle, block):
    """the whole 32768 x 8192 tableau on one GPU: 16 standard pivots through
    the persistent selection (256 blocks, two own rows per lane)"""
    T, want, olog = cfg4_oracle
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(block)
    st, done = e.run(_lib.RULE_STANDARD, 16)
    assert st == _lib.PIVOTED and done == 16
    assert e.exchange_path() == (_lib.PATH_PERSISTENT, 0)
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), want)
    e.close()


def test_cfg4_eight_shards_bit_exact(cfg4_oracle):
    """cfg4 as 8 in-process row shards of 4096 rows (the 8-GPU layout on one
    device): one persistent cross-shard selection launch per group, same
    pivots and rows as the unsharded oracle"""
    T, want, olog = cfg4_oracle
    grp = _lib.create_group(T.shape[0] - 1, T.shape[1] - 1, 8)
    for g in grp:
        g.upload(T)
        g.set_block(32)
    st, done = grp[0].run(_lib.RULE_STANDARD, 16)
    assert done == 16
    assert grp[0].exchange_path() == (_lib.PATH_PEER, 0)
    assert grp[0].log().tolist() == olog.tolist()
    assert np.array_equal(grp[0].rows(0, 1), want[:1])
    for g in grp:
        b, c = g.row_begin, g.row_count
        assert c == 4096
        assert np.array_equal(g.rows(1 + b, c), want[1 + b:1 + b + c])
    for g in reversed(grp):
        g.close()


# ------------------------------------------------------- timeout recovery
@pytest.mark.parametrize("launch,t", [(1, 0), (1, 5), (3, 2)])
@pytest.mark.parametrize("mode", ["run", "solve"])
def test_timeout_recovery_redoes_the_group(monkeypatch, launch, t, mode):
    """LPGPU_FAULT=<launch>:<t>: block 1 of that persistent launch withholds
    pivot t's ratio summary, the launch times out after LPGPU_SPIN_MAX polls,
    the host restores the group's start and redoes it on the per-pivot
    kernels: pivot sequence, stall counters and tableau as without a fault"""
    monkeypatch.setenv("LPGPU_FAULT", f"{launch}:{t}")
    monkeypatch.setenv("LPGPU_SPIN_MAX", "20000")
    monkeypatch.delenv("LPGPU_STRICT")
    if mode == "run":
        T = gen.tableau("mixed", 300, 200, 5)
    else:
        fx = next(x for x in SMALL["solve"] if x["name"] == "km_deg_d10")
        T = fixture_input(fx)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(8)
    o = F64Tableau(T)
    if mode == "run":
        st, done = e.run(_lib.RULE_STANDARD, 60)
        ost, olog = o.run(0, 60)
    else:
        st, npiv, nstd = e.solve()
        ost, olog, onstd = o.solve()
        assert st == ost == _lib.OPTIMAL
        assert nstd == onstd == fx["nstd"]
        assert olog.tolist() == fx["seq"]
    assert e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download(), o.T)
    path, fallbacks = e.exchange_path()
    assert fallbacks == 1 and path == _lib.PATH_KERNELS
    assert "timed out" in e.lib.lp_last_error(e.h).decode()
    e.close()


def test_timeout_recovery_shard_group(monkeypatch):
    """the same for in-process row shards (cross-shard persistent selection):
    every shard restores the group's start and continues with one (emulated)
    collective per pivot"""
    monkeypatch.setenv("LPGPU_FAULT", "2:3")
    monkeypatch.setenv("LPGPU_SPIN_MAX", "20000")
    monkeypatch.delenv("LPGPU_STRICT")
    monkeypatch.setenv("LPGPU_XWAIT_MS", "200")
    T = gen.tableau("mixed", 400, 150, 8)
    grp = _lib.create_group(T.shape[0] - 1, T.shape[1] - 1, 3)
    for g in grp:
        g.upload(T)
        g.set_block(8)
    st, done = grp[0].run(_lib.RULE_STANDARD, 50)
    o = F64Tableau(T)
    _, olog = o.run(0, 50)
    assert grp[0].log().tolist() == olog.tolist()
    for g in grp:
        b, c = g.row_begin, g.row_count
        assert np.array_equal(g.rows(1 + b, c), o.T[1 + b:1 + b + c])
    assert grp[0].exchange_path() == (_lib.PATH_COLLECTIVE, 1)
    for g in reversed(grp):
        g.close()


# ------------------------------------------------- the reference's asserts
def _start(fx):
    rows = [[Fraction(x) for x in r] for r in fx["start"]]
    return np.array([[float(x) for x in r] for r in rows])


@pytest.mark.parametrize("select", ["persistent", "kernels"])
@pytest.mark.parametrize("fx", R2["raises"], ids=_ids(R2["raises"]))
def test_solve_objective_assertion(fx, select, monkeypatch):
    """Simplex(tab), then setB with a negative entry, then solve(): the
    reference's AssertionError('objective value increased') after the same
    pivots, leaving the same tableau (simplex.py:133)"""
    monkeypatch.setenv("LPGPU_SELECT", select)
    tab = Tableau.fromArray(_start(fx))
    s = Simplex(tab)
    tab.setB(fx["new_b"])
    with pytest.raises(AssertionError, match=fx["message"].replace("(", r"\(").replace(")", r"\)")):
        s.solve()
    assert tab._engine().log().tolist() == fx["seq"]
    want = np.array([[float(Fraction(x)) for x in r] for r in fx["final"]])
    assert np.allclose(tab.toArray(), want, rtol=1e-12, atol=1e-12)


# -------------------------------------------------------------- JSON I/O
def _num(x):
    return float(Fraction(x))


@pytest.mark.parametrize("fx", R2["json"], ids=_ids(R2["json"]))
def test_json_device_solve_matches_reference(fx, tmp_path):
    """loadJson(reference saveJson before) -> Simplex(tab).solve() on the GPU
    -> saveJson == the reference's saveJson after, key by key: sizes, names
    and basis marks exactly; numbers exactly where the reference's values are
    dyadic, else within 1e-9 relative of its exact rationals"""
    tab = Tableau(1, 1)
    tab.loadJson(fx["before"])
    s = Simplex(tab)
    s.solve()
    got, want = tab.saveJson(), fx["after"]
    assert set(got) == set(want)
    for k in ("m", "n", "cl", "cm"):
        assert got[k] == want[k], k
    assert s.getBasicSequence() == fx["bfs"]
    flat = lambda d: [d["z"]] + d["c"] + d["b"] + [x for r in d["a"] for x in r]  # noqa: E731
    for g, w in zip(flat(got), flat(want)):
        if fx["dyadic"]:
            assert g == w
        else:
            assert abs(_num(g) - _num(w)) <= 1e-9 * max(1.0, abs(_num(w)))
    # and back through a file
    p = tmp_path / "after.json"
    tab.saveFile(str(p))
    u = Tableau(1, 1)
    u.loadFile(str(p))
    assert np.array_equal(u.toArray(), tab.toArray())


# ------------------------------------------------- sweep grid switches
@pytest.mark.parametrize("env", [{"LPGPU_SWEEP_TAIL": "2"}, {"LPGPU_SWEEP_TAIL": "0"}], ids=["tail", "no-tail"])
def test_sweep_grid_modes_bit_exact(env):
    """the sweep's last strip dealt out to every workgroup (on by default only
    for long runs, cfg4) forced on and off for small shapes, with both sweep
    kernels: pivots and every row identical to oracle/lp_f64.c (one child
    process per setting: the switches are read once per process)"""
    import os
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(__file__), "_sweep_env_worker.py")
    run = subprocess.run([sys.executable, "-u", worker], env=dict(os.environ, **env), capture_output=True,
                         text=True, timeout=110)
    assert run.returncode == 0 and "ALL OK" in run.stdout, run.stdout + run.stderr
