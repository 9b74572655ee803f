import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "linear-program-solver_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblpgpu.so)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def fixture_input(fx):
    """float64 engine-layout tableau of a golden fixture."""
    from lpsol_amd import generators as gen
    from oracle import exact
    if "gen" in fx:
        g = fx["gen"]
        return gen.tableau(g["kind"], g["m"], g["ns"], g["seed"])
    if "exact" in fx:
        e = fx["exact"]
        rows = exact.from_strings(e["z"], e["c"], e["b"], e["a"])
        return np.array([[float(x) for x in r] for r in rows])
    if "phase1" in fx:
        g = fx["phase1"]
        return gen.phase1_lp(g["kind"], g["m"], g["ns"], g["seed"])
    return np.asarray(fx["array"], dtype=np.float64)


def fixture_exact(fx):
    """exact rows of a golden fixture (Fractions)."""
    from oracle import exact
    if "exact" in fx:
        e = fx["exact"]
        return exact.from_strings(e["z"], e["c"], e["b"], e["a"])
    return exact.from_array(fixture_input(fx))


@pytest.fixture(autouse=True)
def strict_engine(monkeypatch):
    """every engine a test creates treats a timed-out persistent selection
    group as an error (lpgpu.cpp, LPGPU_STRICT): the silent recovery onto
    the per-pivot kernels would keep the results right and hide a
    co-residency bug; the fault-injection tests switch it off"""
    monkeypatch.setenv("LPGPU_STRICT", "1")


@pytest.fixture(scope="session")
def small_golden():
    return load_golden("small.json")


@pytest.fixture(scope="session")
def big_golden():
    return load_golden("big.json")
