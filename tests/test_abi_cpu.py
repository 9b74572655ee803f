"""C-ABI library and host front-end checks that need no GPU."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from conftest import ROOT

from lpsol_amd import LinProg, Simplex, Tableau, _lib
from lpsol_amd.tableau import _fmt

HEADER = os.path.join(ROOT, "include", "lpgpu.h")
DIAG_HEADER = os.path.join(ROOT, "include", "lpgpu_diag.h")


def declared_symbols(path=HEADER, prefix="lp_"):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_symbols()
    assert len(names) >= 20
    for name in names:
        assert hasattr(lib, name), name
    assert set(names) == set(_lib.EXPORTS), "ctypes prototypes out of sync with the header"


def test_library_exports_every_declared_diagnostic():
    """include/lpgpu_diag.h: every diagnostic the library exports is declared
    there, and every declared one is exported"""
    lib = _lib.load()
    names = declared_symbols(DIAG_HEADER, "lpdiag_")
    assert len(names) >= 7
    for name in names:
        assert hasattr(lib, name), name
    src = open(os.path.join(ROOT, "linear-program-solver_amd", "csrc", "lpgpu.cpp")).read()
    assert sorted(set(re.findall(r'extern "C" int (lpdiag_\w+)\(', src))) == names
    # null handles are refused without touching a device
    assert lib.lpdiag_geometry(None, None) == _lib.BAD_ARG
    assert lib.lpdiag_stamps(None, None) == _lib.BAD_ARG
    assert lib.lpdiag_bstamps(None, None) == _lib.BAD_ARG
    assert lib.lpdiag_sweep_buffers(None, None) == _lib.BAD_ARG
    n = ctypes.c_int(0)
    assert lib.lpdiag_sweep_clocks(None, None, 4, ctypes.byref(n)) == _lib.BAD_ARG
    assert lib.lpdiag_sweep_block_clocks(None, None, 4, ctypes.byref(n)) == _lib.BAD_ARG
    assert lib.lpdiag_set_xcd_shards(None, 1) == _lib.BAD_ARG


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_default_tolerances():
    t = _lib.default_tol().as_dict()
    assert t == dict(cost=1e-9, cost_tie=1e-12, pivot=1e-9, zero=1e-9, ratio_tie=1e-12,
                     stall=1e-12)


def test_create_rejects_bad_shape_without_gpu():
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.lp_create(0, 4, 0, ctypes.byref(h)) == _lib.BAD_ARG
    assert lib.lp_create(3, -1, 0, ctypes.byref(h)) == _lib.BAD_ARG
    assert b"m > 0" in lib.lp_last_error(None)
    # 32-bit multiplier offsets: at most 4194302 rows per device
    assert lib.lp_create(1 << 22, 4, 0, ctypes.byref(h)) == _lib.BAD_ARG
    assert b"too large" in lib.lp_last_error(None)


def test_no_cpu_fallback():
    """The product path fails loudly without a GPU instead of computing on
    the host."""
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    t = Tableau(2, 4)
    t.setC([-1, -1, 0, 0])
    t.setB([1, 1])
    t.setA([[1, 0, 1, 0], [0, 1, 0, 1]])
    with pytest.raises(_lib.EngineUnavailable):
        t.pivot(0, 0)
    with pytest.raises(_lib.EngineUnavailable):
        Simplex(t).solve()


def test_reference_constructor_errors():
    with pytest.raises(ValueError):
        Tableau(0, 3)
    with pytest.raises(ValueError):
        Tableau(3, 0)


def _tab1a():
    t = Tableau(2, 4)
    t.setVarNames(["x1", "x2", "s1", "s2"])
    t.setZ(0)
    t.setC(["-40", "-30", "0", "0"])
    t.setB([12, 16])
    t.setA([[1, 1, 1, 0], [2, 1, 0, 1]])
    return t


def test_getters_setters_match_reference_semantics():
    """test_tableau.py:60-137 on the host side of the front-end"""
    t = _tab1a()
    assert t.getTableauSize() == (2, 4)
    assert t.getZ() == 0
    assert t.getC() == [-40, -30, 0, 0]
    assert t.getB() == [12, 16]
    assert t.getA() == [[1, 1, 1, 0], [2, 1, 0, 1]]
    assert t.getAij(1, 0) == 2
    with pytest.raises(IndexError):
        t.getCj(4)
    with pytest.raises(IndexError):
        t.getBi(2)
    with pytest.raises(IndexError):
        t.getAij(2, 0)
    with pytest.raises(IndexError):
        t.getVarName(4)
    t.setZ(5)
    assert t.getZ() == 5 and t.toArray()[0, 0] == -5      # stored negated
    t.setAij(0, 1, "1/2")
    assert t.getAij(0, 1) == 0.5
    t.toggleVarMark(2)
    assert t.getVarMarks() == [False, False, True, False]


def test_form_checks():
    t = _tab1a()
    bc = [0, 0]
    assert t.isCanonical(bc) and bc == [2, 3]
    assert not t.isOptimal()
    assert not t.isUnbounded() and not t.isInfeasible() and not t.isDegenerate()
    t.setBi(0, -1)
    bc = [7, 7]
    assert not t.isCanonical(bc) and bc == [7, 7]   # untouched, like tableau.py:474-475


def test_json_roundtrip_reference_format(tmp_path):
    t = _tab1a()
    t.setAij(0, 0, "3/64")
    d = t.saveJson()
    assert d["z"] == "0" and d["a"][0][0] == "3/64" and d["c"][0] == "-40"
    p = tmp_path / "t.json"
    t.saveFile(str(p))
    assert json.loads(p.read_text()) == d
    u = Tableau(1, 1)
    u.loadFile(str(p))
    assert u == t


def test_printing_and_shape_edits():
    t = _tab1a()
    text = t.printText()
    assert "-40" in text and "x1" in text
    assert t.printCSV().splitlines()[0] == ",x1,x2,s1,s2"
    assert "\\begin{tabular}" in t.printLatex()
    assert _fmt(0.5) == "1/2" and _fmt(3.0) == "3"
    c = t.copy()
    c.addVars(["y"])
    c.addCon()
    assert c.getTableauSize() == (3, 5) and t.getTableauSize() == (2, 4)
    c.permuteCols([4, 3, 2, 1, 0])
    assert c.getVarNames()[0] == "y"
    with pytest.raises(ValueError):
        c.permuteRows([0, 0, 1])


def test_linprog_stub_importable():
    LinProg()
