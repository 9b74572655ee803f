"""Round 5 GPU tests (MI355X, through the C-ABI):

* the sweep's tail piece of <= 4 columns, rows across
  lanes, must cover every row of a block's tail, however many -- a tall
  narrow tableau on a grid sized for 8 CUs (LPGPU_SWEEP_CUS) gives tails of
  several times 64 W rows per block (8- and 4-wave sweeps, 1 and 3 tail
  columns), every bit as oracle/lp_f64.c's.

Reference: /root/reference/lpsol/tableau.py:269-280 (rowAdd, the rank-1
update the sweep applies for every pivot of a group).
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shapes", [
    "tall,20000,512,100,64",      # 8 waves, 1 tail column, 2504-row tails (64 W = 512)
    "tall,20000,514,80,64",       # 8 waves, 3 tail columns
    "tall,9000,256,80,64",        # 4 waves, 1 tail column, 568-row tails (64 W = 256)
])
def test_sweep_tail_rows_beyond_one_pass(shapes):
    worker = os.path.join(os.path.dirname(__file__), "_sweep_env_worker.py")
    env = dict(os.environ, LPGPU_SWEEP_CUS="8", SWEEP_SHAPES=shapes)
    run = subprocess.run([sys.executable, "-u", worker], env=env, capture_output=True, text=True, timeout=280)
    assert run.returncode == 0 and "ALL OK" in run.stdout, run.stdout + run.stderr


@pytest.mark.parametrize("kind,m,ns,k,blocks,ipl", [
    ("tall", 8192, 8192, 136, 64, 2),     # a 4-GPU rank of cfg4: 1024 rows per XCD shard, 2 columns per lane
    ("tall", 9000, 6000, 100, 64, 2),     # 1125-row shards, 18 rows per block (the last 9)
    ("tall", 12000, 3000, 80, 64, 1),     # 1500-row shards, one column per lane
])
def test_xcd_shards_at_64_blocks_bit_exact(kind, m, ns, k, blocks, ipl):
    """k_sel's XCD shards take 64 blocks where they fit (round 5, sel_geom):
    shards of 1024-1500 rows, 2 or 1 columns per lane instead of 4 -- the
    pivot sequence and every bit of the tableau as oracle/lp_f64.c's, no
    fallback (simplex.py:251-284, tableau.py:295-308)"""
    import numpy as np

    from lpsol_amd import _lib, generators as gen
    from oracle.f64 import F64Tableau

    T = gen.tableau(kind, m, ns, 5)
    e = _lib.Engine(T.shape[0] - 1, T.shape[1] - 1)
    e.upload(T)
    e.set_block(64)
    st, done = e.run(_lib.RULE_STANDARD, k)
    geo = e.geometry()
    assert geo["kernel"] == "k_sel" and geo["xcd_shards"] == 8, geo
    assert (geo["blocks"], geo["ipl"]) == (blocks, ipl), geo
    assert e.exchange_path()[1] == 0
    o = F64Tableau(T.copy())
    ost, olog = o.run(0, k)
    assert done == len(olog) and e.log().tolist() == olog.tolist()
    assert np.array_equal(e.download().view(np.uint64), o.T.view(np.uint64))
    e.close()
