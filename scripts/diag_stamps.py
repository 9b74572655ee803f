"""k_group phase breakdown (diagnostic build path: LPGPU_STAMPS=1)."""
import ctypes as C
import os
import sys

os.environ["LPGPU_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "linear-program-solver_amd"))
from lpsol_amd import _lib, generators as gen  # noqa: E402

T = gen.tableau("mixed", 4096, 4096, 3)
e = _lib.Engine(4096, 8192)
e.upload(T)
e.set_block(16)
e.run(0, 64)
e.run(0, 16)
buf = (C.c_longlong * (32 * 8))()
assert e.lib.lpdiag_stamps(e.h, buf) == 0
names = ["enter", "ratio", "bar1", "leave", "prow", "bar2", "col0"]
rows = []
for t in range(16):
    st = [buf[t * 8 + k] for k in range(8)]
    d = [(st[k + 1] - st[k]) * 10 / 1000 for k in range(7)]   # 100 MHz ticks -> us
    rows.append(d)
    print(t, " ".join(f"{n}={x:5.2f}" for n, x in zip(names, d)))
avg = [sum(r[k] for r in rows[1:]) / (len(rows) - 1) for k in range(7)]
print("avg", " ".join(f"{n}={x:5.2f}" for n, x in zip(names, avg)), "sum", round(sum(avg), 2))
