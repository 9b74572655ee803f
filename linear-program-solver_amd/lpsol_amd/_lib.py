"""ctypes binding of liblpgpu.so (C-ABI: include/lpgpu.h).

This is the only module that touches the shared library.  There is no CPU
fallback: if the library is missing or no GPU is visible, every device
operation raises ``EngineUnavailable`` loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# LPGPU_LIB selects another build of the same library (A/B timing of variants)
LIB_PATH = os.environ.get("LPGPU_LIB") or os.path.join(HERE, "_lib", "liblpgpu.so")

# lp_status
PIVOTED, OPTIMAL, UNBOUNDED = 0, 1, 2
ZERO_PIVOT, BAD_ARG, DEVICE_ERROR, CAP_REACHED, BAD_PIVOT = -1, -2, -3, -4, -5
OBJ_INCREASED = -6
STATUS_NAMES = {PIVOTED: "pivoted", OPTIMAL: "optimal", UNBOUNDED: "unbounded",
                ZERO_PIVOT: "zero_pivot", BAD_ARG: "bad_arg", DEVICE_ERROR: "device_error",
                CAP_REACHED: "cap_reached", BAD_PIVOT: "bad_pivot",
                OBJ_INCREASED: "objective_increased"}
# lp_exchange_path
PATH_KERNELS, PATH_PERSISTENT, PATH_PEER, PATH_COLLECTIVE = 0, 1, 2, 3
PATH_NAMES = {PATH_KERNELS: "per-pivot kernels", PATH_PERSISTENT: "persistent selection",
              PATH_PEER: "persistent selection, device-side peer exchange",
              PATH_COLLECTIVE: "per-pivot kernels, one collective per pivot"}
# lp_rule
RULE_STANDARD, RULE_MIN_INDEX = 0, 1


class EngineUnavailable(RuntimeError):
    """liblpgpu.so could not be loaded or no GPU is visible."""


class DeviceError(RuntimeError):
    """A HIP/RCCL call failed inside the engine."""


class Tol(C.Structure):
    _fields_ = [("cost", C.c_double), ("cost_tie", C.c_double), ("pivot", C.c_double),
                ("zero", C.c_double), ("ratio_tie", C.c_double), ("stall", C.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


_H = C.c_void_p
_I64 = C.c_int64
_P64 = C.POINTER(C.c_int64)
_PD = C.POINTER(C.c_double)

_PROTOS = {
    "lp_default_tol": (None, [C.POINTER(Tol)]),
    "lp_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "lp_create": (C.c_int, [_I64, _I64, C.c_int, C.POINTER(_H)]),
    "lp_comm_unique_id": (C.c_int, [C.c_void_p]),
    "lp_create_sharded": (C.c_int, [_I64, _I64, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                    C.POINTER(_H)]),
    "lp_create_group": (C.c_int, [_I64, _I64, C.c_int, C.c_int, C.POINTER(_H)]),
    "lp_shard_rows": (C.c_int, [_H, _P64, _P64]),
    "lp_destroy": (C.c_int, [_H]),
    "lp_set_tol": (C.c_int, [_H, C.POINTER(Tol)]),
    "lp_get_tol": (C.c_int, [_H, C.POINTER(Tol)]),
    "lp_upload_rows": (C.c_int, [_H, _I64, _I64, _PD, _I64]),
    "lp_download_rows": (C.c_int, [_H, _I64, _I64, _PD, _I64]),
    "lp_pivot": (C.c_int, [_H, _I64, _I64]),
    "lp_find_pivot": (C.c_int, [_H, C.c_int, C.c_int, _P64, _P64]),
    "lp_pivot_checked": (C.c_int, [_H, _I64, _I64]),
    "lp_solve": (C.c_int, [_H, _I64, _P64, _P64]),
    "lp_run": (C.c_int, [_H, C.c_int, _I64, _P64]),
    "lp_pivot_log": (C.c_int, [_H, _P64, _I64, _P64]),
    "lp_objective": (C.c_int, [_H, _PD]),
    "lp_set_block": (C.c_int, [_H, C.c_int]),
    "lp_get_block": (C.c_int, [_H, C.POINTER(C.c_int)]),
    "lp_profile": (C.c_int, [_H, C.c_int]),
    "lp_update_time": (C.c_int, [_H, _PD, _P64]),
    "lp_select_time": (C.c_int, [_H, _PD, _P64]),
    "lp_find_pivot_max_increase": (C.c_int, [_H, C.c_int, _P64, _P64]),
    "lp_find_pivot_all": (C.c_int, [_H, _P64, _I64, _P64]),
    "lp_form_checks": (C.c_int, [_H, C.POINTER(C.c_int32), _P64]),
    "lp_peer_handle": (C.c_int, [_H, C.c_char_p]),
    "lp_peer_open": (C.c_int, [_H, C.c_char_p]),
    "lp_peer_enable": (C.c_int, [_H, C.c_int]),
    "lp_set_host_allgather": (C.c_int, [_H, C.c_void_p, C.c_void_p]),
    "lp_exchange_path": (C.c_int, [_H, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "lp_xwait": (C.c_int, [_H, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "lp_last_error": (C.c_char_p, [_H]),
}

EXPORTS = tuple(_PROTOS)

_lib = None


def load(path: str = LIB_PATH):
    """Load liblpgpu.so (no GPU needed to load it)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise EngineUnavailable(
            f"{path} is missing: build it with `make -C linear-program-solver_amd/csrc` "
            "or __graft_entry__.build() (there is no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, argt) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = argt
    if path == LIB_PATH:
        _lib = lib
    return lib


def default_tol() -> Tol:
    t = Tol()
    load().lp_default_tol(C.byref(t))
    return t


def device_count() -> int:
    n = C.c_int(0)
    load().lp_device_count(C.byref(n))
    return n.value


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_PD)


class Engine:
    """One device tableau (or one shard of a row-sharded one).

    Thin, typed wrapper of an ``lp_handle``: every method is one C-ABI call.
    ``rows()``/``put_rows()`` use GLOBAL row numbers (row 0 = objective)."""

    def __init__(self, m: int, n: int, device: int = 0, *, _handle=None):
        self.lib = load()
        self.m, self.n = int(m), int(n)
        self.device = device
        if _handle is not None:
            self.h = _handle
        else:
            if device_count() <= device:
                raise EngineUnavailable(
                    f"no GPU {device} visible (lp_device_count = {device_count()}); "
                    "the engine has no CPU fallback")
            h = _H()
            self._check(self.lib.lp_create(self.m, self.n, device, C.byref(h)), None)
            self.h = h
        b, c = C.c_int64(), C.c_int64()
        self.lib.lp_shard_rows(self.h, C.byref(b), C.byref(c))
        self.row_begin, self.row_count = b.value, c.value

    # -- plumbing ---------------------------------------------------------
    def _check(self, st: int, h) -> int:
        if st in (BAD_ARG,):
            raise ValueError(self._err(h))
        if st == DEVICE_ERROR:
            raise DeviceError(self._err(h))
        return st

    def _err(self, h) -> str:
        msg = self.lib.lp_last_error(h)
        return msg.decode() if msg else ""

    def close(self):
        if getattr(self, "h", None):
            self.lib.lp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- tolerances ---------------------------------------------------------
    def set_tol(self, **kw):
        t = self.get_tol()
        for k, v in kw.items():
            if not hasattr(t, k):
                raise KeyError(k)
            setattr(t, k, float(v))
        self.lib.lp_set_tol(self.h, C.byref(t))

    def get_tol(self) -> Tol:
        t = Tol()
        self.lib.lp_get_tol(self.h, C.byref(t))
        return t

    # -- data ---------------------------------------------------------------
    def put_rows(self, row0: int, rows: np.ndarray):
        a = np.ascontiguousarray(rows, dtype=np.float64)
        if a.ndim != 2 or a.shape[1] != self.n + 1:
            raise ValueError(f"rows must be (k, {self.n + 1}) float64")
        self._check(self.lib.lp_upload_rows(self.h, row0, a.shape[0], _ptr(a), a.shape[1]), self.h)

    def rows(self, row0: int, nrows: int) -> np.ndarray:
        out = np.empty((nrows, self.n + 1), dtype=np.float64)
        if nrows:
            self._check(self.lib.lp_download_rows(self.h, row0, nrows, _ptr(out), self.n + 1),
                        self.h)
        return out

    def upload(self, T: np.ndarray):
        """Whole tableau (single device) or row 0 + this shard's rows taken
        from a full-size array."""
        T = np.asarray(T, dtype=np.float64)
        if T.shape != (self.m + 1, self.n + 1):
            raise ValueError(f"tableau must be {(self.m + 1, self.n + 1)}")
        self.put_rows(0, T[:1])
        b = self.row_begin
        self.put_rows(1 + b, T[1 + b:1 + b + self.row_count])

    def download(self) -> np.ndarray:
        """Whole tableau (single device only)."""
        if self.row_count != self.m:
            raise ValueError("download() needs an unsharded engine; use rows()")
        return self.rows(0, self.m + 1)

    def objective(self) -> float:
        z = C.c_double()
        self._check(self.lib.lp_objective(self.h, C.byref(z)), self.h)
        return z.value

    # -- pivots -------------------------------------------------------------
    def pivot(self, r: int, c: int) -> int:
        return self._check(self.lib.lp_pivot(self.h, r, c), self.h)

    def pivot_checked(self, r: int, c: int) -> int:
        return self._check(self.lib.lp_pivot_checked(self.h, r, c), self.h)

    def find(self, rule: int, do_pivot: bool):
        """-> (r, c) | 'optimal' | 'unbounded'"""
        r, c = C.c_int64(), C.c_int64()
        st = self._check(self.lib.lp_find_pivot(self.h, rule, int(bool(do_pivot)),
                                                C.byref(r), C.byref(c)), self.h)
        if st == OPTIMAL:
            return "optimal"
        if st == UNBOUNDED:
            return "unbounded"
        if st != PIVOTED:
            raise DeviceError(f"unexpected status {STATUS_NAMES.get(st, st)}")
        return r.value, c.value

    def find_max_increase(self, do_pivot: bool):
        """findPivotMaxIncrease -> (r, c) | 'optimal' | 'unbounded'"""
        r, c = C.c_int64(), C.c_int64()
        st = self._check(self.lib.lp_find_pivot_max_increase(self.h, int(bool(do_pivot)),
                                                             C.byref(r), C.byref(c)), self.h)
        if st == OPTIMAL:
            return "optimal"
        if st == UNBOUNDED:
            return "unbounded"
        if st != PIVOTED:
            raise DeviceError(f"unexpected status {STATUS_NAMES.get(st, st)}")
        return r.value, c.value

    def find_all(self) -> list[tuple[int, int]]:
        """findPivotAll -> [(r, c), ...] column-major"""
        cnt = C.c_int64()
        self._check(self.lib.lp_find_pivot_all(self.h, None, 0, C.byref(cnt)), self.h)
        if cnt.value == 0:
            return []
        out = np.zeros(2 * cnt.value, dtype=np.int64)
        self._check(self.lib.lp_find_pivot_all(self.h, out.ctypes.data_as(_P64), cnt.value,
                                               C.byref(cnt)), self.h)
        return [(int(out[2 * k]), int(out[2 * k + 1])) for k in range(cnt.value)]

    def form_checks(self):
        """-> dict(canonical, optimal, unbounded, infeasible, degenerate, bcols)"""
        flags = (C.c_int32 * 5)()
        bcols = np.full(self.m, -2, dtype=np.int64)
        self._check(self.lib.lp_form_checks(self.h, flags, bcols.ctypes.data_as(_P64)), self.h)
        keys = ("canonical", "optimal", "unbounded", "infeasible", "degenerate")
        out = {k: bool(flags[i]) for i, k in enumerate(keys)}
        out["bcols"] = None if np.all(bcols == -2) and self.m else [int(x) for x in bcols]
        return out

    def solve(self, max_pivots: int = -1):
        """-> (status, npiv, nstd)"""
        a, b = C.c_int64(), C.c_int64()
        st = self._check(self.lib.lp_solve(self.h, max_pivots, C.byref(a), C.byref(b)), self.h)
        return st, a.value, b.value

    def run(self, rule: int, k: int):
        """-> (status, pivots done)"""
        d = C.c_int64()
        st = self._check(self.lib.lp_run(self.h, rule, k, C.byref(d)), self.h)
        return st, d.value

    def log(self) -> np.ndarray:
        cnt = C.c_int64()
        self.lib.lp_pivot_log(self.h, None, 0, C.byref(cnt))
        out = np.zeros((cnt.value, 2), dtype=np.int64)
        if cnt.value:
            self._check(self.lib.lp_pivot_log(self.h, out.ctypes.data_as(_P64), cnt.value,
                                              C.byref(cnt)), self.h)
        return out

    def exchange_path(self):
        """-> (lp_exchange_path of the last solve/run, timed-out groups redone)"""
        p, f = C.c_int(), C.c_int()
        self.lib.lp_exchange_path(self.h, C.byref(p), C.byref(f))
        return p.value, f.value

    def xwait(self):
        """-> (cross-rank hop seconds, pivots) of the row-sharded persistent
        selection, cumulative (lp_xwait: block 0, 100 MHz device clock)"""
        t, n = C.c_int64(), C.c_int64()
        self.lib.lp_xwait(self.h, C.byref(t), C.byref(n))
        return t.value * 1e-8, n.value

    def set_block(self, pivots_per_sweep: int):
        """pivots deferred into one sweep of the tableau (1..64; 0 = auto)"""
        self._check(self.lib.lp_set_block(self.h, int(pivots_per_sweep)), self.h)

    def geometry(self) -> dict:
        """diagnostics (lpdiag_geometry): the persistent selection's launch
        geometry for this handle and what its last launch found on the device"""
        out = (C.c_longlong * 9)()
        self._check(self.lib.lpdiag_geometry(self.h, out), self.h)
        keys = ("blocks", "ipl", "rpl", "nr", "one_xcd_grid", "two_level_variant", "sel", "flags", "xcd_shards")
        d = dict(zip(keys, list(out)))
        d["kernel"] = "none" if d["blocks"] == 0 else "k_sel" if d["sel"] else "k_group"
        d["on_one_xcd"] = bool(d["flags"] & 1)
        d["two_level_engaged"] = bool(d["flags"] & 2)
        d["xcd_shards_engaged"] = bool(d["flags"] & 16)
        return d

    def sweep_buffers(self) -> int:
        """diagnostics (lpdiag_sweep_buffers): 2 when the sweeps run out of
        place (a second tableau buffer), 1 in place"""
        nb = C.c_int(0)
        self._check(self.lib.lpdiag_sweep_buffers(self.h, C.byref(nb)), self.h)
        return nb.value

    def sweep_clocks(self, cap: int = 1024) -> np.ndarray:
        """diagnostics (lpdiag_sweep_clocks): per 64-pivot sweep launch, its
        block 0's (launch number, shader cycles, 100 MHz ticks, start tick),
        the latest `cap` launches oldest first -- cycles / (ticks / 1e8) is
        the shader clock during that launch"""
        buf = (C.c_ulonglong * (4 * cap))()
        n = C.c_int(0)
        self._check(self.lib.lpdiag_sweep_clocks(self.h, buf, C.c_int(cap), C.byref(n)), self.h)
        return np.array(buf[:4 * n.value], dtype=np.uint64).reshape(-1, 4).astype(np.int64)

    def sweep_block_clocks(self, cap: int = 8192) -> np.ndarray:
        """diagnostics (lpdiag_sweep_block_clocks): every block's pass in the
        latest 64-pivot sweep launch -- (block, start tick, pass-end tick,
        shader cycles), 100 MHz ticks"""
        buf = (C.c_ulonglong * (4 * cap))()
        n = C.c_int(0)
        self._check(self.lib.lpdiag_sweep_block_clocks(self.h, buf, C.c_int(cap), C.byref(n)), self.h)
        return np.array(buf[:4 * n.value], dtype=np.uint64).reshape(-1, 4).astype(np.int64)

    def set_xcd_shards(self, on: bool):
        """diagnostics / A/B (lpdiag_set_xcd_shards): a tall single-device
        tableau runs k_sel as one row shard per XCD (default) or k_group"""
        self._check(self.lib.lpdiag_set_xcd_shards(self.h, 1 if on else 0), self.h)

    def get_block(self) -> int:
        """pivots per sweep in use (the auto choice resolved)"""
        b = C.c_int()
        self.lib.lp_get_block(self.h, C.byref(b))
        return b.value

    # -- timing -------------------------------------------------------------
    def profile(self, enable: bool, every: int = 1):
        """time the launches (every `every`-th of each kernel) with HIP events"""
        self.lib.lp_profile(self.h, max(1, int(every)) if enable else 0)

    def update_time(self):
        """-> (total ms, launches) of the rank-1 update kernel since profile()."""
        ms, n = C.c_double(), C.c_int64()
        self.lib.lp_update_time(self.h, C.byref(ms), C.byref(n))
        return ms.value, n.value

    # ---- device-side exchange between the ranks of a sharded job
    PEER_HANDLE_BYTES = 64

    def peer_handle(self) -> bytes:
        """This rank's exchange-buffer IPC handle (all-gather it in rank order)."""
        buf = C.create_string_buffer(self.PEER_HANDLE_BYTES)
        self._check(self.lib.lp_peer_handle(self.h, buf), self.h)
        return buf.raw

    def peer_open(self, handles: bytes):
        """Open every rank's buffer and check the exchange (collective)."""
        self._check(self.lib.lp_peer_open(self.h, handles), self.h)

    def peer_enable(self, enable: bool):
        self._check(self.lib.lp_peer_enable(self.h, 1 if enable else 0), self.h)

    def set_host_allgather(self, fn):
        """Give a multi-process shard the host's all-gather: fn(bytes) -> list
        of every rank's bytes in rank order (e.g. torch.distributed over gloo,
        see gloo_allgather).  The column scans combine through it; a handle
        without an RCCL communicator also runs its per-pivot exchanges
        through it."""
        cb = allgather_callback(fn)
        self._check(self.lib.lp_set_host_allgather(self.h, C.cast(cb, C.c_void_p), None), self.h)
        self._allgather_cb = cb     # the library holds the pointer: keep it alive

    def select_time(self):
        """-> (total ms, launches) of the pivot-selection kernel since profile()."""
        ms, n = C.c_double(), C.c_int64()
        self.lib.lp_select_time(self.h, C.byref(ms), C.byref(n))
        return ms.value, n.value


_ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)


def allgather_callback(fn):
    """The C callback (lp_allgather_fn) around fn(bytes) -> [bytes per rank]."""
    def tramp(ctx, send, recv, nbytes):
        try:
            parts = fn(C.string_at(send, nbytes))
            blob = b"".join(parts)
            if len(blob) != nbytes * len(parts):
                return 1
            C.memmove(recv, blob, len(blob))
            return 0
        except Exception:       # noqa: BLE001 - no exception may cross the C ABI
            return 1
    return _ALLGATHER_FN(tramp)


def gloo_allgather(group=None):
    """A host all-gather over torch.distributed (CPU tensors: gloo) for
    Engine.set_host_allgather."""
    import torch
    import torch.distributed as dist

    def fn(data: bytes) -> list[bytes]:
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(out, t, group=group)
        return [o.numpy().tobytes() for o in out]
    return fn


def create_group(m: int, n: int, nshards: int, device: int = 0) -> list[Engine]:
    """In-process emulation of an nshards-rank row-sharded job on one GPU."""
    lib = load()
    if device_count() <= device:
        raise EngineUnavailable("no GPU visible; the engine has no CPU fallback")
    hs = (_H * nshards)()
    st = lib.lp_create_group(m, n, device, nshards, hs)
    if st != PIVOTED:
        raise (ValueError if st == BAD_ARG else DeviceError)(lib.lp_last_error(None).decode())
    engines = [Engine(m, n, device, _handle=_H(hs[k])) for k in range(nshards)]
    # destroy in reverse order: shard 0 owns the shared stream
    for e in engines[1:]:
        e._keep = engines[0]
    return engines


def comm_unique_id() -> bytes:
    """128-byte RCCL unique id (call on rank 0, broadcast to all ranks)."""
    buf = C.create_string_buffer(128)
    st = load().lp_comm_unique_id(buf)
    if st != PIVOTED:
        raise DeviceError(load().lp_last_error(None).decode())
    return buf.raw


def create_sharded(m: int, n: int, rank: int, nranks: int, uid: bytes,
                   device: int = 0) -> Engine:
    """One rank's shard of an nranks-process row-sharded tableau (RCCL)."""
    lib = load()
    if device_count() <= device:
        raise EngineUnavailable("no GPU visible; the engine has no CPU fallback")
    if uid is not None and len(uid) != 128:
        raise ValueError("uid must be the 128-byte RCCL unique id (or None: no RCCL)")
    h = _H()
    st = lib.lp_create_sharded(m, n, device, rank, nranks, uid, C.byref(h))
    if st != PIVOTED:
        raise (ValueError if st == BAD_ARG else DeviceError)(lib.lp_last_error(None).decode())
    return Engine(m, n, device, _handle=h)
