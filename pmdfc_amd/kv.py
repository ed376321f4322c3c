"""Python mirror of the per-op front-end (include/pmdfc_kv.h, libpmdfc_gpucceh.so).

`KV` mirrors the reference's `KVStore` (server/IKV.h:9-23) as KV implements it
(server/KV.cpp:100-158): `Insert(key, value)` and `Get(key)` one op at a
time, blocking, served by the persistent device wave through the host ring
(BatchCore, pmdfc_amd/host/batch_core.h).  `ops` / `ops_async` push whole op
streams through the same ring -- per-op calls, contiguous runs, or async calls
(the flood hand-off) -- and return every op's `place | ring << 48`.  Each
serving wave owns a ring and the keys of one hash prefix; within a ring the
place is the serial order the device applied, and different rings touch
disjoint segments (so ops keep call order within a ring only; replay a stream
serially in (ring, place) order).  No CPU fallback: without the library or a
GPU, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .engine import OP_GET, OP_INSERT, PMDFC_ERR_SIZE, ST_HIT, PmdfcError, Stats, _require_gpu, depth_for_hybrid, depth_for_src, load_library

_HERE = os.path.dirname(os.path.abspath(__file__))
KV_LIB_PATH = os.path.join(_HERE, "lib", "libpmdfc_gpucceh.so")
NPHASE = 8

# every symbol include/pmdfc_kv.h declares (checked by tests/test_capi.py)
KV_EXPORTS = [
    "pmdfc_kv_create", "pmdfc_kv_destroy", "pmdfc_kv_insert", "pmdfc_kv_get", "pmdfc_kv_ops",
    "pmdfc_kv_ops_async", "pmdfc_kv_flush", "pmdfc_kv_utilization", "pmdfc_kv_capacity",
    "pmdfc_kv_find_anyway", "pmdfc_kv_stats", "pmdfc_kv_dump", "pmdfc_kv_phase", "pmdfc_kv_last_error",
    "pmdfc_kv_create_error",
]

_kvlib = None


class KVConfig(C.Structure):
    _fields_ = [("initial_depth", C.c_uint32), ("max_batch", C.c_uint32), ("max_segments", C.c_uint64),
                ("device", C.c_int32), ("flags", C.c_uint32), ("ring_size", C.c_uint32),
                ("flood_ops", C.c_uint32), ("caller_spin_us", C.c_uint32), ("serve_waves", C.c_uint32)]


def load_kv_library(path: str = KV_LIB_PATH) -> C.CDLL:
    """Load libpmdfc_gpucceh.so (after libpmdfc_cceh.so) and declare its C signatures."""
    global _kvlib
    if _kvlib is not None:
        return _kvlib
    load_library()
    if not os.path.exists(path):
        raise PmdfcError(f"{path} missing: run `make` first")
    L = C.CDLL(path)
    P, u64, u32, i32, i64 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int, C.c_int64
    sig = {
        "pmdfc_kv_create": (i32, [C.POINTER(KVConfig), C.POINTER(P)]),
        "pmdfc_kv_destroy": (i32, [P]),
        "pmdfc_kv_insert": (i32, [P, u64, u64, P]),
        "pmdfc_kv_get": (i32, [P, u64, P, P]),
        "pmdfc_kv_ops": (i64, [P, P, P, P, P, P, u64, u32, P]),
        "pmdfc_kv_ops_async": (i64, [P, P, P, P, P, P, u64, P]),
        "pmdfc_kv_flush": (i32, [P]),
        "pmdfc_kv_utilization": (i32, [P, C.POINTER(C.c_double)]),
        "pmdfc_kv_capacity": (i32, [P, C.POINTER(u64)]),
        "pmdfc_kv_find_anyway": (i32, [P, u64, P, P]),
        "pmdfc_kv_stats": (i32, [P, C.POINTER(Stats)]),
        "pmdfc_kv_dump": (i32, [P, u64, u64, P, P, P, P, P, C.POINTER(u64), C.POINTER(u64)]),
        "pmdfc_kv_create_error": (C.c_char_p, []),
        "pmdfc_kv_phase": (i32, [P, P]),
        "pmdfc_kv_last_error": (C.c_char_p, [P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _kvlib = L
    return L


class KV:
    """The served per-op front-end over one GPU index (KVStore, server/KV.cpp).

    `init_cap` with `convention` "hybrid" (CCEH_hybrid(initCap), NUMA_KV) or
    "src" (src/cceh.cpp's CCEH(initCap), KV), or `depth` directly.
    ring_size: ring places; flood_ops: unanswered places that switch the
    backlog to engine batches (0: never); serve_waves: serving waves."""

    def __init__(self, init_cap: int | None = None, *, depth: int | None = None, convention: str = "hybrid",
                 max_batch: int = 1 << 16, max_segments: int = 0, device: int = 0, upsert: bool = False,
                 ring_size: int = 1 << 13, flood_ops: int = 1024, serve_waves: int = 8, caller_spin_us: int = 10):
        L = load_kv_library()
        _require_gpu(device)
        if depth is None:
            if init_cap is None:
                raise ValueError("give init_cap or depth")
            depth = depth_for_hybrid(init_cap) if convention == "hybrid" else depth_for_src(init_cap)
        cfg = KVConfig(initial_depth=depth, max_batch=max_batch, max_segments=max_segments, device=device,
                       flags=1 if upsert else 0, ring_size=ring_size, flood_ops=flood_ops,
                       caller_spin_us=caller_spin_us, serve_waves=serve_waves)
        h = C.c_void_p()
        rc = L.pmdfc_kv_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise PmdfcError(f"pmdfc_kv_create failed ({rc}): {L.pmdfc_kv_create_error().decode()}")
        self._h = h
        self.initial_depth = depth

    def close(self):
        if getattr(self, "_h", None):
            load_kv_library().pmdfc_kv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, what: str, rc: int):
        msg = load_kv_library().pmdfc_kv_last_error(self._h)
        raise PmdfcError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    # ---- KVStore (server/IKV.h:13-21), one op at a time
    def Insert(self, key: int, value: int) -> int:
        st = C.c_uint8()
        load_kv_library().pmdfc_kv_insert(self._h, key, value, C.byref(st))
        return st.value

    def Get(self, key: int) -> int:
        """The value, or 0 (NONE) on a miss (KV::Get, server/KV.cpp:145-158)."""
        v, st = C.c_uint64(), C.c_uint8()
        load_kv_library().pmdfc_kv_get(self._h, key, C.byref(v), C.byref(st))
        return v.value if st.value == ST_HIT else 0

    def FindAnyway(self, key: int) -> int:
        v, st = C.c_uint64(), C.c_uint8()
        rc = load_kv_library().pmdfc_kv_find_anyway(self._h, key, C.byref(v), C.byref(st))
        if rc != 0:
            self._err("find_anyway", rc)
        return v.value

    def Utilization(self) -> float:
        r = C.c_double()
        rc = load_kv_library().pmdfc_kv_utilization(self._h, C.byref(r))
        if rc != 0:
            self._err("utilization", rc)
        return r.value

    def Capacity(self) -> int:
        r = C.c_uint64()
        load_kv_library().pmdfc_kv_capacity(self._h, C.byref(r))
        return r.value

    # ---- op streams through the ring
    @staticmethod
    def _arrays(ops, keys, values):
        o = np.ascontiguousarray(ops, dtype=np.uint8)
        k = np.ascontiguousarray(keys, dtype=np.uint64)
        v = np.ascontiguousarray(values, dtype=np.uint64)
        if not (o.size == k.size == v.size):
            raise ValueError("ops, keys, values differ in length")
        return o, k, v

    def ops(self, ops, keys, values, run: int = 0):
        """n ops from this thread: run 0 = one blocking call per op, run k =
        contiguous runs of k ops.  -> (values_out, status, places)."""
        o, k, v = self._arrays(ops, keys, values)
        n = o.size
        vo = np.zeros(n, np.uint64)
        st = np.zeros(n, np.uint8)
        pl = np.zeros(n, np.uint64)
        rc = load_kv_library().pmdfc_kv_ops(self._h, o.ctypes.data, k.ctypes.data, v.ctypes.data, vo.ctypes.data,
                                            st.ctypes.data, n, run, pl.ctypes.data)
        if rc < 0:
            self._err("ops", rc)
        return vo, st, pl

    def ops_async(self, ops, keys, values):
        """n ops queued as async calls, then a wait.  -> (values_out, status, places)."""
        o, k, v = self._arrays(ops, keys, values)
        n = o.size
        vo = np.zeros(n, np.uint64)
        st = np.zeros(n, np.uint8)
        pl = np.zeros(n, np.uint64)
        rc = load_kv_library().pmdfc_kv_ops_async(self._h, o.ctypes.data, k.ctypes.data, v.ctypes.data,
                                                  vo.ctypes.data, st.ctypes.data, n, pl.ctypes.data)
        if rc < 0:
            self._err("ops_async", rc)
        return vo, st, pl

    def flush(self):
        load_kv_library().pmdfc_kv_flush(self._h)

    def stats(self) -> dict:
        s = Stats()
        rc = load_kv_library().pmdfc_kv_stats(self._h, C.byref(s))
        if rc != 0:
            self._err("stats", rc)
        return {n: getattr(s, n) for n, _ in Stats._fields_}

    def phase(self) -> dict:
        a = np.zeros(NPHASE, np.uint64)
        load_kv_library().pmdfc_kv_phase(self._h, a.ctypes.data)
        names = ["wave_starts", "chunks", "flood_batches", "flood_ops", "failed_ops", "ops_completed",
                 "serve_waves", "header_reloads"]
        return {n: int(x) for n, x in zip(names, a)}

    def dump(self) -> dict:
        """Canonical dump (segments in directory order), like CCEH.dump()."""
        L = load_kv_library()
        n, nd = C.c_uint64(), C.c_uint64()
        rc = L.pmdfc_kv_dump(self._h, 0, 0, None, None, None, None, None, C.byref(n), C.byref(nd))
        while True:
            if rc != 0:
                self._err("dump", rc)
            # other threads' ops may grow the table before the filling call:
            # the library checks the capacities and we size up and retry
            nseg, ndir = n.value, nd.value
            dir_canon = np.empty(ndir, np.uint32)
            ld = np.empty(nseg, np.uint32)
            prefix = np.empty(nseg, np.uint64)
            keys = np.empty(nseg * 1024, np.uint64)
            vals = np.empty(nseg * 1024, np.uint64)
            rc = L.pmdfc_kv_dump(self._h, ndir, nseg, dir_canon.ctypes.data, ld.ctypes.data, prefix.ctypes.data,
                                 keys.ctypes.data, vals.ctypes.data, C.byref(n), C.byref(nd))
            if rc == PMDFC_ERR_SIZE:
                rc = 0
                continue
            if rc != 0:
                self._err("dump", rc)
            break
        nseg = n.value
        d = ndir.bit_length() - 1
        return {"depth": d, "dir_canon": dir_canon, "local_depth": ld[:nseg], "prefix": prefix[:nseg],
                "keys": keys[:nseg * 1024], "values": vals[:nseg * 1024]}


__all__ = ["KV", "KV_EXPORTS", "load_kv_library", "OP_GET", "OP_INSERT"]
