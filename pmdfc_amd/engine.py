"""Python host mirror of the reference index interfaces over the HIP C-ABI.

`CCEH` mirrors `IHash`/`ICCEH` as implemented by CCEH_hybrid
(server/IHash.h:9-22, server/ICCEH.h:9-27, server/CCEH_hybrid.cpp) but every
call takes a whole batch.  `BloomFilter` mirrors client/bloom_filter.c.
All compute runs in libpmdfc_cceh.so (include/pmdfc_cceh.h); there is no CPU
fallback: if the library or a GPU is missing, construction raises.

Inputs may be torch tensors already on the engine's device (zero copy, the
work is enqueued on torch's current stream) or numpy/host arrays (copied in
and out, synchronous).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

try:  # torch first: its bundled libamdhip64 then serves the engine too
    import torch
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# PMDFC_LIB: an A/B build of the same engine (Makefile target `ab`)
LIB_PATH = os.environ.get("PMDFC_LIB") or os.path.join(_HERE, "lib", "libpmdfc_cceh.so")

OP_GET, OP_INSERT = 0, 1
PMDFC_ERR_SIZE = -5  # an output buffer is smaller than the result (include/pmdfc_cceh.h)
(ST_MISS, ST_HIT, ST_INSERTED, ST_RESERVED_KEY, ST_UNSPLITTABLE, ST_DEPTH_LIMIT, ST_CAPACITY,
 ST_FILTERED, ST_WRONG_SHARD, ST_ROUTE_OVERFLOW, ST_SPLIT_LOST, ST_UPDATED) = range(12)
CFG_UPSERT = 1  # pmdfc_cceh_config_t.flags: last-writer-wins Insert
K_NAMES = ["get", "prep", "route", "final", "process", "split", "parked", "mixed_get", "bloom"]

_lib = None
# pmdfc_comm_create_host's transport functions
_XCHG = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)
_AMAX = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64))


class PmdfcError(RuntimeError):
    pass


class Config(C.Structure):
    _fields_ = [("initial_depth", C.c_uint32), ("shard_bits", C.c_uint32), ("shard_id", C.c_uint32),
                ("max_batch", C.c_uint32), ("max_segments", C.c_uint64), ("device", C.c_int32),
                ("flags", C.c_uint32)]


class RouterConfig(C.Structure):
    _fields_ = [("shard_bits", C.c_uint32), ("max_batch", C.c_uint32), ("cap", C.c_uint64),
                ("carry_cap", C.c_uint64), ("device", C.c_int32), ("flags", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("depth", C.c_uint32), ("phys_depth", C.c_uint32), ("segments", C.c_uint64),
                ("capacity", C.c_uint64), ("max_segments", C.c_uint64), ("splits", C.c_uint64),
                ("doublings", C.c_uint64), ("split_loss", C.c_uint64), ("insert_passes", C.c_uint64),
                ("batches", C.c_uint64), ("segment_runs", C.c_uint64), ("deferred_ops", C.c_uint64),
                ("bucket_bits", C.c_uint32), ("max_rounds", C.c_uint32), ("insert_lines", C.c_uint64),
                ("error_flags", C.c_uint32), ("fast_declined", C.c_uint32)]


# every symbol include/pmdfc_cceh.h declares (checked by tests/test_capi.py)
EXPORTS = [
    "pmdfc_depth_for_hybrid", "pmdfc_depth_for_src", "pmdfc_abi_version", "pmdfc_last_error",
    "pmdfc_cceh_create", "pmdfc_cceh_destroy", "pmdfc_cceh_reset", "pmdfc_cceh_insert",
    "pmdfc_cceh_insert_batches",
    "pmdfc_cceh_get", "pmdfc_cceh_get_batches", "pmdfc_cceh_find_anyway", "pmdfc_cceh_mixed", "pmdfc_cceh_mixed_batches", "pmdfc_cceh_mixed_host", "pmdfc_cceh_stats",
    "pmdfc_cceh_utilization", "pmdfc_cceh_dump", "pmdfc_cceh_timing_enable",
    "pmdfc_cceh_timing_read", "pmdfc_cceh_last_get_lines", "pmdfc_hash64", "pmdfc_gen_keys",
    "pmdfc_route_by_shard", "pmdfc_cceh_debug_stamps", "pmdfc_bloom_create", "pmdfc_bloom_destroy", "pmdfc_bloom_clear",
    "pmdfc_bloom_add", "pmdfc_bloom_probe", "pmdfc_bloom_bitmap", "pmdfc_bloom_set_bitmap_host",
    "pmdfc_bloom_get_bitmap_host", "pmdfc_bloom_probe_then_get", "pmdfc_ubench_gather64", "pmdfc_ubench_gather", "pmdfc_ubench_scatter16",
    "pmdfc_router_create", "pmdfc_router_destroy", "pmdfc_router_rows", "pmdfc_router_pack", "pmdfc_router_unpack",
    "pmdfc_router_carried", "pmdfc_router_end_call", "pmdfc_router_overflow_count", "pmdfc_router_reset",
    "pmdfc_router_dedupe", "pmdfc_router_fill", "pmdfc_route_split", "pmdfc_route_respond",
    "pmdfc_cceh_insert_records", "pmdfc_cceh_get_records",
    "pmdfc_cbf_create", "pmdfc_cbf_destroy", "pmdfc_cbf_clear", "pmdfc_cbf_insert", "pmdfc_cbf_insert_ops",
    "pmdfc_cbf_delete", "pmdfc_cbf_query", "pmdfc_cbf_pack", "pmdfc_cbf_query_bits",
    "pmdfc_cbf_export", "pmdfc_cbf_counters", "pmdfc_cbf_get_counters_host",
    "pmdfc_cbf_get_bitmap_host", "pmdfc_cceh_insert_extent", "pmdfc_cceh_get_extent", "pmdfc_trace_create", "pmdfc_trace_destroy", "pmdfc_trace_parse",
    "pmdfc_cceh_serve_start", "pmdfc_cceh_serve_start_n", "pmdfc_cceh_serve_waves_max", "pmdfc_comm_id", "pmdfc_comm_create", "pmdfc_comm_create_host", "pmdfc_comm_destroy",
    "pmdfc_route_batches",
    "pmdfc_route_mixed_batches",
]


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load libpmdfc_cceh.so and declare its C signatures (no GPU needed)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise PmdfcError(f"{path} missing: run `make` (or __graft_entry__.build()) first")
    L = C.CDLL(path)
    P, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
    sig = {
        "pmdfc_depth_for_hybrid": (u32, [u64]),
        "pmdfc_depth_for_src": (u32, [u64]),
        "pmdfc_abi_version": (i32, []),
        "pmdfc_last_error": (C.c_char_p, []),
        "pmdfc_cceh_create": (i32, [C.POINTER(Config), C.POINTER(P)]),
        "pmdfc_cceh_destroy": (i32, [P]),
        "pmdfc_cceh_reset": (i32, [P, P]),
        "pmdfc_cceh_insert": (i32, [P, P, P, P, u64, P]),
        "pmdfc_cceh_insert_batches": (i32, [P, P, P, P, P, u32, P]),
        "pmdfc_cceh_get": (i32, [P, P, P, P, u64, P]),
        "pmdfc_cceh_find_anyway": (i32, [P, P, P, P, u64, P]),
        "pmdfc_cceh_mixed": (i32, [P, P, P, P, P, P, u64, P]),
        "pmdfc_cceh_get_batches": (i32, [P, P, P, P, P, u32, P]),
        "pmdfc_cceh_mixed_batches": (i32, [P, P, P, P, P, P, P, u32, P]),
        "pmdfc_cceh_mixed_host": (i32, [P, P, P, P, P, P, u64]),
        "pmdfc_cceh_stats": (i32, [P, C.POINTER(Stats)]),
        "pmdfc_cceh_utilization": (i32, [P, C.POINTER(C.c_double)]),
        "pmdfc_cceh_dump": (i32, [P, P, P, P, P, P, C.POINTER(u64)]),
        "pmdfc_cceh_timing_enable": (i32, [P, i32]),
        "pmdfc_cceh_timing_read": (i32, [P, P, P, i32]),
        "pmdfc_cceh_last_get_lines": (i32, [P, C.POINTER(u64)]),
        "pmdfc_cceh_debug_stamps": (i32, [P, P, u64, C.POINTER(u32)]),
        "pmdfc_hash64": (i32, [P, P, u64, P]),
        "pmdfc_gen_keys": (i32, [u64, u64, P, u64, P]),
        "pmdfc_route_by_shard": (i32, [P, u64, u32, P, P, i32, P]),
        "pmdfc_bloom_create": (i32, [u64, u32, i32, C.POINTER(P)]),
        "pmdfc_bloom_destroy": (i32, [P]),
        "pmdfc_bloom_clear": (i32, [P, P]),
        "pmdfc_bloom_add": (i32, [P, P, u64, P]),
        "pmdfc_bloom_probe": (i32, [P, P, P, u64, P]),
        "pmdfc_bloom_bitmap": (i32, [P, C.POINTER(P), C.POINTER(u64)]),
        "pmdfc_bloom_probe_then_get": (i32, [P, P, P, P, P, u64, P]),
        "pmdfc_bloom_set_bitmap_host": (i32, [P, P, u64]),
        "pmdfc_bloom_get_bitmap_host": (i32, [P, P, u64]),
        "pmdfc_ubench_gather64": (i32, [P, u64, P, u32, u64, u64, P, P]),
        "pmdfc_ubench_gather": (i32, [P, u64, u32, u32, P, u32, u64, u64, P, u64, P]),
        "pmdfc_ubench_scatter16": (i32, [P, u64, u32, u64, u64, P]),
        "pmdfc_router_create": (i32, [C.POINTER(RouterConfig), C.POINTER(P)]),
        "pmdfc_router_destroy": (i32, [P]),
        "pmdfc_router_rows": (u64, [P]),
        "pmdfc_router_pack": (i32, [P, P, P, P, P, u64, u32, u32, P, P, P, P, P]),
        "pmdfc_router_unpack": (i32, [P, P, u32, P, P, P, P]),
        "pmdfc_router_carried": (i32, [P, P, P]),
        "pmdfc_router_end_call": (i32, [P]),
        "pmdfc_router_overflow_count": (i32, [P, C.POINTER(u64), P]),
        "pmdfc_router_reset": (i32, [P, P]),
        "pmdfc_router_dedupe": (i32, [P, P, P, u64, u32, P, P, P]),
        "pmdfc_router_fill": (i32, [P, u64, P, P, i32, P]),
        "pmdfc_route_split": (i32, [P, u64, u32, P, P, P, i32, P]),
        "pmdfc_route_respond": (i32, [P, P, u64, P, i32, P]),
        "pmdfc_cceh_insert_records": (i32, [P, P, P, u64, P]),
        "pmdfc_cceh_get_records": (i32, [P, P, P, u64, P]),
        "pmdfc_cbf_create": (i32, [u64, u32, i32, C.POINTER(P)]),
        "pmdfc_cbf_destroy": (i32, [P]),
        "pmdfc_cbf_clear": (i32, [P, P]),
        "pmdfc_cbf_insert": (i32, [P, P, u64, P]),
        "pmdfc_cbf_insert_ops": (i32, [P, P, P, u64, P]),
        "pmdfc_cbf_delete": (i32, [P, P, P, u64, P]),
        "pmdfc_cbf_query": (i32, [P, P, P, u64, P]),
        "pmdfc_cbf_pack": (i32, [P, P]),
        "pmdfc_cbf_query_bits": (i32, [P, P, P, u64, P]),
        "pmdfc_cbf_export": (i32, [P, P, P]),
        "pmdfc_cbf_counters": (i32, [P, C.POINTER(P), C.POINTER(P), C.POINTER(u64)]),
        "pmdfc_cbf_get_counters_host": (i32, [P, P, u64]),
        "pmdfc_cbf_get_bitmap_host": (i32, [P, P, u64]),
        "pmdfc_cceh_insert_extent": (i32, [P, i32, P, P, P, P, u64, C.POINTER(u64), P]),
        "pmdfc_cceh_get_extent": (i32, [P, i32, P, P, P, P, u64, P]),
        "pmdfc_trace_create": (i32, [i32, C.POINTER(P)]),
        "pmdfc_trace_destroy": (i32, [P]),
        "pmdfc_trace_parse": (i32, [P, P, u64, u64, P, P, P, P]),
        "pmdfc_cceh_serve_start": (i32, [P, P, P, P, u64, u64, P, P]),
        "pmdfc_cceh_serve_start_n": (i32, [P, u32, P, P, P, u64, P, P]),
        "pmdfc_cceh_serve_waves_max": (u32, [P]),
        "pmdfc_comm_id": (i32, [P]),
        "pmdfc_comm_create": (i32, [P, i32, i32, i32, C.POINTER(P)]),
        "pmdfc_comm_create_host": (i32, [i32, i32, i32, _XCHG, _AMAX, P, C.POINTER(P)]),
        "pmdfc_comm_destroy": (i32, [P]),
        "pmdfc_route_batches": (i32, [P, P, P, u32, P, P, P, u64, u32, P, P, P]),
        "pmdfc_route_mixed_batches": (i32, [P, P, P, P, P, P, P, u64, P, P, P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str):
    if rc != 0:
        msg = load_library().pmdfc_last_error()
        raise PmdfcError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def _require_gpu(device: int):
    if torch is None or not torch.cuda.is_available():
        raise PmdfcError("pmdfc_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    if device >= torch.cuda.device_count():
        raise PmdfcError(f"device {device} not present")


def depth_for_hybrid(init_cap: int) -> int:
    """CCEH_hybrid(initCap) -> floor(log2(initCap)) (CCEH_hybrid.cpp:80)."""
    return load_library().pmdfc_depth_for_hybrid(init_cap)


def depth_for_src(init_cap: int) -> int:
    """src/cceh.cpp CCEH(initCap) -> floor(log2(initCap/1024)) (src/cceh.cpp:82)."""
    return load_library().pmdfc_depth_for_src(init_cap)


class _Dev:
    """Move batch arguments to the device; remember which outputs to copy back."""

    def __init__(self, device: int):
        self.device = torch.device("cuda", device)

    def u64(self, x):
        if isinstance(x, torch.Tensor):
            if x.device != self.device or x.dtype not in (torch.int64, torch.uint64):
                raise PmdfcError("device tensors must be int64/uint64 on the engine's device")
            return x.contiguous()
        a = np.ascontiguousarray(x, dtype=np.uint64)
        return torch.from_numpy(a.view(np.int64)).to(self.device)

    def u8(self, x):
        if isinstance(x, torch.Tensor):
            return x.to(self.device, torch.uint8).contiguous()
        return torch.from_numpy(np.ascontiguousarray(x, dtype=np.uint8)).to(self.device)

    def stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)


def _host_out(t: torch.Tensor, kind: str):
    a = t.cpu().numpy()
    return a.view(np.uint64) if kind == "u64" else a


class CCEH:
    """Batched CCEH index on one GPU (one shard of the key space).

    Parameters mirror the reference constructors: give `init_cap` with
    `convention="hybrid"` for CCEH_hybrid(initCap) or `"src"` for src/cceh.cpp's
    CCEH(initCap); or give the initial global `depth` directly.
    `upsert=True` selects last-writer-wins Insert (the reference's Insert with
    its commented-out overwrite clause, CCEH_hybrid.cpp:153, enabled): an
    Insert of a stored key overwrites its value in place (ST_UPDATED).
    """

    def __init__(self, init_cap: int | None = None, *, depth: int | None = None,
                 convention: str = "hybrid", shard_bits: int = 0, shard_id: int = 0,
                 max_batch: int = 1 << 20, max_segments: int = 0, device: int = 0,
                 upsert: bool = False):
        L = load_library()
        _require_gpu(device)
        if depth is None:
            if init_cap is None:
                raise ValueError("give init_cap or depth")
            depth = depth_for_hybrid(init_cap) if convention == "hybrid" else depth_for_src(init_cap)
        cfg = Config(initial_depth=depth, shard_bits=shard_bits, shard_id=shard_id,
                     max_batch=max_batch, max_segments=max_segments, device=device,
                     flags=CFG_UPSERT if upsert else 0)
        h = C.c_void_p()
        _check(L.pmdfc_cceh_create(C.byref(cfg), C.byref(h)), "pmdfc_cceh_create")
        self._h = h
        self.device = device
        self.initial_depth = depth
        self.shard_bits = shard_bits
        self.shard_id = shard_id
        self.max_batch = max_batch
        self.convention = convention
        self.upsert = upsert
        self._d = _Dev(device)

    def close(self):
        if getattr(self, "_h", None):
            load_library().pmdfc_cceh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---- extents (CCEH_hybrid.cpp:90-105,330-341; src/cceh.cpp:308-330,381-391)
    def Insert_extent(self, keys, lens, values, clusters=None, convention: str | None = None) -> int:
        """Insert_extent for a batch of extents, in batch order.  hybrid:
        (key, value, len); src: (key, cluster, len, value).  Returns the number
        of index entries (sub-extent heads) inserted."""
        conv = 1 if (convention or self.convention) == "src" else 0
        k, ln, v = self._d.u64(keys), self._d.u64(lens), self._d.u64(values)
        c = self._d.u64(clusters) if clusters is not None else None
        ne = C.c_uint64(0)
        _check(load_library().pmdfc_cceh_insert_extent(self._h, conv, k.data_ptr(), c.data_ptr() if c is not None else None,
                                                       ln.data_ptr(), v.data_ptr(), k.numel(), C.byref(ne),
                                                       self._d.stream()), "pmdfc_cceh_insert_extent")
        return ne.value

    def Get_extent(self, keys, clusters=None, convention: str | None = None):
        """Get_extent for a batch: (values, status), NONE/ST_MISS when absent."""
        dev_in = isinstance(keys, torch.Tensor)
        conv = 1 if (convention or self.convention) == "src" else 0
        k = self._d.u64(keys)
        c = self._d.u64(clusters) if clusters is not None else None
        out = torch.empty(k.numel(), dtype=torch.int64, device=self._d.device)
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        _check(load_library().pmdfc_cceh_get_extent(self._h, conv, k.data_ptr(), c.data_ptr() if c is not None else None,
                                                    out.data_ptr(), st.data_ptr(), k.numel(), self._d.stream()),
               "pmdfc_cceh_get_extent")
        if dev_in:
            return out, st
        return _host_out(out, "u64"), _host_out(st, "u8")

    # ---- batched IHash operations ------------------------------------
    def Insert(self, keys, values):
        """IHash::Insert for a batch, applied in batch order.  Returns per-op
        status (ST_INSERTED, ...).  Torch inputs -> torch output (async)."""
        dev_in = isinstance(keys, torch.Tensor)
        k, v = self._d.u64(keys), self._d.u64(values)
        if k.numel() != v.numel():
            raise ValueError("keys/values length mismatch")
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        if k.numel() <= self.max_batch:
            if k.numel():
                _check(load_library().pmdfc_cceh_insert(self._h, k.data_ptr(), v.data_ptr(), st.data_ptr(),
                                                        k.numel(), self._d.stream()), "pmdfc_cceh_insert")
        else:  # consecutive max_batch batches, pipelined (pmdfc_cceh_insert_batches)
            self._insert_batches(k, v, st, list(range(0, k.numel(), self.max_batch)) + [k.numel()])
        return st if dev_in else _host_out(st, "u8")

    def InsertBatches(self, keys, values, bounds):
        """Insert batches [bounds[i], bounds[i+1]) in order: the same as one
        Insert per batch, with batch i+1 partitioned while batch i is applied."""
        dev_in = isinstance(keys, torch.Tensor)
        k, v = self._d.u64(keys), self._d.u64(values)
        if k.numel() != v.numel() or bounds[0] != 0 or bounds[-1] != k.numel():
            raise ValueError("keys/values/bounds mismatch")
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        self._insert_batches(k, v, st, list(bounds))
        return st if dev_in else _host_out(st, "u8")

    def _insert_batches(self, k, v, st, bounds):
        b = (C.c_uint64 * len(bounds))(*bounds)
        _check(load_library().pmdfc_cceh_insert_batches(self._h, k.data_ptr(), v.data_ptr(), st.data_ptr(), b,
                                                        len(bounds) - 1, self._d.stream()),
               "pmdfc_cceh_insert_batches")

    def Get(self, keys):
        """IHash::Get for a batch.  Returns (values, status); value 0 and
        ST_MISS on a miss (the reference returns NONE = 0)."""
        dev_in = isinstance(keys, torch.Tensor)
        k = self._d.u64(keys)
        out = torch.empty(k.numel(), dtype=torch.int64, device=self._d.device)
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        for off in range(0, k.numel(), self.max_batch):
            m = min(self.max_batch, k.numel() - off)
            _check(load_library().pmdfc_cceh_get(self._h, k[off:].data_ptr(), out[off:].data_ptr(),
                                                 st[off:].data_ptr(), m, self._d.stream()),
                   "pmdfc_cceh_get")
        if dev_in:
            return out, st
        return _host_out(out, "u64"), _host_out(st, "u8")

    def GetBatches(self, keys, bounds):
        """Get batches [bounds[i], bounds[i+1]): the same as one Get per batch,
        as one launch over their union (pmdfc_cceh_get_batches)."""
        dev_in = isinstance(keys, torch.Tensor)
        k = self._d.u64(keys)
        if bounds[0] != 0 or bounds[-1] != k.numel():
            raise ValueError("keys/bounds mismatch")
        out = torch.empty(k.numel(), dtype=torch.int64, device=self._d.device)
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        b = (C.c_uint64 * len(bounds))(*bounds)
        _check(load_library().pmdfc_cceh_get_batches(self._h, k.data_ptr(), out.data_ptr(), st.data_ptr(), b,
                                                     len(bounds) - 1, self._d.stream()),
               "pmdfc_cceh_get_batches")
        if dev_in:
            return out, st
        return _host_out(out, "u64"), _host_out(st, "u8")

    def FindAnyway(self, keys):
        """CCEH::FindAnyway (CCEH_hybrid.cpp:482-496) for a batch: the first
        copy of each key in directory order, then slot order 0..1023 (not
        Get's probe order).  Returns (values, status) like Get."""
        dev_in = isinstance(keys, torch.Tensor)
        k = self._d.u64(keys)
        out = torch.empty(k.numel(), dtype=torch.int64, device=self._d.device)
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        if k.numel():
            _check(load_library().pmdfc_cceh_find_anyway(self._h, k.data_ptr(), out.data_ptr(), st.data_ptr(),
                                                         k.numel(), self._d.stream()), "pmdfc_cceh_find_anyway")
        if dev_in:
            return out, st
        return _host_out(out, "u64"), _host_out(st, "u8")

    def InsertRecords(self, records: torch.Tensor) -> torch.Tensor:
        """Insert of n interleaved {key, value} records (a [2n] int64 device
        tensor, e.g. rows received from a routed exchange) -> status [n]."""
        r = records.contiguous()
        if r.device != self._d.device or r.dtype not in (torch.int64, torch.uint64) or r.numel() % 2:
            raise PmdfcError("records: int64 device tensor of 2n words on the engine's device")
        n = r.numel() // 2
        st = torch.empty(n, dtype=torch.uint8, device=self._d.device)
        if n > self.max_batch:
            raise PmdfcError(f"InsertRecords: n {n} > max_batch {self.max_batch}")
        _check(load_library().pmdfc_cceh_insert_records(self._h, r.data_ptr(), st.data_ptr(), n,
                                                         self._d.stream()), "pmdfc_cceh_insert_records")
        return st

    def GetRecords(self, keys: torch.Tensor) -> torch.Tensor:
        """Get of n device keys -> [2n] int64 {value, status} response records."""
        k = self._d.u64(keys)
        resp = torch.empty(2 * k.numel(), dtype=torch.int64, device=self._d.device)
        for off in range(0, k.numel(), self.max_batch):
            m = min(self.max_batch, k.numel() - off)
            _check(load_library().pmdfc_cceh_get_records(self._h, k[off:].data_ptr(), resp[2 * off:].data_ptr(), m,
                                                         self._d.stream()), "pmdfc_cceh_get_records")
        return resp

    def Mixed(self, ops, keys, values):
        """Interleaved Insert/Get batch (op 1 = Insert, 0 = Get) in batch
        order.  Returns (get_values, status)."""
        dev_in = isinstance(keys, torch.Tensor)
        o, k, v = self._d.u8(ops), self._d.u64(keys), self._d.u64(values)
        out = torch.empty(k.numel(), dtype=torch.int64, device=self._d.device)
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        if k.numel() <= self.max_batch:
            _check(load_library().pmdfc_cceh_mixed(self._h, o.data_ptr(), k.data_ptr(), v.data_ptr(),
                                                   out.data_ptr(), st.data_ptr(), k.numel(), self._d.stream()),
                   "pmdfc_cceh_mixed")
        else:  # consecutive max_batch batches (pmdfc_cceh_mixed_batches)
            self._mixed_batches(o, k, v, out, st, list(range(0, k.numel(), self.max_batch)) + [k.numel()])
        if dev_in:
            return out, st
        return _host_out(out, "u64"), _host_out(st, "u8")

    def MixedBatches(self, ops, keys, values, bounds):
        """Mixed batches [bounds[i], bounds[i+1]) in order: the same as one
        Mixed per batch, in one call (pmdfc_cceh_mixed_batches)."""
        dev_in = isinstance(keys, torch.Tensor)
        o, k, v = self._d.u8(ops), self._d.u64(keys), self._d.u64(values)
        if not (o.numel() == k.numel() == v.numel()) or bounds[0] != 0 or bounds[-1] != k.numel():
            raise ValueError("ops/keys/values/bounds mismatch")
        out = torch.empty(k.numel(), dtype=torch.int64, device=self._d.device)
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        self._mixed_batches(o, k, v, out, st, list(bounds))
        if dev_in:
            return out, st
        return _host_out(out, "u64"), _host_out(st, "u8")

    def _mixed_batches(self, o, k, v, out, st, bounds):
        b = (C.c_uint64 * len(bounds))(*bounds)
        _check(load_library().pmdfc_cceh_mixed_batches(self._h, o.data_ptr(), k.data_ptr(), v.data_ptr(),
                                                       out.data_ptr(), st.data_ptr(), b, len(bounds) - 1,
                                                       self._d.stream()),
               "pmdfc_cceh_mixed_batches")

    def Delete(self, keys):
        """CCEH::Delete is an unimplemented stub returning false
        (CCEH_hybrid.cpp:322-324); kept for interface parity."""
        n = len(keys)
        return np.zeros(n, dtype=bool)

    def Recovery(self) -> bool:
        """CCEH::Recovery (CCEH_hybrid.cpp:391-410) repairs directory entries of
        a crashed PMEM image; the device index is volatile, nothing to repair."""
        return False

    def Utilization(self) -> float:
        r = C.c_double()
        _check(load_library().pmdfc_cceh_utilization(self._h, C.byref(r)), "utilization")
        return r.value

    def Capacity(self) -> int:
        return self.stats()["capacity"]

    # ---- introspection -------------------------------------------------
    def stats(self) -> dict:
        s = Stats()
        _check(load_library().pmdfc_cceh_stats(self._h, C.byref(s)), "stats")
        return {n: getattr(s, n) for n, _ in Stats._fields_}

    def reset(self):
        _check(load_library().pmdfc_cceh_reset(self._h, self._d.stream()), "reset")

    def dump(self) -> dict:
        """Canonical dump (segments in directory order), like oracle.dump()."""
        L = load_library()
        n = C.c_uint64()
        _check(L.pmdfc_cceh_dump(self._h, None, None, None, None, None, C.byref(n)), "dump")
        st = self.stats()
        d = st["depth"]
        nseg = n.value
        dir_canon = np.empty(1 << (d - self.shard_bits), np.uint32)
        ld = np.empty(nseg, np.uint32)
        prefix = np.empty(nseg, np.uint64)
        keys = np.empty(nseg * 1024, np.uint64)
        vals = np.empty(nseg * 1024, np.uint64)
        _check(L.pmdfc_cceh_dump(self._h, dir_canon.ctypes.data, ld.ctypes.data, prefix.ctypes.data,
                                 keys.ctypes.data, vals.ctypes.data, C.byref(n)), "dump")
        return {"depth": d, "dir_canon": dir_canon, "local_depth": ld, "prefix": prefix,
                "keys": keys, "values": vals}

    def timing(self, events: bool = True, count_lines: bool = False):
        flags = (1 if events else 0) | (2 if count_lines else 0)
        _check(load_library().pmdfc_cceh_timing_enable(self._h, flags), "timing_enable")

    def timing_read(self, reset: bool = True) -> dict:
        ms = (C.c_double * len(K_NAMES))()
        cnt = (C.c_uint64 * len(K_NAMES))()
        _check(load_library().pmdfc_cceh_timing_read(self._h, ms, cnt, int(reset)), "timing_read")
        return {K_NAMES[i]: (ms[i], cnt[i]) for i in range(len(K_NAMES))}

    def last_get_lines(self) -> int:
        r = C.c_uint64()
        _check(load_library().pmdfc_cceh_last_get_lines(self._h, C.byref(r)), "last_get_lines")
        return r.value

    def debug_stamps(self, max_batch: int):
        """Phase stamps (100 MHz wall clock) of the last insert/mixed batch:
        (bucket [2^p1, 16], partition [blocks, 8], split [8192, 8]) -- needs
        PMDFC_STAMPS=1."""
        nblk = (max_batch + 8191) // 8192  # (kPartTile)
        nb = C.c_uint32()
        buf = np.zeros(16 * 16384 + 8 * nblk + 8 * 8192, np.uint64)
        _check(load_library().pmdfc_cceh_debug_stamps(self._h, buf.ctypes.data, buf.size, C.byref(nb)),
               "debug_stamps")
        n = nb.value
        o = 16 * n + 8 * nblk
        return (buf[: 16 * n].reshape(n, 16), buf[16 * n: o].reshape(nblk, 8),
                buf[o: o + 8 * 8192].reshape(8192, 8))


class BloomFilter:
    """client/bloom_filter.c as a device bitmap (MSB-first u64 words)."""

    def __init__(self, nbits: int = 1000000000, k: int = 4, device: int = 0):
        L = load_library()
        _require_gpu(device)
        h = C.c_void_p()
        _check(L.pmdfc_bloom_create(nbits, k, device, C.byref(h)), "pmdfc_bloom_create")
        self._h = h
        self.nbits, self.k, self.device = nbits, k, device
        self._d = _Dev(device)

    def close(self):
        if getattr(self, "_h", None):
            load_library().pmdfc_bloom_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, keys):
        k = self._d.u64(keys)
        _check(load_library().pmdfc_bloom_add(self._h, k.data_ptr(), k.numel(), self._d.stream()), "bloom_add")

    def probe(self, keys):
        dev_in = isinstance(keys, torch.Tensor)
        k = self._d.u64(keys)
        out = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        _check(load_library().pmdfc_bloom_probe(self._h, k.data_ptr(), out.data_ptr(), k.numel(),
                                                self._d.stream()), "bloom_probe")
        return out if dev_in else _host_out(out, "u8")

    def bitmap(self) -> np.ndarray:
        """The MSB-first u64 bitmap (what rdma_svr.cpp:157-251 ships)."""
        n = (self.nbits + 63) // 64
        out = np.empty(n, np.uint64)
        _check(load_library().pmdfc_bloom_get_bitmap_host(self._h, out.ctypes.data, n), "bloom_bitmap")
        return out

    def set_bitmap(self, words: np.ndarray):
        """bloom_filter_set (client/bloom_filter.c:119-124)."""
        w = np.ascontiguousarray(words, dtype=np.uint64)
        _check(load_library().pmdfc_bloom_set_bitmap_host(self._h, w.ctypes.data, w.size), "bloom_set")

    def probe_then_get(self, index: CCEH, keys):
        """Fused client path: bloom-negative -> ST_FILTERED, else index Get."""
        dev_in = isinstance(keys, torch.Tensor)
        k = self._d.u64(keys)
        out = torch.empty(k.numel(), dtype=torch.int64, device=self._d.device)
        st = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        _check(load_library().pmdfc_bloom_probe_then_get(self._h, index.handle, k.data_ptr(),
                                                         out.data_ptr(), st.data_ptr(), k.numel(),
                                                         self._d.stream()), "bloom_probe_then_get")
        if dev_in:
            return out, st
        return _host_out(out, "u64"), _host_out(st, "u8")


class CountingBloomFilter:
    """The server's CountingBloomFilter<Key_t> (server/util/counting_bloom_filter.h)
    on the GPU: u8 counters + the packed MSB-first bitmap.  Method names follow
    the reference (Insert/Delete/Query/QueryBitBloom/ToOrdinaryBloomFilter);
    each call takes a batch and equals the reference applied key by key."""

    def __init__(self, numHashes: int = 4, numBits: int = 1000000000, device: int = 0):
        L = load_library()
        _require_gpu(device)
        h = C.c_void_p()
        _check(L.pmdfc_cbf_create(numBits, numHashes, device, C.byref(h)), "pmdfc_cbf_create")
        self._h = h
        self.k, self.nbits, self.device = numHashes, numBits, device
        self._d = _Dev(device)

    def close(self):
        if getattr(self, "_h", None):
            load_library().pmdfc_cbf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def Insert(self, keys):
        k = self._d.u64(keys)
        _check(load_library().pmdfc_cbf_insert(self._h, k.data_ptr(), k.numel(), self._d.stream()), "cbf_insert")

    def InsertOps(self, ops, keys):
        """Count only the Insert ops of a mixed batch (KV::Insert, server/KV.cpp:113-114)."""
        k, o = self._d.u64(keys), self._d.u8(ops)
        _check(load_library().pmdfc_cbf_insert_ops(self._h, o.data_ptr(), k.data_ptr(), k.numel(),
                                                   self._d.stream()), "cbf_insert_ops")

    def _u8_call(self, fn, keys, what):
        dev_in = isinstance(keys, torch.Tensor)
        k = self._d.u64(keys)
        out = torch.empty(k.numel(), dtype=torch.uint8, device=self._d.device)
        _check(fn(self._h, k.data_ptr(), out.data_ptr(), k.numel(), self._d.stream()), what)
        return out if dev_in else _host_out(out, "u8")

    def Delete(self, keys):
        """Deleted flags (Query at the key's turn in batch order)."""
        return self._u8_call(load_library().pmdfc_cbf_delete, keys, "cbf_delete")

    def Query(self, keys):
        return self._u8_call(load_library().pmdfc_cbf_query, keys, "cbf_query")

    def QueryBitBloom(self, keys):
        return self._u8_call(load_library().pmdfc_cbf_query_bits, keys, "cbf_query_bits")

    def ToOrdinaryBloomFilter(self):
        _check(load_library().pmdfc_cbf_pack(self._h, self._d.stream()), "cbf_pack")

    def export(self, bloom: "BloomFilter"):
        """send_bf (rdma_svr.cpp:157-251) to a client filter on the same GPU."""
        _check(load_library().pmdfc_cbf_export(self._h, bloom._h, self._d.stream()), "cbf_export")

    def Clear(self):
        _check(load_library().pmdfc_cbf_clear(self._h, self._d.stream()), "cbf_clear")

    def counters(self) -> np.ndarray:
        out = np.empty(self.nbits, np.uint8)
        _check(load_library().pmdfc_cbf_get_counters_host(self._h, out.ctypes.data, self.nbits), "cbf_counters")
        return out

    def bitmap(self) -> np.ndarray:
        n = (self.nbits + 63) // 64
        out = np.empty(n, np.uint64)
        _check(load_library().pmdfc_cbf_get_bitmap_host(self._h, out.ctypes.data, n), "cbf_bitmap")
        return out


class TraceReader:
    """replay_KV trace ingestion on the GPU (server/replay_KV.cpp:209-247):
    text lines 'seq ts OP inode inode_size offset size' -> the first
    num_data (op, key) of the reference's page expansion, as device tensors
    (op PMDFC_OP_INSERT for 'W' pages, PMDFC_OP_GET for 'R' pages)."""

    def __init__(self, device: int = 0):
        L = load_library()
        _require_gpu(device)
        h = C.c_void_p()
        _check(L.pmdfc_trace_create(device, C.byref(h)), "pmdfc_trace_create")
        self._h = h
        self._d = _Dev(device)

    def close(self):
        if getattr(self, "_h", None):
            load_library().pmdfc_trace_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def parse(self, text, num_data: int):
        """text: bytes, a numpy u8 array or a device u8 tensor.  Returns
        (ops u8, keys int64 bit-pattern u64, info dict)."""
        if isinstance(text, torch.Tensor):
            t = text.to(self._d.device, torch.uint8).contiguous()
        else:
            a = np.frombuffer(text, np.uint8) if isinstance(text, (bytes, bytearray)) else np.asarray(text, np.uint8)
            t = torch.from_numpy(a.copy()).to(self._d.device)
        ops = torch.empty(max(num_data, 1), dtype=torch.uint8, device=self._d.device)
        keys = torch.empty(max(num_data, 1), dtype=torch.int64, device=self._d.device)
        info = (C.c_uint64 * 5)()
        _check(load_library().pmdfc_trace_parse(self._h, t.data_ptr(), t.numel(), num_data, ops.data_ptr(),
                                                keys.data_ptr(), info, self._d.stream()), "trace_parse")
        names = ("ops", "lines", "trace_ops", "stop_line", "first_bad_line")
        return ops[:num_data], keys[:num_data], dict(zip(names, [int(x) for x in info]))


def replay(index: "CCEH", ops: torch.Tensor, keys: torch.Tensor, batch: int | None = None) -> dict:
    """replay_KV's run (server/replay_KV.cpp:262-275) in trace order: 'W'
    pages Insert(key, value=key), 'R' pages Get(key) and count a failed
    search when the value is not the key.  Batches of index.max_batch."""
    batch = batch or index.max_batch
    failed = torch.zeros((), dtype=torch.int64, device=keys.device)
    for a in range(0, keys.numel(), batch):
        o, k = ops[a:a + batch], keys[a:a + batch]
        v, _ = index.Mixed(o, k, k)
        failed += ((o == OP_GET) & (v != k)).sum()
    puts = int((ops == OP_INSERT).sum())
    return {"failedSearch": int(failed), "put": puts, "get": int(ops.numel()) - puts}


def hash64(keys):
    """h() of every key on the GPU (std::_Hash_bytes, seed 0xc70697)."""
    d = _Dev(keys.device.index or 0) if isinstance(keys, torch.Tensor) else _Dev(0)
    k = d.u64(keys)
    out = torch.empty_like(k)
    _check(load_library().pmdfc_hash64(k.data_ptr(), out.data_ptr(), k.numel(), d.stream()), "hash64")
    return out if isinstance(keys, torch.Tensor) else _host_out(out, "u64")


def gen_keys(seed: int, start: int, n: int, device: int = 0):
    """Device splitmix64 key stream == workload.uniform_keys(seed, start, n)."""
    d = _Dev(device)
    out = torch.empty(n, dtype=torch.int64, device=d.device)
    _check(load_library().pmdfc_gen_keys(seed, start, out.data_ptr(), n, d.stream()), "gen_keys")
    return out


def route_by_shard(keys: torch.Tensor, shard_bits: int):
    """Stable grouping of a device key batch by owner shard (top shard_bits of
    h()).  Returns (perm int32 device tensor, counts list)."""
    d = _Dev(keys.device.index or 0)
    n = keys.numel()
    perm = torch.empty(n, dtype=torch.int32, device=d.device)
    counts = (C.c_uint64 * (1 << shard_bits))()
    _check(load_library().pmdfc_route_by_shard(keys.data_ptr(), n, shard_bits, perm.data_ptr(), counts,
                                               d.device.index, d.stream()), "route_by_shard")
    return perm, [int(c) for c in counts]


def route_capacity(max_batch: int, shard_bits: int, slack: float = 1 / 16) -> int:
    """Record slots per owner block for batches of up to max_batch ops: the
    mean share plus `slack` of it plus 1024, a multiple of 256.  Uniform
    hashing puts an owner's count within a few sqrt(mean) of the mean, so the
    default is tens of standard deviations above it at 1M-op batches."""
    G = 1 << shard_bits
    mean = -(-max_batch // G)
    if shard_bits == 0:
        return max(256, -(-max_batch // 256) * 256)
    return -(-(int(mean * (1 + slack)) + 1024) // 256) * 256


class BlockPacker:
    """Device side of the fixed-capacity routing protocol (route.hip through
    the C-ABI pmdfc_router_*): one router handle with its per-owner FIFO
    carry, sized once for batches of max_batch ops, reused batch after batch
    on the current stream.  pmdfc_amd.dist.BlockRouter drives it; the CPU
    restatement tests/route_ref.py has the same methods."""

    def __init__(self, device: int, max_batch: int, shard_bits: int, cap: int | None = None,
                 carry_cap: int | None = None):
        _require_gpu(device)
        self._d = _Dev(device)
        self.sbits = shard_bits
        self.G = 1 << shard_bits
        self.max_batch = max_batch
        self.cap = cap or route_capacity(max_batch, shard_bits)
        self.carry_cap = carry_cap or max_batch
        self.rows = self.G * self.cap
        cfg = RouterConfig(shard_bits, max_batch, self.cap, self.carry_cap, device, 0)
        h = C.c_void_p()
        _check(load_library().pmdfc_router_create(C.byref(cfg), C.byref(h)), "pmdfc_router_create")
        self._h = h
        self.keys = torch.empty(self.rows, dtype=torch.int64, device=self._d.device)
        self.vals = torch.empty(self.rows, dtype=torch.int64, device=self._d.device)
        self.ops = torch.empty(self.rows, dtype=torch.uint8, device=self._d.device)

    def close(self):
        if getattr(self, "_h", None):
            load_library().pmdfc_router_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _ptr(t):
        return t.data_ptr() if t is not None else None

    def pack(self, keys, vals, ops, width: int, keep=None, base: int = 0, vals_out=None, st_out=None):
        """Pack this batch (ops base .. base + n - 1 of the call's outputs)
        behind the carried ops -> (send [rows * width] int64, rowpos [rows]
        int32), fresh tensors (an async all-to-all may still read the previous
        batch's).  keys None: a drain pack (n = 0).  Ops kept home (keep == 0)
        or dropped on a full carry get their status (ST_FILTERED /
        ST_ROUTE_OVERFLOW) in st_out right away."""
        n = 0 if keys is None else keys.numel()
        if n > self.max_batch:
            raise PmdfcError(f"routed batch of {n} > max_batch {self.max_batch}")
        if n and st_out is None:
            raise PmdfcError("pack: st_out (the call's status output) is required")
        dev = self._d.device
        send = torch.empty(self.rows * width, dtype=torch.int64, device=dev)
        rowpos = torch.empty(self.rows, dtype=torch.int32, device=dev)
        kp = keep.to(dev, torch.uint8).contiguous() if keep is not None else None
        _check(load_library().pmdfc_router_pack(
            self._h, self._ptr(keys), self._ptr(vals) if width > 1 else None, self._ptr(ops) if width > 2 else None,
            self._ptr(kp), n, width, base, send.data_ptr(), rowpos.data_ptr(), self._ptr(vals_out),
            self._ptr(st_out), self._d.stream()), "pmdfc_router_pack")
        return send, rowpos

    def unpack(self, back, resp_width: int, rowpos, vals_out, st_out):
        """returned response rows -> the call's outputs (scatter by rowpos)"""
        _check(load_library().pmdfc_router_unpack(self._h, back.data_ptr(), resp_width, rowpos.data_ptr(),
                                                  self._ptr(vals_out), st_out.data_ptr(), self._d.stream()),
               "pmdfc_router_unpack")

    def carried(self) -> torch.Tensor:
        """ops waiting in the carry after the last pack: int64 [1] device tensor (no sync)"""
        out = torch.empty(1, dtype=torch.int64, device=self._d.device)
        _check(load_library().pmdfc_router_carried(self._h, out.data_ptr(), self._d.stream()), "pmdfc_router_carried")
        return out

    def end_call(self):
        _check(load_library().pmdfc_router_end_call(self._h), "pmdfc_router_end_call")

    def overflow_count(self) -> int:
        """ops dropped on a full carry since create / reset (synchronises)"""
        v = C.c_uint64()
        _check(load_library().pmdfc_router_overflow_count(self._h, C.byref(v), self._d.stream()),
               "pmdfc_router_overflow_count")
        return v.value

    def reset(self):
        _check(load_library().pmdfc_router_reset(self._h, self._d.stream()), "pmdfc_router_reset")

    def dedupe(self, keys, keep=None, base: int = 0, lead_out=None):
        """Get batch: keep mask of the first Get of every key (and keep);
        lead_out[base + i] = base + that first Get's index."""
        n = keys.numel()
        if n > self.max_batch:
            raise PmdfcError(f"routed batch of {n} > max_batch {self.max_batch}")
        dev = self._d.device
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        kp = keep.to(dev, torch.uint8).contiguous() if keep is not None else None
        _check(load_library().pmdfc_router_dedupe(self._h, keys.data_ptr(), self._ptr(kp), n, base, out.data_ptr(),
                                                  lead_out.data_ptr(), self._d.stream()), "pmdfc_router_dedupe")
        return out

    def fill(self, lead, vals_out, st_out):
        """followers take their leader's result"""
        _check(load_library().pmdfc_router_fill(lead.data_ptr(), lead.numel(), self._ptr(vals_out), st_out.data_ptr(),
                                                self._d.device.index, self._d.stream()), "pmdfc_router_fill")

    def route_batches(self, index, comm, width: int, keys, values, bounds, dedupe: bool, vals_out, st_out):
        """The whole routed call in C++ (pmdfc_route_batches): the same packs,
        exchanges (RCCL, the communicator's stream), carries and drains as
        BlockRouter's Python loop, so the same results."""
        nb = len(bounds) - 1
        b = (C.c_uint64 * len(bounds))(*bounds)
        _check(load_library().pmdfc_route_batches(
            self._h, index.handle, comm.handle, width, keys.data_ptr(), self._ptr(values) if width > 1 else None,
            b, nb, 1 if dedupe else 0, self._ptr(vals_out), st_out.data_ptr(), self._d.stream()),
            "pmdfc_route_batches")

    def route_mixed_batches(self, index, comm, ops, keys, values, bounds, vals_out, st_out):
        """Routed mixed batches in C++ (pmdfc_route_mixed_batches), the same
        packs, exchanges and drains as BlockRouter.mixed_batches."""
        nb = len(bounds) - 1
        b = (C.c_uint64 * len(bounds))(*bounds)
        _check(load_library().pmdfc_route_mixed_batches(
            self._h, index.handle, comm.handle, ops.data_ptr(), keys.data_ptr(), values.data_ptr(), b, nb,
            vals_out.data_ptr(), st_out.data_ptr(), self._d.stream()), "pmdfc_route_mixed_batches")

    def split(self, recv, width: int):
        """received rows -> (keys, values | None, ops | None), rows each"""
        _check(load_library().pmdfc_route_split(recv.data_ptr(), self.rows, width, self.keys.data_ptr(),
                                                self.vals.data_ptr(), self.ops.data_ptr(),
                                                self._d.device.index, self._d.stream()), "pmdfc_route_split")
        return self.keys, (self.vals if width > 1 else None), (self.ops if width > 2 else None)

    def respond(self, vals, st):
        """engine (value, status) rows -> [rows * 2] int64 response records (fresh)"""
        resp = torch.empty(self.rows * 2, dtype=torch.int64, device=self._d.device)
        _check(load_library().pmdfc_route_respond(vals.data_ptr(), st.data_ptr(), self.rows, resp.data_ptr(),
                                                  self._d.device.index, self._d.stream()), "pmdfc_route_respond")
        return resp


class Comm:
    """An RCCL communicator of the engine's own (pmdfc_comm_*), for
    pmdfc_route_batches: one rank per GPU, the id made by rank 0 and
    broadcast through the torch.distributed group (any backend), or a
    one-rank communicator without a group."""

    def __init__(self, device: int, group=None, host_staged: bool = False):
        """host_staged: exchanges through the torch.distributed group on host
        copies (pmdfc_comm_create_host; any backend, e.g. gloo with two ranks
        on one GPU) instead of an RCCL communicator -- the same routed loop
        and protocol, only the transport differs."""
        _require_gpu(device)
        import torch.distributed as dist
        L = load_library()
        init = dist.is_available() and dist.is_initialized()
        world = dist.get_world_size(group) if init else 1
        rank = dist.get_rank(group) if init else 0
        if host_staged:
            self._fns = self._host_transport(dist, group, world)
            h = C.c_void_p()
            _check(L.pmdfc_comm_create_host(world, rank, device, self._fns[0], self._fns[1], None, C.byref(h)),
                   "pmdfc_comm_create_host")
            self._h = h
            self.world, self.rank, self.device = world, rank, device
            self.exchanges = 0
            return
        idb = (C.c_uint8 * 128)()
        if rank == 0:
            _check(L.pmdfc_comm_id(idb), "pmdfc_comm_id")
        if world > 1:
            t = torch.tensor(list(idb), dtype=torch.uint8)
            if dist.get_backend(group) != "gloo":
                t = t.to(torch.device("cuda", device))
            dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
            idb = (C.c_uint8 * 128)(*t.cpu().tolist())
        h = C.c_void_p()
        _check(L.pmdfc_comm_create(idb, world, rank, device, C.byref(h)), "pmdfc_comm_create")
        self._h = h
        self.world, self.rank, self.device = world, rank, device

    def _host_transport(self, dist, group, world):
        def xchg(ctx, send, recv, nbytes):
            try:
                tot = nbytes * world
                s = np.ctypeslib.as_array((C.c_uint8 * tot).from_address(send))
                r = np.ctypeslib.as_array((C.c_uint8 * tot).from_address(recv))
                out = torch.empty(tot, dtype=torch.uint8)
                dist.all_to_all_single(out, torch.from_numpy(s.copy()), group=group)
                r[:] = out.numpy()
                self.exchanges += 1
                return 0
            except Exception:  # pragma: no cover - reported as the call's error
                return 1

        def amax(ctx, v):
            try:
                t = torch.tensor([int(v[0])], dtype=torch.int64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
                v[0] = int(t.item())
                return 0
            except Exception:  # pragma: no cover
                return 1

        return _XCHG(xchg), _AMAX(amax)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            load_library().pmdfc_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ubench_gather(buf: torch.Tensor, n_ops: int, line: int, depth: int, table: torch.Tensor | None = None,
                  seed: int = 1, out: torch.Tensor | None = None):
    """Random-line gather ceiling at scale (pmdfc_ubench_gather): n_ops lines
    of `line` bytes (64/128), `depth` (1/2/4) lines in flight per lane group."""
    d = _Dev(buf.device.index or 0)
    if out is None:
        out = torch.empty(1 << 20, dtype=torch.int64, device=d.device)
    tp = table.data_ptr() if table is not None else None
    tm = (table.numel() - 1) if table is not None else 0
    _check(load_library().pmdfc_ubench_gather(buf.data_ptr(), buf.numel() * buf.element_size(), line, depth, tp, tm,
                                              n_ops, seed, out.data_ptr(), out.numel() - 1, d.stream()),
           "ubench_gather")
    return out


def ubench_scatter16(buf: torch.Tensor, n_ops: int, depth: int = 4, seed: int = 1):
    """Random 16-B store ceiling (pmdfc_ubench_scatter16): n_ops stores into
    random 16-B slots of buf, `depth` (1/4) per lane."""
    d = _Dev(buf.device.index or 0)
    _check(load_library().pmdfc_ubench_scatter16(buf.data_ptr(), buf.numel() * buf.element_size(), depth, n_ops, seed,
                                                 d.stream()), "ubench_scatter16")


def ubench_gather64(buf: torch.Tensor, n_ops: int, table: torch.Tensor | None = None, seed: int = 1,
                    out: torch.Tensor | None = None):
    """Random 64-B line gather ceiling (k_get's access shape); returns `out`."""
    d = _Dev(buf.device.index or 0)
    nlines = buf.numel() * buf.element_size() // 64
    if out is None:
        out = torch.empty(n_ops, dtype=torch.int64, device=d.device)
    tp = table.data_ptr() if table is not None else None
    tm = (table.numel() - 1) if table is not None else 0
    _check(load_library().pmdfc_ubench_gather64(buf.data_ptr(), nlines, tp, tm, n_ops, seed,
                                                out.data_ptr(), d.stream()), "ubench_gather64")
    return out
