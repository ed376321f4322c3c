"""ctypes binding for oracle/liboracle.so -- the CPU restatement of the
reference's serial CCEH_hybrid (see cceh_oracle.h).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product package pmdfc_amd never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

ST_MISS, ST_HIT, ST_INSERTED, ST_RESERVED_KEY, ST_UNSPLITTABLE, ST_DEPTH_LIMIT, ST_CAPACITY, ST_FILTERED = range(8)
ST_UPDATED = 11
OP_GET, OP_INSERT = 0, 1


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "splits", "doublings", "split_loss", "gets", "get_hits", "get_lines",
        "get_lines_full", "inserts", "insert_lines", "early_exit_mismatch")]


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "cceh_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return path


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = C.CDLL(build())
        L = _LIB
        P = C.c_void_p
        u64p = np.ctypeslib.ndpointer(np.uint64, flags="C")
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C")
        L.oc_hash64.restype = C.c_uint64
        L.oc_hash64.argtypes = [C.c_uint64]
        L.oc_murmur2.restype = C.c_uint32
        L.oc_murmur2.argtypes = [C.c_uint64, C.c_uint32]
        L.oc_hash64_batch.argtypes = [u64p, u64p, C.c_size_t]
        L.oc_murmur2_batch.argtypes = [u64p, C.c_uint32, u32p, C.c_size_t]
        L.oc_create.restype = P
        L.oc_create.argtypes = [C.c_uint32, C.c_size_t]
        L.oc_destroy.argtypes = [P]
        L.oc_set_upsert.argtypes = [P, C.c_int]
        L.oc_depth_for_hybrid.restype = C.c_uint32
        L.oc_depth_for_hybrid.argtypes = [C.c_uint64]
        L.oc_depth_for_src.restype = C.c_uint32
        L.oc_depth_for_src.argtypes = [C.c_uint64]
        L.oc_insert.restype = C.c_int
        L.oc_insert.argtypes = [P, C.c_uint64, C.c_uint64]
        L.oc_get.restype = C.c_int
        L.oc_get.argtypes = [P, C.c_uint64, C.POINTER(C.c_uint64)]
        L.oc_mixed.argtypes = [P, u8p, u64p, u64p, C.c_size_t, u64p, u8p]
        L.oc_insert_batch.argtypes = [P, u64p, u64p, C.c_size_t, u8p]
        L.oc_get_batch.argtypes = [P, u64p, C.c_size_t, u64p, u8p]
        L.oc_find_anyway_batch.argtypes = [P, u64p, C.c_size_t, u64p, u8p]
        L.oc_depth.restype = C.c_uint32
        L.oc_depth.argtypes = [P]
        L.oc_num_segments.restype = C.c_uint32
        L.oc_num_segments.argtypes = [P]
        L.oc_get_stats.argtypes = [P, C.POINTER(Stats)]
        L.oc_utilization.restype = C.c_double
        L.oc_utilization.argtypes = [P]
        L.oc_capacity.restype = C.c_uint64
        L.oc_capacity.argtypes = [P]
        L.oc_dump.argtypes = [P, u32p, u32p, u64p, u64p, u64p]
        L.oc_bloom_add_batch.argtypes = [u64p, C.c_uint64, C.c_uint32, u64p, C.c_size_t]
        L.oc_bloom_check_batch.argtypes = [u64p, C.c_uint64, C.c_uint32, u64p, C.c_size_t, u8p,
                                           C.POINTER(C.c_uint64)]
        L.oc_cbf_insert.argtypes = [u8p, C.c_uint64, C.c_uint32, C.c_uint64]
        L.oc_cbf_query.restype = C.c_int
        L.oc_cbf_query.argtypes = [u8p, C.c_uint64, C.c_uint32, C.c_uint64]
        L.oc_cbf_delete.restype = C.c_int
        L.oc_cbf_delete.argtypes = [u8p, C.c_uint64, C.c_uint32, C.c_uint64]
        L.oc_cbf_to_bitmap.argtypes = [u8p, C.c_uint64, u64p]
        L.oc_cbf_insert_batch.argtypes = [u8p, C.c_uint64, C.c_uint32, u64p, C.c_uint64]
        L.oc_cbf_delete_batch.argtypes = [u8p, C.c_uint64, C.c_uint32, u64p, C.c_uint64, u8p]
        L.oc_time_insert.restype = C.c_double
        L.oc_time_insert.argtypes = [P, u64p, C.c_size_t, C.c_int]
        L.oc_time_get.restype = C.c_double
        L.oc_time_get.argtypes = [P, u64p, C.c_size_t, C.c_int, C.POINTER(C.c_uint64)]
        L.oc_mt_bench.restype = C.c_int
        L.oc_mt_bench.argtypes = [C.c_uint32, u64p, C.c_size_t, C.c_int, P, C.c_int, C.POINTER(MtResult)]
    return _LIB


class MtResult(C.Structure):
    _fields_ = [("insert_s", C.c_double), ("get_s", C.c_double), ("failed", C.c_uint64),
                ("depth", C.c_uint32), ("segments", C.c_uint64)]


def mt_bench(initial_depth: int, keys, threads: int, cpus=None, flush_ns: int = 10) -> dict:
    """The concurrent CCEH_hybrid restatement (cceh_mt.c) under test_KV's
    harness: `threads` threads pinned to `cpus` (None: unpinned), insert
    (value = key) then Get.  Returns seconds per phase, failedSearch, and the
    final depth / segment count."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    r = MtResult()
    cp = None
    if cpus is not None:
        arr = (C.c_int * threads)(*[int(c) for c in cpus[:threads]])
        cp = C.cast(arr, C.c_void_p)
    rc = lib().oc_mt_bench(initial_depth, keys, keys.size, threads, cp, flush_ns, C.byref(r))
    if rc:
        raise ValueError("oc_mt_bench failed")
    return {n: getattr(r, n) for n, _ in MtResult._fields_}


def hash64(keys) -> np.ndarray:
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    out = np.empty_like(keys)
    lib().oc_hash64_batch(keys, out, keys.size)
    return out


def murmur2(keys, seed: int) -> np.ndarray:
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    out = np.empty(keys.size, dtype=np.uint32)
    lib().oc_murmur2_batch(keys, seed, out, keys.size)
    return out


class OracleCCEH:
    """Serial CCEH_hybrid restatement.  initial_depth as in CCEH_hybrid(initCap)
    (use depth_for_hybrid / depth_for_src to convert an initCap)."""

    def __init__(self, initial_depth: int, reserve_segments: int = 0, upsert: bool = False):
        self._t = lib().oc_create(initial_depth, reserve_segments)
        if not self._t:
            raise ValueError("bad initial depth")
        if upsert:  # last-writer-wins: CCEH_hybrid.cpp:153's overwrite clause enabled
            lib().oc_set_upsert(self._t, 1)

    def close(self):
        if getattr(self, "_t", None):
            lib().oc_destroy(self._t)
            self._t = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter teardown
            pass

    @staticmethod
    def depth_for_hybrid(init_cap: int) -> int:
        return lib().oc_depth_for_hybrid(init_cap)

    @staticmethod
    def depth_for_src(init_cap: int) -> int:
        return lib().oc_depth_for_src(init_cap)

    def insert(self, keys, values) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        values = np.ascontiguousarray(values, dtype=np.uint64)
        st = np.empty(keys.size, dtype=np.uint8)
        lib().oc_insert_batch(self._t, keys, values, keys.size, st)
        return st

    def get(self, keys):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        vals = np.empty(keys.size, dtype=np.uint64)
        st = np.empty(keys.size, dtype=np.uint8)
        lib().oc_get_batch(self._t, keys, keys.size, vals, st)
        return vals, st

    def find_anyway(self, keys):
        """CCEH::FindAnyway (CCEH_hybrid.cpp:482-496) per key: (values, status)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        vals = np.empty(keys.size, dtype=np.uint64)
        st = np.empty(keys.size, dtype=np.uint8)
        lib().oc_find_anyway_batch(self._t, keys, keys.size, vals, st)
        return vals, st

    def mixed(self, ops, keys, values):
        ops = np.ascontiguousarray(ops, dtype=np.uint8)
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        values = np.ascontiguousarray(values, dtype=np.uint64)
        out = np.empty(keys.size, dtype=np.uint64)
        st = np.empty(keys.size, dtype=np.uint8)
        lib().oc_mixed(self._t, ops, keys, values, keys.size, out, st)
        return out, st

    @property
    def depth(self) -> int:
        return lib().oc_depth(self._t)

    @property
    def num_segments(self) -> int:
        return lib().oc_num_segments(self._t)

    def stats(self) -> dict:
        s = Stats()
        lib().oc_get_stats(self._t, C.byref(s))
        return {n: getattr(s, n) for n, _ in Stats._fields_}

    def utilization(self) -> float:
        return lib().oc_utilization(self._t)

    def capacity(self) -> int:
        return lib().oc_capacity(self._t)

    def dump(self) -> dict:
        """Canonical dump: segments in directory order."""
        d = self.depth
        n = self.num_segments
        dir_canon = np.empty(1 << d, dtype=np.uint32)
        ld = np.empty(n, dtype=np.uint32)
        prefix = np.empty(n, dtype=np.uint64)
        keys = np.empty(n * 1024, dtype=np.uint64)
        vals = np.empty(n * 1024, dtype=np.uint64)
        lib().oc_dump(self._t, dir_canon, ld, prefix, keys, vals)
        return {"depth": d, "dir_canon": dir_canon, "local_depth": ld, "prefix": prefix,
                "keys": keys, "values": vals}

    def time_insert(self, keys, flush_ns: int = 10) -> float:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        return lib().oc_time_insert(self._t, keys, keys.size, flush_ns)

    def time_get(self, keys, threads: int = 1):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        m = C.c_uint64(0)
        t = lib().oc_time_get(self._t, keys, keys.size, threads, C.byref(m))
        return t, m.value


def bloom_add(bitmap: np.ndarray, nbits: int, k: int, keys) -> None:
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    lib().oc_bloom_add_batch(bitmap, nbits, k, keys, keys.size)


def bloom_check(bitmap: np.ndarray, nbits: int, k: int, keys):
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    out = np.empty(keys.size, dtype=np.uint8)
    tp = C.c_uint64(0)
    lib().oc_bloom_check_batch(bitmap, nbits, k, keys, keys.size, out, C.byref(tp))
    return out, tp.value


class OracleCBF:
    """Serial CountingBloomFilter<Key_t> (server/util/counting_bloom_filter.h):
    u8 counters (Insert :109-118 saturating, Delete :120-131 query-then-decrement
    with uint8 wrap, Query :133-143) and ToOrdinaryBloomFilter (:202-215)."""

    def __init__(self, nbits: int, k: int):
        self.m, self.k = nbits, k
        self.counters = np.zeros(nbits, np.uint8)

    def insert(self, keys) -> None:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        lib().oc_cbf_insert_batch(self.counters, self.m, self.k, keys, keys.size)

    def delete(self, keys) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.empty(keys.size, np.uint8)
        lib().oc_cbf_delete_batch(self.counters, self.m, self.k, keys, keys.size, out)
        return out

    def query(self, keys) -> np.ndarray:
        return np.array([lib().oc_cbf_query(self.counters, self.m, self.k, int(x)) for x in
                         np.asarray(keys, np.uint64)], np.uint8)

    def bitmap(self) -> np.ndarray:
        bm = np.zeros((self.m + 63) // 64, np.uint64)
        lib().oc_cbf_to_bitmap(self.counters, self.m, bm)
        return bm


def _stoull(tok: bytes):
    """std::stoull(tok) base 10: optional sign, >= 1 digit, trailing chars
    ignored, '-' negates mod 2^64; None where the reference throws."""
    i, neg = 0, False
    if tok[:1] in (b"+", b"-"):
        neg, i = tok[:1] == b"-", 1
    j = i
    while j < len(tok) and 48 <= tok[j] <= 57:
        j += 1
    if j == i:
        return None
    v = int(tok[i:j])
    if v >= 1 << 64:
        return None
    return (-v) % (1 << 64) if neg else v


def parse_replay_trace(text: bytes, num_data: int):
    """server/replay_KV.cpp:209-247, line by line: fields split on isspace;
    key = (INODE << 32) + OFFSET (:24-31, :222-224); 'W' -> ceil(SIZE/4096)
    Inserts (op 1), 'R' -> as many Gets (op 0) of key + 4096*b (:226-243);
    stop after the line that brings the count to num_data (:245-246).
    Returns (ops u8, keys u64) of the first num_data ops; raises ValueError
    where the reference throws / reads out of range."""
    ops, keys = [], []
    lines = text.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()  # getline: no empty line after a final newline
    done = 0
    for ln in lines:
        e = ln.split()
        if len(e) < 6:
            raise ValueError("malformed line")
        inode, off = _stoull(e[3]), _stoull(e[5])
        if inode is None or off is None:
            raise ValueError("malformed line")
        key = ((inode << 32) + off) % (1 << 64)
        batch, op = 0, 0
        if e[2][:1] in (b"W", b"R"):
            if len(e) < 7 or _stoull(e[6]) is None:
                raise ValueError("malformed line")
            size = _stoull(e[6])
            batch = size // 4096 + (1 if size % 4096 else 0)
            op = 1 if e[2][:1] == b"W" else 0
        for b in range(batch):
            ops.append(op)
            keys.append((key + 4096 * b) % (1 << 64))
        done += batch
        if done >= num_data:
            break
    if len(ops) < num_data:
        raise ValueError("trace shorter than num_data")
    return np.array(ops[:num_data], np.uint8), np.array(keys[:num_data], np.uint64)


def _ffs32(x: int) -> int:  # ffs((int)x)
    lo = x & 0xFFFFFFFF
    return (lo & -lo).bit_length() if lo else 0


def extent_heads(key: int, length: int, cluster: int = 0, convention: str = "hybrid"):
    """Sub-extent heads of one Insert_extent call, in insertion order.
    hybrid: CCEH_hybrid.cpp:90-105 (cover = 1 << (ffs((int)head) - 1) as
    unsigned int, 0 -> 1 << EXTENT_MAX_HEIGHT(30), halved while > len);
    src: src/cceh.cpp:308-330 (odd -> 1; 0 -> len/2; else
    1 << ctz((unsigned)min(len, 1 << ((ffs-1) & 63))))."""
    M = (1 << 64) - 1
    out = []
    head = (key + cluster) & M if convention == "src" else key
    while length > 0:
        out.append(head)
        if length == 1:
            break
        if convention == "src":
            if head & 1:
                sub = 1
            elif head == 0:
                sub = length // 2
            else:
                order = (_ffs32(head) - 1) & M
                lim = min(length, 1 << (order & 63))
                l32 = lim & 0xFFFFFFFF
                sub = 1 << ((l32 & -l32).bit_length() - 1 if l32 else 32)
        else:
            f = _ffs32(head)
            cover = ((1 << (f - 1)) & 0xFFFFFFFF) if f else 0
            if cover == 0:
                cover = 1 << 30
            while cover > length:
                cover >>= 1
            sub = cover
        head = (head + sub) & M
        length -= sub
    return out


def extent_targets(key: int, cluster: int = 0, convention: str = "hybrid"):
    """Get_extent probe targets in order: src Get(key + cluster)
    (src/cceh.cpp:381-391); hybrid key - key % 2^h, h < 30 (CCEH_hybrid.cpp:330-341);
    the first nonzero Get result is returned."""
    if convention == "src":
        return [(key + cluster) & ((1 << 64) - 1)]
    return [key - key % (1 << h) for h in range(30)]
