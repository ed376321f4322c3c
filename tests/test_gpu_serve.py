"""Op-by-op parity of the SERVED per-op front-end (include/pmdfc_kv.h over
BatchCore and the persistent k_serve wave) with the serial oracle.

The reference's callers reach the index one op at a time (server/KV.cpp:
100-158 from the RDMA poll threads, server/rdma_svr.cpp:755-835).  Here the
reference fixture streams go through the ring exactly as such callers would:
  * one blocking call per op;
  * contiguous runs of ragged sizes (many past the wave's 64-op chunk) in a
    256-place ring, so the stream wraps the ring hundreds of times;
  * async calls, whose backlog the control thread serves as engine batches
    (the flood hand-off) interleaved with the wave's chunks;
  * concurrent caller threads, whose interleaving the ring places record;
  * one ring or several (serve_waves: a serving wave per hash prefix, each
    owning its directory buckets).
Every op's status and Get value is compared with the oracle run in ring
order (places; ring-major with several rings, whose ops commute), and the
final table (dump) with the oracle's.  The small
tables (CCEH_hybrid(2)) grow through splits and sub-directory growth inside
the ordered path, so the wave's LDS copy of the directory bucket headers is
reloaded between chunks (checked: header_reloads > 0).  Bit-exact throughout.
"""
import json
import os
import threading

import numpy as np
import pytest

import scenarios as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import pmdfc_amd as P  # noqa: E402
from pmdfc_amd.kv import KV  # noqa: E402

NAMES = ["split_loss_mixed", "split_loss", "dup_wrap", "dup32", "cap2_ins3k", "mixed_cap2_30k_ins80"]
UPSERT_NAMES = ["up_dup_wrap", "up_dup_many", "up_reinserts_cap2", "up_split_loss_mixed"]


@pytest.fixture(scope="module")
def golden(golden_dir):
    with open(os.path.join(golden_dir, "cceh_scenarios.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def scen():
    return S.scenarios(O.hash64)


@pytest.fixture(scope="module")
def upscen():
    return S.upsert_scenarios(O.hash64)


def _runs(n, seed):
    """Ragged run lengths: singles, sub-chunk and past-chunk runs (<= 200)."""
    rng = np.random.default_rng(seed)
    out, o = [], 0
    while o < n:
        r = int(rng.choice([1, 3, 17, 63, 64, 65, 100, 129, 200]))
        out.append((o, min(n, o + r)))
        o += r
    return out


def _drive(kv, mode, ops, keys, vals, seed=0):
    n = ops.size
    if mode == "single":
        return kv.ops(ops, keys, vals, run=0)
    if mode == "burst":
        vo = np.zeros(n, np.uint64)
        st = np.zeros(n, np.uint8)
        pl = np.zeros(n, np.uint64)
        for a, b in _runs(n, seed):
            vo[a:b], st[a:b], pl[a:b] = kv.ops(ops[a:b], keys[a:b], vals[a:b], run=b - a)
        return vo, st, pl
    if mode == "async":
        return kv.ops_async(ops, keys, vals)
    raise ValueError(mode)


def _check_table(kv, o):
    d, od = kv.dump(), o.dump()
    assert d["depth"] == od["depth"]
    assert np.array_equal(d["local_depth"], od["local_depth"])
    assert np.array_equal(d["keys"], od["keys"]) and np.array_equal(d["values"], od["values"])
    return d


KV_CFG = {"single": dict(ring_size=1 << 13), "burst": dict(ring_size=256),
          "async": dict(ring_size=1 << 13, flood_ops=1024)}


def _ring_order(pl, waves):
    """The serial order the device applied: ring-major, place order within a
    ring (ring = place >> 48; rings own disjoint directory buckets, so ops of
    different rings commute).  One caller: each ring's places are consecutive
    in call order."""
    ring = pl >> np.uint64(48)
    assert int(ring.max()) < waves
    for g in np.unique(ring):
        p = pl[ring == g] & np.uint64((1 << 48) - 1)
        assert np.array_equal(p, np.arange(p.size, dtype=np.uint64) + p[0])
    return np.argsort(pl, kind="stable")


@pytest.mark.parametrize("waves", [1, 4])
@pytest.mark.parametrize("mode", ["single", "burst", "async"])
@pytest.mark.parametrize("name", NAMES)
def test_served_stream_matches_oracle(name, mode, waves, scen, golden):
    """waves 4: the front-end's rings per hash prefix (at most the table's
    starting directory buckets: CCEH_hybrid(2) gets 2, dup32's (4) 4)."""
    init_cap, conv, ops, keys, vals = scen[name]
    kv = KV(init_cap, convention=conv, max_batch=8192, max_segments=8192, serve_waves=waves, **KV_CFG[mode])
    vo, st, pl = _drive(kv, mode, ops, keys, vals, seed=len(name))
    nw = kv.phase()["serve_waves"]
    assert nw == min(waves, 1 << kv.initial_depth)
    order = _ring_order(pl, nw)
    o = O.OracleCCEH(kv.initial_depth)
    ov, ost = o.mixed(ops[order], keys[order], vals[order])
    st, vo = st[order], vo[order]
    bad = np.nonzero((st != ost) | (vo != ov))[0]
    assert bad.size == 0, (name, mode, bad[:8], st[bad[:8]], ost[bad[:8]])
    d = _check_table(kv, o)
    g = golden[name]
    assert S.sha(d["keys"]) == g["keys_sha"] and S.sha(d["values"]) == g["values_sha"]
    ph = kv.phase()
    assert ph["failed_ops"] == 0
    assert ph["ops_completed"] >= ops.size
    if init_cap == 2 and mode != "async":
        # the ordered path grew sub-directories between chunks: the wave's
        # header copy was reloaded, and the table is far past its 2 segments
        assert ph["header_reloads"] > 0, ph
        assert d["depth"] > 1
    if mode == "async" and ops.size >= 4096:
        assert ph["flood_batches"] > 0, ph  # the hand-off ran
    assert kv.stats()["error_flags"] == 0
    kv.close()


@pytest.mark.parametrize("delivery,waves", [(2, 4), (4, 4), (8, 8)])
@pytest.mark.parametrize("name", ["mixed_cap16_60k", "dup_pairs"])
def test_async_delivery_threads_match_oracle(name, delivery, waves, scen, monkeypatch):
    """Async ops whose callbacks run on several delivery threads
    (BatchingConfig::delivery_threads via PMDFC_DELIVERY_THREADS: ring g's
    callbacks on thread g mod n, concurrently with the other rings'): every
    op's result and the final table still equal the oracle's ring-major
    replay, and every place of every ring is freed."""
    monkeypatch.setenv("PMDFC_DELIVERY_THREADS", str(delivery))
    init_cap, conv, ops, keys, vals = scen[name]
    kv = KV(init_cap, convention=conv, max_batch=8192, max_segments=8192, serve_waves=waves, **KV_CFG["async"])
    vo, st, pl = _drive(kv, "async", ops, keys, vals)
    order = _ring_order(pl, kv.phase()["serve_waves"])
    o = O.OracleCCEH(kv.initial_depth)
    ov, ost = o.mixed(ops[order], keys[order], vals[order])
    bad = np.nonzero((st[order] != ost) | (vo[order] != ov))[0]
    assert bad.size == 0, (name, delivery, bad[:8])
    _check_table(kv, o)
    ph = kv.phase()
    assert ph["failed_ops"] == 0 and ph["ops_completed"] >= ops.size
    kv.close()


@pytest.mark.parametrize("mode", ["single", "burst"])
@pytest.mark.parametrize("name", UPSERT_NAMES)
def test_served_upsert_matches_oracle(name, mode, upscen):
    """Last-writer-wins (PMDFC_CFG_UPSERT) through the ring: the oracle is the
    reference with its :153 overwrite clause enabled (pinned by
    upsert_scenarios.json in test_gpu_parity.py)."""
    init_cap, conv, ops, keys, vals = upscen[name]
    kv = KV(init_cap, convention=conv, max_batch=8192, max_segments=8192, upsert=True, **KV_CFG[mode])
    vo, st, pl = _drive(kv, mode, ops, keys, vals, seed=len(name))
    order = _ring_order(pl, kv.phase()["serve_waves"])
    o = O.OracleCCEH(kv.initial_depth, upsert=True)
    ov, ost = o.mixed(ops[order], keys[order], vals[order])
    st, vo = st[order], vo[order]
    bad = np.nonzero((st != ost) | (vo != ov))[0]
    assert bad.size == 0, (name, mode, bad[:8], st[bad[:8]], ost[bad[:8]])
    _check_table(kv, o)
    kv.close()


@pytest.mark.parametrize("name,threads,run,waves", [("mixed_cap2_30k_ins80", 8, 0, 1),
                                                    ("mixed_cap2_30k_ins80", 16, 0, 1),
                                                    ("mixed_cap2_30k_ins80", 6, 37, 1),
                                                    ("mixed_cap2_30k_ins80", 16, 0, 2),
                                                    ("mixed_cap16_60k", 16, 0, 8),
                                                    ("mixed_cap16_60k", 8, 29, 16)])
def test_concurrent_callers_match_oracle_in_ring_order(name, threads, run, waves, scen):
    """T caller threads push disjoint slices of a mixed stream at once (the
    reference's concurrent poll threads), through one ring or several (one
    serving wave each, by hash prefix).  Their interleaving is whatever the
    rings recorded: the oracle replays all ops ring-major in place order and
    must agree on every op and on the final table."""
    init_cap, conv, ops, keys, vals = scen[name]
    n = ops.size
    kv = KV(init_cap, convention=conv, max_batch=8192, max_segments=8192, ring_size=1024, serve_waves=waves)
    assert kv.phase()["serve_waves"] == waves
    vo = np.zeros(n, np.uint64)
    st = np.zeros(n, np.uint8)
    pl = np.zeros(n, np.uint64)
    part = np.arange(n) % threads
    errs = []

    def caller(t):
        try:
            idx = np.nonzero(part == t)[0]
            a, b, c = kv.ops(ops[idx], keys[idx], vals[idx], run=run)
            vo[idx], st[idx], pl[idx] = a, b, c
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=caller, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    order = np.argsort(pl, kind="stable")
    ring = pl >> np.uint64(48)
    for g in np.unique(ring):  # every place of every ring once
        p = np.sort(pl[ring == g] & np.uint64((1 << 48) - 1))
        assert np.array_equal(p, np.arange(p.size, dtype=np.uint64) + p[0])
    o = O.OracleCCEH(kv.initial_depth)
    ov, ost = o.mixed(ops[order], keys[order], vals[order])
    assert np.array_equal(st[order], ost)
    assert np.array_equal(vo[order], ov)
    _check_table(kv, o)
    kv.close()


def test_served_single_op_calls_and_introspection(scen):
    """KVStore's per-op calls (Insert, Get, FindAnyway, Utilization,
    Capacity) interleaved: each introspection call stops the wave, runs on the
    engine and restarts the wave for the next op."""
    init_cap, conv, ops, keys, vals = scen["dup_wrap"]
    kv = KV(init_cap, convention=conv, max_batch=8192, max_segments=8192)
    o = O.OracleCCEH(kv.initial_depth)
    for i in range(0, min(ops.size, 3000)):
        if ops[i] == S.OP_INSERT:
            assert kv.Insert(int(keys[i]), int(vals[i])) == P.ST_INSERTED
            o.insert(keys[i:i + 1], vals[i:i + 1])
        else:
            ov, _ = o.get(keys[i:i + 1])
            assert kv.Get(int(keys[i])) == int(ov[0])
        if i % 701 == 0:
            assert abs(kv.Utilization() - o.utilization()) < 1e-9
            assert kv.Capacity() == o.capacity()
            fv, _ = o.find_anyway(keys[i:i + 1])
            assert kv.FindAnyway(int(keys[i])) == int(fv[0])
    _check_table(kv, o)
    assert kv.phase()["wave_starts"] > 1
    kv.close()


def test_dump_while_other_threads_insert(scen):
    """KV.dump() from one thread while others insert and split segments
    (a dump sized by one call and filled by another could write
    past the caller's buffers when the table grew in between).  pmdfc_kv_dump
    now sizes and fills under one stop of the serving waves and answers
    PMDFC_ERR_SIZE, with the sizes, when the buffers are too small: every
    dump is self-consistent (its directory points at its own segments, its
    segment count never shrinks), and the last one, after the callers are
    done, holds every inserted key exactly once."""
    init_cap, conv, ops, keys, vals = scen["cap2_ins100k"]
    ins = ops == S.OP_INSERT
    k, v = keys[ins][:60000], vals[ins][:60000]
    kv = KV(init_cap, convention=conv, max_batch=8192, max_segments=8192, serve_waves=2)
    stop = threading.Event()
    errs, dumps = [], []

    def caller(t):
        try:
            sl = slice(t, k.size, 4)
            kv.ops(np.ones(k[sl].size, np.uint8), k[sl], v[sl], run=61)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    def dumper():
        try:
            while not stop.is_set():
                d = kv.dump()
                nseg = d["local_depth"].size
                assert d["keys"].size == nseg * 1024 and d["dir_canon"].size == 1 << d["depth"]
                assert int(d["dir_canon"].max()) < nseg
                dumps.append(nseg)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=caller, args=(t,)) for t in range(4)]
    dt = threading.Thread(target=dumper)
    dt.start()
    for x in th:
        x.start()
    for x in th:
        x.join()
    stop.set()
    dt.join()
    assert not errs, errs
    assert len(dumps) >= 2 and dumps[-1] >= dumps[0]
    d = kv.dump()
    stored = d["keys"][d["keys"] != np.uint64(0xFFFFFFFFFFFFFFFF)]
    assert np.array_equal(np.sort(stored), np.sort(k))  # (distinct keys: every insert stored once)
    kv.close()
