"""GPU parity of the server counting bloom filter (server/util/counting_bloom_filter.h)
through the C-ABI (pmdfc_cbf_*): the reference-generated fixtures
(tests/golden/cbf_seq.json, bloom.json) and the oracle (OracleCBF) on larger
seeded inputs, bit-exact."""
import json
import os

import numpy as np
import pytest

import scenarios as S
from oracle import oracle as O
from pmdfc_amd.workload import uniform_keys

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import pmdfc_amd as P  # noqa: E402


@pytest.fixture(scope="module")
def cbf_golden(golden_dir):
    with open(os.path.join(golden_dir, "cbf_seq.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def bloom_golden(golden_dir):
    with open(os.path.join(golden_dir, "bloom.json")) as f:
        return json.load(f)


def _cuts(n, parts):
    if parts == 1:
        return [(0, n)]
    b = np.linspace(0, n, parts + 1).astype(int)
    return list(zip(b[:-1], b[1:]))


@pytest.mark.parametrize("parts", [1, 3])
@pytest.mark.parametrize("name", ["sat_conflict", "tiny_wrap", "fastpath", "bftest_seq"])
def test_cbf_sequences_match_reference(cbf_golden, name, parts):
    """Insert batch(es), then Delete batch(es) in order: counters, per-key
    Delete results and the packed bitmap equal the reference's."""
    g = cbf_golden[name]
    k, m, ins, dels = S.cbfseq_cases()[name]
    f = P.CountingBloomFilter(k, m)
    for a, b in _cuts(ins.size, parts):
        f.Insert(ins[a:b])
    c = f.counters()
    assert S.sha(c) == g["counters_sha"]
    d = np.concatenate([f.Delete(dels[a:b]) for a, b in _cuts(dels.size, parts)])
    assert np.packbits(d).tobytes().hex() == g["deleted"]
    assert int(d.sum()) == g["n_deleted"]
    assert S.sha(f.counters()) == g["counters_after_delete_sha"]
    f.ToOrdinaryBloomFilter()
    assert S.sha(f.bitmap()) == g["bitmap_sha"]
    f.close()


def test_cbf_bftest_queries(bloom_golden):
    """server/bftest.cpp's scenario: Query / QueryBitBloom before and after
    Delete(t[0]) equal the reference's answers."""
    g = bloom_golden["bftest"]
    k, m = 2, 100000
    t = np.arange(10000, dtype=np.uint64) * np.uint64(14)
    qs = np.concatenate([t, uniform_keys(31, 0, 2000)])
    f = P.CountingBloomFilter(k, m)
    f.Insert(t[:9999])
    f.ToOrdinaryBloomFilter()
    assert np.packbits(f.Query(qs)).tobytes().hex() == g["query"]
    assert np.packbits(f.QueryBitBloom(qs)).tobytes().hex() == g["querybb"]
    assert S.sha(f.bitmap()) == g["bitmap_sha"]
    assert f.Delete(t[:1])[0] == 1
    assert np.packbits(f.Query(qs)).tobytes().hex() == g["query_after_delete"]
    f.ToOrdinaryBloomFilter()
    assert S.sha(f.bitmap()) == g["bitmap_after_delete_sha"]


def test_cbf_client_shape_bitmap(bloom_golden):
    """k=4, 1e9 bits (client/rdpma.h:33-35): the packed bitmap equals the
    reference's ToOrdinaryBloomFilter output, and exported to a client filter
    it answers bloom_filter_check as the reference's QueryBitBloom."""
    g = bloom_golden["k4_m1e9"]
    m, k = 1000000000, 4
    ins = uniform_keys(32, 0, 100000)
    q = np.concatenate([uniform_keys(32, 0, 20000), uniform_keys(32, 100000, 20000)])
    f = P.CountingBloomFilter(k, m)
    f.Insert(ins)
    f.ToOrdinaryBloomFilter()
    bm = f.bitmap()
    assert S.sha(bm) == g["bitmap_sha"]
    b = P.BloomFilter(m, k)
    f.export(b)
    assert np.packbits(b.probe(q)).tobytes().hex() == g["querybb"]
    assert np.packbits(f.Query(q)).tobytes().hex() == g["query"]
    f.close()
    b.close()


@pytest.mark.parametrize("m,k,n_ins,n_del", [(1 << 20, 4, 400000, 200000),  # dense: conflicts
                                              (100000007, 4, 2000000, 500000),  # sparse: fast path
                                              (4099, 3, 50000, 30000)])  # saturation, wraps
def test_cbf_random_vs_oracle(m, k, n_ins, n_del):
    rng = np.random.default_rng(m)
    ins = uniform_keys(50, 0, n_ins)
    ins = np.concatenate([ins, ins[rng.integers(0, n_ins, n_ins // 4)]])  # repeated keys
    dels = np.concatenate([ins[rng.integers(0, ins.size, n_del)], uniform_keys(51, 0, n_del // 5)])
    rng.shuffle(dels)
    f, o = P.CountingBloomFilter(k, m), O.OracleCBF(m, k)
    f.Insert(ins)
    o.insert(ins)
    assert np.array_equal(f.counters(), o.counters)
    d = np.concatenate([f.Delete(dels[a:b]) for a, b in _cuts(dels.size, 4)])
    od = o.delete(dels)
    assert np.array_equal(d, od)
    assert np.array_equal(f.counters(), o.counters)
    f.ToOrdinaryBloomFilter()
    assert np.array_equal(f.bitmap(), o.bitmap())
    qs = np.concatenate([ins[:5000], uniform_keys(52, 0, 5000)])
    assert np.array_equal(f.Query(qs), o.query(qs))
    bb, _ = O.bloom_check(o.bitmap(), m, k, qs)
    assert np.array_equal(f.QueryBitBloom(qs), bb)
    f.close()


def test_cbf_pack_tail_and_clear():
    """nbits not a multiple of 64 (or of the 4 KiB pack step): the last word's
    unused bits stay 0; Clear empties counters and bitmap."""
    for m in [1, 63, 65, 4095, 4097, 12345]:
        f, o = P.CountingBloomFilter(3, m), O.OracleCBF(m, 3)
        keys = uniform_keys(60, 0, 3 * m)
        f.Insert(keys)
        o.insert(keys)
        f.ToOrdinaryBloomFilter()
        assert np.array_equal(f.counters(), o.counters)
        assert np.array_equal(f.bitmap(), o.bitmap()), m
        f.Clear()
        f.ToOrdinaryBloomFilter()
        assert not f.counters().any() and not f.bitmap().any()
        f.close()


def test_cbf_rejects_bad_geometry():
    with pytest.raises(P.PmdfcError):
        P.CountingBloomFilter(4, 1 << 31)
    with pytest.raises(P.PmdfcError):
        P.CountingBloomFilter(0, 1000)


def test_cbf_feeds_fused_probe_then_get():
    """KV::Insert path (server/KV.cpp:100-121): index Insert + counting-BF
    Insert per batch, pack, ship to the client filter, then the fused
    client probe: absent keys are FILTERED unless false-positive, present
    keys hit."""
    t = P.CCEH(depth=8, max_batch=1 << 16, max_segments=4096)
    f = P.CountingBloomFilter(4, 10000019)
    b = P.BloomFilter(10000019, 4)
    keys = uniform_keys(70, 0, 100000)
    for a in range(0, keys.size, 1 << 16):
        kk = keys[a:a + (1 << 16)]
        t.Insert(kk, kk)
        f.Insert(kk)
    f.ToOrdinaryBloomFilter()
    f.export(b)
    q = np.concatenate([keys[:20000], uniform_keys(71, 0, 20000)])
    v, st = b.probe_then_get(t, q)
    assert np.all(st[:20000] == P.ST_HIT) and np.array_equal(v[:20000], keys[:20000])
    o = O.OracleCBF(10000019, 4)
    o.insert(keys)
    bb, _ = O.bloom_check(o.bitmap(), 10000019, 4, q[20000:])
    assert np.array_equal(st[20000:] == P.ST_FILTERED, bb == 0)
    assert np.all(st[20000:][bb == 1] == P.ST_MISS)


def test_cbf_insert_ops_counts_only_inserts():
    """Mixed batch: only ops == PMDFC_OP_INSERT increment (KV::Insert)."""
    rng = np.random.default_rng(5)
    keys = uniform_keys(80, 0, 300000)
    ops = (rng.random(keys.size) < 0.3).astype(np.uint8)
    f, o = P.CountingBloomFilter(4, 1 << 22), O.OracleCBF(1 << 22, 4)
    f.InsertOps(ops, keys)
    o.insert(keys[ops == 1])
    assert np.array_equal(f.counters(), o.counters)
