"""Pin the CPU oracle (oracle/cceh_oracle.c) to golden vectors produced by the
reference's own code (tests/golden/gen_golden.py -> oracle/_ref/ref_driver)."""
import json
import os

import numpy as np
import pytest

import scenarios as S
from oracle import oracle as O


@pytest.fixture(scope="module")
def kat(golden_dir):
    return np.load(os.path.join(golden_dir, "hash_kat.npz"))


@pytest.fixture(scope="module")
def cceh_golden(golden_dir):
    with open(os.path.join(golden_dir, "cceh_scenarios.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def bloom_golden(golden_dir):
    with open(os.path.join(golden_dir, "bloom.json")) as f:
        return json.load(f)


def test_hash64_kat(kat):
    h = O.hash64(kat["keys"])
    assert np.array_equal(h, kat["h"])
    # SURVEY §8a a1 published KATs
    assert O.lib().oc_hash64(0) == 0xc7e834dfe9778643
    assert O.lib().oc_hash64(1) == 0x59338fd0956c55bd
    assert O.lib().oc_hash64(42) == 0x4c60d11342c38e05
    assert O.lib().oc_hash64((1 << 64) - 1) == 0x0f8dcb1772df2c17


def test_murmur2_kat(kat):
    for s in range(4):
        assert np.array_equal(O.murmur2(kat["keys"], s), kat["murmur2"][:, s])
    assert [O.lib().oc_murmur2(0, s) for s in range(4)] == [0x93b132bc, 0xb6136249, 0xcd3f883f, 0x2627ecf5]
    # bloom indices of key 42 at m = 1e9
    assert [O.lib().oc_murmur2(42, s) % 1000000000 for s in range(4)] == [
        219936211, 915845167, 985558426, 225417891]


SCEN = None


def _scen():
    global SCEN
    if SCEN is None:
        SCEN = S.scenarios(O.hash64)
    return SCEN


@pytest.mark.parametrize("name", [
    "cap2_ins3k", "cap8_ins20k", "cap1024_ins100k", "cap2_ins100k", "cap256_ins400k",
    "mixed_cap16_60k", "mixed_cap2_30k_ins80", "dup_wrap", "dup32", "dup_pairs", "src_cap2m_ins50k",
    "split_loss", "split_loss_mixed"])
def test_oracle_matches_reference(name, cceh_golden):
    g = cceh_golden[name]
    init_cap, conv, ops, keys, vals = _scen()[name]
    depth = O.OracleCCEH.depth_for_hybrid(init_cap) if conv == "hybrid" else O.OracleCCEH.depth_for_src(init_cap)
    t = O.OracleCCEH(depth)
    out, st = t.mixed(ops, keys, vals)
    d = t.dump()
    rec = S.summarize(d["depth"], d["local_depth"], d["prefix"], d["keys"], d["values"], out, ops)
    for k, v in rec.items():
        assert v == g[k], (name, k)
    assert abs(t.utilization() - g["utilization"]) < 1e-9
    assert t.capacity() == g["capacity"]
    if "get_values_sample" in g:
        assert out[g["get_positions_sample"]].tolist() == g["get_values_sample"]
    stats = t.stats()
    # early exit at the first empty slot never changes a Get result
    assert stats["early_exit_mismatch"] == 0
    ins = ops == S.OP_INSERT
    assert np.all(st[ins] == O.ST_INSERTED)
    assert np.all((st[~ins] == O.ST_HIT) == (out[~ins] != 0))
    # Insert4split's silent drops (CCEH_hybrid.cpp:18-28): the reference's
    # final table holds every inserted key but the dropped ones (scenarios
    # without duplicate inserts)
    if not name.startswith("dup"):
        assert stats["split_loss"] == int(ins.sum()) - g["occupied"]
    if name.startswith("split_loss"):
        assert stats["split_loss"] == 4


@pytest.fixture(scope="module")
def findany_golden(golden_dir):
    with open(os.path.join(golden_dir, "findany.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", S.FINDANY_CASES)
def test_oracle_find_anyway_matches_reference(name, findany_golden):
    """CCEH::FindAnyway (CCEH_hybrid.cpp:482-496): the reference's own answers
    after each stream, including the wrap-reorder key of dup_wrap whose first
    copy in slot order is not Get's first copy in probe order."""
    g = findany_golden[name]
    init_cap, conv, ops, keys, vals = _scen()[name]
    depth = O.OracleCCEH.depth_for_hybrid(init_cap) if conv == "hybrid" else O.OracleCCEH.depth_for_src(init_cap)
    t = O.OracleCCEH(depth)
    t.mixed(ops, keys, vals)
    q = S.findany_queries(keys)
    assert S.sha(q) == g["query_sha"]
    fa, fst = t.find_anyway(q)
    gv, _ = t.get(q)
    assert S.sha(fa) == g["find_sha"] and S.sha(gv) == g["get_sha"]
    assert int(np.count_nonzero(fa)) == g["find_hits"]
    assert np.array_equal(fst == O.ST_HIT, fa != 0)
    div = np.nonzero(fa != gv)[0]
    assert [[int(i), int(fa[i]), int(gv[i])] for i in div] == g["diverge"]
    if name == "dup_wrap":
        assert g["n_diverge"] == 1  # the wrapped window: slot order != probe order


@pytest.fixture(scope="module")
def upsert_golden(golden_dir):
    with open(os.path.join(golden_dir, "upsert_scenarios.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["up_dup_wrap", "up_dup_many", "up_dup_pairs", "up_reinserts_cap2",
                                  "up_reinserts_cap256", "up_split_loss_mixed"])
def test_oracle_upsert_matches_reference(name, upsert_golden):
    """Last-writer-wins: the oracle's upsert mode equals the reference's
    CCEH_hybrid.cpp with its overwrite clause (:153) enabled
    (oracle/CCEH_hybrid.upsert.patch, built as oracle/_ref/ref_driver_upsert)."""
    g = upsert_golden[name]
    init_cap, conv, ops, keys, vals = S.upsert_scenarios(O.hash64)[name]
    t = O.OracleCCEH(O.OracleCCEH.depth_for_hybrid(init_cap), upsert=True)
    out, st = t.mixed(ops, keys, vals)
    d = t.dump()
    rec = S.summarize(d["depth"], d["local_depth"], d["prefix"], d["keys"], d["values"], out, ops)
    for k, v in rec.items():
        assert v == g[k], (name, k)
    assert abs(t.utilization() - g["utilization"]) < 1e-9
    ins = ops == S.OP_INSERT
    assert np.all(np.isin(st[ins], [O.ST_INSERTED, O.ST_UPDATED]))
    # last-writer-wins against a dictionary model (where no split dropped the key)
    last = {}
    want = np.zeros(keys.size, np.uint64)
    for i in range(keys.size):
        if ops[i] == S.OP_INSERT:
            last[int(keys[i])] = int(vals[i])
        else:
            want[i] = last.get(int(keys[i]), 0)
    g_ = ~ins
    if t.stats()["split_loss"] == 0:
        assert np.array_equal(out[g_], want[g_])
    # an update never takes a second slot: one copy of every key
    occ = d["keys"][d["keys"] != np.uint64(2**64 - 1)]
    assert occ.size == np.unique(occ).size


def test_dup33_is_unsplittable():
    """The 33rd copy of a key hangs the reference; the build
    contract reports UNSPLITTABLE and leaves the table unchanged."""
    t = O.OracleCCEH(2)
    k = np.full(33, 12345, np.uint64)
    st = t.insert(k, np.arange(1, 34, dtype=np.uint64))
    assert np.all(st[:32] == O.ST_INSERTED) and st[32] == O.ST_UNSPLITTABLE
    v, s = t.get(np.array([12345], np.uint64))
    assert s[0] == O.ST_HIT and v[0] == 1


def test_reserved_keys_rejected():
    t = O.OracleCCEH(2)
    st = t.insert(np.array([2**64 - 1, 2**64 - 2], np.uint64), np.array([1, 2], np.uint64))
    assert np.all(st == O.ST_RESERVED_KEY)
    v, s = t.get(np.array([2**64 - 1], np.uint64))
    assert s[0] == O.ST_RESERVED_KEY


def test_bftest_known_answers(bloom_golden):
    """server/bftest.cpp:9-55 assertions, restated on the oracle, and the
    reference's counter/bitmap state for the same inputs."""
    g = bloom_golden["bftest"]
    k, m = 2, 100000
    t = np.arange(10000, dtype=np.uint64) * np.uint64(14)
    cnt = np.zeros(m, np.uint8)
    lib = O.lib()
    for key in t[:9999]:
        lib.oc_cbf_insert(cnt, m, k, int(key))
    assert lib.oc_cbf_query(cnt, m, k, int(t[0])) == 1
    assert lib.oc_cbf_query(cnt, m, k, int(t[9999])) == 0
    bm = np.zeros((m + 63) // 64, np.uint64)
    lib.oc_cbf_to_bitmap(cnt, m, bm)
    assert S.sha(bm) == g["bitmap_sha"]
    from pmdfc_amd.workload import uniform_keys
    qs = np.concatenate([t, uniform_keys(31, 0, 2000)])
    assert S.sha(qs) == g["query_sha"]
    q = np.array([lib.oc_cbf_query(cnt, m, k, int(x)) for x in qs], np.uint8)
    assert np.packbits(q).tobytes().hex() == g["query"]
    qbb, _ = O.bloom_check(bm, m, k, qs)
    assert np.packbits(qbb).tobytes().hex() == g["querybb"]
    assert qbb[0] == 1 and qbb[9999] == 0
    assert lib.oc_cbf_delete(cnt, m, k, int(t[0])) == 1
    assert lib.oc_cbf_query(cnt, m, k, int(t[0])) == 0
    q2 = np.array([lib.oc_cbf_query(cnt, m, k, int(x)) for x in qs], np.uint8)
    assert np.packbits(q2).tobytes().hex() == g["query_after_delete"]
    lib.oc_cbf_to_bitmap(cnt, m, bm)
    assert S.sha(bm) == g["bitmap_after_delete_sha"]


@pytest.mark.slow
def test_bloom_k4_m1e9(bloom_golden):
    """Client filter shape (client/rdpma.h:33-35): k=4, 1e9 bits, MSB-first."""
    g = bloom_golden["k4_m1e9"]
    from pmdfc_amd.workload import uniform_keys
    m, k = 1000000000, 4
    ins = uniform_keys(32, 0, 100000)
    bm = np.zeros((m + 63) // 64, np.uint64)
    O.bloom_add(bm, m, k, ins)
    assert S.sha(bm) == g["bitmap_sha"]
    qs = np.concatenate([uniform_keys(32, 0, 20000), uniform_keys(32, 100000, 20000)])
    out, _ = O.bloom_check(bm, m, k, qs)
    assert np.packbits(out).tobytes().hex() == g["querybb"]


@pytest.fixture(scope="module")
def cbf_golden(golden_dir):
    with open(os.path.join(golden_dir, "cbf_seq.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["sat_conflict", "tiny_wrap", "fastpath", "bftest_seq"])
def test_cbf_sequences(cbf_golden, name):
    """Counting-BF Insert-then-Delete sequences against the reference's own
    counting_bloom_filter.h run by oracle/_ref/ref_driver (mode cbfseq)."""
    g = cbf_golden[name]
    k, m, ins, dels = S.cbfseq_cases()[name]
    assert (k, m) == (g["k"], g["m"])
    assert S.sha(ins) == g["insert_sha"] and S.sha(dels) == g["delete_sha"]
    f = O.OracleCBF(m, k)
    f.insert(ins)
    assert S.sha(f.counters) == g["counters_sha"]
    d = f.delete(dels)
    assert np.packbits(d).tobytes().hex() == g["deleted"]
    assert S.sha(f.counters) == g["counters_after_delete_sha"]
    assert S.sha(f.bitmap()) == g["bitmap_sha"]


@pytest.fixture(scope="module")
def replay_golden(golden_dir):
    with open(os.path.join(golden_dir, "replay.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["small", "mid", "crlf_tiny_table", "big"])
def test_replay_trace_matches_reference(replay_golden, name):
    """The oracle's replay_KV restatement (trace parse + serial CCEH over
    src/cceh.cpp) reproduces the reference replay_KV's failedSearch and
    put/get counts on the same synthetic trace."""
    g = replay_golden[name]
    text = S.replay_trace(g["seed"], g["n_lines"], crlf=g["crlf"])
    assert S.sha(np.frombuffer(text, np.uint8)) == g["text_sha"]
    ops, keys = O.parse_replay_trace(text, g["num_data"])
    assert int((ops == 1).sum()) == g["put"] and int((ops == 0).sum()) == g["get"]
    t = O.OracleCCEH(O.OracleCCEH.depth_for_src(g["tablesize"]))
    v, st = t.mixed(ops, keys, keys)
    assert int(((ops == 0) & (v != keys)).sum()) == g["failedSearch"]
    # per-op Get results equal the reference's src/cceh.cpp on the same stream
    gv = np.where(ops == 0, v, 0).astype(np.uint64)
    assert S.sha(gv) == g["get_values_sha"] and int(np.count_nonzero(gv)) == g["get_hits"]


def test_replay_trace_parse_edges():
    txt = b"0 t W 1 9 0 4097\n1 t O 2 9 7\n2 t R +1 9 -4096 1\n3 t X 5 9 0 99999\n4 t W 3 9 0 0\n5 t R 1 9 4096 10\n"
    ops, keys = O.parse_replay_trace(txt, 4)
    assert ops.tolist() == [1, 1, 0, 0]
    assert keys.tolist() == [1 << 32, (1 << 32) + 4096, (1 << 32) - 4096, (1 << 32) + 4096]
    with pytest.raises(ValueError):
        O.parse_replay_trace(b"0 t W 1 9\n", 1)  # missing fields
    with pytest.raises(ValueError):
        O.parse_replay_trace(b"0 t W x 9 0 1\n", 1)  # no digits
    with pytest.raises(ValueError):
        O.parse_replay_trace(txt, 100)  # shorter than num_data
    ops, _ = O.parse_replay_trace(b"0 t W 1 9 0 4096\n\n", 1)  # stops before the empty line
    assert ops.tolist() == [1]


@pytest.fixture(scope="module")
def extent_golden(golden_dir):
    with open(os.path.join(golden_dir, "extent.json")) as f:
        return json.load(f)


def oracle_extent_run(case):
    conv, cap, keys, cl, lens, vals, qk, qc = case
    depth = O.OracleCCEH.depth_for_src(cap) if conv == "src" else O.OracleCCEH.depth_for_hybrid(cap)
    t = O.OracleCCEH(depth)
    hk, hv = S.extent_expand(conv, keys, cl, lens, vals, O.extent_heads)
    t.insert(hk, hv)
    per = 1 if conv == "src" else 30
    tk = np.array([x for k, c in zip(qk.tolist(), qc.tolist()) for x in O.extent_targets(k, c, conv)], np.uint64)
    v, st = t.get(tk)
    v = np.where(st == O.ST_HIT, v, 0).reshape(-1, per)
    first = np.argmax(v != 0, axis=1)
    res = np.where((v != 0).any(axis=1), v[np.arange(v.shape[0]), first], 0).astype(np.uint64)
    return t, res, hk


@pytest.mark.parametrize("name", ["hyb_cap1024", "hyb_cap2", "src_cap2m", "src_cap4096"])
def test_extent_matches_reference(extent_golden, name):
    """Insert_extent / Get_extent restated (oracle.extent_heads / extent_targets
    over the serial CCEH) equal the reference's own extent API."""
    g = extent_golden[name]
    t, res, _ = oracle_extent_run(S.extent_cases()[name])
    d = t.dump()
    rec = S.summarize(d["depth"], d["local_depth"], d["prefix"], d["keys"], d["values"],
                      np.zeros(0, np.uint64), np.zeros(0, np.uint8))
    for k, v in rec.items():
        assert v == g[k], (k, v, g[k])
    assert S.sha(res) == g["results_sha"]
