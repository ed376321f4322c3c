"""Fixed-capacity routing (route.hip, the N>1 path of bench.py) on one GPU.

* the HIP packer against the CPU restatement (tests/route_ref.py): send
  buffers (records and INVALID padding), row positions, carried ops across
  packs and drain packs, full-carry drops, keep masks and Get dedupe,
  bit-exact, for 1..16 owners, widths 1..3, reserved keys and ragged tile
  tails;
* split / respond / unpack against the restatement;
* a whole routed exchange among G in-process shards (separate engines on one
  GPU, the all-to-all done as a block transpose): per-op results and the
  union of the shards equal ONE serial oracle run over the rank-major
  concatenation of the ranks' batches -- the protocol BlockRouter runs over
  RCCL, minus the wire.
"""
import numpy as np
import pytest

import scenarios as S
from oracle import oracle as O
from route_ref import INVALID, TorchBlockPacker

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import pmdfc_amd as P  # noqa: E402


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64))


def _batch(seed, n):
    rng = np.random.default_rng(seed)
    keys = np.array(S.uniform_keys(seed, 0, n), dtype=np.uint64)
    if n > 10:
        keys[rng.integers(0, n, 3)] = INVALID  # reserved keys route like any other
        keys[rng.integers(0, n, 2)] = INVALID - np.uint64(1)
    vals = rng.integers(0, 2**63, n, dtype=np.int64).view(np.uint64)
    ops = rng.integers(0, 2, n).astype(np.uint8)
    return keys, vals, ops


def _pair(n_out, sbits, max_batch, cap=None, carry_cap=None):
    hp = P.BlockPacker(0, max_batch, sbits, cap=cap, carry_cap=carry_cap)
    rp = TorchBlockPacker(max_batch, sbits, cap=hp.cap, carry_cap=carry_cap)
    d = torch.device("cuda", 0)
    outs = (torch.full((n_out,), 77, dtype=torch.int64, device=d), torch.full((n_out,), 99, dtype=torch.uint8, device=d),
            torch.full((n_out,), 77, dtype=torch.int64), torch.full((n_out,), 99, dtype=torch.uint8))
    return hp, rp, outs


def _pack_both(hp, rp, outs, keys, vals, ops, width, base, keep=None):
    d = torch.device("cuda", 0)
    n = 0 if keys is None else keys.size
    hv, hs, rv, rs_ = outs
    if n:
        kp = torch.from_numpy(keep).to(d) if keep is not None else None
        send, rowpos = hp.pack(_t(keys).to(d), _t(vals).to(d) if width > 1 else None,
                               torch.from_numpy(ops).to(d) if width > 2 else None, width, kp, base, hv, hs)
        rs, rrow = rp.pack(_t(keys), _t(vals), torch.from_numpy(ops), width, keep, base, rv, rs_)
    else:
        send, rowpos = hp.pack(None, None, None, width, None, 0, hv, hs)
        rs, rrow = rp.pack(None, None, None, width, None, 0, rv, rs_)
    torch.cuda.synchronize()
    assert np.array_equal(send.cpu().numpy(), rs.numpy())
    assert np.array_equal(rowpos.cpu().numpy(), rrow.numpy())
    assert int(hp.carried().item()) == int(rp.carried()[0])
    return send, rowpos, rrow


@pytest.mark.parametrize("sbits", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("width", [1, 2, 3])
@pytest.mark.parametrize("n", [1, 4095, 4097, 50000])
def test_pack_matches_restatement(sbits, width, n):
    """send rows (records and INVALID padding) and rowpos bit-exact, at a
    nonzero call base"""
    keys, vals, ops = _batch(sbits * 100 + width * 10 + n % 7, n)
    hp, rp, outs = _pair(n + 1000, sbits, 65536)
    _pack_both(hp, rp, outs, keys, vals, ops, width, 1000)
    assert hp.overflow_count() == 0


@pytest.mark.parametrize("sbits", [0, 2, 4])
def test_pack_reused_across_batch_sizes(sbits):
    """One packer over a run of ragged batch sizes (the carry buffers flip
    every pack) matches the restatement on every call."""
    sizes = [50000, 1, 1 << 20, 4097, 0, 777777, 1025]
    hp, rp, outs = _pair(sum(sizes), sbits, 1 << 20)
    base = 0
    for i, n in enumerate(sizes):
        keys, vals, ops = _batch(900 + sbits * 10 + i, n)
        _pack_both(hp, rp, outs, keys if n else None, vals, ops, 2, base)
        base += n
    hp.end_call()


@pytest.mark.parametrize("sbits", [1, 3])
@pytest.mark.parametrize("width", [1, 3])
def test_pack_carry_matches_restatement(sbits, width):
    """Owner blocks far too small for the batches: each pack sends the
    carried ops first and carries the rest (FIFO per owner), drain packs
    (n = 0) empty the carry; send, rowpos, carried counts bit-exact with the
    restatement, and every op is sent exactly once."""
    n, nb = 40000, 3
    cap = max(256, (n >> sbits) // 3)
    hp, rp, outs = _pair(n * nb, sbits, n, cap=cap, carry_cap=n * nb)
    sent = []
    for e in range(nb):
        keys, vals, ops = _batch(11 + sbits + 7 * e, n)
        _, _, rrow = _pack_both(hp, rp, outs, keys, vals, ops, width, e * n)
        sent.append(rrow.numpy())
    for _ in range(100):
        if int(hp.carried().item()) == 0:
            break
        _, _, rrow = _pack_both(hp, rp, outs, None, None, None, width, 0)
        sent.append(rrow.numpy())
    assert int(hp.carried().item()) == 0
    hp.end_call()
    allrows = np.concatenate(sent)
    allrows = allrows[allrows >= 0]
    assert np.array_equal(np.sort(allrows), np.arange(n * nb))
    assert hp.overflow_count() == 0


def test_pack_full_carry_matches_restatement():
    """A carry of carry_cap ops per owner: the ops past it come back
    ST_ROUTE_OVERFLOW (value 0) in the call outputs, counted."""
    sbits, n = 2, 40000
    hp, rp, outs = _pair(2 * n, sbits, n, cap=2048, carry_cap=4096)
    for e in range(2):
        keys, vals, ops = _batch(31 + e, n)
        _pack_both(hp, rp, outs, keys, vals, ops, 2, e * n)
    hv, hs, rv, rs_ = outs
    assert np.array_equal(hs.cpu().numpy(), rs_.numpy()) and np.array_equal(hv.cpu().numpy(), rv.numpy())
    assert hp.overflow_count() == rp.overflow_count() > 0
    assert (hs.cpu().numpy() == P.ST_ROUTE_OVERFLOW).sum() == rp.overflow_count()
    hp.reset()
    assert hp.overflow_count() == 0 and int(hp.carried().item()) == 0


def test_split_respond_unpack_match_restatement():
    sbits, n = 2, 30000
    keys, vals, ops = _batch(3, n)
    d = torch.device("cuda", 0)
    hp, rp, outs = _pair(n, sbits, n)
    rng = np.random.default_rng(9)
    recv = rng.integers(-2**63, 2**63 - 1, hp.rows * 3, dtype=np.int64)
    hk, hv, ho = hp.split(torch.from_numpy(recv).to(d), 3)
    rk, rv, ro = rp.split(torch.from_numpy(recv), 3)
    assert np.array_equal(hk.cpu().numpy(), rk.numpy())
    assert np.array_equal(hv.cpu().numpy(), rv.numpy())
    assert np.array_equal(ho.cpu().numpy(), ro.numpy())
    gv = rng.integers(-2**63, 2**63 - 1, hp.rows, dtype=np.int64)
    gs = rng.integers(0, 9, hp.rows).astype(np.uint8)
    hr = hp.respond(torch.from_numpy(gv).to(d), torch.from_numpy(gs).to(d))
    rr = rp.respond(torch.from_numpy(gv), torch.from_numpy(gs))
    assert np.array_equal(hr.cpu().numpy(), rr.numpy())
    _, rowpos, rrow = _pack_both(hp, rp, outs, keys, vals, ops, 1, 0)
    hv2, hs2, rv2, rs2 = outs
    hp.unpack(hr, 1, rowpos, hv2, hs2)
    rp.unpack(rr, 1, rrow, rv2, rs2)
    assert np.array_equal(hv2.cpu().numpy(), rv2.numpy())
    assert np.array_equal(hs2.cpu().numpy(), rs2.numpy())
    st = torch.from_numpy((np.arange(hp.rows) % 9).astype(np.uint8))
    hp.unpack(st.to(d), 0, rowpos, None, hs2)
    rp.unpack(st, 0, rrow, None, rs2)
    assert np.array_equal(hs2.cpu().numpy(), rs2.numpy())


def test_dedupe_matches_restatement():
    """Get dedupe: leader = first Get of each key in its 1024-Get tile;
    INVALID keys and kept-home Gets lead themselves; fill copies the leader's
    result."""
    n = 200000
    rng = np.random.default_rng(4)
    pool = np.array(S.uniform_keys(12, 0, 500), dtype=np.uint64)
    keys = pool[rng.integers(0, pool.size, n)]
    keys[rng.integers(0, n, 50)] = INVALID
    keep = (rng.random(n) < 0.9).astype(np.uint8)
    d = torch.device("cuda", 0)
    hp, rp, _ = _pair(n, 2, n)
    base = 123
    hl = torch.full((n + base,), -5, dtype=torch.int32, device=d)
    rl = torch.full((n + base,), -5, dtype=torch.int32)
    hk = hp.dedupe(_t(keys).to(d), torch.from_numpy(keep).to(d), base, hl)
    rk = rp.dedupe(_t(keys), keep, base, rl)
    assert np.array_equal(hk.cpu().numpy(), rk.numpy())
    assert np.array_equal(hl.cpu().numpy(), rl.numpy())
    assert int(hk.sum()) < 0.5 * n  # ~440 distinct of 500 keys per 1024-Get tile
    vals = torch.arange(n + base, dtype=torch.int64, device=d)
    st = (torch.arange(n + base, device=d) % 7).to(torch.uint8)
    hp.fill(hl[base:] - base, vals[base:], st[base:])  # a call whose outputs start at 0
    lv = (rl.numpy()[base:] - base).astype(np.int64)
    assert np.array_equal(vals.cpu().numpy()[base:], lv + base)
    assert np.array_equal(st.cpu().numpy()[base:], ((lv + base) % 7).astype(np.uint8))


class _Exchange:
    """G in-process ranks on one GPU: an equal-split all-to-all is a block
    transpose of the ranks' send buffers."""

    def __init__(self, G):
        self.G = G

    def a2a(self, sends):
        chunks = [s.view(self.G, -1) for s in sends]
        return [torch.cat([chunks[src][dst] for src in range(self.G)]) for dst in range(self.G)]


@pytest.mark.parametrize("records", [False, True])
@pytest.mark.parametrize("sbits", [1, 2])
def test_routed_exchange_equals_global_serial(sbits, records):
    """records=True: the owners run pmdfc_cceh_insert_records / get_records
    straight on the received rows (what BlockRouter does with the engine)."""
    G, depth, B = 1 << sbits, 6, 6000
    d = torch.device("cuda", 0)
    pk = [P.BlockPacker(0, B, sbits) for _ in range(G)]
    rows = pk[0].rows
    eng = [P.CCEH(depth=depth, shard_bits=sbits, shard_id=r, max_batch=rows, max_segments=4096, device=0)
           for r in range(G)]
    ex = _Exchange(G)
    # per rank: an insert batch, a mixed batch, a get batch (step-major, rank-major)
    streams = []
    for r in range(G):
        ops, keys, vals = S.mixed(300 + r, B, 0.6)
        ins = S.insert_then_get(400 + r, B, 0)
        streams.append([(None, ins[1][:B], ins[2][:B]), (ops, keys, vals),
                        ("get", np.concatenate([ins[1][:B // 2], keys[:B // 2]]), None)])
    g = O.OracleCCEH(depth)
    for bi in range(3):
        kind = streams[0][bi][0]
        W = 2 if kind is None else (1 if isinstance(kind, str) else 3)
        sends, rows, outs = [], [], []
        for r in range(G):
            ops, keys, vals = streams[r][bi]
            vo = torch.empty(keys.size, dtype=torch.int64, device=d)
            so = torch.empty(keys.size, dtype=torch.uint8, device=d)
            s, p = pk[r].pack(_t(keys).to(d), _t(vals).to(d) if W > 1 else None,
                              torch.from_numpy(ops).to(d) if W > 2 else None, W, None, 0, vo, so)
            assert int(pk[r].carried().item()) == 0
            sends.append(s.clone())
            rows.append(p.clone())
            outs.append((vo, so))
        recvs = ex.a2a(sends)
        resps = []
        for r in range(G):
            if W == 1 and records:
                resps.append(eng[r].GetRecords(recvs[r]))
            elif W == 2 and records:
                resps.append(eng[r].InsertRecords(recvs[r]))
            elif W == 1:
                v, st = eng[r].Get(recvs[r])
                resps.append(pk[r].respond(v, st).clone())
            else:
                k, v, o = pk[r].split(recvs[r], W)
                if W == 2:
                    resps.append(eng[r].Insert(k, v).clone())
                else:
                    gv, st = eng[r].Mixed(o, k, v)
                    resps.append(pk[r].respond(gv, st).clone())
        backs = ex.a2a(resps)
        for r in range(G):
            ops, keys, vals = streams[r][bi]
            vv, st = outs[r]
            pk[r].unpack(backs[r], 0 if W == 2 else 1, rows[r], vv, st)
            pk[r].end_call()
            if W == 2:
                assert np.array_equal(st.cpu().numpy(), g.insert(keys, vals)), (bi, r)
            elif W == 1:
                ov, os_ = g.get(keys)
                assert np.array_equal(st.cpu().numpy(), os_) and np.array_equal(vv.cpu().numpy().view(np.uint64), ov)
            else:
                ov, os_ = g.mixed(ops, keys, vals)
                assert np.array_equal(st.cpu().numpy(), os_) and np.array_equal(vv.cpu().numpy().view(np.uint64), ov)
    gd = g.dump()
    ks, vs = [], []
    for r in range(G):
        dd = eng[r].dump()
        ks.append(dd["keys"])
        vs.append(dd["values"])
        eng[r].close()
    assert np.array_equal(np.concatenate(ks), gd["keys"])
    assert np.array_equal(np.concatenate(vs), gd["values"])


def test_record_entry_points_equal_array_ones():
    """InsertRecords / GetRecords == Insert / Get on the same ops (statuses,
    values, final table), including reserved keys."""
    d = torch.device("cuda", 0)
    ops, keys, vals = S.insert_then_get(21, 30000, 3000)
    keys[[5, 77, 1234]] = INVALID
    ins_k, ins_v = keys[:30000], vals[:30000]
    a = P.CCEH(depth=4, max_batch=1 << 15, max_segments=2048)
    b = P.CCEH(depth=4, max_batch=1 << 15, max_segments=2048)
    sa = a.Insert(_t(ins_k).to(d), _t(ins_v).to(d))
    rec = torch.from_numpy(np.stack([ins_k, ins_v], axis=1).reshape(-1).view(np.int64)).to(d)
    sb = b.InsertRecords(rec)
    assert np.array_equal(sa.cpu().numpy(), sb.cpu().numpy())
    da, db = a.dump(), b.dump()
    assert np.array_equal(da["keys"], db["keys"]) and np.array_equal(da["values"], db["values"])
    gk = _t(keys[30000:]).to(d)
    v, st = a.Get(gk)
    resp = b.GetRecords(gk).view(-1, 2).cpu().numpy()
    assert np.array_equal(resp[:, 0], v.cpu().numpy())
    assert np.array_equal(resp[:, 1].astype(np.uint8), st.cpu().numpy())
    a.close()
    b.close()


@pytest.mark.parametrize("sbits", [0, 2])
def test_pack_keep_matches_restatement(sbits):
    """Keep mask (bloom-negatives stay home): same send blocks and rowpos as
    the CPU restatement; kept-home ops are ST_FILTERED, value 0, at once."""
    n = 50000
    keys, vals, ops = _batch(77 + sbits, n)
    keep = (np.random.default_rng(sbits).random(n) < 0.6).astype(np.uint8)
    hp, rp, outs = _pair(n, sbits, n)
    _, rowpos, rrow = _pack_both(hp, rp, outs, keys, vals, ops, 2, 0, keep=keep)
    hv, hs, rv, rs_ = outs
    resp = torch.arange(hp.rows * 2, dtype=torch.int64)
    hp.unpack(resp.to(torch.device("cuda", 0)), 1, rowpos, hv, hs)
    rp.unpack(resp, 1, rrow, rv, rs_)
    assert np.array_equal(hs.cpu().numpy(), rs_.numpy()) and np.array_equal(hv.cpu().numpy(), rv.numpy())
    assert np.all(hs.cpu().numpy()[keep == 0] == P.ST_FILTERED)
    assert np.all(hv.cpu().numpy()[keep == 0] == 0)


def test_block_router_bloom_get_one_gpu():
    """BlockRouter.bloom_get on one GPU with the HIP packer, bloom and index:
    equals the fused single-GPU probe_then_get."""
    from pmdfc_amd.dist import BlockRouter
    B = 1 << 16
    pk = P.BlockPacker(0, B, 0)
    idx = P.CCEH(depth=8, max_batch=pk.rows, max_segments=4096)
    r = BlockRouter(idx, pk)
    bf = P.BloomFilter(1 << 20, 4)
    keys = np.array(S.uniform_keys(90, 0, B), dtype=np.uint64)
    d = torch.device("cuda", 0)
    kd = _t(keys).to(d)
    idx.Insert(kd, kd)
    bf.add(kd)
    q = _t(np.concatenate([keys[: B // 2], np.array(S.uniform_keys(91, 0, B // 2), dtype=np.uint64)])).to(d)
    v, st = r.bloom_get(bf, q)
    v2, st2 = bf.probe_then_get(idx, q)
    assert torch.equal(st, st2) and torch.equal(v, v2)
    assert int((st == P.ST_FILTERED).sum()) > B // 4


def _native_pair(B, cap=None, depth=8, segs=1 << 14):
    """(index + native router, index + Python router) with the same packer shape"""
    from pmdfc_amd.dist import BlockRouter
    pk_n = P.BlockPacker(0, B, 0, cap=cap)
    pk_p = P.BlockPacker(0, B, 0, cap=cap)
    idx_n = P.CCEH(depth=depth, max_batch=pk_n.rows, max_segments=segs)
    idx_p = P.CCEH(depth=depth, max_batch=pk_p.rows, max_segments=segs)
    comm = P.Comm(0)
    return BlockRouter(idx_n, pk_n, comm=comm), BlockRouter(idx_p, pk_p), comm


@pytest.mark.parametrize("cap", [None, 7000])
def test_native_routed_batches_equal_python_loop(cap):
    """pmdfc_route_batches (the whole routed call in C++ over a one-rank RCCL
    communicator) against BlockRouter's Python loop on the same batches:
    identical statuses and Get results, and both equal a direct engine; with
    cap < batch every exchange carries ops (FIFO, so the same serial order)
    and the call ends with drains."""
    B, nb = 1 << 13, 6
    rn, rp, _ = _native_pair(B, cap=cap)
    d = torch.device("cuda", 0)
    keys = [_t(np.array(S.uniform_keys(300 + i, 0, B), dtype=np.uint64)).to(d) for i in range(nb)]
    keys[2][:7] = keys[1][:7]  # repeats across batches: the second insert of a key is stored again
    st_n = rn.insert_batches([(k, k) for k in keys])
    st_p = rp.insert_batches([(k, k) for k in keys])
    direct = P.CCEH(depth=8, max_batch=B, max_segments=1 << 14)
    for a, b, k in zip(st_n, st_p, keys):
        assert torch.equal(a, b)
        assert torch.equal(a, direct.Insert(k, k))
    q = [torch.cat([k[: B // 2], _t(np.array(S.uniform_keys(400 + i, 0, B // 2), dtype=np.uint64)).to(d)])
         for i, k in enumerate(keys)]
    g_n = rn.get_batches(q)
    g_p = rp.get_batches(q)
    for (vn, sn), (vp, sp), qq in zip(g_n, g_p, q):
        vd, sd = direct.Get(qq)
        assert torch.equal(sn, sp) and torch.equal(vn, vp)
        assert torch.equal(sn, sd) and torch.equal(vn, vd)
    assert int(sum((s == P.ST_HIT).sum() for _, s in g_n)) == nb * B // 2


def test_native_routed_gets_dedupe_hot_keys():
    """Gets with hot keys through the native loop with dedupe on: every Get
    equals the direct engine's answer."""
    B = 1 << 13
    rn, _, _ = _native_pair(B)
    d = torch.device("cuda", 0)
    base = np.array(S.uniform_keys(500, 0, B), dtype=np.uint64)
    kd = _t(base).to(d)
    rn.insert_batches([(kd, kd)])
    rng = np.random.default_rng(5)
    hot = base[rng.integers(0, 16, B)]  # 16 hot keys
    qd = _t(np.where(rng.random(B) < 0.7, hot, np.array(S.uniform_keys(501, 0, B), dtype=np.uint64))).to(d)
    (v, s), = rn.get_batches([qd])
    direct = P.CCEH(depth=8, max_batch=B, max_segments=1 << 14)
    direct.Insert(kd, kd)
    vd, sd = direct.Get(qd)
    assert torch.equal(s, sd) and torch.equal(v, vd)


@pytest.mark.parametrize("cap", [None, 7000])
def test_native_routed_mixed_equal_python_loop(cap):
    """pmdfc_route_mixed_batches against BlockRouter's Python loop on the same
    50/50 mixed batches (fresh inserts, repeats, Gets of stored, absent and
    same-batch keys): identical values and statuses, and both equal a direct
    engine taking the batches in order; cap < batch forces carries and drains."""
    B, nb = 1 << 13, 5
    rn, rp, _ = _native_pair(B, cap=cap)
    d = torch.device("cuda", 0)
    rng = np.random.default_rng(17)
    stored = np.zeros(0, dtype=np.uint64)
    batches = []
    for i in range(nb):
        fresh = np.array(S.uniform_keys(600 + i, 0, B), dtype=np.uint64)
        absent = np.array(S.uniform_keys(700 + i, 0, B), dtype=np.uint64)
        ops = (rng.random(B) < 0.5).astype(np.uint8)  # 1: Insert, 0: Get
        keys = fresh.copy()
        if stored.size:
            old = stored[rng.integers(0, stored.size, B)]
            pick = rng.random(B)
            keys = np.where(ops == 0, np.where(pick < 0.6, old, np.where(pick < 0.8, absent, fresh)), keys)
            keys = np.where((ops == 1) & (pick < 0.05), old, keys)  # an insert of a stored key
        vals = np.array(S.uniform_keys(800 + i, 0, B), dtype=np.uint64)
        stored = np.concatenate([stored, keys[ops == 1]])
        batches.append((_t(keys).to(d), _t(vals).to(d), torch.from_numpy(ops).to(d)))
    out_n = rn.mixed_batches(batches)
    out_p = rp.mixed_batches(batches)
    direct = P.CCEH(depth=8, max_batch=B, max_segments=1 << 14)
    for (vn, sn), (vp, sp), (k, v, o) in zip(out_n, out_p, batches):
        vd, sd = direct.Mixed(o, k, v)
        assert torch.equal(sn, sp) and torch.equal(vn, vp)
        assert torch.equal(sn, sd) and torch.equal(vn, vd)
    assert int(sum((s == P.ST_HIT).sum() for _, s in out_n)) > nb * B // 8
