"""Fixed-capacity routing (route.hip, the N>1 path of bench.py) on one GPU.

* the HIP packer against the CPU restatement (tests/route_ref.py): send
  buffers (records and INVALID padding), positions and overflow, bit-exact,
  for 1..16 owners, widths 1..3, reserved keys and ragged tile tails;
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


@pytest.mark.parametrize("sbits", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("width", [1, 2, 3])
@pytest.mark.parametrize("n", [1, 4095, 4097, 50000])
def test_pack_matches_restatement(sbits, width, n):
    keys, vals, ops = _batch(sbits * 100 + width * 10 + n % 7, n)
    hp = P.BlockPacker(0, 65536, sbits)
    rp = TorchBlockPacker(65536, sbits, cap=hp.cap)
    d = torch.device("cuda", 0)
    send, pos = hp.pack(_t(keys).to(d), _t(vals).to(d) if width > 1 else None,
                        torch.from_numpy(ops).to(d) if width > 2 else None, width)
    rs, rpos = rp.pack(_t(keys), _t(vals), torch.from_numpy(ops), width)
    assert np.array_equal(send.cpu().numpy(), rs.numpy())
    assert np.array_equal(pos.cpu().numpy(), rpos.numpy())
    assert not hp.overflowed()


@pytest.mark.parametrize("sbits", [0, 2, 4])
def test_pack_reused_across_batch_sizes(sbits):
    """One packer over a run of ragged batch sizes: k_route_count's in-place
    tile scan (done counter left at 0 for the next pack, several tiles per scan
    thread at 1000+ tiles) matches the restatement on every call."""
    hp = P.BlockPacker(0, 1 << 20, sbits)
    rp = TorchBlockPacker(1 << 20, sbits, cap=hp.cap)
    d = torch.device("cuda", 0)
    for i, n in enumerate([50000, 1, 1 << 20, 4097, 0, 777777, 1025]):
        keys, vals, ops = _batch(900 + sbits * 10 + i, n)
        send, pos = hp.pack(_t(keys).to(d), _t(vals).to(d), None, 2)
        rs, rpos = rp.pack(_t(keys), _t(vals), None, 2)
        assert np.array_equal(send.cpu().numpy(), rs.numpy()), n
        assert np.array_equal(pos.cpu().numpy(), rpos.numpy()), n
        assert not hp.overflowed()


@pytest.mark.parametrize("sbits", [1, 3])
def test_pack_overflow(sbits):
    n = 40000
    keys, vals, ops = _batch(11 + sbits, n)
    cap = (n >> sbits) - 300  # every owner block overflows
    hp = P.BlockPacker(0, n, sbits, cap=cap)
    rp = TorchBlockPacker(n, sbits, cap=cap)
    d = torch.device("cuda", 0)
    send, pos = hp.pack(_t(keys).to(d), _t(vals).to(d), None, 2)
    rs, rpos = rp.pack(_t(keys), _t(vals), None, 2)
    assert np.array_equal(send.cpu().numpy(), rs.numpy())
    assert np.array_equal(pos.cpu().numpy(), rpos.numpy())
    assert hp.overflowed() and (rpos.numpy() < 0).sum() > 0
    st = (np.arange(hp.rows) % 9).astype(np.uint8)  # any status but ROUTE_OVERFLOW
    _, a = hp.unpack(torch.from_numpy(st).to(d), 0, pos, n)
    _, b = rp.unpack(torch.from_numpy(st), 0, rpos, n)
    assert np.array_equal(a.cpu().numpy(), b.numpy())
    assert (a.cpu().numpy() == P.ST_ROUTE_OVERFLOW).sum() == (rpos.numpy() < 0).sum()


def test_split_respond_unpack_match_restatement():
    sbits, n = 2, 30000
    keys, vals, ops = _batch(3, n)
    d = torch.device("cuda", 0)
    hp = P.BlockPacker(0, n, sbits)
    rp = TorchBlockPacker(n, sbits, cap=hp.cap)
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
    _, pos = hp.pack(_t(keys).to(d), None, None, 1)
    _, rpos = rp.pack(_t(keys), None, None, 1)
    hv2, hs2 = hp.unpack(hr, 1, pos, n)
    rv2, rs2 = rp.unpack(rr, 1, rpos, n)
    assert np.array_equal(hv2.cpu().numpy(), rv2.numpy())
    assert np.array_equal(hs2.cpu().numpy(), rs2.numpy())


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
        sends, poss = [], []
        for r in range(G):
            ops, keys, vals = streams[r][bi]
            s, p = pk[r].pack(_t(keys).to(d), _t(vals).to(d) if W > 1 else None,
                              torch.from_numpy(ops).to(d) if W > 2 else None, W)
            sends.append(s.clone())
            poss.append(p.clone())
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
            vv, st = pk[r].unpack(backs[r], 0 if W == 2 else 1, poss[r], keys.size)
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
    """Keep mask (bloom-negatives stay home): same send blocks and pos as the
    CPU restatement, kept-home ops unpack as ST_FILTERED."""
    n = 50000
    keys, vals, ops = _batch(77 + sbits, n)
    keep = (np.random.default_rng(sbits).random(n) < 0.6).astype(np.uint8)
    hp = P.BlockPacker(0, n, sbits)
    rp = TorchBlockPacker(n, sbits, cap=hp.cap)
    d = torch.device("cuda", 0)
    send, pos = hp.pack(_t(keys).to(d), _t(vals).to(d), None, 2, keep=torch.from_numpy(keep).to(d))
    rs, rpos = rp.pack(_t(keys), _t(vals), None, 2, keep=keep)
    assert np.array_equal(send.cpu().numpy(), rs.numpy())
    assert np.array_equal(pos.cpu().numpy(), rpos.numpy())
    resp = torch.arange(hp.rows * 2, dtype=torch.int64)
    v, st = hp.unpack(resp.to(d), 1, pos, n)
    v2, st2 = rp.unpack(resp, 1, rpos, n)
    assert np.array_equal(st.cpu().numpy(), st2.numpy()) and np.array_equal(v.cpu().numpy(), v2.numpy())
    assert np.all(st.cpu().numpy()[keep == 0] == P.ST_FILTERED)


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
