"""SURVEY §8d configs 3 and 4 at their full sizes on one MI355X, through the
same code paths bench.py times, checked by size-independent properties, plus
reduced variants bit-exact against the serial oracle.

* config 4, one shard of the 8-GPU job: 2^28 keys owned by shard 0 of 8
  (shard_bits = 3) preloaded, then 50/50 mixed batches of 1M, all routed by
  BlockRouter over a 1-rank RCCL process group (pack -> all_to_all_single ->
  the engine on the received rows -> all_to_all_single -> unpack);
* config 3: 2^28 replay-shape keys preloaded, mixed batches of 1M with 95 %
  Zipf(0.99) Gets and 5 % fresh Inserts.

Properties: every Get of a stored key hits with its value, every fresh
Insert is INSERTED, no op comes back ROUTE_OVERFLOW, the carries drain, the
fresh keys are all readable afterwards, no split dropped an entry, and the
stats agree with the op counts.
"""
import os
import socket

import numpy as np
import pytest

import scenarios as S
from oracle import oracle as O
from pmdfc_amd.workload import uniform_keys

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402

import pmdfc_amd as P  # noqa: E402
from pmdfc_amd.dist import BlockRouter  # noqa: E402


@pytest.fixture(scope="module")
def rccl1():
    """A 1-rank RCCL (backend "nccl") process group on GPU 0."""
    if dist.is_initialized():
        yield
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def _shard_keys(seed, n, sbits, shard, start=0, chunk=1 << 24):
    """The first n keys of the splitmix stream `seed` (from `start`) whose
    hash prefix is `shard`, on the GPU."""
    out, got, off = [], 0, start
    while got < n:
        k = P.gen_keys(seed, off, chunk)
        h = P.hash64(k)
        sel = k[(h >> (64 - sbits)) & ((1 << sbits) - 1) == shard] if sbits else k
        out.append(sel[: n - got])
        got += out[-1].numel()
        off += chunk
    return torch.cat(out), off


def _mixed_batches(pre, fresh, nb, B, seed):
    """nb batches of B: 50 % Gets of uniform preloaded keys, 50 % fresh
    Inserts (value = key)."""
    dev = pre.device
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    out, f = [], 0
    for _ in range(nb):
        is_ins = torch.rand(B, device=dev, generator=g) < 0.5
        r = torch.randint(0, pre.numel(), (B,), device=dev, generator=g)
        ni = int(is_ins.sum())
        k = pre[r].clone()
        k[is_ins] = fresh[f:f + ni]
        f += ni
        out.append((k, k, is_ins.to(torch.uint8)))
    return out, f


def test_config4_shard_full_size_routed(rccl1):
    """One config-4 shard at full size: 2^28 preloaded keys of shard 0 of 8,
    eight 50/50 mixed batches of 1M, routed over RCCL (1-rank group)."""
    B, n_pre, nb, sbits = 1 << 20, 1 << 28, 8, 3
    pre, nxt = _shard_keys(4000, n_pre, sbits, 0)
    fresh, _ = _shard_keys(4000, nb * B, sbits, 0, start=nxt)
    pk = P.BlockPacker(0, B, 0)
    idx = P.CCEH(65536, shard_bits=sbits, shard_id=0, max_batch=pk.rows,
                 max_segments=int((n_pre + nb * B) / 480) + 65536)
    r = BlockRouter(idx, pk, strict=True)
    for i in range(0, n_pre, 16 * B):
        sts = r.insert_batches([(pre[j:j + B], pre[j:j + B]) for j in range(i, min(n_pre, i + 16 * B), B)])
        assert all(bool((s == P.ST_INSERTED).all()) for s in sts)
    batches, nf = _mixed_batches(pre, fresh, nb, B, 7)
    outs = r.mixed_batches(batches)
    n_get = n_ins = 0
    for (k, _, o), (v, st) in zip(batches, outs):
        gm = o == 0
        assert bool(((st[gm] == P.ST_HIT) & (v[gm] == k[gm])).all())
        assert bool((st[~gm] == P.ST_INSERTED).all())
        n_get += int(gm.sum())
        n_ins += int((~gm).sum())
    assert n_ins == nf and n_get + n_ins == nb * B
    assert int(pk.carried().item()) == 0 and pk.overflow_count() == 0
    # every fresh key is readable through the routed Get path (deduped rows)
    for j in range(0, nf, B):
        v, st = r.get(fresh[j:min(nf, j + B)])
        assert bool((st == P.ST_HIT).all()) and torch.equal(v, fresh[j:min(nf, j + B)])
    # Gets of keys no one inserted miss; keys of another shard are refused
    other, _ = _shard_keys(4100, 4096, sbits, 5)
    absent, _ = _shard_keys(4200, 4096, sbits, 0)
    v, st = r.get(absent)
    assert bool((st == P.ST_MISS).all()) and bool((v == 0).all())
    st = idx.Get(other)[1]
    assert bool((st == P.ST_WRONG_SHARD).all())
    s = idx.stats()
    assert s["split_loss"] == 0 and s["error_flags"] == 0
    assert s["segments"] * 1024 >= n_pre + nf
    assert 30.0 < idx.Utilization() <= 100.0  # percent, as CCEH_hybrid.cpp:412-427
    idx.close()
    pk.close()


def test_config4_shard_reduced_vs_oracle(rccl1):
    """The same shard workload at oracle size: 2^20 preloaded shard-0 keys,
    four 50/50 mixed batches of 64k with read-after-write Gets of keys the
    batch inserts, routed over RCCL; every result and the shard's table equal
    the serial oracle's global table restricted to shard 0."""
    B, n_pre, nb, sbits, depth = 1 << 16, 1 << 20, 4, 3, 10
    pre, nxt = _shard_keys(4300, n_pre, sbits, 0)
    fresh, _ = _shard_keys(4300, nb * B, sbits, 0, start=nxt)
    pk = P.BlockPacker(0, B, 0)
    idx = P.CCEH(depth=depth, shard_bits=sbits, shard_id=0, max_batch=pk.rows, max_segments=1 << 14)
    o = O.OracleCCEH(depth)
    r = BlockRouter(idx, pk, strict=True)
    r.insert_batches([(pre[j:j + B], pre[j:j + B]) for j in range(0, n_pre, B)])
    pn = pre.cpu().numpy().view(np.uint64)
    o.insert(pn, pn)
    batches, _ = _mixed_batches(pre, fresh, nb, B, 8)
    rng = np.random.default_rng(8)
    for k, _, op in batches:  # Gets of keys the batch itself inserts (either side of the insert)
        ins = torch.nonzero(op).flatten()
        gets = torch.nonzero(op == 0).flatten()
        pick = torch.from_numpy(rng.integers(0, ins.numel(), 2000)).to(k.device)
        k[gets[:2000]] = k[ins[pick]]
    outs = r.mixed_batches([(k, k, op) for k, _, op in batches])
    for (k, _, op), (v, st) in zip(batches, outs):
        kn = k.cpu().numpy().view(np.uint64)
        ov, os_ = o.mixed(op.cpu().numpy(), kn, kn)
        assert np.array_equal(st.cpu().numpy(), os_)
        assert np.array_equal(v.cpu().numpy().view(np.uint64), ov)
    d, od = idx.dump(), o.dump()
    own = (od["prefix"].astype(np.uint64) >> (od["local_depth"].astype(np.uint64) - np.uint64(sbits))) == 0
    assert np.array_equal(d["keys"], od["keys"].reshape(-1, 1024)[own].ravel())
    assert np.array_equal(d["values"], od["values"].reshape(-1, 1024)[own].ravel())
    idx.close()
    pk.close()


def test_config3_full_size(tmp_path):
    """Config 3 at full size on one GPU: 2^28 replay-shape keys preloaded,
    four mixed batches of 1M (95 % Zipf(0.99) Gets over the preloaded ranks,
    5 % fresh Inserts), then every fresh key read back."""
    from pmdfc_amd.workload import scramble, zipf_ranks
    dev = torch.device("cuda", 0)
    B, n_pre = 1 << 20, 1 << 28

    def rkey(rank):
        return ((1 + (rank >> 8)) << 32) + ((rank & 255) << 12)

    idx = P.CCEH(65536, max_batch=B, max_segments=int(n_pre / 500) + 65536 + 262144)
    for off in range(0, n_pre, B):
        k = rkey(torch.arange(off, off + B, dtype=torch.int64, device=dev))
        st = idx.Insert(k, k)
        if off % (64 * B) == 0:
            assert bool((st == P.ST_INSERTED).all())
    s0 = idx.stats()
    rng = np.random.default_rng(3)
    fresh = 0
    hot_hits = 0
    all_fresh = []
    for _ in range(4):
        is_ins = rng.random(B) < 0.05
        r = scramble(zipf_ranks(rng, n_pre, 0.99, B), n_pre, 33)
        nf = int(is_ins.sum())
        r[is_ins] = n_pre + fresh + np.arange(nf)
        fresh += nf
        k = rkey(torch.from_numpy(r).to(dev))
        op = torch.from_numpy(is_ins.astype(np.uint8)).to(dev)
        v, st = idx.Mixed(op, k, k)
        g = op == 0
        assert bool(((st[g] == P.ST_HIT) & (v[g] == k[g])).all())
        assert bool((st[~g] == P.ST_INSERTED).all())
        hot_hits = max(hot_hits, int(np.unique(r[~is_ins], return_counts=True)[1].max()))
        all_fresh.append(k[~g])
    assert hot_hits > B // 100  # the Zipf head really is hot
    fk = torch.cat(all_fresh)
    assert fk.numel() == fresh
    v, st = idx.Get(fk)
    assert bool((st == P.ST_HIT).all()) and torch.equal(v, fk)
    s = idx.stats()
    assert s["split_loss"] == 0 and s["error_flags"] == 0
    assert s["segments"] >= s0["segments"] and s["segments"] * 1024 >= n_pre + fresh
    idx.close()


def test_config5_bloom_at_full_fill(rccl1):
    """Config 5 at its specified fill: the client filter (1e9
    bits, k = 4, MSB-first) built from config 2's 2^26 inserted keys -- fill
    1 - e^(-4 * 2^26 / 1e9) = 23.5 %, FPR 0.235^4 = 0.31 % -- and 1M probes, 50 %
    present / 50 % absent, fused ahead of the index Get (client/rdpma.c:
    1050-1061).  The bitmap equals the oracle's (client/bloom_filter.c:61-80)
    bit for bit, every probe equals the oracle's bloom_filter_check (:82-117),
    negatives never reach the index (ST_FILTERED), false positives miss in it,
    and the routed path (BlockRouter.bloom_get over a 1-rank RCCL group) gives
    the same answers as the fused kernel."""
    B, n, m, kh = 1 << 20, 1 << 26, 1000000000, 4
    keys = P.gen_keys(5, 0, n)
    pk = P.BlockPacker(0, B, 0)
    idx = P.CCEH(65536, max_batch=pk.rows, max_segments=1 << 18)
    st = idx.Insert(keys, keys)
    assert bool((st == P.ST_INSERTED).all())
    bf = P.BloomFilter(m, kh)
    bf.add(keys)
    bm = bf.bitmap()
    fill = int(np.unpackbits(bm.view(np.uint8)).sum()) / m
    assert abs(fill - (1 - np.exp(-kh * n / m))) < 0.002
    obm = np.zeros_like(bm)
    O.bloom_add(obm, m, kh, uniform_keys(5, 0, n))
    assert np.array_equal(bm, obm)
    del obm
    g = torch.Generator(device="cuda")
    g.manual_seed(55)
    present = keys[torch.randint(0, n, (B // 2,), device="cuda", generator=g)]
    absent = P.gen_keys(5, n, B // 2)
    qs = torch.cat([present, absent])[torch.randperm(B, device="cuda", generator=g)]
    qn = qs.cpu().numpy().view(np.uint64)
    pos, _ = O.bloom_check(bm, m, kh, qn)
    assert np.array_equal(bf.probe(qs).cpu().numpy(), pos)
    is_abs = np.isin(qn, absent.cpu().numpy().view(np.uint64))
    fpr = pos[is_abs].mean()
    assert 0.0022 < fpr < 0.004, fpr  # 0.235^4 = 0.0031
    v, s = bf.probe_then_get(idx, qs)
    v, s = v.cpu().numpy().view(np.uint64), s.cpu().numpy()
    assert np.all((s == P.ST_FILTERED) == (pos == 0))
    assert np.all(s[~is_abs] == P.ST_HIT) and np.array_equal(v[~is_abs], qn[~is_abs])
    assert np.all(s[is_abs & (pos == 1)] == P.ST_MISS) and not v[is_abs].any()
    rv, rs = BlockRouter(idx, pk, strict=True).bloom_get(bf, qs)
    assert np.array_equal(rs.cpu().numpy(), s) and np.array_equal(rv.cpu().numpy().view(np.uint64), v)
    idx.close()
    pk.close()
