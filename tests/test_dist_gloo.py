"""The N>1 exchange protocol (pmdfc_amd/dist.py) on CPU with gloo, world 2 and 4.

Each rank owns the hash-prefix shard `rank`; its local index is the oracle
(CPU restatement) standing in for the GPU engine, the bucketing is a numpy
stable sort by owner.  The routed result must equal ONE serial oracle run on
the rank-major concatenation of all ranks' batches (the global batch order
dist.py promises), and the union of the shards must equal that global table.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import scenarios as S
from oracle import oracle as O
from pmdfc_amd.workload import uniform_keys


class OracleIndex:
    """Oracle behind the same batched interface as pmdfc_amd.CCEH (torch CPU tensors)."""

    def __init__(self, depth):
        self.o = O.OracleCCEH(depth)

    @staticmethod
    def _u(t):
        return t.numpy().view(np.uint64)

    def Insert(self, k, v):
        return torch.from_numpy(self.o.insert(self._u(k), self._u(v)))

    def Get(self, k):
        v, s = self.o.get(self._u(k))
        return torch.from_numpy(v.view(np.int64)), torch.from_numpy(s)

    def Mixed(self, ops, k, v):
        out, s = self.o.mixed(ops.numpy(), self._u(k), self._u(v))
        return torch.from_numpy(out.view(np.int64)), torch.from_numpy(s)


def bucket_np(sbits):
    def f(keys):
        h = O.hash64(keys.numpy().view(np.uint64))
        own = (h >> np.uint64(64 - sbits)).astype(np.int64)
        perm = np.argsort(own, kind="stable")
        return torch.from_numpy(perm), np.bincount(own, minlength=1 << sbits).tolist()
    return f


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, depth, streams, q, kind="sorted"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pmdfc_amd.dist import BlockRouter, ShardRouter
    sbits = world.bit_length() - 1
    idx = OracleIndex(depth)
    if kind.startswith("block"):
        from route_ref import TorchBlockPacker
        r = BlockRouter(idx, TorchBlockPacker(4096, sbits))
    else:
        r = ShardRouter(idx, sbits, bucket_np(sbits))
    outs = []
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64))
    if kind == "block_pipe":  # runs of same-kind batches through the pipelined calls
        i = 0
        st = streams[rank]
        while i < len(st):
            j = i
            while j < len(st) and type(st[j][0]) is type(st[i][0]):
                j += 1
            run = st[i:j]
            if run[0][0] is None:
                for s_ in r.insert_batches([(t(k), t(v)) for _, k, v in run]):
                    outs.append(("ins", s_.numpy().copy()))
            elif isinstance(run[0][0], str):
                for v, s_ in r.get_batches([t(k) for _, k, _ in run]):
                    outs.append(("get", v.numpy().view(np.uint64).copy(), s_.numpy().copy()))
            else:
                for v, s_ in r.mixed_batches([(t(k), t(v), torch.from_numpy(o)) for o, k, v in run]):
                    outs.append(("mix", v.numpy().view(np.uint64).copy(), s_.numpy().copy()))
            i = j
        streams = {rank: []}
    for ops, keys, vals in streams[rank]:
        if ops is None:
            st = r.insert(t(keys), t(vals))
            outs.append(("ins", st.numpy().copy()))
        elif isinstance(ops, str):
            v, st = r.get(t(keys))
            outs.append(("get", v.numpy().view(np.uint64).copy(), st.numpy().copy()))
        else:
            v, st = r.mixed(torch.from_numpy(ops), t(keys), t(vals))
            outs.append(("mix", v.numpy().view(np.uint64).copy(), st.numpy().copy()))
    d = idx.o.dump()
    q.put((rank, outs, d["keys"], d["values"], d["local_depth"], d["prefix"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["sorted", "block", "block_pipe"])
@pytest.mark.parametrize("world", [2, 4])
def test_routed_batches_equal_global_serial(world, kind):
    """kind "sorted": ShardRouter (variable splits, counts on the host);
    "block": BlockRouter (fixed-capacity owner blocks, equal splits, no host
    sync) with the CPU restatement of route.hip's packer; "block_pipe": the
    same through insert_batches / mixed_batches / get_batches (async
    all-to-alls, batch i+1 in flight while batch i is applied)."""
    depth = 6
    # per rank: insert batches, mixed batches, get batches
    streams = []
    for r in range(world):
        ops, keys, vals = S.mixed(100 + r, 3000, 0.6)
        ops2, keys2, vals2 = S.mixed(500 + r, 2000, 0.5)
        ins = S.insert_then_get(200 + r, 3000, 0)
        streams.append([(None, ins[1][:2000], ins[2][:2000]), (None, ins[1][2000:3000], ins[2][2000:3000]),
                        (ops, keys, vals), (ops2, keys2, vals2),
                        ("get", np.concatenate([ins[1][:2000], keys[:500]]), None),
                        ("get", np.concatenate([keys2[:700], ins[1][2500:3000]]), None)])
    nbatch = len(streams[0])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, depth, streams, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, outs, k, v, ld, pf = q.get(timeout=120)
        res[rank] = (outs, k, v, ld, pf)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # global serial reference: batch i of every rank, rank-major
    g = O.OracleCCEH(depth)
    for bi in range(nbatch):
        for r in range(world):
            ops, keys, vals = streams[r][bi]
            if ops is None:
                st = g.insert(keys, vals)
                assert np.array_equal(res[r][0][bi][1], st)
            elif isinstance(ops, str):
                v, st = g.get(keys)
                assert np.array_equal(res[r][0][bi][1], v) and np.array_equal(res[r][0][bi][2], st)
            else:
                v, st = g.mixed(ops, keys, vals)
                assert np.array_equal(res[r][0][bi][1], v) and np.array_equal(res[r][0][bi][2], st)
    # NB: within one step every rank's batch goes before the next step's, so
    # the serial order is step-major then rank-major, as applied above.
    gd = g.dump()
    sbits = world.bit_length() - 1
    ks, vs = [], []
    for r in range(world):
        _, k, v, ld, pf = res[r]
        own = (pf.astype(np.uint64) >> (ld.astype(np.uint64) - np.uint64(sbits))) == np.uint64(r)
        k = k.reshape(-1, 1024)[own]
        v = v.reshape(-1, 1024)[own]
        ks.append(k.ravel())
        vs.append(v.ravel())
    assert np.array_equal(np.concatenate(ks), gd["keys"])
    assert np.array_equal(np.concatenate(vs), gd["values"])


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int64))


def test_block_router_carry_single_rank():
    """An owner block that fills up leaves the rest in the carry; the call
    drains it, so every op is applied, in batch order (world 1, no process
    group: the exchange is the identity)."""
    from pmdfc_amd.dist import BlockRouter
    from route_ref import ST_ROUTE_OVERFLOW, TorchBlockPacker
    idx = OracleIndex(4)
    pk = TorchBlockPacker(1000, 0, cap=256)
    r = BlockRouter(idx, pk)
    _, keys, vals = S.insert_then_get(5, 1000, 0)
    st = r.insert(_t(keys[:1000]), _t(vals[:1000])).numpy()
    g = O.OracleCCEH(4)
    assert np.array_equal(st, g.insert(keys[:1000], vals[:1000]))
    assert np.array_equal(g.dump()["keys"], idx.o.dump()["keys"])
    v, st = r.get(_t(keys[:1000]))
    assert (st.numpy() == O.ST_HIT).all() and np.array_equal(v.numpy().view(np.uint64), vals[:1000])
    assert not (st.numpy() == ST_ROUTE_OVERFLOW).any() and int(pk.carried()[0]) == 0


def test_block_router_full_carry_single_rank():
    """Ops that find the carry full (carry_cap ops waiting) come back
    ST_ROUTE_OVERFLOW unapplied -- the queue positions past cap + carry_cap
    -- and a strict router raises."""
    from pmdfc_amd.dist import BlockRouter, RouteOverflowError
    from route_ref import ST_ROUTE_OVERFLOW, TorchBlockPacker
    idx = OracleIndex(4)
    r = BlockRouter(idx, TorchBlockPacker(1000, 0, cap=300, carry_cap=200))
    _, keys, vals = S.insert_then_get(5, 1000, 0)
    st = r.insert(_t(keys[:1000]), _t(vals[:1000])).numpy()
    assert (st[:500] == O.ST_INSERTED).all() and (st[500:] == ST_ROUTE_OVERFLOW).all()
    g = O.OracleCCEH(4)
    g.insert(keys[:500], vals[:500])
    assert np.array_equal(g.dump()["keys"], idx.o.dump()["keys"])
    rs = BlockRouter(OracleIndex(4), TorchBlockPacker(1000, 0, cap=300, carry_cap=200), strict=True)
    with pytest.raises(RouteOverflowError):
        rs.insert(_t(keys[:1000]), _t(vals[:1000]))


def _owner_skewed(seed, n, sbits, hot_owner, frac):
    """n distinct keys, `frac` of them owned by `hot_owner`: owner skew with
    no repeated key (what dedupe cannot remove)."""
    from route_ref import owners
    k = uniform_keys(seed, 0, 8 * n)
    own = owners(k, sbits)
    hot = k[own == hot_owner]
    cold = k[own != hot_owner]
    nh = int(n * frac)
    out = np.concatenate([hot[:nh], cold[:n - nh]])
    return out[np.random.default_rng(seed).permutation(n)]


def _skew_worker(rank, world, port, streams, cap, carry_cap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pmdfc_amd.dist import BlockRouter
    from route_ref import TorchBlockPacker
    sbits = world.bit_length() - 1
    idx = OracleIndex(6)
    pk = TorchBlockPacker(4096, sbits, cap=cap, carry_cap=carry_cap)
    r = BlockRouter(idx, pk)
    outs = []
    mine = streams[rank]
    if isinstance(mine[0][0], str):
        for v, st in r.get_batches([_t(k) for _, k, _ in mine]):
            outs.append((v.numpy().view(np.uint64).copy(), st.numpy().copy()))
    else:
        for v, st in r.mixed_batches([(_t(k), _t(v), torch.from_numpy(o)) for o, k, v in mine]):
            outs.append((v.numpy().view(np.uint64).copy(), st.numpy().copy()))
    d = idx.o.dump()
    q.put((rank, outs, d["keys"], d["values"], d["local_depth"], d["prefix"], int(pk.carried()[0])))
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(target, world, args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        out = q.get(timeout=240)
        res[out[0]] = out[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _shards_equal(res, world, g):
    gd = g.dump()
    sbits = world.bit_length() - 1
    ks, vs = [], []
    for r in range(world):
        _, k, v, ld, pf, _ = res[r]
        own = (pf.astype(np.uint64) >> (ld.astype(np.uint64) - np.uint64(sbits))) == np.uint64(r)
        ks.append(k.reshape(-1, 1024)[own].ravel())
        vs.append(v.reshape(-1, 1024)[own].ravel())
    return np.array_equal(np.concatenate(ks), gd["keys"]) and np.array_equal(np.concatenate(vs), gd["values"])


@pytest.mark.parametrize("cap", [None, 600])
def test_block_router_owner_skew_world4(cap):
    """World 4, mixed batches whose keys pile onto owner 0 (60% of every
    rank's distinct keys): owner 0's blocks overflow, the rest waits in the
    carries and drains.  No op comes back ST_ROUTE_OVERFLOW, and every result
    and the union of the shards equal ONE serial oracle run in the order the
    protocol promises (tests/route_ref.py serial_order, restated from the
    queues, not from the packer).  cap 600 forces several carried exchanges
    per batch."""
    from route_ref import ST_ROUTE_OVERFLOW, route_capacity, serial_order
    world, sbits, nb, n = 4, 2, 3, 3000
    capv = cap or route_capacity(4096, sbits)
    streams = []
    for r in range(world):
        bs = []
        for e in range(nb):
            keys = _owner_skewed(700 + 10 * r + e, n, sbits, 0, 0.6)
            rng = np.random.default_rng(900 + 10 * r + e)
            ops = (rng.random(n) < 0.5).astype(np.uint8)
            # Gets of this rank's earlier keys (hits), of its later keys (misses
            # or read-after-write), of other ranks' keys (cross-rank order)
            pool = np.concatenate([keys, _owner_skewed(700 + 10 * ((r + 1) % world) + e, n, sbits, 0, 0.6)])
            gk = pool[rng.integers(0, pool.size, n)]
            keys = np.where(ops == 1, keys, gk)
            vals = np.where(ops == 1, S._vals(keys), np.uint64(0))
            bs.append((ops, keys, vals))
        streams.append(bs)
    res = _run_ranks(_skew_worker, world, (streams, capv, None))
    order, dropped = serial_order([[b[1] for b in streams[r]] for r in range(world)], sbits, capv, 4096)
    assert not dropped
    if cap:
        assert len(order) == world * nb * n
    g = O.OracleCCEH(6)
    o = np.array([streams[r][e][0][i] for r, e, i in order], np.uint8)
    k = np.array([streams[r][e][1][i] for r, e, i in order], np.uint64)
    v = np.array([streams[r][e][2][i] for r, e, i in order], np.uint64)
    gv, gs = g.mixed(o, k, v)
    exp = {(r, e): (np.zeros(n, np.uint64), np.zeros(n, np.uint8)) for r in range(world) for e in range(nb)}
    for j, (r, e, i) in enumerate(order):
        exp[(r, e)][0][i] = gv[j]
        exp[(r, e)][1][i] = gs[j]
    for r in range(world):
        assert res[r][5] == 0  # carries drained
        for e in range(nb):
            got_v, got_s = res[r][0][e]
            assert not (got_s == ST_ROUTE_OVERFLOW).any()
            assert np.array_equal(got_s, exp[(r, e)][1]), (r, e)
            assert np.array_equal(got_v, exp[(r, e)][0]), (r, e)
    assert _shards_equal(res, world, g)


def test_block_router_zipf_gets_world4():
    """World 4, Zipf(0.99) Gets (SURVEY §8d config 3's skew) over keys all
    ranks inserted: Get dedupe routes one row per distinct key, so the hot
    keys' owners do not overflow; the results equal one serial oracle (a
    Get-only batch changes nothing) with no ST_ROUTE_OVERFLOW."""
    from pmdfc_amd.workload import zipf_ranks
    from route_ref import ST_ROUTE_OVERFLOW
    world, nb, n = 4, 3, 4096
    base = [uniform_keys(300 + r, 0, 2500) for r in range(world)]
    allk = np.concatenate(base)
    ins = [[(np.ones(2500, np.uint8), base[r], S._vals(base[r]))] for r in range(world)]
    rng = np.random.default_rng(5)
    pool = np.concatenate([allk, uniform_keys(999, 0, 500)])  # some absent keys
    gets = [[("get", pool[zipf_ranks(rng, pool.size, 0.99, n)], None) for _ in range(nb)] for _ in range(world)]
    res = _run_ranks(_zipf_worker, world, (ins, gets))
    g = O.OracleCCEH(6)
    for r in range(world):
        g.insert(base[r], S._vals(base[r]))
    hot = 0
    for r in range(world):
        for e in range(nb):
            keys = gets[r][e][1]
            ev, es = g.get(keys)
            got_v, got_s = res[r][0][e]
            assert not (got_s == ST_ROUTE_OVERFLOW).any()
            assert np.array_equal(got_s, es) and np.array_equal(got_v, ev)
            hot = max(hot, np.unique(keys, return_counts=True)[1].max())
        assert res[r][1] == 0  # no exchange needed a carry: dedupe kept the blocks within cap
    assert hot > n // 20  # the hottest key really is hot


def _zipf_worker(rank, world, port, ins, gets, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pmdfc_amd.dist import BlockRouter
    from route_ref import TorchBlockPacker
    from route_ref import route_capacity
    sbits = world.bit_length() - 1
    idx = OracleIndex(6)
    pk = TorchBlockPacker(4096, sbits, cap=route_capacity(4096, sbits) // 2)  # little slack for a hot key
    r = BlockRouter(idx, pk)
    r.mixed_batches([(_t(k), _t(v), torch.from_numpy(o)) for o, k, v in ins[rank]])
    outs = []
    carried_any = 0

    class Spy:  # records whether any exchange of the Get call left ops in a carry
        def __init__(self, p):
            self.p = p

        def __getattr__(self, a):
            return getattr(self.p, a)

        def pack(self, *a, **kw):
            out = self.p.pack(*a, **kw)
            nonlocal carried_any
            carried_any += int(self.p.carried()[0])
            return out

    r.p = Spy(pk)
    for v, st in r.get_batches([_t(k) for _, k, _ in gets[rank]]):
        outs.append((v.numpy().view(np.uint64).copy(), st.numpy().copy()))
    q.put((rank, outs, carried_any))
    dist.barrier()
    dist.destroy_process_group()


class CPUBloom:
    """Replicated client bloom filter (the oracle's client/bloom_filter.c
    restatement) with the probe() interface BlockRouter.bloom_get expects."""

    def __init__(self, keys, nbits=1 << 16, k=4):
        self.bm = np.zeros((nbits + 63) // 64, np.uint64)
        self.nbits, self.k = nbits, k
        O.bloom_add(self.bm, nbits, k, keys)

    def probe(self, keys):
        out, _ = O.bloom_check(self.bm, self.nbits, self.k, keys.numpy().view(np.uint64))
        return torch.from_numpy(out)


def _bloom_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pmdfc_amd.dist import BlockRouter
    from route_ref import TorchBlockPacker
    sbits = world.bit_length() - 1
    idx = OracleIndex(4)
    r = BlockRouter(idx, TorchBlockPacker(4096, sbits))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64))
    mine = uniform_keys(500 + rank, 0, 3000)
    r.insert(t(mine), t(mine))
    allk = np.concatenate([uniform_keys(500 + i, 0, 3000) for i in range(world)])
    bf = CPUBloom(allk)
    qk = np.concatenate([allk[rank::world][:1500], uniform_keys(600 + rank, 0, 1500)])
    v, st = r.bloom_get(bf, t(qk))
    q.put((rank, qk, v.numpy().view(np.uint64).copy(), st.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_block_router_bloom_get_world2():
    """bloom-negatives stay home (ST_FILTERED, no exchange); the
    rest are routed Gets equal to one serial oracle over all ranks' inserts."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bloom_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    allk = np.concatenate([uniform_keys(500 + i, 0, 3000) for i in range(world)])
    o = O.OracleCCEH(4)
    o.insert(allk, allk)
    bm = np.zeros((1 << 16) // 64, np.uint64)
    O.bloom_add(bm, 1 << 16, 4, allk)
    for rank, qk, v, st in res:
        pos, _ = O.bloom_check(bm, 1 << 16, 4, qk)
        ov, os_ = o.get(qk)
        assert np.all(st[pos == 0] == 7) and np.all(v[pos == 0] == 0)
        assert np.array_equal(st[pos == 1], os_[pos == 1]) and np.array_equal(v[pos == 1], ov[pos == 1])
        assert (pos == 0).sum() > 100 and np.all(st[:1500] == O.ST_HIT)
