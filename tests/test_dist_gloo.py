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


def test_block_router_overflow_single_rank():
    """An op whose owner block is full comes back ST_ROUTE_OVERFLOW and is not
    applied; the ops that fit are applied in batch order (world 1, no
    process group: the exchange is the identity)."""
    from pmdfc_amd.dist import BlockRouter
    from route_ref import ST_ROUTE_OVERFLOW, TorchBlockPacker
    idx = OracleIndex(4)
    pk = TorchBlockPacker(1000, 0, cap=600)
    r = BlockRouter(idx, pk)
    _, keys, vals = S.insert_then_get(5, 1000, 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64))
    st = r.insert(t(keys[:1000]), t(vals[:1000])).numpy()
    assert (st[:600] == O.ST_INSERTED).all() and (st[600:] == ST_ROUTE_OVERFLOW).all()
    g = O.OracleCCEH(4)
    g.insert(keys[:600], vals[:600])
    assert np.array_equal(g.dump()["keys"], idx.o.dump()["keys"])
    v, st = r.get(t(keys[:1000]))
    assert (st.numpy()[:600] == O.ST_HIT).all() and (st.numpy()[600:] == ST_ROUTE_OVERFLOW).all()
    assert np.array_equal(v.numpy()[:600].view(np.uint64), vals[:600])


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
