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


def _worker(rank, world, port, depth, streams, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pmdfc_amd.dist import ShardRouter
    sbits = world.bit_length() - 1
    idx = OracleIndex(depth)
    r = ShardRouter(idx, sbits, bucket_np(sbits))
    outs = []
    for ops, keys, vals in streams[rank]:
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64))
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


@pytest.mark.parametrize("world", [2, 4])
def test_routed_batches_equal_global_serial(world):
    depth = 6
    rng = np.random.default_rng(world)
    # per rank: an insert batch, a mixed batch, a get batch
    streams = []
    for r in range(world):
        ops, keys, vals = S.mixed(100 + r, 3000, 0.6)
        ins = S.insert_then_get(200 + r, 2000, 0)
        streams.append([(None, ins[1][:2000], ins[2][:2000]), (ops, keys, vals),
                        ("get", np.concatenate([ins[1][:2000], keys[:500]]), None)])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, depth, streams, q)) for r in range(world)]
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
    for bi in range(3):
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
