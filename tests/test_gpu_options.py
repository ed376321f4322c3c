"""The engine's optional pass layouts, each in a child process with its
environment knob set (the engine reads them once per process): results equal
the serial oracle op by op and table by table, as the default layout's do in
test_gpu_parity.py.  The options are off by default because they measured
slower, not because they differ:
  PMDFC_SPLIT_TEAM_MAX=0        every split by one wave (no four-wave teams);
  PMDFC_SPLIT_TEAM_MAX=1000000  every split by a team of four waves;
  PMDFC_PIPE_GROUP=1            the insert pipeline with an event pair per batch.
(The round-5 fused layouts -- split round + parked pass, parked + final pass
-- measured slower and were removed in round 6.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys, numpy as np
sys.path.insert(0, "tests")
import scenarios as S
from oracle import oracle as O
import pmdfc_amd as P
scen = S.scenarios(O.hash64)
out = {}
for name, batch in (("cap2_ins100k", 1 << 14), ("cap256_ins400k", 1 << 16), ("mixed_cap16_60k", 10000),
                    ("split_loss", 1 << 12), ("dup_pairs", 9000)):
    init_cap, conv, ops, keys, vals = scen[name]
    n = keys.size
    t = P.CCEH(init_cap, convention=conv, max_batch=batch, max_segments=16384)
    o = O.OracleCCEH(t.initial_depth)
    ins = ops == S.OP_INSERT
    if ins.all() or (ins[: ins.sum()].all() and name != "mixed_cap16_60k"):
        k, v = keys[ins], vals[ins]
        st = t.InsertBatches(k, v, list(range(0, k.size, batch)) + [k.size])
        ost = o.insert(k, v)
        ok = bool(np.array_equal(st, ost))
        g = keys[~ins]
        if g.size:
            gv, gs = t.Get(g)
            ov, os_ = o.get(g)
            ok = ok and bool(np.array_equal(gv, ov) and np.array_equal(gs, os_))
    else:
        vo, st = t.MixedBatches(ops, keys, vals, list(range(0, n, batch)) + [n])
        ov, ost = o.mixed(ops, keys, vals)
        ok = bool(np.array_equal(st, ost) and np.array_equal(vo, ov))
    d, od = t.dump(), o.dump()
    ok = ok and d["depth"] == od["depth"] and all(np.array_equal(d[f], od[f]) for f in ("local_depth", "keys", "values"))
    ok = ok and t.stats()["error_flags"] == 0
    out[name] = ok
    t.close()
print(json.dumps(out))
'''


@pytest.mark.parametrize("env", [{"PMDFC_SPLIT_TEAM_MAX": "0"}, {"PMDFC_SPLIT_TEAM_MAX": "1000000"},
                                 {"PMDFC_PIPE_GROUP": "1"}])
def test_optional_layouts_match_oracle(env):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=REPO, env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert all(res.values()), (env, res)


# Mixed batches tell their Gets whether the batch inserts their key in one of
# two exact ways, chosen per batch from the last batch's insert count
# (cceh_engine.hip mixed_join_mode): the insert set, or the Get-side join.
# Each forced for every batch, over the mixed fixture streams at three batch
# cuttings (every op and the final table against the serial oracle), plus a
# stream whose Gets hit wrapping windows of keys the same batch re-inserts
# and misses of keys inserted once or twice in the batch (the join's cases).
CHILD_MIXED = r'''
import json, sys, numpy as np
sys.path.insert(0, "tests")
import scenarios as S
from oracle import oracle as O
import pmdfc_amd as P
scen = dict(S.scenarios(O.hash64))
rng = np.random.default_rng(77)
base = rng.integers(1, 1 << 62, 40000, dtype=np.uint64)
h = O.hash64(base)
wrap = base[(h & np.uint64(0xFF)) >= np.uint64(249)]
pre = base[:30000]
ops = [np.ones(30000, np.uint8)]
keys = [pre]
for r in range(4):
    k = np.concatenate([rng.choice(pre, 12000), rng.choice(wrap, 3000), base[30000 + r * 2000: 32000 + r * 2000],
                        rng.choice(base[30000:], 3000)])
    o = (rng.random(k.size) < 0.45).astype(np.uint8)
    p = rng.permutation(k.size)
    ops.append(o[p]); keys.append(k[p])
ops = np.concatenate(ops); keys = np.concatenate(keys)
vals = keys ^ np.uint64(0x5555)
scen["join_cases"] = (64, "hybrid", np.where(ops == 1, S.OP_INSERT, S.OP_GET).astype(np.uint8), keys, vals)
out = {}
for name in ("mixed_cap16_60k", "mixed_cap2_30k_ins80", "split_loss_mixed", "dup_wrap", "join_cases"):
    init_cap, conv, ops, keys, vals = scen[name]
    n = keys.size
    for batch in (9000, 20000, 65536):
        t = P.CCEH(init_cap, convention=conv, max_batch=batch, max_segments=16384)
        o = O.OracleCCEH(t.initial_depth)
        vo, st = t.MixedBatches(ops, keys, vals, list(range(0, n, batch)) + [n])
        ov, ost = o.mixed(ops, keys, vals)
        ok = bool(np.array_equal(st, ost) and np.array_equal(vo, ov))
        d, od = t.dump(), o.dump()
        ok = ok and d["depth"] == od["depth"] and all(np.array_equal(d[f], od[f]) for f in ("local_depth", "keys", "values"))
        ok = ok and t.stats()["error_flags"] == 0
        out[f"{name}/{batch}"] = ok
        t.close()
print(json.dumps(out))
'''


@pytest.mark.parametrize("mode", ["0", "1"])
def test_mixed_modes_match_oracle(mode):
    e = dict(os.environ)
    e["PMDFC_MIXED_JOIN"] = mode
    r = subprocess.run([sys.executable, "-c", CHILD_MIXED], cwd=REPO, env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert all(res.values()), (mode, res)


# The routed call forced through its pack / exchange / unpack on one rank
# (PMDFC_ROUTE_DIRECT=0: on one rank the routed call is otherwise the direct
# call), at the bench's batch geometry: three 1M-op insert batches, then Get
# batches (half stored keys, half absent) with and without the per-tile
# dedupe, then 50/50 mixed batches -- every status and value equal to a
# direct engine fed the same batches.
CHILD_ROUTE = r'''
import json, sys, torch, numpy as np
import pmdfc_amd as P
from pmdfc_amd.dist import BlockRouter
B, nb = 1 << 20, 3
pk = P.BlockPacker(0, B, 0)
idx = P.CCEH(depth=16, max_batch=pk.rows, max_segments=1 << 17, device=0)
comm = P.Comm(0)
r = BlockRouter(idx, pk, comm=comm)
assert r._native()
direct = P.CCEH(depth=16, max_batch=B, max_segments=1 << 17, device=0)
keys = [P.gen_keys(900 + i, 0, B, device=0) for i in range(nb)]
out = {}
st_r = r.insert_batches([(k, k) for k in keys])
out["insert"] = all(bool(torch.equal(a, direct.Insert(k, k))) for a, k in zip(st_r, keys))
q = [torch.cat([k[: B // 2], P.gen_keys(950 + i, 0, B // 2, device=0)]) for i, k in enumerate(keys)]
ok = True
for dd in (True, False):
    r.dedupe_gets = dd
    for (v, s), qq in zip(r.get_batches(q), q):
        vd, sd = direct.Get(qq)
        ok = ok and bool(torch.equal(v, vd) and torch.equal(s, sd))
out["get"] = ok
rng = np.random.default_rng(5)
mb = []
for i in range(nb):
    o = torch.from_numpy((rng.random(B) < 0.5).astype(np.uint8)).to("cuda:0")
    fresh = P.gen_keys(980 + i, 0, B, device=0)
    k = torch.where(o.bool(), fresh, keys[i][torch.randint(0, B, (B,), device="cuda:0")])
    mb.append((k, k ^ 5, o))
ok = True
for (v, s), (k, vv, o) in zip(r.mixed_batches(mb), mb):
    vd, sd = direct.Mixed(o, k, vv)
    ok = ok and bool(torch.equal(v, vd) and torch.equal(s, sd))
out["mixed"] = ok
print(json.dumps(out))
'''


def test_routed_forced_one_rank_bench_geometry():
    e = dict(os.environ)
    e["PMDFC_ROUTE_DIRECT"] = "0"
    r = subprocess.run([sys.executable, "-c", CHILD_ROUTE], cwd=REPO, env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert all(res.values()), res
