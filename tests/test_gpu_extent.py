"""GPU extent API (pmdfc_cceh_insert_extent / get_extent, both reference
variants) against the reference's own Insert_extent / Get_extent fixtures
(tests/golden/extent.json): final table images and Get_extent results."""
import json
import os

import numpy as np
import pytest

import scenarios as S

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import pmdfc_amd as P  # noqa: E402


@pytest.fixture(scope="module")
def extent_golden(golden_dir):
    with open(os.path.join(golden_dir, "extent.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("parts", [1, 3])
@pytest.mark.parametrize("name", ["hyb_cap1024", "hyb_cap2", "src_cap2m", "src_cap4096"])
def test_extent_matches_reference(extent_golden, name, parts):
    g = extent_golden[name]
    conv, cap, keys, cl, lens, vals, qk, qc = S.extent_cases()[name]
    t = P.CCEH(cap, convention=conv, max_batch=1 << 14, max_segments=8192)
    b = np.linspace(0, keys.size, parts + 1).astype(int)
    n = 0
    for a, e in zip(b[:-1], b[1:]):
        n += t.Insert_extent(keys[a:e], lens[a:e], vals[a:e], clusters=cl[a:e] if conv == "src" else None)
    assert n == g["occupied"]  # every sub-extent head stored (no duplicates, no split loss)
    d = t.dump()
    rec = S.summarize(d["depth"], d["local_depth"], d["prefix"], d["keys"], d["values"],
                      np.zeros(0, np.uint64), np.zeros(0, np.uint8))
    for k, v in rec.items():
        assert v == g[k], (k, v, g[k])
    v, st = t.Get_extent(qk, clusters=qc if conv == "src" else None)
    assert S.sha(v) == g["results_sha"]
    assert np.array_equal(st == P.ST_HIT, v != 0)


def test_extent_device_tensors_and_empty():
    t = P.CCEH(1024, max_batch=4096, max_segments=1024)
    assert t.Insert_extent(np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.uint64)) == 0
    k = torch.tensor([64, 1 << 32], dtype=torch.int64, device="cuda")
    n = t.Insert_extent(k, torch.tensor([100, 7], dtype=torch.int64, device="cuda"),
                        torch.tensor([11, 13], dtype=torch.int64, device="cuda"))
    q = torch.tensor([64, 100, 163, 164, (1 << 32) + 6, (1 << 32) + 7], dtype=torch.int64, device="cuda")
    v, st = t.Get_extent(q)
    from oracle import oracle as O
    o = O.OracleCCEH(10)
    hk = O.extent_heads(64, 100) + O.extent_heads(1 << 32, 7)
    assert n == len(hk)
    o.insert(np.array(hk, np.uint64), np.array([11] * len(O.extent_heads(64, 100)) + [13] * len(O.extent_heads(1 << 32, 7)), np.uint64))
    exp = []
    for x in q.tolist():
        ov, os_ = o.get(np.array(O.extent_targets(x), np.uint64))
        hits = [int(a) for a, b in zip(ov, os_) if b == O.ST_HIT and a]
        exp.append(hits[0] if hits else 0)
    assert v.tolist() == exp and exp[0] == 11 and exp[4] == 13
