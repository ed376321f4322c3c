"""GPU trace ingestion (replay_KV format, server/replay_KV.cpp:209-247) through
the C-ABI (pmdfc_trace_parse): op/key streams bit-exact with the oracle's
restatement, the replayed run's failedSearch / put / get equal the reference
replay_KV's on the same traces, and every per-op Get result equals the
reference's src/cceh.cpp on that op stream (tests/golden/replay.json)."""
import json
import os

import numpy as np
import pytest

import scenarios as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import pmdfc_amd as P  # noqa: E402


@pytest.fixture(scope="module")
def replay_golden(golden_dir):
    with open(os.path.join(golden_dir, "replay.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def reader():
    r = P.TraceReader()
    yield r
    r.close()


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("batch", [997, 65536])
@pytest.mark.parametrize("name", ["small", "mid", "crlf_tiny_table", "big"])
def test_replay_matches_reference(replay_golden, reader, name, batch):
    g = replay_golden[name]
    text = S.replay_trace(g["seed"], g["n_lines"], crlf=g["crlf"])
    ops, keys, info = reader.parse(text, g["num_data"])
    oo, ok = O.parse_replay_trace(text, g["num_data"])
    assert np.array_equal(ops.cpu().numpy(), oo) and np.array_equal(_u64(keys), ok)
    assert info["ops"] == g["num_data"] and info["first_bad_line"] == 2**64 - 1
    idx = P.CCEH(g["tablesize"], convention="src", max_batch=batch, max_segments=8192)
    r = P.replay(idx, ops, keys)
    assert r == {"failedSearch": g["failedSearch"], "put": g["put"], "get": g["get"]}
    # per-op Get results: equal to the reference's src/cceh.cpp on the same
    # op stream (replay.json get_values_sha, tests/golden/gen_golden.py)
    idx2 = P.CCEH(g["tablesize"], convention="src", max_batch=batch, max_segments=8192)
    gv = np.concatenate([_u64(idx2.Mixed(ops[a:a + batch], keys[a:a + batch], keys[a:a + batch])[0])
                         for a in range(0, keys.numel(), batch)])
    gv = np.where(ops.cpu().numpy() == 0, gv, 0).astype(np.uint64)
    assert S.sha(gv) == g["get_values_sha"] and int(np.count_nonzero(gv)) == g["get_hits"]


def test_parse_edges(reader):
    txt = b"0 t W 1 9 0 4097\n1 t O 2 9 7\n2 t R +1 9 -4096 1\n3 t X 5 9 0 99999\n4 t W 3 9 0 0\n5 t R 1 9 4096 10"
    for nd in [1, 2, 3, 4]:
        ops, keys, info = reader.parse(txt, nd)
        oo, ok = O.parse_replay_trace(txt, nd)
        assert np.array_equal(ops.cpu().numpy(), oo) and np.array_equal(_u64(keys), ok)
    assert info["lines"] == 6 and info["trace_ops"] == 4  # unterminated last line counts
    with pytest.raises(P.PmdfcError):
        reader.parse(txt, 5)  # fewer ops than num_data
    with pytest.raises(P.PmdfcError):
        reader.parse(b"0 t W 1 9\n0 t W 1 9 0 1\n", 1)  # malformed line before the stop line
    with pytest.raises(P.PmdfcError):
        reader.parse(b"0 t W x 9 0 1\n", 1)
    ops, keys, info = reader.parse(b"0 t W 1 9 0 4096\n\ngarbage\n", 1)  # stops before them
    assert ops.tolist() == [1] and info["first_bad_line"] == 1 and info["stop_line"] == 0
    ops, keys, info = reader.parse(b"", 0)
    assert ops.numel() == 0 and info["lines"] == 0
    # stoull: overflow is malformed, leading zeros and trailing junk are not
    with pytest.raises(P.PmdfcError):
        reader.parse(b"0 t R 1 9 0 99999999999999999999\n", 1)
    ops, keys, _ = reader.parse(b"0 t R 0007x 9 12abc 1\n", 1)
    assert _u64(keys).tolist() == [(7 << 32) + 12]


def test_large_trace_parse_matches_oracle(reader):
    text = S.replay_trace(9, 150000, n_inodes=50000)
    n = int(S.replay_trace_ops(text))
    ops, keys, info = reader.parse(text, n)
    oo, ok = O.parse_replay_trace(text, n)
    assert info["trace_ops"] == n and info["lines"] == 150000
    assert np.array_equal(ops.cpu().numpy(), oo) and np.array_equal(_u64(keys), ok)


def test_long_lines_and_unaligned_text(reader):
    """Lines of > 64 pages (the wave-per-line expansion), a 16 KiB-tile
    boundary inside a line, and a text that does not start 16-byte aligned
    (the byte path of the newline pass)."""
    rng = np.random.default_rng(3)
    parts = []
    for i in range(3000):
        size = int(rng.choice([4096 * 1000, 4096 * 65, 4096 * 64, 8191, 1])) if i % 7 == 0 else int(rng.integers(1, 40000))
        op = b"W" if i % 3 else b"R"
        parts.append(b"%d 0.0 %s %d 77 %d %d" % (i, op, i + 1, 4096 * (i % 13), size))
    text = b"\n".join(parts) + b"\n"
    n = int(S.replay_trace_ops(text))
    ops, keys, info = reader.parse(text, n)
    oo, ok = O.parse_replay_trace(text, n)
    assert np.array_equal(ops.cpu().numpy(), oo) and np.array_equal(_u64(keys), ok)
    d = torch.from_numpy(np.frombuffer(b"x" + text, np.uint8).copy()).cuda()
    ops2, keys2, _ = reader.parse(d[1:], n - 5)
    assert np.array_equal(ops2.cpu().numpy(), oo[: n - 5]) and np.array_equal(_u64(keys2), ok[: n - 5])
