"""Golden CCEH scenarios shared by tests/golden/gen_golden.py (which runs the
reference's own CCEH_hybrid.cpp on them) and the parity tests (which run the
oracle restatement and the HIP engine on them).

A scenario is a serial op stream (ops, keys, values) applied to
CCEH_hybrid(init_cap) in order; op 1 = Insert, op 0 = Get.  Values are never 0
(0 is NONE, the reference's miss value, server/util/pair.h:11).
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pmdfc_amd.workload import uniform_keys  # noqa: E402

OP_GET, OP_INSERT = 0, 1


def _vals(keys, salt=0x1234):
    v = keys ^ np.uint64(salt)
    v[v == 0] = np.uint64(1)
    return v


def insert_then_get(seed, n_ins, n_absent):
    ins = uniform_keys(seed, 0, n_ins)
    absent = uniform_keys(seed, n_ins, n_absent)
    keys = np.concatenate([ins, ins, absent])
    vals = np.concatenate([_vals(ins), np.zeros(n_ins + n_absent, np.uint64)])
    ops = np.concatenate([np.full(n_ins, OP_INSERT, np.uint8), np.zeros(n_ins + n_absent, np.uint8)])
    return ops, keys, vals


def mixed(seed, n_ops, p_insert=0.5):
    """Random interleaving: inserts of fresh keys; gets drawn from a pool that
    holds keys inserted earlier, keys inserted LATER in the stream and keys
    never inserted -- exercises Get-after-Insert ordering inside a batch."""
    rng = np.random.default_rng(seed)
    is_ins = rng.random(n_ops) < p_insert
    n_ins = int(is_ins.sum())
    fresh = uniform_keys(seed, 0, n_ins)
    never = uniform_keys(seed, n_ins, n_ops)
    pool = np.concatenate([fresh, never[: n_ins // 4 + 1]])
    keys = np.empty(n_ops, np.uint64)
    keys[is_ins] = fresh
    keys[~is_ins] = pool[rng.integers(0, pool.size, int((~is_ins).sum()))]
    vals = np.where(is_ins, _vals(keys), np.uint64(0)).astype(np.uint64)
    return is_ins.astype(np.uint8), keys, vals


def _find_key_with_low_byte(seed, want_low, hash64, count=1, start=0):
    out = []
    pos = start
    while len(out) < count:
        ks = uniform_keys(seed, pos, 1 << 14)
        h = hash64(ks)
        sel = ks[(h & np.uint64(0xFF)) == np.uint64(want_low)]
        out.extend(sel.tolist())
        pos += 1 << 14
    return np.array(out[:count], dtype=np.uint64)


def dup_wrap(seed, hash64, n_fill=6000):
    """duplicates of a key whose window wraps (y = 1020); the
    first copy in probe order changes after the segment splits."""
    k = _find_key_with_low_byte(seed + 7, 255, hash64)[0]
    fill = uniform_keys(seed, 0, n_fill)
    ops, keys, vals = [], [], []
    for i in range(5):
        ops.append(OP_INSERT); keys.append(k); vals.append(100 + i)
    ops.append(OP_GET); keys.append(k); vals.append(0)
    for j, f in enumerate(fill):
        ops.append(OP_INSERT); keys.append(f); vals.append(int(f ^ np.uint64(0x77)) or 1)
        if j % 500 == 0:
            ops.append(OP_GET); keys.append(k); vals.append(0)
    ops.append(OP_GET); keys.append(k); vals.append(0)
    return np.array(ops, np.uint8), np.array(keys, np.uint64), np.array(vals, np.uint64)


def dup32(seed, n_fill=3000):
    """32 copies of one key (the 33rd would hang the reference)."""
    k = uniform_keys(seed + 11, 0, 1)[0]
    fill = uniform_keys(seed, 0, n_fill)
    ops = [OP_INSERT] * 32 + [OP_GET] + [OP_INSERT] * n_fill + [OP_GET]
    keys = [k] * 32 + [k] + fill.tolist() + [k]
    vals = list(range(1, 33)) + [0] + [int(f ^ np.uint64(0x99)) or 1 for f in fill] + [0]
    return np.array(ops, np.uint8), np.array(keys, np.uint64), np.array(vals, np.uint64)


def dup_pairs(seed, n=20000):
    """Uniform stream where ~5% of inserts re-insert an earlier key (re-puts of
    the same longkey reach the server: client/julee.c:25)."""
    rng = np.random.default_rng(seed)
    base = uniform_keys(seed, 0, n)
    keys = base.copy()
    rep = rng.random(n) < 0.05
    rep[0] = False
    idx = np.arange(n)
    src = (rng.random(n) * idx).astype(np.int64)
    keys[rep] = base[src[rep]]
    ops = np.ones(n, np.uint8)
    vals = (np.arange(n, dtype=np.uint64) + np.uint64(1))
    q = np.concatenate([base, uniform_keys(seed, n, 1000)])
    return (np.concatenate([ops, np.zeros(q.size, np.uint8)]),
            np.concatenate([keys, q]),
            np.concatenate([vals, np.zeros(q.size, np.uint64)]))


def _find_keys(seed, hash64, want_low, want_top2, count):
    """`count` keys with h & 0xFF == want_low and h >> 62 == want_top2."""
    out, pos = [], 0
    while len(out) < count:
        ks = uniform_keys(seed, pos, 1 << 16)
        h = hash64(ks)
        sel = ks[((h & np.uint64(0xFF)) == np.uint64(want_low)) & ((h >> np.uint64(62)) == np.uint64(want_top2))]
        out.extend(sel.tolist())
        pos += 1 << 16
    return np.array(out[:count], dtype=np.uint64)


def split_loss(seed, hash64, mixed=False, n_fill=3000):
    """Insert4split's silent drop (CCEH_hybrid.cpp:18-28), through
    the wrap unit.  CCEH_hybrid(2): segment 0 holds hash prefix 0; every key
    here has h >> 62 == 0 (segment 0, and child 0 of its first split).
      A: 32 keys of home line 248 fill the window [992, 1024);
      B: 28 keys of home line 255 (window [1020, 1052) mod 1024) find
         1020..1023 taken and wrap to slots 0..27;
      C: keys of home line 248 find their window full -> split.
    The split replays the parent in slot order: B's wrapped entries (slots
    0..27) go first and take 1020..1023 and 0..23 of the child, so A's window
    [992, 1024) keeps 28 free slots for 32 entries -- 4 are dropped.  Then
    fill keys (more splits elsewhere) and Gets of everything.  mixed=True
    interleaves Gets of A and B before, between and after the splits (a
    mixed batch may answer a Get early against the pre-batch image; the
    engine places the drop before or after it through its drop log,
    DESIGN §2)."""
    a = _find_keys(seed, hash64, 248, 0, 36)
    b = _find_keys(seed + 1, hash64, 255, 0, 28)
    c, a = a[32:], a[:32]
    fill = uniform_keys(seed + 2, 0, n_fill)
    absent = uniform_keys(seed + 3, 0, 100)
    ops, keys = [], []

    def ins(ks):
        ops.extend([OP_INSERT] * len(ks))
        keys.extend(ks.tolist())

    def get(ks):
        ops.extend([OP_GET] * len(ks))
        keys.extend(ks.tolist())

    ins(a)
    ins(b)
    if mixed:
        get(a)
        get(b)
        for k in c:  # each trigger followed by Gets of A (some are dropped by now)
            ins(np.array([k], np.uint64))
            get(a[::3])
        ins(fill[: n_fill // 2])
        get(np.concatenate([a, b]))
        ins(fill[n_fill // 2:])
    else:
        ins(c)
        ins(fill)
    get(np.concatenate([a, b, c, fill, absent]))
    ops = np.array(ops, np.uint8)
    keys = np.array(keys, np.uint64)
    vals = np.where(ops == OP_INSERT, _vals(keys), np.uint64(0)).astype(np.uint64)
    return ops, keys, vals


def scenarios(hash64):
    """name -> (init_cap, convention, ops, keys, values)."""
    s = {}
    s["cap2_ins3k"] = (2, "hybrid") + insert_then_get(1, 3000, 1000)
    s["cap8_ins20k"] = (8, "hybrid") + insert_then_get(2, 20000, 5000)
    s["cap1024_ins100k"] = (1024, "hybrid") + insert_then_get(3, 100000, 20000)
    s["cap2_ins100k"] = (2, "hybrid") + insert_then_get(4, 100000, 10000)
    s["cap256_ins400k"] = (256, "hybrid") + insert_then_get(5, 400000, 50000)
    s["mixed_cap16_60k"] = (16, "hybrid") + mixed(6, 60000)
    s["mixed_cap2_30k_ins80"] = (2, "hybrid") + mixed(7, 30000, 0.8)
    s["dup_wrap"] = (2, "hybrid") + dup_wrap(8, hash64)
    s["dup32"] = (4, "hybrid") + dup32(9)
    s["dup_pairs"] = (32, "hybrid") + dup_pairs(10)
    # src/cceh.cpp twin: CCEH(initCap) -> depth floor(log2(initCap/1024))
    s["src_cap2m_ins50k"] = (2 << 20, "src") + insert_then_get(12, 50000, 5000)
    # Insert4split's drop (CCEH_hybrid.cpp:18-28) through the wrap unit
    s["split_loss"] = (2, "hybrid") + split_loss(13, hash64)
    s["split_loss_mixed"] = (2, "hybrid") + split_loss(13, hash64, mixed=True)
    return s


# CCEH::FindAnyway fixtures (tests/golden/findany.json): scenarios whose
# final table the reference scans for these queries
FINDANY_CASES = ["dup_wrap", "dup32", "split_loss", "cap2_ins3k", "mixed_cap2_30k_ins80", "src_cap2m_ins50k"]


def findany_queries(keys):
    """The stream's distinct keys in first-occurrence order (at most 4000) and
    64 keys it never holds."""
    _, first = np.unique(keys, return_index=True)
    q = keys[np.sort(first)][:4000]
    return np.concatenate([q, uniform_keys(4242, 0, 64)]).astype(np.uint64)


def upsert_reinserts(seed, n=30000, p_re=0.15, p_get=0.3):
    """A mixed stream where ~15% of the inserts re-insert an earlier key with a
    new value (the client re-puts a longkey, client/julee.c:25) and Gets ask
    for inserted, re-inserted and absent keys: last-writer-wins must return
    the latest value."""
    rng = np.random.default_rng(seed)
    fresh = uniform_keys(seed, 0, n)
    absent = uniform_keys(seed, n, n // 10)
    ops = np.empty(n, np.uint8)
    keys = np.empty(n, np.uint64)
    nf = 0
    for i in range(n):
        r = rng.random()
        if r < p_get and nf:
            ops[i] = OP_GET
            keys[i] = fresh[rng.integers(0, nf)] if rng.random() < 0.9 else absent[rng.integers(0, absent.size)]
        elif r < p_get + p_re and nf:
            ops[i] = OP_INSERT
            keys[i] = fresh[rng.integers(0, nf)]
        else:
            ops[i] = OP_INSERT
            keys[i] = fresh[nf]
            nf += 1
    vals = np.where(ops == OP_INSERT, np.arange(1, n + 1, dtype=np.uint64), np.uint64(0)).astype(np.uint64)
    return ops, keys, vals


def dup_many(seed, copies=100, n_fill=3000):
    """100 copies of one key interleaved with fill inserts and Gets: in upsert
    mode a key never holds more than one slot (the reference as shipped hangs
    at the 33rd copy)."""
    k = uniform_keys(seed + 11, 0, 1)[0]
    fill = uniform_keys(seed, 0, n_fill)
    ops, keys, vals = [], [], []
    per = n_fill // copies
    for c in range(copies):
        ops += [OP_INSERT, OP_GET]
        keys += [int(k), int(k)]
        vals += [c + 1, 0]
        for f in fill[c * per:(c + 1) * per]:
            ops.append(OP_INSERT); keys.append(int(f)); vals.append(int(f ^ np.uint64(0x99)) or 1)
    ops.append(OP_GET); keys.append(int(k)); vals.append(0)
    return np.array(ops, np.uint8), np.array(keys, np.uint64), np.array(vals, np.uint64)


def upsert_scenarios(hash64):
    """Last-writer-wins scenarios, pinned by the reference's CCEH_hybrid.cpp
    with its overwrite clause (:153) enabled (oracle/_ref/ref_driver_upsert).
    name -> (init_cap, convention, ops, keys, values)."""
    s = {}
    s["up_dup_wrap"] = (2, "hybrid") + dup_wrap(8, hash64)
    s["up_dup_many"] = (4, "hybrid") + dup_many(9)
    s["up_dup_pairs"] = (32, "hybrid") + dup_pairs(10)
    s["up_reinserts_cap2"] = (2, "hybrid") + upsert_reinserts(14)
    s["up_reinserts_cap256"] = (256, "hybrid") + upsert_reinserts(15, n=120000, p_re=0.25)
    s["up_split_loss_mixed"] = (2, "hybrid") + split_loss(13, hash64, mixed=True)
    return s


def sha(a) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def summarize(depth, local_depth, prefix, keys, values, get_values, ops):
    """Fixture record for a final table state + the Get results of a stream.
    keys/values are the canonical segment images (values 0 where key INVALID),
    get_values[i] is the Get result for op i (0 for inserts and misses)."""
    gv = np.where(np.asarray(ops) == OP_GET, get_values, 0).astype(np.uint64)
    return {
        "depth": int(depth),
        "nseg": int(len(local_depth)),
        "local_depth_sha": sha(np.asarray(local_depth, np.uint64)),
        "prefix_sha": sha(np.asarray(prefix, np.uint64)),
        "keys_sha": sha(np.asarray(keys, np.uint64)),
        "values_sha": sha(np.asarray(values, np.uint64)),
        "get_values_sha": sha(gv),
        "get_hits": int(np.count_nonzero(gv)),
        "occupied": int(np.count_nonzero(np.asarray(keys, np.uint64) != np.uint64(0xFFFFFFFFFFFFFFFF))),
    }


def cbfseq_cases():
    """Counting-BF insert-then-delete sequences (counting_bloom_filter.h:109-131):
    saturation at 255, deletes that conflict inside one batch, a key whose k
    hashes repeat an index (uint8 wrap on Delete), absent keys."""
    rng = np.random.default_rng(77)
    a = np.array([0x1234567], np.uint64)
    pool = uniform_keys(40, 0, 1500)
    dels = np.concatenate([a, a, pool[rng.integers(0, 1500, 400)], uniform_keys(41, 0, 100)])
    rng.shuffle(dels)
    t = (np.arange(10000, dtype=np.uint64) * np.uint64(14))
    big = uniform_keys(42, 0, 50000)
    return {
        "sat_conflict": (3, 1000, np.concatenate([np.repeat(a, 300), pool]), dels),
        "tiny_wrap": (4, 7, uniform_keys(43, 0, 3), uniform_keys(43, 0, 40)[rng.integers(0, 40, 30)]),
        "fastpath": (4, 1000000, big, np.concatenate([big[rng.permutation(50000)[:10000]],
                                                       uniform_keys(44, 0, 2000)])),
        "bftest_seq": (2, 100000, t[:9999], np.concatenate([t[:5000], t[9999:]])),
    }


def replay_trace(seed: int, n_lines: int, n_inodes: int = 2000, crlf: bool = False) -> bytes:
    """Synthetic trace in replay_KV's format (server/replay_KV.cpp:24-31):
    'seq ts OP inode inode_size offset size' with O/C/F/R/W ops, sizes that
    are 0, sub-page, page-multiple and ragged, some unaligned offsets, mixed
    spaces/tabs.  Reads mostly revisit written ranges.  No page is written
    more than 8 times (the reference hangs on a key's 33rd copy)."""
    rng = np.random.default_rng(seed)
    wcount = {}
    written = []
    out = []
    for i in range(n_lines):
        op = rng.choice([b"W", b"W", b"R", b"R", b"R", b"O", b"C", b"F"])
        if op == b"R" and written and rng.random() < 0.8:
            ino, off = written[int(rng.integers(0, len(written)))]
        else:
            ino = int(rng.integers(1, n_inodes + 1))
            off = 4096 * int(rng.integers(0, 256)) + (int(rng.integers(1, 4096)) if rng.random() < 0.05 else 0)
        size = int(rng.choice([0, 100, 4096, 5000, 8192, 12288, 20000, 65536]))
        if op == b"W":
            np_ = size // 4096 + (1 if size % 4096 else 0)
            pages = [((ino << 32) + off + 4096 * b) for b in range(np_)]
            if any(wcount.get(p, 0) >= 8 for p in pages):
                op = b"R"
            else:
                for p in pages:
                    wcount[p] = wcount.get(p, 0) + 1
                written.append((ino, off))
        sep = b"\t" if rng.random() < 0.1 else b" "
        fields = [str(i).encode(), b"%d.%06d" % (i // 1000, i % 1000), op, str(ino).encode(),
                  str(int(rng.integers(1, 1 << 30))).encode(), str(off).encode(), str(size).encode()]
        out.append(sep.join(fields) + (b"  " if rng.random() < 0.05 else b""))
    end = b"\r\n" if crlf else b"\n"
    return end.join(out) + end


def replay_trace_ops(text: bytes) -> int:
    """Ops in the whole trace (W/R pages), for num_data = everything."""
    tot = 0
    for ln in text.split(b"\n"):
        e = ln.split()
        if len(e) >= 7 and e[2][:1] in (b"W", b"R"):
            s = int(e[6])
            tot += s // 4096 + (1 if s % 4096 else 0)
    return tot


def extent_cases():
    """Extent streams for Insert_extent / Get_extent (both reference variants):
    non-overlapping extents (no duplicate heads), lens 1..300 plus a few long
    ones, heads with zero low 32 bits (inode << 32 shape, ffs((int)head) = 0)
    and head 0; queries inside and outside the extents.
    name -> (convention, init_cap, keys, clusters, lens, values, qkeys, qclusters)."""
    out = {}
    for name, conv, cap, n, seed in [("hyb_cap1024", "hybrid", 1024, 3000, 1),
                                     ("hyb_cap2", "hybrid", 2, 1500, 2),
                                     ("src_cap2m", "src", 1 << 21, 3000, 3),
                                     ("src_cap4096", "src", 4096, 1500, 4)]:
        rng = np.random.default_rng(seed)
        lens = rng.integers(1, 300, n).astype(np.uint64)
        lens[rng.integers(0, n, 5)] = rng.integers(1000, 5000, 5).astype(np.uint64)
        gaps = rng.integers(0, 64, n).astype(np.uint64)
        keys = np.cumsum(lens + gaps).astype(np.uint64) - lens
        keys[: n // 10] = (np.arange(1, n // 10 + 1, dtype=np.uint64) << np.uint64(32))  # low 32 bits zero
        keys[n // 10] = 0
        keys[n // 10 + 1:] += np.uint64(1 << 33)
        clusters = np.zeros(n, np.uint64)
        if conv == "src":
            clusters = (rng.integers(0, 3, n) * rng.integers(0, 8, n)).astype(np.uint64)
            clusters = np.minimum(clusters, lens - np.uint64(1))
            lens = lens - clusters  # src extents: the remaining pages from cluster
        vals = uniform_keys(seed + 100, 0, n) | np.uint64(1)
        qi = rng.integers(0, n, 4000)
        qoff = (rng.random(4000) * lens[qi].astype(np.float64)).astype(np.uint64)
        if conv == "src":
            qk, qc = keys[qi], clusters[qi] + qoff
        else:
            qk, qc = keys[qi] + qoff, np.zeros(4000, np.uint64)
        qk = np.concatenate([qk, uniform_keys(seed + 200, 0, 500)])
        qc = np.concatenate([qc, np.zeros(500, np.uint64)])
        out[name] = (conv, cap, keys, clusters, lens, vals, qk, qc)
    return out


def extent_expand(conv, keys, clusters, lens, vals, heads_fn):
    """Concatenated sub-extent heads/values of a batch of Insert_extent calls."""
    hk, hv = [], []
    for k, c, ln, v in zip(keys.tolist(), clusters.tolist(), lens.tolist(), vals.tolist()):
        h = heads_fn(k, ln, c, conv)
        hk.extend(h)
        hv.extend([v] * len(h))
    return np.array(hk, np.uint64), np.array(hv, np.uint64)
