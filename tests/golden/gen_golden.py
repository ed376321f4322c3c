"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's own
code: oracle/_ref/ref_driver (our driver + /root/reference/server/CCEH_hybrid.cpp,
util/hash.h, util/counting_bloom_filter.h) and oracle/_ref/ref_driver_src
(+ src/cceh.cpp).  Build recipe: oracle/Makefile target `ref`.

Run in the build container (the reference never travels to the GPU box):
    python tests/golden/gen_golden.py
Compiler: g++ 11.4 -O2 -std=c++17 (recorded in meta.json).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)

import scenarios as S  # noqa: E402
from oracle import oracle as O  # noqa: E402  (only for finding wrap keys)
from pmdfc_amd.workload import uniform_keys  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref")


def run(mode, binary, payload: bytes, timeout=600) -> bytes:
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fin, "wb") as f:
            f.write(payload)
        subprocess.run([os.path.join(REF, binary), mode, fin, fout], check=True, timeout=timeout)
        with open(fout, "rb") as f:
            return f.read()


def gen_hash():
    special = np.array([0, 1, 42, 1 << 63, (1 << 64) - 1, (1 << 64) - 2, (1 << 32), 0xdeadbeef,
                        4096, (1 << 20) << 32], dtype=np.uint64)
    keys = np.concatenate([special, uniform_keys(99, 0, 4096 - special.size)])
    out = run("hash", "ref_driver", np.uint64(keys.size).tobytes() + keys.tobytes())
    rec = np.frombuffer(out, dtype=np.dtype([("h", "<u8"), ("m", "<u4", (4,))]))
    np.savez_compressed(os.path.join(HERE, "hash_kat.npz"), keys=keys, h=rec["h"].copy(),
                        murmur2=rec["m"].copy())
    print("hash_kat:", keys.size, "keys; h(0)=%#x" % rec["h"][0])


def gen_cceh(upsert=False):
    table = {}
    scen = S.upsert_scenarios(O.hash64) if upsert else S.scenarios(O.hash64)
    for name, (init_cap, conv, ops, keys, vals) in scen.items():
        n = keys.size
        payload = (np.array([init_cap, n], np.uint64).tobytes() + keys.astype("<u8").tobytes()
                   + vals.astype("<u8").tobytes() + ops.astype(np.uint8).tobytes())
        binary = "ref_driver" if conv == "hybrid" else "ref_driver_src"
        if upsert:
            assert conv == "hybrid"
            binary = "ref_driver_upsert"  # CCEH_hybrid.cpp with :153 enabled
        out = run("cceh", binary, payload)
        p = 0
        depth, nseg = np.frombuffer(out, "<u8", 2, p); p += 16
        meta = np.frombuffer(out, "<u8", 2 * int(nseg), p).reshape(-1, 2); p += 16 * int(nseg)
        skeys = np.frombuffer(out, "<u8", int(nseg) * 1024, p); p += 8 * int(nseg) * 1024
        svals = np.frombuffer(out, "<u8", int(nseg) * 1024, p); p += 8 * int(nseg) * 1024
        gv = np.frombuffer(out, "<u8", n, p); p += 8 * n
        util = float(np.frombuffer(out, "<f8", 1, p)[0]); p += 8
        cap = int(np.frombuffer(out, "<u8", 1, p)[0]); p += 8
        assert p == len(out)
        rec = S.summarize(depth, meta[:, 0], meta[:, 1], skeys, svals, gv, ops)
        rec.update(init_cap=int(init_cap), convention=conv, n_ops=int(n),
                   utilization=util, capacity=cap)
        if n <= 10000 or name.startswith("dup"):
            sel = np.nonzero(ops == S.OP_GET)[0]
            rec["get_positions_sample"] = sel[:64].tolist()
            rec["get_values_sample"] = gv[sel[:64]].tolist()
        table[name] = rec
        print(name, "depth", int(depth), "nseg", int(nseg), "hits", rec["get_hits"], "util %.3f" % util)
    fn = "upsert_scenarios.json" if upsert else "cceh_scenarios.json"
    with open(os.path.join(HERE, fn), "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)


def cbf_payload(k, m, ins, qs, dels):
    parts = [np.array([k, m, ins.size], np.uint64), ins, np.array([qs.size], np.uint64), qs,
             np.array([dels.size], np.uint64), dels]
    return b"".join(np.ascontiguousarray(x, dtype="<u8").tobytes() for x in parts)


def gen_bloom():
    recs = {}
    # server/bftest.cpp:9-19: t[i] = 14*i, k=2, m=100000, insert t[0..9998]
    t = (np.arange(10000, dtype=np.uint64) * np.uint64(14))
    extra = uniform_keys(31, 0, 2000)
    qs = np.concatenate([t, extra])
    for name, k, m, ins, q, dels in [
        ("bftest", 2, 100000, t[:9999], qs, t[:1]),
        ("k4_m1e9", 4, 1000000000, uniform_keys(32, 0, 100000),
         np.concatenate([uniform_keys(32, 0, 20000), uniform_keys(32, 100000, 20000)]), np.zeros(0, np.uint64)),
    ]:
        out = run("cbf", "ref_driver", cbf_payload(k, m, ins, q, dels), timeout=1200)
        nl = (m + 63) // 64
        p = 0
        query = np.frombuffer(out, np.uint8, q.size, p); p += q.size
        querybb = np.frombuffer(out, np.uint8, q.size, p); p += q.size
        bm = np.frombuffer(out, "<u8", nl, p); p += 8 * nl
        query2 = np.frombuffer(out, np.uint8, q.size, p); p += q.size
        bm2 = np.frombuffer(out, "<u8", nl, p); p += 8 * nl
        assert p == len(out)
        recs[name] = {"k": k, "m": m, "insert_sha": S.sha(ins), "query_sha": S.sha(q),
                      "query": np.packbits(query).tobytes().hex(),
                      "querybb": np.packbits(querybb).tobytes().hex(),
                      "query_after_delete": np.packbits(query2).tobytes().hex(),
                      "bitmap_sha": S.sha(bm), "bitmap_after_delete_sha": S.sha(bm2),
                      "bitmap_popcount": int(np.unpackbits(bm.view(np.uint8)).sum()),
                      "n_query": int(q.size)}
        print(name, "positives", int(querybb.sum()), "/", q.size)
    with open(os.path.join(HERE, "bloom.json"), "w") as f:
        json.dump(recs, f, indent=1, sort_keys=True)


def gen_cbfseq():
    recs = {}
    for name, (k, m, ins, dels) in S.cbfseq_cases().items():
        out = run("cbfseq", "ref_driver", cbf_payload(k, m, ins, dels, np.zeros(0, np.uint64))[:-8])
        nl = (m + 63) // 64
        p = 0
        c1 = np.frombuffer(out, np.uint8, m, p); p += m
        dd = np.frombuffer(out, np.uint8, dels.size, p); p += dels.size
        c2 = np.frombuffer(out, np.uint8, m, p); p += m
        bm = np.frombuffer(out, "<u8", nl, p); p += 8 * nl
        assert p == len(out)
        rec = {"k": k, "m": m, "insert_sha": S.sha(ins), "delete_sha": S.sha(dels),
               "counters_sha": S.sha(c1), "deleted": np.packbits(dd).tobytes().hex(),
               "n_deleted": int(dd.sum()), "counters_after_delete_sha": S.sha(c2),
               "bitmap_sha": S.sha(bm), "saturated": int((c1 == 255).sum())}
        if m <= 1000:
            rec["counters"] = c1.tolist()
            rec["counters_after_delete"] = c2.tolist()
        recs[name] = rec
        print(name, "deleted", int(dd.sum()), "/", dels.size, "saturated", rec["saturated"])
    with open(os.path.join(HERE, "cbf_seq.json"), "w") as f:
        json.dump(recs, f, indent=1, sort_keys=True)


REPLAY_CASES = {  # name: (seed, n_lines, crlf, num_data, tablesize)
    "small": (1, 400, False, 800, 1 << 20),
    "mid": (2, 6000, False, 12000, 1 << 20),
    "crlf_tiny_table": (3, 3000, True, 6000, 2048),
    "big": (4, 40000, False, 90000, 1 << 21),
}


def gen_replay():
    """The reference's own replay_KV (one network thread on CPU 0, so ops run
    serially in trace order) on synthetic traces: failedSearch, put/get."""
    import re
    recs = {}
    for name, (seed, nl, crlf, nd, ts) in REPLAY_CASES.items():
        text = S.replay_trace(seed, nl, crlf=crlf)
        with tempfile.TemporaryDirectory() as td:
            fin = os.path.join(td, "t.trace")
            with open(fin, "wb") as f:
                f.write(text)
            r = subprocess.run([os.path.join(REF, "replay_KV"), "-d", fin, "-n", str(nd), "-t", str(ts),
                                "-W", "0", "-h"], capture_output=True, text=True, timeout=600, check=True)
        fs = int(re.search(r"(\d+) failedSearch", r.stdout).group(1))
        put, get = map(int, re.search(r"Total put = (\d+), get = (\d+)", r.stdout).groups())
        # per-op Get results: the same op stream (the restated parser, pinned by
        # put/get/failedSearch above) through the reference's src/cceh.cpp
        # CCEH(tablesize), what KV links, serially, value = key as replay_KV
        # inserts (server/replay_KV.cpp:262-270)
        ops, keys = O.parse_replay_trace(text, nd)
        payload = (np.array([ts, nd], np.uint64).tobytes() + keys.astype("<u8").tobytes()
                   + keys.astype("<u8").tobytes() + ops.astype(np.uint8).tobytes())
        out = run("cceh", "ref_driver_src", payload)
        nseg = int(np.frombuffer(out, "<u8", 2, 0)[1])
        p = 16 + 16 * nseg + 16 * nseg * 1024
        gv = np.frombuffer(out, "<u8", nd, p)
        gv = np.where(ops == S.OP_GET, gv, 0).astype(np.uint64)
        assert int(((ops == S.OP_GET) & (gv != keys)).sum()) == fs  # the two reference runs agree
        recs[name] = {"seed": seed, "n_lines": nl, "crlf": crlf, "num_data": nd, "tablesize": ts,
                      "text_sha": S.sha(np.frombuffer(text, np.uint8)), "failedSearch": fs,
                      "put": put, "get": get, "get_values_sha": S.sha(gv),
                      "get_hits": int(np.count_nonzero(gv))}
        print(name, recs[name])
    with open(os.path.join(HERE, "replay.json"), "w") as f:
        json.dump(recs, f, indent=1, sort_keys=True)


def gen_extent():
    recs = {}
    for name, (conv, cap, keys, cl, lens, vals, qk, qc) in S.extent_cases().items():
        parts = [np.array([cap, keys.size], np.uint64), keys, cl, lens, vals,
                 np.array([qk.size], np.uint64), qk, qc]
        payload = b"".join(np.ascontiguousarray(x, dtype="<u8").tobytes() for x in parts)
        out = run("extent", "ref_driver" if conv == "hybrid" else "ref_driver_src", payload)
        p = 0
        depth, nseg = np.frombuffer(out, "<u8", 2, p); p += 16
        meta = np.frombuffer(out, "<u8", 2 * int(nseg), p).reshape(-1, 2); p += 16 * int(nseg)
        skeys = np.frombuffer(out, "<u8", int(nseg) * 1024, p); p += 8 * int(nseg) * 1024
        svals = np.frombuffer(out, "<u8", int(nseg) * 1024, p); p += 8 * int(nseg) * 1024
        res = np.frombuffer(out, "<u8", qk.size, p); p += 8 * qk.size
        assert p == len(out)
        rec = S.summarize(depth, meta[:, 0], meta[:, 1], skeys, svals, np.zeros(0, np.uint64),
                          np.zeros(0, np.uint8))
        rec.update(convention=conv, init_cap=int(cap), results_sha=S.sha(res),
                   results_hits=int(np.count_nonzero(res)), results_sample=res[:32].tolist())
        recs[name] = rec
        print(name, "depth", int(depth), "nseg", int(nseg), "occupied", rec["occupied"], "hits", rec["results_hits"])
    with open(os.path.join(HERE, "extent.json"), "w") as f:
        json.dump(recs, f, indent=1, sort_keys=True)


def gen_findany():
    """CCEH::FindAnyway (CCEH_hybrid.cpp:482-496 / src/cceh.cpp:457-471) of the
    reference after each stream, next to its Get: slot order vs probe order."""
    scen = S.scenarios(O.hash64)
    recs = {}
    for name in S.FINDANY_CASES:
        init_cap, conv, ops, keys, vals = scen[name]
        q = S.findany_queries(keys)
        payload = (np.array([init_cap, keys.size], np.uint64).tobytes() + keys.astype("<u8").tobytes()
                   + vals.astype("<u8").tobytes() + ops.astype(np.uint8).tobytes()
                   + np.uint64(q.size).tobytes() + q.astype("<u8").tobytes())
        out = run("findany", "ref_driver" if conv == "hybrid" else "ref_driver_src", payload)
        fa = np.frombuffer(out, "<u8", q.size, 0)
        gv = np.frombuffer(out, "<u8", q.size, 8 * q.size)
        div = np.nonzero(fa != gv)[0]
        recs[name] = {"n_query": int(q.size), "query_sha": S.sha(q), "find_sha": S.sha(fa), "get_sha": S.sha(gv),
                      "find_hits": int(np.count_nonzero(fa)),
                      "diverge": [[int(i), int(fa[i]), int(gv[i])] for i in div[:64]], "n_diverge": int(div.size)}
        print(name, "queries", q.size, "hits", recs[name]["find_hits"], "FindAnyway != Get:", int(div.size))
    with open(os.path.join(HERE, "findany.json"), "w") as f:
        json.dump(recs, f, indent=1, sort_keys=True)


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("reference not present; fixtures are generated in the build container only")
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"])
    if sys.argv[1:] == ["cbfseq"]:
        return gen_cbfseq()
    if sys.argv[1:] == ["replay"]:
        return gen_replay()
    if sys.argv[1:] == ["extent"]:
        return gen_extent()
    if sys.argv[1:] == ["findany"]:
        return gen_findany()
    if sys.argv[1:] == ["cceh"]:
        return gen_cceh()
    if sys.argv[1:] == ["upsert"]:
        return gen_cceh(upsert=True)
    gen_hash()
    gen_cceh()
    gen_cceh(upsert=True)
    gen_bloom()
    gen_cbfseq()
    gen_replay()
    gen_extent()
    gen_findany()
    cc = subprocess.run(["g++", "--version"], capture_output=True, text=True).stdout.splitlines()[0]
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_golden.py", "compiler": cc,
                   "flags": "-std=c++17 -O2", "reference_files": [
                       "server/CCEH_hybrid.cpp", "server/src/cceh.cpp", "server/util/hash.h",
                       "server/util/counting_bloom_filter.h", "server/replay_KV.cpp", "server/KV.cpp"],
                   "upsert_pin": "server/CCEH_hybrid.cpp + oracle/CCEH_hybrid.upsert.patch"}, f, indent=1)


if __name__ == "__main__":
    main()
