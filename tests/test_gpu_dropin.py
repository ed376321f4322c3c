"""The drop-in claim, end to end on the GPU: the reference's OWN front-ends and
harnesses, built from /root/reference with only the maintainer patches of
integration/ (a -DGPUCCEH backend branch, oracle/Makefile target `dropin`),
run over the MI355X engine:

* server/test_KV.cpp + server/KV.cpp -> GpuCCEH : IHash    (_ref/julee_kv_gpu)
* server/replay_KV.cpp + server/KV.cpp -> GpuCCEH          (_ref/replay_kv_gpu)
* server/NuMA_KV.cpp -> GpuCCEHHybrid : ICCEH + our driver (_ref/numa_kv_gpu)

plus our own C++ harnesses of the batching front-end (tests/cpp/test_gpu_kv.cpp,
tools/bench_frontend.cpp at the server's 32 poll threads).  The binaries are
built in the build container and travel with the tree; without them (no
reference at build time) the reference-linked tests skip.
"""
import json
import os
import re
import subprocess

import pytest

import scenarios as S
from conftest import REPO

pytestmark = pytest.mark.gpu

REF = os.path.join(REPO, "oracle", "_ref")
LIB = os.path.join(REPO, "pmdfc_amd", "lib")


def _bin(name):
    p = os.path.join(REF, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (needs the reference at build time: make -C oracle dropin)")
    return p


def _cpus(n):
    return sorted(os.sched_getaffinity(0))[:n]


def test_reference_test_kv_over_gpucceh(tmp_path):
    """server/test_KV.cpp, unmodified, with KV's -DGPUCCEH backend: 8 pinned
    network threads insert then search 200k keys (value = key); the
    reference's own pass criterion is "0 failedSearch" (:305-308).  -b also
    runs KV's host counting BF on every Insert (server/KV.cpp:113-121)."""
    exe = _bin("julee_kv_gpu")
    from pmdfc_amd.workload import uniform_keys
    n = 200000
    keys = uniform_keys(2024, 0, n)
    f = tmp_path / "keys.txt"
    f.write_text("\n".join(str(int(k)) for k in keys) + "\n")
    cpus = ",".join(str(c) for c in _cpus(8))
    r = subprocess.run([exe, "-d", str(f), "-n", str(n), "-W", cpus, "-h", "-b"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    fs = int(re.search(r"(\d+) failedSearch", r.stdout).group(1))
    put, get = map(int, re.search(r"Total put = (\d+), get = (\d+)", r.stdout).groups())
    assert fs == 0 and put == n and get == n, r.stdout


@pytest.fixture(scope="module")
def replay_golden(golden_dir):
    with open(os.path.join(golden_dir, "replay.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["small", "mid", "crlf_tiny_table", "big"])
def test_reference_replay_kv_over_gpucceh(replay_golden, name, tmp_path):
    """server/replay_KV.cpp, unmodified, with KV's -DGPUCCEH backend, on the
    traces whose failedSearch/put/get the CPU reference replay_KV produced
    (tests/golden/replay.json): one network thread, so ops run in trace order."""
    exe = _bin("replay_kv_gpu")
    g = replay_golden[name]
    text = S.replay_trace(g["seed"], g["n_lines"], crlf=g["crlf"])
    f = tmp_path / "t.trace"
    f.write_bytes(text)
    r = subprocess.run([exe, "-d", str(f), "-n", str(g["num_data"]), "-t", str(g["tablesize"]), "-W",
                        str(_cpus(1)[0]), "-h"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    fs = int(re.search(r"(\d+) failedSearch", r.stdout).group(1))
    put, get = map(int, re.search(r"Total put = (\d+), get = (\d+)", r.stdout).groups())
    assert (fs, put, get) == (g["failedSearch"], g["put"], g["get"]), r.stdout


def test_reference_numa_kv_over_gpucceh_hybrid():
    """server/NuMA_KV.cpp with the ICCEH backend GpuCCEHHybrid: 8 pinned
    threads of per-op NUMA_KV::Insert / Get (:85-132), then InsertExtent /
    GetExtent page by page (:69-116)."""
    exe = _bin("numa_kv_gpu")
    cpus = _cpus(8)
    r = subprocess.run([exe, "200000", str(len(cpus)), str(cpus[0])], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failedSearch" in r.stdout and "extent_bad 0" in r.stdout


@pytest.mark.parametrize("delivery", [None, "4"])
def test_gpu_kv_harness_zero_failed_search(delivery):
    """Our C++ harness of both facades outside the reference tree: 8 threads,
    counting BF attached (and untouched by extent heads), failure reporting,
    upsert mode, hybrid extents, completion callbacks that block (refused) or
    queue more async ops into a full ring (held, then published)
    (tests/cpp/test_gpu_kv.cpp); delivery "4": the callbacks on four delivery
    threads (PMDFC_DELIVERY_THREADS), the chained ops queued from them into
    other threads' rings."""
    exe = os.path.join(LIB, "test_gpu_kv")
    env = dict(os.environ)
    if delivery:
        env["PMDFC_DELIVERY_THREADS"] = delivery
    r = subprocess.run([exe, "200000", "8"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    for line in ("0 failedSearch", "false_hits 0", "bf_negatives 0", "extent_cbf_changed 0", "extent_bad 0",
                 "failure_report_bad 0", "upsert_bad 0", "callback_block_bad 0", "callback_chain_bad 0", "flood_bad 0",
                 "findany_bad 0", "failed_ops 0"):
        assert line in r.stdout, (line, r.stdout)


def test_frontend_32_callers():
    """The batching front-end at the server's concurrency: 32 per-op callers
    (NUM_CLIENT x NUM_QUEUES, server/rdma_svr.h:17-18)."""
    exe = os.path.join(LIB, "bench_frontend")
    r = subprocess.run([exe, "32", "8192"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["failedSearch"] == 0 and res["failed_ops"] == 0
    assert res["insert_avg_batch"] > 1 and res["get_avg_batch"] > 1  # calls really share batches
