"""Calibration of the CPU baseline (build container only; TEST INFRASTRUCTURE).

bench.py's cpu_baseline times oracle/cceh_mt.c, the concurrent restatement of
CCEH_hybrid, because the reference source never travels to the GPU box.  This
script times it beside the reference's own CCEH_hybrid.cpp (oracle/_ref/
ref_driver, `bench` mode: test_KV's thread pattern, clflush emulation compiled
in as in the reference) on the same keys and thread counts, and writes
profiles/r02/cpu_calibration.json.  Both unpinned (ref_driver does not pin).
usage: python oracle/bench_cpu.py [n_keys] [threads ...]"""
import json
import math
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

from oracle import oracle as O  # noqa: E402
from pmdfc_amd.workload import uniform_keys  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 23
    ts = [int(x) for x in sys.argv[2:]] or [1, 4, 8]
    ref = os.path.join(HERE, "_ref", "ref_driver")
    if not os.path.exists(ref):
        sys.exit("oracle/_ref/ref_driver missing: make -C oracle ref (needs /root/reference)")
    init_cap = max(2, n // 1024)  # config 2's load trajectory (64M keys into 65536)
    depth = int(math.log2(init_cap))
    keys = uniform_keys(1000, 0, n)  # == ref_driver's splitmix stream with seed 1000
    rows = []
    for T in ts:
        out = subprocess.run([ref, "bench", str(n), str(T), str(init_cap), "1000"], capture_output=True, text=True,
                             check=True, timeout=1200).stdout.split()
        ri, rg, rf = float(out[0]), float(out[1]), int(out[2])
        p = O.mt_bench(depth, keys, T, cpus=None, flush_ns=10)
        row = {"threads": T,
               "reference": {"insert_mops": round(n / ri / 1e6, 3), "get_mops": round(n / rg / 1e6, 3),
                             "mops": round(2 * n / (ri + rg) / 1e6, 3), "failedSearch": rf},
               "port": {"insert_mops": round(n / p["insert_s"] / 1e6, 3), "get_mops": round(n / p["get_s"] / 1e6, 3),
                        "mops": round(2 * n / (p["insert_s"] + p["get_s"]) / 1e6, 3), "failedSearch": p["failed"]}}
        row["port_over_reference"] = round(row["port"]["mops"] / row["reference"]["mops"], 3)
        rows.append(row)
        print(json.dumps(row), flush=True)
    res = {"what": "oracle/cceh_mt.c (port, -O3) vs the reference CCEH_hybrid.cpp (oracle/_ref/ref_driver, -O2), "
                   f"same {n} keys (rank-0 stream), CCEH_hybrid({init_cap}), insert (clflush emulation on) then Get, "
                   "unpinned threads, build container", "cpus": os.cpu_count(), "rows": rows}
    out = os.path.join(REPO, "profiles", "r02", "cpu_calibration.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
