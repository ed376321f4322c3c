"""Mean per-dispatch PMC values per kernel from rocprofv3 counter CSVs
(one counter pass each, e.g. FETCH_SIZE and WRITE_SIZE), written as JSON.

HBM traffic per launch follows the MI355X guide's rocprofv3 section: the
TCC-derived FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced streaming reads, so it is doubled ("upper":
all reads counted as if streaming) and also kept as counted ("lower").
usage: pmc_summary.py OUT.json PASS_DIR [PASS_DIR ...]"""
import collections
import csv
import json
import os
import sys

out = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[2:]:
    for x in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = x["Kernel_Name"].split("(")[0].replace("pmdfc::", "").replace("void ", "")
        vals[k][x["Counter_Name"]].append(float(x["Counter_Value"]))
res = {}
for k, cs in vals.items():
    if not k.startswith("k_"):
        continue
    r = {c: sum(v) / len(v) for c, v in cs.items()}
    r["dispatches"] = max(len(v) for v in cs.values())
    if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
        f, w = r["FETCH_SIZE"] * 1024, r["WRITE_SIZE"] * 1024
        r["hbm_bytes_lower"] = int(f + w)
        r["hbm_bytes_upper"] = int(2 * f + w)
    res[k] = r
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps({k: {c: round(v, 1) for c, v in r.items()} for k, r in res.items()}, indent=1))
