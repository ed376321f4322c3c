"""Counter calibration factors from tools/calib_fetch.py's two PMC passes:
algorithmic bytes / counted bytes per access shape (FETCH_SIZE and WRITE_SIZE
in KiB, MI355X_MICROARCH.md rocprofv3 section).  The k_gather dispatches
are matched in launch order; the streaming copy is the last dispatch that
is not a k_gather.  usage: calib_summary.py OUT.json PLAN.json FETCH_DIR WRITE_DIR"""
import csv
import json
import os
import sys

out, plan_f, fdir, wdir = sys.argv[1:5]
plan = json.loads(open(plan_f).read().strip().splitlines()[0])


def rows(d, counter):
    r = [x for x in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))) if x["Counter_Name"] == counter]
    r.sort(key=lambda x: int(x.get("Dispatch_Id") or x.get("Correlation_Id") or 0))
    return r


res = {"source": "tools/calib_fetch.py under rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)",
       "shapes": []}
for counter, d in (("FETCH_SIZE", fdir), ("WRITE_SIZE", wdir)):
    rs = rows(d, counter)
    g = [x for x in rs if "k_gather" in x["Kernel_Name"]]
    other = [x for x in rs if "k_gather" not in x["Kernel_Name"]]
    gi = 0
    for p in plan:
        if p["kernel"] == "k_gather":
            x = g[gi]
            gi += 1
        else:
            x = other[-1]
        key = "read_bytes" if counter == "FETCH_SIZE" else "write_bytes"
        counted = float(x["Counter_Value"]) * 1024
        p.setdefault("counted", {})[counter] = int(counted)
        if p[key]:
            p.setdefault("algorithmic_over_counted", {})[counter] = round(p[key] / counted, 4)
res["shapes"] = plan
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
