"""Summarise tools/clock_probe.sh output: per fa_fwd dispatch, effective clock and MFMA utilisation.

    python tools/clock_summary.py <outdir> [<outdir> ...]
"""
import collections
import csv
import glob
import json
import sys

res = {}
for out in sys.argv[1:]:
    cc = glob.glob(f"{out}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(cc)):
        if "fa_fwd" not in r["Kernel_Name"]:
            continue
        d = per[r["Dispatch_Id"]]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["_start"], d["_end"] = int(r.get("Start_Timestamp", 0) or 0), int(r.get("End_Timestamp", 0) or 0)
    rows = []
    for k, d in per.items():
        dur = (d["_end"] - d["_start"]) * 1e-9
        if dur <= 0:
            continue
        clk = d["GRBM_GUI_ACTIVE"] / 8 / dur
        util = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * d["GRBM_GUI_ACTIVE"] / 8)
        rows.append((dur * 1e6, clk / 1e9, util))
    rows.sort()
    med = rows[len(rows) // 2]
    res[out] = {"dispatches": len(rows), "us_med": round(med[0], 1), "clock_GHz": round(med[1], 3),
                "mfma_pipe_util": round(med[2], 3)}
print(json.dumps(res, indent=1))
