"""Average the PMC counters of one kernel over the passes written by tools/pmc_sweep.sh.

    python tools/pmc_summary.py <outdir> [kernel-substring]
"""
import collections
import csv
import glob
import json
import sys

out = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "fa_fwd_kernel"
agg = collections.defaultdict(list)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
print(json.dumps(res, indent=1))
