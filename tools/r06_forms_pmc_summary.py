"""Summarise tools/r05/forms_pmc.sh output (tools only): per leg, each counter averaged over the dispatches
of the forward kernel (fa_fwd_d64p_*), plus MFMA busy per SIMD-cycle, co-execution share and wave-cycle
waits.   python tools/r06_forms_pmc_summary.py gpurun_out/<tag>/forms_pmc > profiles/<...>.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
out = {"config": "north star forward B8 H12 S2048 D64 bf16, tools/r05/forms_pmc.sh (tiles_run, 5 launches after "
                 "0.05 s warm-up), averages per kernel launch", "legs": {}}
for leg in sorted(os.listdir(root)):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(root, leg, "p*", "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "fa_fwd_d64p" in r["Kernel_Name"]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not vals:
        continue
    d = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
        d["mfma_busy"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (d["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_VALU_MFMA_COEXEC_CYCLES" in d and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
        d["coexec_over_mfma_busy"] = d["SQ_VALU_MFMA_COEXEC_CYCLES"] / d["SQ_VALU_MFMA_BUSY_CYCLES"]
    if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d:
        d["wait_any_over_wave_cycles"] = d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
        d["wait_inst_any_over_wave_cycles"] = d.get("SQ_WAIT_INST_ANY", 0) / d["SQ_WAVE_CYCLES"]
    out["legs"][leg] = d
print(json.dumps(out, indent=1))
