"""Copy one round-end profile run (tools/round_end_profile.sh) into profiles/ under a round tag.

    python tools/collect_profiles.py gpurun_out/<tag> <round>      e.g. gpurun_out/r02a r02

Writes <round>_fwd_bench_kernel_stats.csv, <round>_{c2,c3,c4,c5}_kernel_stats.csv, <round>_bench.json
and <round>_fwd_pmc.json (HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE with the gfx950 FETCH
correction of MI355X_MICROARCH.md §HBM; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs /
(GRBM_GUI_ACTIVE / 8 XCDs)).
"""
import csv
import glob
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")


def one(pattern):
    f = glob.glob(os.path.join(src, pattern), recursive=True)
    return f[0] if f else None


f = one("prof_bench/**/*kernel_stats.csv")
if f:
    shutil.copy(f, os.path.join(prof, f"{tag}_fwd_bench_kernel_stats.csv"))
for c in ("c2", "c3", "c4", "c5"):
    f = one(f"prof_{c}/**/*kernel_stats.csv")
    if f:
        shutil.copy(f, os.path.join(prof, f"{tag}_{c}_kernel_stats.csv"))
b = os.path.join(src, "bench.json.log")
bench = None
if os.path.exists(b):
    line = [l for l in open(b) if l.startswith("{")][-1]
    bench = json.loads(line)
    json.dump(bench, open(os.path.join(prof, f"{tag}_bench.json"), "w"), indent=1)
KERN = (bench or {}).get("roofline", {}).get("kernel") or "fa_fwd_d64p_bf16_asm"

# the bench line recomputed from the rocprofv3 kernel-trace summary of the same command, same lease
f = one("prof_bench/**/*kernel_stats.csv")
if bench and f:
    row = next((r for r in csv.DictReader(open(f)) if r["Name"] == KERN), None)
    if row:
        rf = bench["roofline"]
        avg_ms = float(row["AverageNs"]) / 1e6
        ach = rf["flops_per_launch"] / (avg_ms * 1e-3) / 1e12
        chk = {"kernel": KERN, "rocprof_calls": int(row["Calls"]), "rocprof_avg_ms": round(avg_ms, 5),
               "bench_avg_kernel_ms": rf["avg_kernel_ms"], "recomputed_achieved_tflops": round(ach, 2),
               "bench_achieved_tflops": rf["achieved"], "recomputed_frac": round(ach / rf["peak"], 4),
               "bench_frac": rf["frac"], "ratio": round(rf["avg_kernel_ms"] / avg_ms, 4)}
        chk["within_2pct"] = abs(chk["ratio"] - 1) <= 0.02
        json.dump(chk, open(os.path.join(prof, f"{tag}_bench_check.json"), "w"), indent=1)
        print(json.dumps(chk, indent=1))


def pmc(pattern, kern=KERN):
    agg = {}
    n = {}
    for f in glob.glob(os.path.join(src, pattern, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                key = (r["Counter_Name"], r["Dispatch_Id"])
                agg[key] = agg.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (name, _), v in agg.items():
        out.setdefault(name, []).append(v)
    return {k: sum(v) / len(v) for k, v in out.items()}


fe, wr, mf = pmc("pmc_fetch"), pmc("pmc_write"), pmc("pmc_mfma")
if fe and wr:
    hbm = 2 * fe["FETCH_SIZE"] * 1024 + wr["WRITE_SIZE"] * 1024
    res = {"kernel": KERN, "config": "B=8 H=12 S=2048 D=64",
           "FETCH_SIZE_KB": round(fe["FETCH_SIZE"], 2), "WRITE_SIZE_KB": round(wr["WRITE_SIZE"], 2),
           "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts half of 16B/lane "
                         "streaming reads, MI355X_MICROARCH.md §HBM)",
           "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes_per_launch": 101449728}
    if mf:
        res.update({"mfma_busy_frac": mf["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (mf["GRBM_GUI_ACTIVE"] / 8),
                    "SQ_INSTS_MFMA": mf["SQ_INSTS_MFMA"], "SQ_INSTS_VALU": mf["SQ_INSTS_VALU"],
                    "GRBM_GUI_ACTIVE": mf["GRBM_GUI_ACTIVE"]})
    res["source"] = f"tools/round_end_profile.sh (separate PMC passes, 5 launches each), {src}"
    json.dump(res, open(os.path.join(prof, f"{tag}_fwd_pmc.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))
