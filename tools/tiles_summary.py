"""Summarise tools/profile_tiles.sh into one JSON per head-dim tile (forward and backward kernels).

    python tools/tiles_summary.py <outdir> > profiles/rNN_tiles_roofline.json

Per kernel: average duration (kernel trace), algorithmic FLOPs and bytes per launch, achieved
TFLOP/s and fraction of the 2516.6 TFLOP/s bf16 MFMA peak, HBM bytes per launch from PMC
(2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md §HBM) and the GB/s
they imply, and MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs).
"""
import collections
import csv
import glob
import json
import sys

OUT = sys.argv[1]
B, H, S = 8, 12, 2048
PEAK_TF, PEAK_GBS = 2516.6, 8000.0


def rows(pattern):
    for f in glob.glob(pattern, recursive=True):
        yield from csv.DictReader(open(f))


def kind(name):
    if "fa_fwd_kernel" in name:
        return "fwd"
    if "fa_bwd_kernel" in name or "fa_bwd_split_kernel" in name:
        return "bwd_main"
    if "fa_bwd_dq_kernel" in name:
        return "bwd_dq"
    if "fa_bwd_dot_kernel" in name:
        return "bwd_delta"
    if "fa_bwd_dq_convert" in name:
        return "bwd_dq_convert"
    return None


res = {}
for D in (32, 64, 128):
    base = f"{OUT}/d{D}"
    dur = collections.defaultdict(list)
    for r in rows(f"{base}/trace/**/*kernel_trace.csv"):
        k = kind(r["Kernel_Name"])
        if k:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)   # us
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ("fetch", "write", "mfma"):
        for r in rows(f"{base}/{sub}/**/*counter_collection.csv"):
            k = kind(r["Kernel_Name"])
            if k:
                pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    fwd_fl = 4.0 * B * H * S * S * D
    # D = 128: the key-major kernel does S, dZ, dV, dK (2.0x forward FLOPs) and no dQ; the
    # query-major dQ pass recomputes S and dP and does dQ (1.5x forward FLOPs), no atomics
    split = D == 128
    alg = {
        "fwd": (fwd_fl, 2 * (2 * B * S * H * D) * 2 + 4 * B * H * S),
        "bwd_main": ((2.0 if split else 2.5) * fwd_fl,
                     (5 * B * S * H * D) * 2 + 8 * B * H * S + (0 if split else 4 * B * S * H * D * (S // 256) * 2)),
        "bwd_dq": (1.5 * fwd_fl, (4 * B * S * H * D) * 2 + 8 * B * H * S),
        "bwd_delta": (0.0, 2 * B * S * H * D * 2 + 4 * B * H * S + 4 * B * S * H * D),
        "bwd_dq_convert": (0.0, 4 * B * S * H * D + 2 * B * S * H * D),
    }
    out = {}
    for k, ds in dur.items():
        ds = sorted(ds)[len(ds) // 5:]       # drop the first (cold) fifth
        us = sum(ds) / len(ds)
        fl, by = alg[k]
        c = {n: sum(v) / len(v) for n, v in pmc[k].items()}
        hbm = 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024 if "FETCH_SIZE" in c and "WRITE_SIZE" in c else None
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        e = {"avg_us": round(us, 2), "flops": fl, "algorithmic_bytes": by,
             "hbm_bytes_pmc": round(hbm) if hbm else None,
             "hbm_GBps_pmc": round(hbm / us / 1e3, 1) if hbm else None,
             "algorithmic_GBps": round(by / us / 1e3, 1), "frac_hbm": round(by / us / 1e3 / PEAK_GBS, 4)}
        if fl:
            e["TFLOPS"] = round(fl / us / 1e6, 1)
            e["frac_mfma_peak"] = round(fl / us / 1e6 / PEAK_TF, 4)
        if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            e["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 4)
        out[k] = e
    res[f"D{D}"] = {"config": f"B={B} H={H} S={S} D={D} bf16 non-causal", "kernels": out}
res["notes"] = ("bwd_main algorithmic bytes count q,k,v,dO reads, dk/dv writes, lse/delta and (D <= 64) the fp32 "
                "dQ atomics (one partial per 256-key block); D = 128 runs the P/dS split kernel plus the query-major "
                "dQ pass (bwd_dq: q,k,v,dO reads, dq write); durations from rocprofv3 kernel trace; PMC passes "
                "run separately (profiled clocks read ~2-5 % low)")
print(json.dumps(res, indent=1))
