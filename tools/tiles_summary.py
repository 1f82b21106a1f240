"""Summarise tools/tiles.sh into profiles/r0N_tiles_roofline.json.

    python tools/tiles_summary.py <outdir> > profiles/r0N_tiles_roofline.json

Per configuration and mode (fwd-only loop / bwd-only loop):
  * per kernel: average duration over the timed (last) dispatches of the kernel-trace pass,
    dispatches per call, PMC per dispatch: HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB counters;
    FETCH_SIZE doubled: the gfx950 correction of MI355X_MICROARCH.md §HBM), MFMA busy =
    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), SQ_INSTS_MFMA/VALU;
  * per call: the trace time (sum over kernels), the driver's HIP-event time and their ratio
    (steady state: within 5 %), algorithmic FLOPs (forward 4 B H Sq Sk D, halved for causal
    Sq == Sk; backward 2.5x that) and bytes (q, k, v, o once each way, lse; backward q, k, v, o,
    dO reads, dq, dk, dv writes, lse / delta), achieved TFLOP/s and fraction of the 2516.6
    TFLOP/s bf16/fp16 MFMA peak, algorithmic and PMC GB/s against 8 TB/s.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tiles_run import CFGS  # noqa: E402

PEAK_TF, PEAK_GBS = 2516.6, 8000.0


def rows(pattern):
    for f in glob.glob(pattern, recursive=True):
        yield from csv.DictReader(open(f))


def driver_line(path):
    for ln in open(path):
        if ln.startswith("{") and '"event_us_per_call"' in ln:
            return json.loads(ln)
    return None


def main(out):
    res = {}
    for cfg, (B, H, Sq, Sk, D, dts, causal, p, kvp) in CFGS.items():
        fwd_fl = 4.0 * B * H * Sq * Sk * D * (0.5 if causal and Sq == Sk else 1.0)
        alg = {"fwd": (fwd_fl, 2 * 2 * B * H * D * (Sq + Sk) + 4 * B * H * Sq),
               "bwd": (2.5 * fwd_fl, 2 * 4 * B * H * D * (Sq + Sk) + 12 * B * H * Sq)}
        entry = {"config": f"B={B} H={H} Sq={Sq} Sk={Sk} D={D} {dts} {'causal' if causal else 'non-causal'}"
                           f"{f' dropout={p}' if p else ''}{' kv-packed' if kvp else ''}"}
        for mode in ("fwd", "bwd"):
            base = f"{out}/{cfg}.{mode}"
            drv = driver_line(f"{out}/{cfg}.{mode}.trace.log") if os.path.exists(f"{out}/{cfg}.{mode}.trace.log") else None
            if not drv:
                continue
            calls = drv["launches"] + drv["warmup_calls"] + (1 if mode == "bwd" else 0)
            disp = collections.defaultdict(list)
            for r in rows(f"{base}/trace/**/*kernel_trace.csv"):
                disp[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            pmc = collections.defaultdict(lambda: collections.defaultdict(list))
            for sub in ("fetch", "write", "mfma"):
                for r in rows(f"{base}/{sub}/**/*counter_collection.csv"):
                    pmc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            kern, total = {}, 0.0
            for name, ds in disp.items():
                per_call = len(ds) / calls
                if per_call < 0.5:          # the single forward of a bwd-mode run, setup kernels
                    continue
                n_timed = int(round(per_call * drv["launches"]))
                ds = sorted(ds)[-n_timed:]
                us = sum(e - s for s, e in ds) / len(ds) / 1e3
                total += us * per_call
                c = {k: sum(v) / len(v) for k, v in pmc[name].items()}
                e = {"avg_us": round(us, 2), "dispatches_per_call": round(per_call, 2), "timed_dispatches": len(ds)}
                if "FETCH_SIZE" in c:
                    e["fetch_bytes_corrected"] = round(2 * c["FETCH_SIZE"] * 1024)
                if "WRITE_SIZE" in c:
                    e["write_bytes"] = round(c["WRITE_SIZE"] * 1024)
                if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                    hbm = 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
                    e["hbm_bytes_pmc"] = round(hbm)
                    e["hbm_GBps_pmc"] = round(hbm / us / 1e3, 1)
                if c.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    e["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 4)
                for k in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU"):
                    if k in c:
                        e[k] = round(c[k])
                kern[name.split("(")[0][:120]] = e
            fl, by = alg[mode]
            ratio = total / drv["event_us_per_call"] if drv["event_us_per_call"] else None
            hbm_call = sum(k.get("hbm_bytes_pmc", 0) * k["dispatches_per_call"] for k in kern.values())
            entry[mode] = {
                "trace_us_per_call": round(total, 2), "event_us_per_call": drv["event_us_per_call"],
                "trace_over_event": round(ratio, 4) if ratio else None,
                "warmup_s": drv["warmup_s"], "timed_calls": drv["launches"],
                "flops": fl, "TFLOPS": round(fl / total / 1e6, 1), "frac_mfma_peak": round(fl / total / 1e6 / PEAK_TF, 4),
                "algorithmic_bytes": by, "algorithmic_GBps": round(by / total / 1e3, 1),
                "hbm_bytes_pmc_per_call": round(hbm_call) or None,
                "hbm_over_algorithmic": round(hbm_call / by, 3) if hbm_call else None,
                "kernels": kern}
        res[cfg] = entry
    res["notes"] = ("durations: rocprofv3 kernel trace of a steady-state single-mode loop (>= 0.3 s warm-up, the last "
                    "200 calls' dispatches); event time: HIP events around the same 200 calls in the same process; PMC "
                    "from separate short passes (10 calls, profiled clocks read a few % low); bwd mode runs the "
                    "backward on one forward's outputs, so its kernels exclude the forward")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
