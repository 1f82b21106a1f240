"""Steady-state driver of one configuration for the per-tile roofline (profiles/r0N_tiles_roofline.json).

    python tools/tiles_run.py --cfg D64 --mode fwd [--launches 200] [--warm 0.3]

Runs the product binding (flash_attn_hip.fwd / .bwd, the calls flash_attn_interface makes) for
one mode only: `fwd` repeats the forward; `bwd` runs one forward, then repeats the backward on
its saved outputs (no forward in the timed loop). A warm-up of at least `--warm` seconds comes
first (clock ramp), then `--launches` calls bracketed by HIP events on the binding's stream; one
JSON line reports the event time per call. Under rocprofv3 the last `--launches` dispatches of
each kernel are the timed ones (tools/tiles_summary.py takes exactly those).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
import torch  # noqa: E402
from flash_attn import flash_attn_hip as hip  # noqa: E402

# name: (B, H, Sq, Sk, D, dtype, causal, dropout, kvpacked)
CFGS = {
    "D32": (8, 12, 2048, 2048, 32, "bf16", False, 0.0, False),
    "D64": (8, 12, 2048, 2048, 64, "bf16", False, 0.0, False),
    "D80": (8, 12, 2048, 2048, 80, "bf16", False, 0.0, False),
    "D96": (8, 12, 2048, 2048, 96, "bf16", False, 0.0, False),
    "D128": (8, 12, 2048, 2048, 128, "bf16", False, 0.0, False),
    "D128b16": (16, 12, 4096, 4096, 128, "bf16", False, 0.0, False),   # C4's shape, non-causal
    "C2": (8, 12, 512, 512, 64, "fp16", False, 0.0, False),
    "C3": (8, 12, 2048, 2048, 64, "bf16", True, 0.1, False),
    "C3nd": (8, 12, 2048, 2048, 64, "bf16", True, 0.0, False),    # C3 without dropout (its cost)
    "C4": (16, 12, 4096, 4096, 128, "bf16", True, 0.0, False),
    "C5": (4, 16, 1024, 4096, 64, "bf16", False, 0.0, True),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", required=True, help="a CFGS name or B,H,Sq,Sk,D[,c] (bf16; c: causal)")
    ap.add_argument("--mode", required=True, choices=["fwd", "bwd"])
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--warm", type=float, default=0.3)
    ap.add_argument("--impl", default="auto", choices=["auto", "hip", "asm4", "asm4p"],
                    help="forward kernel family (FaFwdArgs.impl)")
    a = ap.parse_args()
    if a.cfg in CFGS:
        B, H, Sq, Sk, D, dts, causal, p, kvpacked = CFGS[a.cfg]
    else:
        f = a.cfg.split(",")
        B, H, Sq, Sk, D = map(int, f[:5])
        dts, causal, p, kvpacked = "bf16", len(f) > 5 and f[5] == "c", 0.0, False
    dt = torch.float16 if dts == "fp16" else torch.bfloat16
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B * Sq, H, D, generator=g, device=dev).to(dt)
    if kvpacked:
        kv = torch.randn(B * Sk, 2, H, D, generator=g, device=dev).to(dt)
        k, v = kv[:, 0], kv[:, 1]
    else:
        k = torch.randn(B * Sk, H, D, generator=g, device=dev).to(dt)
        v = torch.randn(B * Sk, H, D, generator=g, device=dev).to(dt)
    cu_q = torch.arange(0, (B + 1) * Sq, Sq, dtype=torch.int32, device=dev)
    cu_k = torch.arange(0, (B + 1) * Sk, Sk, dtype=torch.int32, device=dev)
    scale = D ** -0.5
    rng = hip.reserve_rng(dev) if p > 0 else None

    def fwd():
        return hip.fwd(q, k, v, cu_q, cu_k, Sq, Sk, p, scale, False, causal, False, None, rng_state=rng,
                       impl=getattr(hip, "FA_IMPL_" + a.impl.upper()))

    if a.mode == "fwd":
        step = fwd
    else:
        out, lse = fwd()
        dout = torch.randn(out.shape, generator=g, device=dev).to(dt)
        dq = torch.empty_like(q)
        if kvpacked:
            dkv = torch.empty_like(kv)
            dk, dv = dkv[:, 0], dkv[:, 1]
        else:
            dk, dv = torch.empty_like(k), torch.empty_like(v)

        def step():
            hip.bwd(dout, q, k, v, out, lse, dq, dk, dv, cu_q, cu_k, Sq, Sk, p, scale, False, causal, None,
                    rng_state=rng)
    # warm-up: at least `warm` seconds of back-to-back calls
    t0 = time.perf_counter()
    n_warm = 0
    while True:
        step()
        n_warm += 1
        if n_warm % 10 == 0:
            torch.cuda.synchronize()
            if time.perf_counter() - t0 >= a.warm:
                break
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.launches):
        step()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / a.launches
    print(json.dumps({"cfg": a.cfg, "mode": a.mode, "impl": a.impl, "launches": a.launches, "warmup_calls": n_warm,
                      "warmup_s": round(time.perf_counter() - t0 - s.elapsed_time(e) / 1e3, 3),
                      "event_us_per_call": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
