"""Where the bench's wall-clock region spends time beyond its kernels (tools only).

bench.py times K forward steps between two torch.cuda.synchronize() calls with perf_counter; its
roofline block times the same steps with HIP events. This script repeats that timed region for
several K and splits the wall time into: the event span (s recorded right after the first
synchronize, e after the last step), the kernels' own time (K x the event time per call of a long
back-to-back run) and the remainder (submission latency before the first kernel, gaps between
kernels, the final synchronize's wake-up).

    python tools/bench_overhead.py > gpurun_out/bench_overhead.txt
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from flash_attn.flash_attn_interface import flash_attn_unpadded_func  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, H, S, D = 8, 12, 2048, 64
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(B * S, H, D, generator=g).bfloat16().to(dev) for _ in range(3))
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=dev)
    step = lambda: flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0)
    for _ in range(300):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
        for _ in range(20):
            step()
        torch.cuda.synchronize()
    # kernel time per call: a long back-to-back run
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(400):
        step()
    e.record()
    torch.cuda.synchronize()
    per_call = s.elapsed_time(e) / 400
    print(json.dumps({"event_ms_per_call_400": round(per_call, 5)}), flush=True)
    # idle synchronize, and the wake-up after an already finished kernel
    t = time.perf_counter()
    for _ in range(100):
        torch.cuda.synchronize()
    idle_sync_us = (time.perf_counter() - t) / 100 * 1e6
    step()
    t = time.perf_counter()
    while time.perf_counter() - t < 0.002:
        pass
    t = time.perf_counter()
    torch.cuda.synchronize()
    done_sync_us = (time.perf_counter() - t) * 1e6
    print(json.dumps({"idle_sync_us": round(idle_sync_us, 2), "sync_after_finished_kernel_us": round(done_sync_us, 2)}),
          flush=True)
    for K in (20, 50, 200, 20, 50, 200):
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        s.record()
        for _ in range(K):
            step()
        e.record()
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        span = s.elapsed_time(e) / 1e3
        print(json.dumps({"K": K, "wall_ms": round(wall * 1e3, 4), "event_span_ms": round(span * 1e3, 4),
                          "kernels_ms": round(K * per_call, 4), "enqueue_ms": round(t_enq * 1e3, 4),
                          "wall_minus_span_us": round((wall - span) * 1e6, 1),
                          "span_minus_kernels_us": round((span - K * per_call * 1e-3) * 1e6, 1),
                          "wall_ms_per_step": round(wall * 1e3 / K, 5)}), flush=True)


if __name__ == "__main__":
    main()
