"""Run one forward configuration N times (profiling driver for rocprofv3; no timing logic).

    python tools/run_fwd.py [--B 8 --H 12 --S 2048 --D 64 --causal 0 --p 0 --iters 20 --bwd 0]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
import torch  # noqa: E402
from flash_attn.flash_attn_interface import flash_attn_unpadded_func  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=8)
ap.add_argument("--H", type=int, default=12)
ap.add_argument("--S", type=int, default=2048)
ap.add_argument("--Sk", type=int, default=0)
ap.add_argument("--D", type=int, default=64)
ap.add_argument("--causal", type=int, default=0)
ap.add_argument("--p", type=float, default=0.0)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--bwd", type=int, default=0)
ap.add_argument("--fp16", type=int, default=0)
ap.add_argument("--time", type=int, default=0)
a = ap.parse_args()
Sk = a.Sk or a.S
dt = torch.float16 if a.fp16 else torch.bfloat16
g = torch.Generator().manual_seed(0)
q = torch.randn(a.B * a.S, a.H, a.D, generator=g).to(dt).cuda().requires_grad_(bool(a.bwd))
k = torch.randn(a.B * Sk, a.H, a.D, generator=g).to(dt).cuda().requires_grad_(bool(a.bwd))
v = torch.randn(a.B * Sk, a.H, a.D, generator=g).to(dt).cuda().requires_grad_(bool(a.bwd))
cq = torch.arange(0, (a.B + 1) * a.S, a.S, dtype=torch.int32, device="cuda")
ck = torch.arange(0, (a.B + 1) * Sk, Sk, dtype=torch.int32, device="cuda")
go = torch.randn_like(q)
def step():
    o = flash_attn_unpadded_func(q, k, v, cq, ck, a.S, Sk, a.p, causal=bool(a.causal))
    if a.bwd:
        torch.autograd.grad(o, (q, k, v), go)


for _ in range(a.iters):
    step()
torch.cuda.synchronize()
if a.time:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        step()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    fl = 4.0 * a.B * a.H * a.S * Sk * a.D / (2 if a.causal else 1) * (3.5 if a.bwd else 1.0)
    print(f"B={a.B} H={a.H} S={a.S} Sk={Sk} D={a.D} causal={a.causal} p={a.p} bwd={a.bwd} "
          f"{ms:.4f} ms  {fl / ms / 1e9:.1f} TFLOPS")
print("done")
