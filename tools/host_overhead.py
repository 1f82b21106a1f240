"""Host-side cost per call of the drop-in interface: tiny inputs (GPU time negligible), so the
wall time of 2000 back-to-back calls is the Python + ctypes + launch cost per call.

    python tools/host_overhead.py [--profile]      (GPU; prints one JSON line)
"""
import cProfile
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
import torch  # noqa: E402
from flash_attn import flash_attn_hip as hip  # noqa: E402
from flash_attn.flash_attention import FlashAttnRotaryQKVFunc  # noqa: E402
from flash_attn.flash_attn_interface import (flash_attn_unpadded_func,  # noqa: E402
                                             flash_attn_unpadded_qkvpacked_func)
from flash_attn.rotary import RotaryEmbedding, apply_rotary_emb_qkv_  # noqa: E402


def per_call_us(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e6, 1)


def main():
    dev = "cuda"
    q = torch.randn(64, 2, 64, device=dev, dtype=torch.bfloat16)
    cu = torch.tensor([0, 64], dtype=torch.int32, device=dev)
    qg, kg, vg = (torch.randn(64, 2, 64, device=dev, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    g = torch.randn(64, 2, 64, device=dev, dtype=torch.bfloat16)
    out = hip.fwd(q, q, q, cu, cu, 64, 64, 0.0, 0.125, False, False, False, None)
    dq, dk, dv = (torch.empty_like(q) for _ in range(3))
    qkv = torch.randn(1, 64, 3, 2, 64, device=dev, dtype=torch.bfloat16)
    cos, sin = RotaryEmbedding(64).to(dev).cos_sin_tables(64, dev, torch.bfloat16)

    class Noop(torch.autograd.Function):
        # torch's own autograd cost: one Function, forward and backward each one tiny kernel
        @staticmethod
        def forward(ctx, x):
            return x.clone()

        @staticmethod
        def backward(ctx, gx):
            return gx.clone()

    def noop_fwd_bwd():
        torch.autograd.grad(Noop.apply(qg), (qg,), g)

    def fwd_bwd():
        o = flash_attn_unpadded_func(qg, kg, vg, cu, cu, 64, 64, 0.0)
        torch.autograd.grad(o, (qg, kg, vg), g)

    cases = {
        "interface_fwd": lambda: flash_attn_unpadded_func(q, q, q, cu, cu, 64, 64, 0.0),
        "interface_fwd_dropout": lambda: flash_attn_unpadded_func(q, q, q, cu, cu, 64, 64, 0.1),
        "hip_fwd": lambda: hip.fwd(q, q, q, cu, cu, 64, 64, 0.0, 0.125, False, False, False, None),
        "hip_bwd": lambda: hip.bwd(q, q, q, q, out[0], out[1], dq, dk, dv, cu, cu, 64, 64, 0.0, 0.125,
                                   False, False, None),
        "autograd_fwd_bwd": fwd_bwd,
        "torch_noop_function_fwd_bwd": noop_fwd_bwd,
        "hip_rotary": lambda: apply_rotary_emb_qkv_(qkv.view(1, 64, -1), cos, sin, 2, 64),
        "rotary_separate_then_fwd": lambda: flash_attn_unpadded_qkvpacked_func(
            apply_rotary_emb_qkv_(qkv.view(1, 64, -1), cos, sin, 2, 64).view(64, 3, 2, 64), cu, 64, 0.0),
        "rotary_fused_fwd": lambda: FlashAttnRotaryQKVFunc.apply(qkv, cos, sin, 0.0, None, False),
    }
    res = {"unit": "us per call (wall, tiny inputs: host-bound)"}
    for name, fn in cases.items():
        res[name] = per_call_us(fn)
    print(json.dumps(res), flush=True)
    if "--profile" in sys.argv:
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(2000):
            cases["interface_fwd"]()
        pr.disable()
        torch.cuda.synchronize()
        pstats.Stats(pr).sort_stats("tottime").print_stats(15)


if __name__ == "__main__":
    main()
