"""Host-side cost per call of the drop-in interface on tiny inputs: the host enqueue time per call
(batches well below the launch-queue depth, no device wait inside a batch) and, for reference,
the wall time of 2000 back-to-back calls (bounded below by the device time of a tiny launch).

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
    """Wall time per call of n back-to-back calls including the final sync: the larger of the
    host cost and the device time per call (tiny kernels still take a few us on the device)."""
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) / n * 1e6, 1)


def host_us(fn, n=100, reps=30):
    """Host (enqueue) cost per call: batches of n calls timed on the host without waiting for the
    device (n is far below the launch queue depth, so the host never blocks), synced between
    batches; median over reps batches."""
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    per = []
    for _ in range(reps):
        t = time.perf_counter()
        for _ in range(n):
            fn()
        per.append((time.perf_counter() - t) / n * 1e6)
        torch.cuda.synchronize()
    per.sort()
    return round(per[len(per) // 2], 2)


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

    C = hip._C
    raw = {}
    if C is not None:
        # the C ABI call alone on a pre-packed argument block (no allocation): validation + launch
        o0, l0 = hip.fwd(q, q, q, cu, cu, 64, 64, 0.0, 0.125, False, False, False, None)
        packer, buf, addr, raw_fwd = hip._fwd_call()
        packer.pack_into(buf, 0, q.data_ptr(), q.data_ptr(), q.data_ptr(), o0.data_ptr(), l0.data_ptr(), 0,
                         cu.data_ptr(), cu.data_ptr(), q.stride(0), q.stride(1), q.stride(0), q.stride(1),
                         q.stride(0), q.stride(1), 128, 64, 1, 2, 64, 64, 64, 64, 0, 0, 0.125, 0.0, 0, 0, 0,
                         0, hip.FA_DTYPE_BF16, 0, 0, 0, 0, 0)
        stream = hip._stream_ptr(q.device)
        raw = {"c_abi_fa_fwd_prepacked": lambda: raw_fwd(addr, stream),
               "compiled_fwd_direct": lambda: C.fwd(q, q, q, cu, cu, 64, 64, 0.0, 0.125, False, False, False, 0, 0, 0, 0),
               "compiled_interface_direct": lambda: C.flash_attn_unpadded_func(q, q, q, cu, cu, 64, 64, 0.0, 0.125,
                                                                               False, 0, 0, None, 0),
               "torch_empty_x2": lambda: (torch.empty(64, 2, 64, device=dev, dtype=torch.bfloat16),
                                          torch.empty(1, 2, 64, device=dev))}

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
    cases.update(raw)
    res = {"unit": "us per call, tiny inputs; host_enqueue_us: host time per call without waiting for the "
                   "device (median of 30 batches of 100); wall_us: back-to-back calls incl. the device time",
           "host_enqueue_us": {}, "wall_us": {}}
    for name, fn in cases.items():
        res["host_enqueue_us"][name] = host_us(fn)
        res["wall_us"][name] = per_call_us(fn)
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
