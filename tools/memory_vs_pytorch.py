"""The reference's memory metric on MI355X: peak device memory of FlashAttention against PyTorch
standard attention (README.md:84-90 chart "10X memory savings at 2K, 20X at 4K"), measured the way
benchmarks/utils.py:119-129 (benchmark_memory) does: empty_cache, reset_peak_memory_stats, one
call, max_memory_allocated. The call is the forward on inputs that require grad (what training
keeps alive for the backward), and separately forward + backward.

    python tools/memory_vs_pytorch.py [--out profiles/r02_memory_vs_pytorch.json]

B=8, H=12, D=64, fp16, no mask, no dropout (the chart notes the footprint is the same with
dropout or masking). PyTorch attention = tools/speedup_vs_pytorch.torch_attention (the benchmark's
expression). Memory in MB (2^20 B): the call's peak growth plus its inputs (qkv and the output
gradient), i.e. what benchmark_memory reports in a process that holds nothing else.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from flash_attn.flash_attn_interface import flash_attn_unpadded_qkvpacked_func  # noqa: E402
from speedup_vs_pytorch import torch_attention  # noqa: E402


def peak_mb(fn, input_bytes):
    """benchmark_memory's max_memory_allocated, made independent of what else the process holds
    (the hipBLAS workspace torch keeps after its first GEMM, earlier iterations' caches): the peak
    growth over the allocation at the call, plus the call's own input bytes."""
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    fn()
    torch.cuda.synchronize()
    m = (torch.cuda.max_memory_allocated() - base + input_bytes) / 2 ** 20
    torch.cuda.empty_cache()
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--seqlens", default="128,256,512,1024,2048,4096")
    args = ap.parse_args()
    B, H, D = 8, 12, 64
    rows = []
    for S in [int(s) for s in args.seqlens.split(",")]:
        qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.float16, requires_grad=True)
        g = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16)
        mask = torch.ones(B, S, dtype=torch.bool, device="cuda")
        qkv_u = qkv.detach().reshape(B * S, 3, H, D).requires_grad_()
        cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device="cuda")
        keep = {}

        def f_fwd():
            keep["o"] = flash_attn_unpadded_qkvpacked_func(qkv_u, cu, S, 0.0)

        def t_fwd():
            keep["o"] = torch_attention(qkv, mask, 0.0)

        def f_fb():
            flash_attn_unpadded_qkvpacked_func(qkv_u, cu, S, 0.0).backward(g.reshape(B * S, H, D))

        def t_fb():
            torch_attention(qkv, mask, 0.0).backward(g)

        inb = qkv.numel() * qkv.element_size() + g.numel() * g.element_size()
        r = {"seqlen": S}
        for name, fn in (("flash_fwd_MB", f_fwd), ("pytorch_fwd_MB", t_fwd), ("flash_fwd_bwd_MB", f_fb),
                         ("pytorch_fwd_bwd_MB", t_fb)):
            keep.clear()
            qkv.grad = None
            qkv_u.grad = None
            r[name] = round(peak_mb(fn, inb), 1)
            keep.clear()
        r["saving_fwd"] = round(r["pytorch_fwd_MB"] / r["flash_fwd_MB"], 2)
        r["saving_fwd_bwd"] = round(r["pytorch_fwd_bwd_MB"] / r["flash_fwd_bwd_MB"], 2)
        rows.append(r)
        print(json.dumps(r), flush=True)
        del qkv, qkv_u, g
    res = {"metric": "peak device memory, FlashAttention vs PyTorch standard attention (benchmark_memory)",
           "config": "B=8 H=12 D=64 fp16, no mask, no dropout", "gpu": torch.cuda.get_device_name(),
           "reference_A100_chart": {"2048": "10x", "4096": "20x"}, "rows": rows}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
