"""The reference's published metric, measured on MI355X: forward+backward speedup of FlashAttention
over PyTorch standard attention (README.md:69-81 charts; benchmarks/benchmark_flash_attention.py).

    python tools/speedup_vs_pytorch.py [--out profiles/rNN_speedup_vs_pytorch.json]

B=8, H=12, D=64, fp16 (the chart's setting), S = 128 ... 4096, three cases as in the charts:
no mask / no dropout, padding mask + dropout 0.1, padding mask only. PyTorch attention is the
benchmark's own expression (q @ (k/sqrt(d)), masked_fill, softmax, F.dropout, @ v) on the padded
batch; FlashAttention runs flash_attn_unpadded_qkvpacked_func on the unpadded qkv, as the
reference benchmark does. Times are medians of CUDA-event timed repeats of forward + backward.
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from flash_attn.bert_padding import unpad_input  # noqa: E402
from flash_attn.flash_attn_interface import flash_attn_unpadded_qkvpacked_func  # noqa: E402


def torch_attention(qkv, attn_mask, dropout_p):
    q, k, v = qkv.unbind(dim=2)
    d = qkv.shape[-1]
    scores = torch.einsum("bthd,bshd->bhts", q, k / math.sqrt(d))
    scores = scores.masked_fill(~attn_mask[:, None, None, :], float("-inf"))
    attention = torch.softmax(scores, dim=-1)
    attention_drop = F.dropout(attention, dropout_p)
    return torch.einsum("bhts,bshd->bthd", attention_drop, v)


def timed(fn, reps=10, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--seqlens", default="128,256,512,1024,2048,4096")
    args = ap.parse_args()
    B, H, D = 8, 12, 64
    dev = "cuda"
    res = {"config": f"B={B} H={H} D={D} fp16, fwd+bwd; speedup = PyTorch ms / FlashAttention ms", "cases": {}}
    for case, (masked, p) in {"no_mask_no_dropout": (False, 0.0), "mask_dropout": (True, 0.1),
                              "mask_only": (True, 0.0)}.items():
        rows = []
        for S in (int(x) for x in args.seqlens.split(",")):
            torch.manual_seed(0)
            qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.float16, requires_grad=True)
            if masked:
                lengths = torch.randint(max(1, S - 20), S + 1, (B, 1), device=dev)
                mask = torch.arange(S, device=dev)[None, :] < lengths
            else:
                mask = torch.ones(B, S, dtype=torch.bool, device=dev)
            g = torch.randn(B, S, H, D, device=dev, dtype=torch.float16)

            def run_torch():
                out = torch_attention(qkv, mask, p)
                torch.autograd.grad(out, (qkv,), g)

            x_u, idx, cu, max_s = unpad_input(qkv.detach().reshape(B, S, -1), mask)
            x_u = x_u.reshape(-1, 3, H, D).requires_grad_()
            g_u = g.reshape(B * S, H, D)[idx]

            def run_flash():
                out = flash_attn_unpadded_qkvpacked_func(x_u, cu, max_s, p)
                torch.autograd.grad(out, (x_u,), g_u)

            t_flash = timed(run_flash)
            try:
                t_torch = timed(run_torch)
            except torch.OutOfMemoryError:
                t_torch = None
            rows.append({"seqlen": S, "flash_ms": round(t_flash, 4), "pytorch_ms": round(t_torch, 4) if t_torch else None,
                         "speedup": round(t_torch / t_flash, 2) if t_torch else None})
            print(case, rows[-1], flush=True)
            del qkv, x_u
            torch.cuda.empty_cache()
        res["cases"][case] = rows
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
