"""Per-block fixed cost and per-tile cost of the asm forward forms, from a linear fit of kernel time
against the key length at a fixed query grid (B, H, Sq): T(Sk) = blocks/CU * (fixed + tiles(Sk) * tile).

    python tools/fixed_cost_fit.py [--shape 8,12,2048] [--sks 256,512,1024,2048,4096] [--forms ASM4,ASM4P]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8,12,2048")
    ap.add_argument("--sks", default="256,512,1024,2048,4096")
    ap.add_argument("--forms", default="ASM4,ASM4P")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--d", type=int, default=64)
    args = ap.parse_args()
    import torch
    from flash_attn import flash_attn_hip as hip
    from flash_attn.flash_attn_interface import flash_attn_unpadded_func
    B, H, Sq = (int(x) for x in args.shape.split(","))
    sks = [int(x) for x in args.sks.split(",")]
    D = args.d
    g = torch.Generator().manual_seed(0)
    q = torch.randn(B * Sq, H, D, generator=g).bfloat16().cuda()
    cq = torch.arange(0, (B + 1) * Sq, Sq, dtype=torch.int32, device="cuda")
    kv = {}
    for sk in sks:
        k = torch.randn(B * sk, H, D, generator=g).bfloat16().cuda()
        v = torch.randn(B * sk, H, D, generator=g).bfloat16().cuda()
        ck = torch.arange(0, (B + 1) * sk, sk, dtype=torch.int32, device="cuda")
        kv[sk] = (k, v, ck)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nblk = (Sq + 255) // 256 * H * B
    res = {}
    for form in args.forms.split(","):
        impl = getattr(hip, f"FA_IMPL_{form}")
        with hip.force_impl(impl):
            for sk in sks:   # warm-up (clock ramp)
                k, v, ck = kv[sk]
                for _ in range(30):
                    flash_attn_unpadded_func(q, k, v, cq, ck, Sq, sk, 0.0)
            torch.cuda.synchronize()
            for rnd in range(3):
                for sk in sks:
                    k, v, ck = kv[sk]
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(args.iters):
                        flash_attn_unpadded_func(q, k, v, cq, ck, Sq, sk, 0.0)
                    e.record()
                    torch.cuda.synchronize()
                    res.setdefault((form, sk), []).append(s.elapsed_time(e) / args.iters * 1e3)
    rounds = nblk / ncu
    for form in args.forms.split(","):
        xs = np.array([sk / 64 for sk in sks])
        ys = np.array([np.median(res[(form, sk)]) for sk in sks])
        slope, icpt = np.polyfit(xs, ys, 1)
        print(f"{form}: " + "  ".join(f"Sk={sk}: {y:.2f} us" for sk, y in zip(sks, ys)))
        print(f"{form}: fit per block-round: fixed {icpt / rounds:.3f} us + {slope / rounds * 1e3:.1f} ns/tile "
              f"({rounds:.2f} block rounds; residual max {np.abs(ys - (slope * xs + icpt)).max():.2f} us)", flush=True)


if __name__ == "__main__":
    main()
