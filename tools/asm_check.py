"""asm_check.py — GPU check of the hand-scheduled assembly forward against the HIP kernel and an
fp32 reference, plus a timing A/B at the BASELINE shapes (one process, interleaved).

    python tools/asm_check.py [--quick]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
import torch  # noqa: E402
from flash_attn import flash_attn_hip as H  # noqa: E402


def ref_attn(q, k, v, cq, ck, scale):
    out = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
    lse = []
    for b in range(len(cq) - 1):
        qs, ks = slice(cq[b], cq[b + 1]), slice(ck[b], ck[b + 1])
        s = torch.einsum("qhd,khd->hqk", q[qs].float(), k[ks].float()) * scale
        if s.shape[-1] == 0:
            lse.append(torch.full(s.shape[:2], -math.inf, device=q.device))
            continue
        p = torch.softmax(s, -1)
        out[qs] = torch.einsum("hqk,khd->qhd", p, v[ks].float())
        lse.append(torch.logsumexp(s, -1))
    return out, lse


def case(B, Hh, sq, sk, D, dtype, ragged=False, seed=0, kvpacked=False, check_ref=True):
    g = torch.Generator(device="cpu").manual_seed(seed)
    if ragged:
        lq = torch.randint(1, sq + 1, (B,), generator=g)
        lk = torch.randint(0, sk + 1, (B,), generator=g)
    else:
        lq = torch.full((B,), sq)
        lk = torch.full((B,), sk)
    cq = [0] + torch.cumsum(lq, 0).tolist()
    ck = [0] + torch.cumsum(lk, 0).tolist()
    dev = "cuda"
    q = torch.randn(cq[-1], Hh, D, generator=g).to(dtype).to(dev)
    if kvpacked:
        kv = torch.randn(ck[-1], 2, Hh, D, generator=g).to(dtype).to(dev)
        k, v = kv[:, 0], kv[:, 1]
    else:
        k = torch.randn(ck[-1], Hh, D, generator=g).to(dtype).to(dev)
        v = torch.randn(ck[-1], Hh, D, generator=g).to(dtype).to(dev)
    cqt = torch.tensor(cq, dtype=torch.int32, device=dev)
    ckt = torch.tensor(ck, dtype=torch.int32, device=dev)
    scale = D ** -0.5
    mq, mk = int(lq.max()), int(lk.max())
    run = lambda impl: H.fwd(q, k, v, cqt, ckt, mq, mk, 0.0, scale, False, False, False, None, impl=impl)
    oa, la = run(H.FA_IMPL_AUTO)
    oh, lh = run(H.FA_IMPL_HIP)
    torch.cuda.synchronize()
    res = {"shape": f"B{B} H{Hh} {sq}x{sk} D{D} {str(dtype)[6:]}{' ragged' if ragged else ''}{' kvpacked' if kvpacked else ''}"}
    res["asm_vs_hip_out"] = (oa.float() - oh.float()).abs().max().item()
    fin = torch.isfinite(lh)
    res["asm_vs_hip_lse"] = (la[fin] - lh[fin]).abs().max().item() if fin.any() else 0.0
    res["lse_inf_match"] = bool(((la == -math.inf) == (lh == -math.inf))[:, :, :mq].all().item()) if not ragged else None
    if check_ref:
        r, rl = ref_attn(q, k, v, cq, ck, scale)
        res["asm_vs_ref"] = (oa.float() - r).abs().max().item()
        res["hip_vs_ref"] = (oh.float() - r).abs().max().item()
        el = 0.0
        for b in range(B):
            n = cq[b + 1] - cq[b]
            a_ = la[b, :, :n]
            fr = torch.isfinite(rl[b])
            if fr.any():
                el = max(el, (a_[fr] - rl[b][fr]).abs().max().item())
            if (~fr).any():
                el = max(el, 0.0 if bool((a_[~fr] == -math.inf).all()) else float("inf"))
        res["asm_lse_vs_ref"] = el
        res["nonfinite_out"] = int((~torch.isfinite(oa)).sum().item())
    return res, run


def timeit(fn, n=50, reps=5):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / n)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--time", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    cases = [(1, 1, 64, 64, 64, torch.bfloat16, False), (2, 2, 130, 200, 64, torch.bfloat16, False),
             (1, 2, 300, 77, 64, torch.float16, False), (4, 3, 257, 190, 64, torch.bfloat16, True),
             (3, 2, 100, 150, 48, torch.bfloat16, True), (2, 2, 1000, 1000, 40, torch.float16, True),
             (1, 1, 1, 1, 64, torch.bfloat16, False), (2, 4, 600, 0, 64, torch.bfloat16, False)]
    if not args.quick:
        cases += [(8, 12, 512, 512, 64, torch.float16, False), (8, 12, 2048, 2048, 64, torch.bfloat16, False)]
    out = []
    for B, Hh, sq, sk, D, dt, rg in cases:
        r, _ = case(B, Hh, sq, sk, D, dt, ragged=rg, check_ref=(B * Hh * sq * sk <= 8 * 12 * 2048 * 2048))
        print(json.dumps(r), flush=True)
        out.append(r)
    r, _ = case(4, 16, 1024, 4096, 64, torch.bfloat16, kvpacked=True)
    print(json.dumps(r), flush=True)
    if args.time:
        for (B, Hh, sq, sk, dt, kvp) in [(8, 12, 2048, 2048, torch.bfloat16, False), (8, 12, 512, 512, torch.float16, False),
                                         (4, 16, 1024, 4096, torch.bfloat16, True), (16, 12, 2048, 2048, torch.bfloat16, False)]:
            _, run = case(B, Hh, sq, sk, 64, dt, kvpacked=kvp, check_ref=False)
            fl = 4.0 * B * Hh * sq * sk * 64
            ta = timeit(lambda: run(H.FA_IMPL_AUTO))
            th = timeit(lambda: run(H.FA_IMPL_HIP))
            ta2 = timeit(lambda: run(H.FA_IMPL_AUTO))
            print(json.dumps({"time": f"B{B} H{Hh} {sq}x{sk} {str(dt)[6:]}", "asm_ms": round(min(ta, ta2), 4),
                              "hip_ms": round(th, 4), "asm_TF": round(fl / min(ta, ta2) / 1e9, 1),
                              "hip_TF": round(fl / th / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
