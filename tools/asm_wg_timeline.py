"""Per-workgroup timeline of the D=64 asm forward (gen_fwd.py --probe stamps): every wave records
s_memrealtime (100 MHz) at entry, after the prologue's first barrier, at the last tile and after
its final stores, plus its CU (HW_ID / XCC_ID). Reports, per workgroup, prologue / loop / epilogue
durations and the gap between consecutive workgroups on one CU (dispatch latency).

    python tools/asm_wg_timeline.py [--shape B,H,Sq,Sk] [--causal]

Status: its first hardware run (round 3) faulted with an illegal address: the stamps probe read its
buffer pointer 8 bytes past the argument block (KARG_BYTES after the += 8). gen_fwd.py now reads it at
KARG_BYTES - 8; the fixed probe has not been run on hardware since. Run it alone, under a short timeout.
"""
import argparse
import ctypes
import json
import os
import struct
import subprocess
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "hazyresearch_flash-attention_amd", "csrc", "asm", "gen_fwd.py")
LLVM = "/opt/rocm/lib/llvm/bin"


def build(out_dir, cyc=False):
    s = os.path.join(out_dir, "stampcyc.s" if cyc else "stamps.s")
    subprocess.check_call([sys.executable, GEN, "--out", s, "--probe", "stamps,stampcyc" if cyc else "stamps"])
    subprocess.check_call([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                           s, "-o", s[:-2] + ".o"])
    subprocess.check_call([f"{LLVM}/ld.lld", "-shared", s[:-2] + ".o", "-o", s[:-2] + ".hsaco"])
    return open(s[:-2] + ".hsaco", "rb").read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8,12,2048,2048")
    ap.add_argument("--causal", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--cycles", action="store_true",
                    help="stamp with s_memtime (shader cycles) instead of s_memrealtime; durations in kcycles")
    args = ap.parse_args()
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    img = build(out_dir, args.cycles)
    import torch
    B, H, Sq, Sk = (int(x) for x in args.shape.split(","))
    D = 64
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    q = torch.randn(B * Sq, H, D, generator=g).bfloat16().to(dev)
    k = torch.randn(B * Sk, H, D, generator=g).bfloat16().to(dev)
    v = torch.randn(B * Sk, H, D, generator=g).bfloat16().to(dev)
    o = torch.empty_like(q)
    lse_stride = (Sq + 15) // 16 * 16
    lse = torch.empty(B, H, lse_stride, device=dev)
    cq = torch.arange(0, (B + 1) * Sq, Sq, dtype=torch.int32, device=dev)
    ck = torch.arange(0, (B + 1) * Sk, Sk, dtype=torch.int32, device=dev)
    nqb = (Sq + 255) // 256
    nwg = nqb * H * B
    mg = lambda d: ((1 << 32) + 2 * d - 1) // (2 * d)
    c = np.float32(D ** -0.5 * 1.4426950408889634)
    per = grp = 0
    if args.causal and (H * B) % 8 == 0:     # fa_asm.cpp's group choice
        nh, want = H * B // 8, (64 + nqb - 1) // nqb
        grp = max(x for x in range(1, min(nh, want) + 1) if nh % x == 0)
        per = grp * nqb
    stamps = torch.zeros(16 + nwg * 4 * 16, dtype=torch.int32, device=dev)
    kb = struct.pack("<7Q4Q4I2I2f2I2I2I2I4IQ", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                     cq.data_ptr(), ck.data_ptr(), D * 2, D * 2, D * 2, D * 2, H * D * 2, H * D * 2, H * D * 2,
                     H * D * 2, H, lse_stride * 4, c, np.float32(8.0 / c), nqb, nwg, mg(nqb), mg(H), D, H * B,
                     int(args.causal), mg(H * B), per, mg(per) if per else 0, grp, mg(grp) if grp else 0,
                     stamps.data_ptr())
    assert len(kb) == 176
    libs = [ln.split()[-1] for ln in open("/proc/self/maps").read().split("\n") if "libamdhip64" in ln]
    hip = ctypes.CDLL(libs[0])
    kbuf = ctypes.create_string_buffer(kb, len(kb))
    size = ctypes.c_size_t(len(kb))
    extra = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbuf), 2, ctypes.addressof(size), 3)
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    buf = ctypes.create_string_buffer(img, len(img))
    assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"fa_fwd_d64_bf16_asm") == 0
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def launch():
        assert hip.hipModuleLaunchKernel(fn, nqb, H, B, 256, 1, 1, 0, stream, None, extra) == 0

    for _ in range(200):     # clock ramp
        stamps.zero_()
        launch()
    torch.cuda.synchronize()
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stamps.zero_()
    s_.record()
    launch()
    e_.record()
    torch.cuda.synchronize()
    ev_us = s_.elapsed_time(e_) * 1e3
    st = stamps.cpu().numpy()
    n = int(st[0])
    assert n == nwg * 4, (n, nwg * 4)
    rec = st[16:16 + n * 16].reshape(n, 16).view(np.uint32).astype(np.int64)
    t0 = rec[:, 0] | (rec[:, 1] << 32)
    t2 = rec[:, 2] | (rec[:, 3] << 32)
    t3 = rec[:, 4] | (rec[:, 5] << 32)
    t1 = rec[:, 12] | (rec[:, 13] << 32)
    hwid, xcc = rec[:, 6], rec[:, 7]
    wg = rec[:, 8] + nqb * (rec[:, 9] + H * rec[:, 10])
    base = t0.min()
    us = (lambda x: (x - base) * 1e-3) if args.cycles else (lambda x: (x - base) * 0.01)
    wgs = defaultdict(list)
    for i in range(n):
        wgs[int(wg[i])].append(i)
    rows = []
    for w, ids in wgs.items():
        ids = np.array(ids)
        cu = (int(xcc[ids[0]]) & 0xF, (int(hwid[ids[0]]) >> 8) & 0xFF)
        rows.append(dict(wg=w, cu=cu, start=us(t0[ids].min()), pro=us(t1[ids].max()) - us(t0[ids].min()),
                         loop=us(t2[ids].max()) - us(t1[ids].max()), epi=us(t3[ids].max()) - us(t2[ids].max()),
                         end=us(t3[ids].max())))
    percu = defaultdict(list)
    for r in rows:
        percu[r["cu"]].append(r)
    gaps, firsts, lasts, counts = [], [], [], []
    for cu, rs in percu.items():
        rs.sort(key=lambda r: r["start"])
        counts.append(len(rs))
        firsts.append(rs[0]["start"])
        lasts.append(rs[-1]["end"])
        for a, b in zip(rs, rs[1:]):
            gaps.append(b["start"] - a["end"])
    med = lambda xs: float(np.median(xs))
    res = {"shape": args.shape, "causal": args.causal, "unit": "kcycles" if args.cycles else "us",
           "event_us": round(ev_us, 2),
           "stamp_span_us": round(max(r["end"] for r in rows), 2), "cus": len(percu),
           "wg_per_cu": [min(counts), max(counts)],
           "prologue_us_med": round(med([r["pro"] for r in rows]), 3),
           "loop_us_med": round(med([r["loop"] for r in rows]), 3),
           "epilogue_us_med": round(med([r["epi"] for r in rows]), 3),
           "gap_us_med": round(med(gaps), 3) if gaps else None,
           "gap_us_p90": round(float(np.percentile(gaps, 90)), 3) if gaps else None,
           "first_start_us_max": round(max(firsts), 3), "last_end_us_min": round(min(lasts), 3),
           "last_end_us_max": round(max(lasts), 3)}
    print(json.dumps(res), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"summary": res, "workgroups": sorted(rows, key=lambda r: r["start"])}, f)


if __name__ == "__main__":
    main()
