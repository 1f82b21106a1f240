"""A/B of the causal XCD group size of the asm forward (fa_asm.cpp: G heads per group, G * nqb ~ 64
workgroups = 2x the CUs of an XCD) at a causal shape, one process, interleaved: the same code object
launched with different (per, group) kernel arguments; per = 0 is the global heaviest-first order.

    python tools/asm_group_ab.py [--shape B,H,S] [--hd 128] [--groups 0,1,2,4]
"""
import argparse
import ctypes
import os
import struct
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "hazyresearch_flash-attention_amd", "csrc", "asm", "gen_fwd.py")
LLVM = "/opt/rocm/lib/llvm/bin"


def build(out_dir, hd):
    s = os.path.join(out_dir, f"grp_d{hd}.s")
    subprocess.check_call([sys.executable, GEN, "--out", s, "--hd", str(hd)])
    subprocess.check_call([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                           s, "-o", s[:-2] + ".o"])
    subprocess.check_call([f"{LLVM}/ld.lld", "-shared", s[:-2] + ".o", "-o", s[:-2] + ".hsaco"])
    return open(s[:-2] + ".hsaco", "rb").read(), f"fa_fwd_d{hd}_bf16_asm"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="16,12,4096")
    ap.add_argument("--hd", type=int, default=128)
    ap.add_argument("--groups", default="0,1,2,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    img, kname = build(out, args.hd)
    import torch
    B, H, S = (int(x) for x in args.shape.split(","))
    D = args.hd
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    q, k, v = (torch.randn(B * S, H, D, generator=g).bfloat16().to(dev) for _ in range(3))
    o = torch.empty_like(q)
    lse_stride = (S + 15) // 16 * 16
    lse = torch.empty(B, H, lse_stride, device=dev)
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=dev)
    nqb = (S + 255) // 256
    nbh = B * H
    mg = lambda d: ((1 << 32) + 2 * d - 1) // (2 * d) if d else 0
    c = np.float32(D ** -0.5 * 1.4426950408889634)
    libs = [ln.split()[-1] for ln in open("/proc/self/maps").read().split("\n") if "libamdhip64" in ln]
    hip = ctypes.CDLL(libs[0])
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    buf = ctypes.create_string_buffer(img, len(img))
    assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, kname.encode()) == 0
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    keep, launches = [], {}
    for grp in (int(x) for x in args.groups.split(",")):
        assert grp == 0 or (nbh // 8) % grp == 0
        per = grp * nqb
        kb = struct.pack("<7Q4Q4I2I2f2I2I2I2I4I", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                         lse.data_ptr(), cu.data_ptr(), cu.data_ptr(), D * 2, D * 2, D * 2, D * 2, H * D * 2,
                         H * D * 2, H * D * 2, H * D * 2, H, lse_stride * 4, c, np.float32(8.0 / c), nqb, nqb * nbh,
                         mg(nqb), mg(H), D, nbh, 1, mg(nbh), per, mg(per), grp, mg(grp))
        kbuf = ctypes.create_string_buffer(kb, len(kb))
        size = ctypes.c_size_t(len(kb))
        extra = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbuf), 2, ctypes.addressof(size), 3)
        keep += [kbuf, size, extra]
        launches[grp] = extra

    def launch(grp):
        assert hip.hipModuleLaunchKernel(fn, nqb, H, B, 256, 1, 1, 0, stream, None, launches[grp]) == 0

    # correctness of each order on sequence 0, two heads (causal, fp32 reference)
    qf, kf, vf = (x[:S, :2].float().transpose(0, 1) for x in (q, k, v))
    sc = torch.matmul(qf, kf.transpose(1, 2)) * D ** -0.5
    sc = sc.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=dev), 1), float("-inf"))
    ref = torch.matmul(torch.softmax(sc, -1), vf).transpose(0, 1)
    for grp in launches:
        o.zero_()
        launch(grp)
        torch.cuda.synchronize()
        print(f"check G={grp}: max|o-ref| {(o[:S, :2].float() - ref).abs().max().item():.3e}", flush=True)
    flops = 2.0 * B * H * S * S * D
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        launch(0)
        torch.cuda.synchronize()
    res = {grp: [] for grp in launches}
    for _ in range(args.rounds):
        for grp in launches:
            launch(grp)
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            for _ in range(args.iters):
                launch(grp)
            e_.record()
            torch.cuda.synchronize()
            res[grp].append(s_.elapsed_time(e_) / args.iters)
    for grp, r in res.items():
        m = float(np.median(r))
        print(f"G={grp:2d} {m * 1e3:9.1f} us  {flops / m / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
