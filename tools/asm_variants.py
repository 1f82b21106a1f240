"""asm_variants.py — timing of assembly-forward variants (gen_fwd.py --probe switches) in one
process, interleaved, at a BASELINE shape. Probe variants compute wrong results by design
(a part is removed to price it); the base variant is the product kernel.

    python tools/asm_variants.py [--shape B,H,S] [--variants ",nomax,noexp"] [--rounds 5]
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


def build(spec, out_dir, hd=64):
    """spec: 'label:generator args' (e.g. 'vp1:--vp1 1 --probe noexp') or a bare probe switch."""
    if ":" in spec:
        tag, args = spec.split(":", 1)
        extra = args.split()
    else:
        tag, extra = spec or "base", (["--probe", spec] if spec else [])
    s = os.path.join(out_dir, f"var_{tag}.s")
    subprocess.check_call([sys.executable, GEN, "--out", s, "--hd", str(hd)] + list(extra))
    subprocess.check_call([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                           s, "-o", s[:-2] + ".o"])
    subprocess.check_call([f"{LLVM}/ld.lld", "-shared", s[:-2] + ".o", "-o", s[:-2] + ".hsaco"])
    txt = open(s).read()
    name = txt.split(".globl ")[1].split()[0]
    threads = int(txt.split(".max_flat_workgroup_size: ")[1].split()[0])
    persist = int(txt.split(".kernarg_segment_size: ")[1].split()[0]) == 176
    return open(s[:-2] + ".hsaco", "rb").read(), name, (threads, persist)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8,12,2048")
    ap.add_argument("--variants", default=",nomax,noexp,nofma,nocvt,nofill,nodma,nolds,nosum,nobar")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--hd", type=int, default=64, choices=[32, 64, 128])
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    # ';'-separated 'label:generator args' specs, or ','-separated probe switches ('' = base)
    variants = args.variants.split(";") if ";" in args.variants else args.variants.split(",")
    images = {v: build(v, out, args.hd) for v in variants}
    import torch
    B, H, S = (int(x) for x in args.shape.split(","))
    D = args.hd
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    q = torch.randn(B * S, H, D, generator=g).bfloat16().to(dev)
    k = torch.randn(B * S, H, D, generator=g).bfloat16().to(dev)
    v = torch.randn(B * S, H, D, generator=g).bfloat16().to(dev)
    o = torch.empty_like(q)
    lse_stride = (S + 15) // 16 * 16
    lse = torch.empty(B, H, lse_stride, device=dev)
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=dev)
    nqb = (S + 255) // 256
    mg = lambda d: ((1 << 32) + 2 * d - 1) // (2 * d)
    c = np.float32(D ** -0.5 * 1.4426950408889634)
    # the whole 168-byte argument block of fa_asm.cpp (FaAsmFwdArgs), non-causal
    kb = struct.pack("<7Q4Q4I2I2f2I2I2I2I4I", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                     lse.data_ptr(), cu.data_ptr(), cu.data_ptr(), D * 2, D * 2, D * 2, D * 2, H * D * 2, H * D * 2,
                     H * D * 2, H * D * 2, H, lse_stride * 4, c, np.float32(8.0 / c), nqb, nqb * H * B, mg(nqb),
                     mg(H), D, H * B, 0, mg(H * B), 0, 0, 0, 0)
    assert len(kb) == 168
    libs = [ln.split()[-1] for ln in open("/proc/self/maps").read().split("\n") if "libamdhip64" in ln]
    hip = ctypes.CDLL(libs[0])
    kbuf = ctypes.create_string_buffer(kb, len(kb))
    size = ctypes.c_size_t(len(kb))
    extra = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbuf), 2, ctypes.addressof(size), 3)
    # persistent kernels: the grid size (one workgroup per CU) in the 8 bytes after the block
    ncu = torch.cuda.get_device_properties(0).multi_processor_count // 8 * 8
    kbp = kb + struct.pack("<2I", ncu, 0)
    kbufp = ctypes.create_string_buffer(kbp, len(kbp))
    sizep = ctypes.c_size_t(len(kbp))
    extrap = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbufp), 2, ctypes.addressof(sizep), 3)
    fns = {}
    keep = []
    threads = {}
    for name, (img, kname, nthr) in images.items():
        mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
        buf = ctypes.create_string_buffer(img, len(img))
        keep.append(buf)
        assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, kname.encode()) == 0
        fns[name] = fn
        threads[fn.value] = nthr
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def launch(fn):
        nthr, persist = threads[fn.value]
        if persist:
            rc = hip.hipModuleLaunchKernel(fn, min(ncu, nqb * H * B), 1, 1, nthr, 1, 1, 0, stream, None, extrap)
        else:
            rc = hip.hipModuleLaunchKernel(fn, nqb, H, B, nthr, 1, 1, 0, stream, None, extra)
        assert rc == 0

    flops = 4.0 * B * H * S * S * D
    # correctness of every variant on sequence 0 (probe variants are wrong by design)
    qf, kf, vf = (x[:S].float().transpose(0, 1) for x in (q, k, v))
    sc = torch.matmul(qf, kf.transpose(1, 2)) * D ** -0.5
    ref = torch.matmul(torch.softmax(sc, -1), vf).transpose(0, 1)
    ref_lse = torch.logsumexp(sc, -1)
    for n in variants:
        o.zero_()
        launch(fns[n])
        torch.cuda.synchronize()
        err = (o[:S].float() - ref).abs().max().item()
        lerr = (lse[0, :, :S] - ref_lse).abs().max().item()
        print(f"check {(n.split(':')[0] if n else 'base'):24s} max|o-ref| {err:.3e}  max|lse-ref| {lerr:.3e}", flush=True)
    # warm the clock
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _ in range(20):
            launch(fns[variants[0]])
        torch.cuda.synchronize()
    res = {n: [] for n in variants}
    for _ in range(args.rounds):
        for n in variants:
            for _ in range(5):
                launch(fns[n])
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            for _ in range(args.iters):
                launch(fns[n])
            e_.record()
            torch.cuda.synchronize()
            res[n].append(s_.elapsed_time(e_) / args.iters)
    base = np.median(res[variants[0]])
    for n in variants:
        m = float(np.median(res[n]))
        print(f"{(n.split(':')[0] if n else 'base'):24s} {m * 1e3:8.2f} us  {flops / m / 1e9:7.1f} TF/s  {100 * (m / base - 1):+6.1f}%", flush=True)


if __name__ == "__main__":
    main()
