"""asm_debug.py — register dumps of the assembly forward on the GPU vs the simulator.

    python tools/asm_debug.py --dump 'pro:v4-v15,v16-v47' [--sq 64 --sk 64] [--dtype bf16]

Generates a debug build of csrc/asm/gen_fwd.py that stores the listed registers of workgroup
(0,0,0) at the dump point and stops, runs it on cuda:0 (hipModuleLaunchKernel through ctypes)
and in tools/asm_sim.py on the same inputs, and prints the registers that differ.
"""
import argparse
import ctypes
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd", "csrc", "asm"))
import asm_sim  # noqa: E402
import gen_fwd  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def build_debug(dtype, dump, out_dir):
    s = os.path.join(out_dir, f"dbg_{dtype}.s")
    o = s[:-2] + ".o"
    h = s[:-2] + ".hsaco"
    extra = ["--dump", dump] if dump.split(":")[0] != "none" else []
    subprocess.check_call([sys.executable, gen_fwd.__file__, "--dtype", dtype, "--out", s] + extra)
    subprocess.check_call([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", s,
                           "-o", o])
    subprocess.check_call([f"{LLVM}/ld.lld", "-shared", o, "-o", h])
    return open(s).read(), open(h, "rb").read()


def karg_bytes(pq, pk, pv, po, pl, pcq, pck, H, Dh, lse_stride, nqb, nwg, c):
    mg = lambda d: ((1 << 32) + 2 * d - 1) // (2 * d)
    return struct.pack("<7Q4Q4I2I2f2I2I2I", pq, pk, pv, po, pl, pcq, pck, Dh * 2, Dh * 2, Dh * 2, Dh * 2,
                       H * Dh * 2, H * Dh * 2, H * Dh * 2, H * Dh * 2, H, lse_stride * 4, c, np.float32(8.0 / c),
                       nqb, nwg, mg(nqb), mg(H), Dh, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump", required=True)
    ap.add_argument("--sq", type=int, default=64)
    ap.add_argument("--sk", type=int, default=64)
    ap.add_argument("--heads", type=int, default=1)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--sim-only", action="store_true")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    txt, image = build_debug(args.dtype, args.dump, args.out)
    regs = gen_fwd.expand_regs(args.dump.split(":")[1])
    H, Dh = args.heads, 64
    rng = np.random.default_rng(0)
    cv = asm_sim.bf16_bits if args.dtype == "bf16" else asm_sim.f16_bits
    q = cv(rng.standard_normal((args.sq, H, Dh)).astype(np.float32)).astype(np.uint16)
    k = cv(rng.standard_normal((args.sk, H, Dh)).astype(np.float32)).astype(np.uint16)
    v = cv(rng.standard_normal((args.sk, H, Dh)).astype(np.float32)).astype(np.uint16)
    lse_stride = max((args.sq + 15) // 16 * 16, 16)
    nbytes_o = max(args.sq * H * Dh * 2, 4 * len(regs) * 256)
    cq = np.array([0, args.sq], np.int32)
    ck = np.array([0, args.sk], np.int32)
    c = np.float32(Dh ** -0.5 * 1.4426950408889634)
    nqb = (args.sq + 255) // 256
    nwg = nqb * H
    # ---- simulator
    mem = asm_sim.Memory()
    pq, pk, pv = mem.alloc(q), mem.alloc(k), mem.alloc(v)
    po = mem.alloc(np.zeros(nbytes_o, np.uint8))
    pl = mem.alloc(np.zeros((1, H, lse_stride), np.float32))
    pcq, pck = mem.alloc(cq), mem.alloc(ck)
    pa = mem.alloc(np.frombuffer(karg_bytes(pq, pk, pv, po, pl, pcq, pck, H, Dh, lse_stride, nqb, nwg, c), np.uint8))
    sim = asm_sim.Sim(txt, args.dtype)
    sim.run((nqb, H, 1), pa, mem)
    simd = mem.get(po)[:4 * len(regs) * 256].view(np.uint32).reshape(4, len(regs), 64)
    sim_o = mem.get(po)[:args.sq * H * Dh * 2].copy()
    if args.sim_only:
        print("sim ok")
        return
    # ---- GPU
    import torch
    dev = torch.device("cuda", 0)
    tq = torch.from_numpy(q.view(np.int16)).to(dev)
    tk = torch.from_numpy(k.view(np.int16)).to(dev)
    tv = torch.from_numpy(v.view(np.int16)).to(dev)
    to = torch.zeros(nbytes_o, dtype=torch.uint8, device=dev)
    tl = torch.zeros((1, H, lse_stride), dtype=torch.float32, device=dev)
    tcq = torch.from_numpy(cq).to(dev)
    tck = torch.from_numpy(ck).to(dev)
    kb = karg_bytes(tq.data_ptr(), tk.data_ptr(), tv.data_ptr(), to.data_ptr(), tl.data_ptr(), tcq.data_ptr(),
                    tck.data_ptr(), H, Dh, lse_stride, nqb, nwg, c)
    # the HIP runtime torch itself loaded (a second runtime would not own torch's allocations)
    libs = [ln.split()[-1] for ln in open("/proc/self/maps").read().split("\n") if "libamdhip64" in ln]
    hip = ctypes.CDLL(libs[0] if libs else "libamdhip64.so")
    print("hip runtime:", hip._name, flush=True)
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    img = ctypes.create_string_buffer(image, len(image))
    assert hip.hipModuleLoadData(ctypes.byref(mod), img) == 0
    name = f"fa_fwd_d64_{args.dtype}_asm".encode()
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, name) == 0
    kbuf = ctypes.create_string_buffer(kb, len(kb))
    size = ctypes.c_size_t(len(kb))
    extra = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbuf), 2, ctypes.addressof(size), 3)
    torch.cuda.synchronize()
    rc = hip.hipModuleLaunchKernel(fn, nqb, H, 1, 256, 1, 1, 0, ctypes.c_void_p(0), None, extra)
    assert rc == 0, rc
    torch.cuda.synchronize()
    if not regs:
        go = to.cpu().numpy()[:args.sq * H * Dh * 2]
        a_ = asm_sim.from16(go.view(np.uint16).astype(np.uint32), args.dtype)
        b_ = asm_sim.from16(sim_o.view(np.uint16).astype(np.uint32), args.dtype)
        print("full kernel: max |gpu - sim| =", float(np.abs(a_ - b_).max()), "gpu finite:", bool(np.isfinite(a_).all()))
        return
    gpud = to.cpu().numpy()[:4 * len(regs) * 256].view(np.uint32).reshape(4, len(regs), 64)
    np.savez(os.path.join(args.out, "dump.npz"), gpu=gpud, sim=simd, regs=np.array(regs))
    bad = 0
    for w in range(4):
        for i, r in enumerate(regs):
            a, b = gpud[w, i], simd[w, i]
            if (a == b).all():
                continue
            fa, fb = a.view(np.float32), b.view(np.float32)
            close = np.isfinite(fa).all() and np.allclose(fa, fb, rtol=2e-3, atol=2e-3)
            if close:
                continue
            bad += 1
            if bad <= 40:
                idx = np.nonzero(a != b)[0]
                print(f"wave {w} {r}: {len(idx)} lanes differ, first lanes {idx[:6].tolist()} "
                      f"gpu {[hex(x) for x in a[idx[:4]]]} sim {[hex(x) for x in b[idx[:4]]]} "
                      f"gpu_f {fa[idx[:4]].tolist()} sim_f {fb[idx[:4]].tolist()}")
    print(f"{bad} register dumps differ of {4 * len(regs)}")


if __name__ == "__main__":
    main()
