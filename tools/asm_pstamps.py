"""Per-block cycle anatomy of the persistent D=64 asm forward (gen_fwd.py --persist 1 --probe pstamps):
every wave stamps s_memtime at block entry, loop start, last-tile entry and the seam; this reports the
median shader cycles of prologue (entry -> loop start), loop (-> last tile, nt - 1 tiles), last tile +
epilogue (-> seam) and the seam-to-next-entry gap, per block round.

    python tools/asm_pstamps.py [--shape B,H,S] [--gen "--prescale 1"]
"""
import argparse
import ctypes
import json
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "hazyresearch_flash-attention_amd", "csrc", "asm", "gen_fwd.py")
LLVM = "/opt/rocm/lib/llvm/bin"


def build(out_dir, extra):
    s = os.path.join(out_dir, "pstamps_" + "".join(c if c.isalnum() else "_" for c in extra) + ".s")
    extra = extra.split()
    probes = ["pstamps"]
    if "--probe" in extra:     # merge the variant's own probe switches with the stamps
        i = extra.index("--probe")
        probes.append(extra[i + 1])
        del extra[i:i + 2]
    subprocess.check_call([sys.executable, GEN, "--out", s, "--persist", "1", "--probe", ",".join(probes)] + extra)
    subprocess.check_call([f"{LLVM}/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c",
                           s, "-o", s[:-2] + ".o"])
    subprocess.check_call([f"{LLVM}/ld.lld", "-shared", s[:-2] + ".o", "-o", s[:-2] + ".hsaco"])
    return open(s[:-2] + ".hsaco", "rb").read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8,12,2048")
    ap.add_argument("--gen", default="")
    ap.add_argument("--hd", type=int, default=64, help="head-dim tile (64, or 32: head_dim 32)")
    args = ap.parse_args()
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    img = build(out_dir, args.gen + (f" --hd {args.hd}" if args.hd != 64 else ""))
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
    nwg = nqb * H * B
    ncu = torch.cuda.get_device_properties(0).multi_processor_count // 8 * 8
    grid = min(ncu, nwg)
    mg = lambda d: ((1 << 32) + 2 * d - 1) // (2 * d)
    c = np.float32(D ** -0.5 * 1.4426950408889634)
    rec = torch.zeros(nwg * 4 * 4, dtype=torch.int64, device=dev)
    kb = struct.pack("<7Q4Q4I2I2f2I2I2I2I4I2IQ", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                     cu.data_ptr(), cu.data_ptr(), D * 2, D * 2, D * 2, D * 2, H * D * 2, H * D * 2, H * D * 2,
                     H * D * 2, H, lse_stride * 4, c, np.float32(8.0 / c), nqb, nwg, mg(nqb), mg(H), D, H * B, 0,
                     mg(H * B), 0, 0, 0, 0, grid, 0, rec.data_ptr())
    assert len(kb) == 184
    libs = [ln.split()[-1] for ln in open("/proc/self/maps").read().split("\n") if "libamdhip64" in ln]
    hip = ctypes.CDLL(libs[0])
    kbuf = ctypes.create_string_buffer(kb, len(kb))
    size = ctypes.c_size_t(len(kb))
    extra = (ctypes.c_void_p * 5)(1, ctypes.addressof(kbuf), 2, ctypes.addressof(size), 3)
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    buf = ctypes.create_string_buffer(img, len(img))
    assert hip.hipModuleLoadData(ctypes.byref(mod), buf) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, f"fa_fwd_d{args.hd}p_bf16_asm".encode()) == 0
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(300):     # clock ramp
        assert hip.hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, 0, stream, None, extra) == 0
    torch.cuda.synchronize()
    rec.zero_()
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_.record()
    assert hip.hipModuleLaunchKernel(fn, grid, 1, 1, 256, 1, 1, 0, stream, None, extra) == 0
    e_.record()
    torch.cuda.synchronize()
    r = rec.cpu().numpy().reshape(nwg, 4, 4).astype(np.int64)
    tb, tl, tt, ts = r[..., 0], r[..., 1], r[..., 2], r[..., 3]
    assert (ts > 0).all(), "missing records"
    rounds = nwg // grid
    res = {"shape": args.shape, "gen": args.gen, "event_us": round(s_.elapsed_time(e_) * 1e3, 2), "grid": grid,
           "kernel_kcycles": round(float((ts.max() - tb.min()) / 1e3), 2)}
    nt = (S + 63) // 64
    for rnd in range(rounds):
        sel = slice(rnd * grid, (rnd + 1) * grid)
        d = {"prologue": np.median(tl[sel] - tb[sel]), "loop": np.median(tt[sel] - tl[sel]),
             "last_epi": np.median(ts[sel] - tt[sel])}
        d["loop_per_tile"] = d["loop"] / (nt - 1)
        if rnd:
            prev = slice((rnd - 1) * grid, rnd * grid)
            d["seam_gap"] = np.median(tb[sel] - ts[prev])
        res[f"round{rnd}"] = {k: round(float(v), 1) for k, v in d.items()}
    # finish spread (--gen "--probe pstrt": stamps on the global 100 MHz clock, so comparable across
    # CUs): per workgroup the seam stamp of its last block (median over waves), us after the first entry
    if rounds and "pstrt" in args.gen:
        last = slice((rounds - 1) * grid, rounds * grid)
        fin = (np.median(ts[last], axis=1) - tb.min()) / 100.0
        res["finish_us"] = {"min": round(float(fin.min()), 2), "med": round(float(np.median(fin)), 2),
                            "p90": round(float(np.percentile(fin, 90)), 2), "max": round(float(fin.max()), 2),
                            "by_wg_mod8_med": [round(float(np.median(fin[x::8])), 2) for x in range(8)]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
