"""A/B harness for forward-kernel structure variants (guide rule 24: interleaved rounds, one process).

    python tools/fwd_variants.py build            # here: compile build/var_<name>.so per variant
    python tools/fwd_variants.py run [--rounds 5]  # on the GPU box: time every variant, interleaved

Each variant recompiles only the head-dim TUs with its -D switches (FA_FWD_PIPE, FA_FWD_SCHED,
FA_FWD_WPS, ...; a key starting with '-' is passed as a raw compiler flag) and links them with the shared objects of the main build. The run
loads each library with ctypes (RTLD_LOCAL) and calls fa_fwd on the same device tensors.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import concurrent.futures as cf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hazyresearch_flash-attention_amd")
sys.path.insert(0, PKG)
BUILD = os.path.join(PKG, "build")

VARIANTS = {
    "base": {},
}
# more variants from the environment: FA_VARIANTS='{"name": {"MACRO": value, "-flag": 1}}'
VARIANTS.update(json.loads(os.environ.get("FA_VARIANTS", "{}")))

CONFIGS = [
    # name, B, H, Sq, Sk, D, causal, dtype
    ("ns_B8_H12_S2048_D64", 8, 12, 2048, 2048, 64, False, "bf16"),
    ("xs_B16_H12_S2048_D64", 16, 12, 2048, 2048, 64, False, "bf16"),   # 1536 workgroups: whole rounds
    ("xs_B4_H12_S2048_D64", 4, 12, 2048, 2048, 64, False, "bf16"),     # 384 workgroups
    ("c4_B16_H12_S4096_D128_causal", 16, 12, 4096, 4096, 128, True, "bf16"),
    ("c5_B4_H16_1024x4096_D64", 4, 16, 1024, 4096, 64, False, "bf16"),
    ("bs_localglobal_B8_H12_S2048_D64", 8, 12, 2048, 2048, 64, False, "bf16"),   # fa_fwd_block
    ("c2_B8_H12_S512_D64_fp16", 8, 12, 512, 512, 64, False, "fp16"),
    ("tiny_B1_H12_S2048_D64", 1, 12, 2048, 2048, 64, False, "bf16"),   # 96 workgroups of 8 waves
    ("tiny_B2_H8_S1024_D64", 2, 8, 1024, 1024, 64, False, "bf16"),     # 64 workgroups of 8 waves
    ("c3_B8_H12_S2048_D64_causal_p0.1", 8, 12, 2048, 2048, 64, True, "bf16", 0.1),
    ("c3nd_B8_H12_S2048_D64_causal", 8, 12, 2048, 2048, 64, True, "bf16", 0.0),
]


def build(names):
    import importlib.util
    spec = importlib.util.spec_from_file_location("fa_build", os.path.join(PKG, "build.py"))
    fb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(fb)
    fb.build(verbose=False)
    VAR_TUS = tuple(fb.KERNEL_TUS)
    shared = [os.path.join(BUILD, s + ".o") for s in fb.SOURCES if s not in VAR_TUS]

    def one(name):
        defs = VARIANTS[name]
        extra = []
        for k, v in defs.items():
            extra += k.split() if k.startswith("-") else [f"-D{k}={v}"]
        objs = []
        for tu in VAR_TUS:
            obj = os.path.join(BUILD, f"var_{name}_{tu}.o")
            cmd = ([fb.hipcc()] + fb.common_flags() + fb.SOURCE_FLAGS.get(tu, []) + extra +
                   ["-x", "hip", "-c", os.path.join(fb.CSRC, tu), "-o", obj])
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode:
                raise RuntimeError(r.stderr)
            objs.append(obj)
        out = os.path.join(BUILD, f"var_{name}.so")
        r = subprocess.run([fb.hipcc(), f"--offload-arch={fb.ARCH}", "-shared", "-fPIC", "-o", out] + shared + objs,
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return out

    with cf.ThreadPoolExecutor(4) as ex:
        for out in ex.map(one, names):
            print("built", out)


def run(names, rounds, iters):
    import torch
    from flash_attn import flash_attn_hip as hip
    libs = {}
    for n in names:
        L = ctypes.CDLL(os.path.join(BUILD, f"var_{n}.so"))
        L.fa_fwd.argtypes = [ctypes.POINTER(hip.FaFwdArgs), ctypes.c_void_p]
        L.fa_fwd.restype = ctypes.c_int
        L.fa_fwd_block.argtypes = [ctypes.POINTER(hip.FaFwdArgs), ctypes.POINTER(hip.FaBlockMask), ctypes.c_void_p]
        L.fa_fwd_block.restype = ctypes.c_int
        libs[n] = L
    results = {}
    only_cfg = os.environ.get("FA_CONFIGS", "")
    for (cname, B, H, Sq, Sk, D, causal, dt, *pdrop) in CONFIGS:
        if only_cfg and not any(cname.startswith(c) for c in only_cfg.split(",")):
            continue
        p = pdrop[0] if pdrop else 0.0
        dtype = torch.bfloat16 if dt == "bf16" else torch.float16
        g = torch.Generator().manual_seed(0)
        q = torch.randn(B * Sq, H, D, generator=g).to(dtype).cuda()
        k = torch.randn(B * Sk, H, D, generator=g).to(dtype).cuda()
        v = torch.randn(B * Sk, H, D, generator=g).to(dtype).cuda()
        cq = torch.arange(0, (B + 1) * Sq, Sq, dtype=torch.int32, device="cuda")
        ck = torch.arange(0, (B + 1) * Sk, Sk, dtype=torch.int32, device="cuda")
        sparse = cname.startswith("bs_")
        lay, m, live = None, None, 1.0
        if sparse:   # sliding window of +-1 256-key block plus a global first block
            rblk = torch.arange((Sq + 15) // 16)[:, None] // 16
            cblk = torch.arange((Sk + 255) // 256)[None, :]
            lay = (((rblk - cblk).abs() <= 1) | (cblk == 0)).to(torch.uint8).cuda()
            live = lay.float().mean().item()
            m, _keep = hip._mask_struct(lay, q.device)
        ref, _lse = hip.fwd(q, k, v, cq, ck, Sq, Sk, p, D ** -0.5, False, causal, False, None, layout=lay,
                            rng_state=(1234, 0))
        outs = {}
        a = hip.FaFwdArgs()
        lse = torch.empty(B, H, (Sq + 15) // 16 * 16, dtype=torch.float32, device="cuda")
        a.q, a.k, a.v = q.data_ptr(), k.data_ptr(), v.data_ptr()
        a.softmax_lse = lse.data_ptr()
        a.cu_seqlens_q, a.cu_seqlens_k = cq.data_ptr(), ck.data_ptr()
        a.q_row_stride, a.q_head_stride = q.stride(0), q.stride(1)
        a.k_row_stride, a.k_head_stride = k.stride(0), k.stride(1)
        a.v_row_stride, a.v_head_stride = v.stride(0), v.stride(1)
        a.o_row_stride, a.o_head_stride = q.stride(0), q.stride(1)
        a.batch, a.nheads, a.head_dim = B, H, D
        a.max_seqlen_q, a.max_seqlen_k, a.lse_stride = Sq, Sk, lse.shape[2]
        a.softmax_scale = D ** -0.5
        a.is_causal = 1 if causal else 0
        a.p_dropout, a.rng_seed, a.rng_offset = p, 1234, 0
        a.dtype = hip.FA_DTYPE_BF16 if dt == "bf16" else hip.FA_DTYPE_FP16
        stream = torch.cuda.current_stream().cuda_stream
        for n in names:
            o = torch.empty_like(q)
            outs[n] = o
        times = {n: [] for n in names}
        flops = 4.0 * B * H * Sq * Sk * D / (2 if causal else 1) * live
        call = ((lambda L: L.fa_fwd_block(ctypes.byref(a), ctypes.byref(m), stream)) if sparse
                else (lambda L: L.fa_fwd(ctypes.byref(a), stream)))
        for r in range(rounds):
            for n in names:
                a.o = outs[n].data_ptr()
                L = libs[n]
                for _ in range(3):
                    call(L)
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(iters):
                    rc = call(L)
                e.record()
                torch.cuda.synchronize()
                assert rc == 0
                times[n].append(s.elapsed_time(e) / iters)
        res = {}
        for n in names:
            ts = sorted(times[n])
            err = (outs[n].float() - ref.float()).abs().max().item()
            res[n] = {"ms_med": round(ts[len(ts) // 2], 4), "ms_min": round(ts[0], 4),
                      "TFLOPS_med": round(flops / ts[len(ts) // 2] / 1e9, 1), "max_diff_vs_main": err}
        results[cname] = res
        print(cname, json.dumps(res), flush=True)
    return results


BWD_CONFIGS = [
    # name, B, H, S, D, causal, p
    ("bwd_ns_B8_H12_S2048_D64", 8, 12, 2048, 64, False, 0.0),
    ("bwd_c3_B8_H12_S2048_D64_causal_p0.1", 8, 12, 2048, 64, True, 0.1),
    ("bwd_c_B8_H12_S2048_D64_causal", 8, 12, 2048, 64, True, 0.0),
    ("bwd_ns_B8_H12_S2048_D32", 8, 12, 2048, 32, False, 0.0),
    ("bwd_ns_B8_H12_S2048_D128", 8, 12, 2048, 128, False, 0.0),
    ("bwd_c_B8_H12_S2048_D128_causal", 8, 12, 2048, 128, True, 0.0),
    ("bwd_c4_B16_H12_S4096_D128_causal", 16, 12, 4096, 128, True, 0.0),
]


def run_bwd(names, rounds, iters):
    """Interleaved A/B of fa_bwd (pre-pass + main + convert) per variant library."""
    import torch
    from flash_attn import flash_attn_hip as hip
    libs = {}
    for n in names:
        L = ctypes.CDLL(os.path.join(BUILD, f"var_{n}.so"))
        L.fa_bwd.argtypes = [ctypes.POINTER(hip.FaBwdArgs), ctypes.c_void_p]
        L.fa_bwd.restype = ctypes.c_int
        libs[n] = L
    results = {}
    only_cfg = os.environ.get("FA_CONFIGS", "")
    for (cname, B, H, S, D, causal, p) in BWD_CONFIGS:
        if only_cfg and not any(cname.startswith(c) for c in only_cfg.split(",")):
            continue
        g = torch.Generator().manual_seed(0)
        q, k, v, do = (torch.randn(B * S, H, D, generator=g).bfloat16().cuda() for _ in range(4))
        cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device="cuda")
        rng = (1234, 0)
        o, lse = hip.fwd(q, k, v, cu, cu, S, S, p, D ** -0.5, False, causal, False, None, rng_state=rng)[:2]
        dq_ref, dk_ref, dv_ref = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        hip.bwd(do, q, k, v, o, lse, dq_ref, dk_ref, dv_ref, cu, cu, S, S, p, D ** -0.5, False, causal, None,
                rng_state=rng)
        sd = torch.empty(B, H, lse.shape[2], dtype=torch.float32, device="cuda")
        acc = torch.empty(B * S, H, D, dtype=torch.float32, device="cuda")
        outs = {n: (torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)) for n in names}
        a = hip.FaBwdArgs()
        a.dout, a.q, a.k, a.v, a.out = do.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr()
        a.softmax_lse, a.softmax_d, a.dq_accum = lse.data_ptr(), sd.data_ptr(), acc.data_ptr()
        a.cu_seqlens_q = a.cu_seqlens_k = cu.data_ptr()
        for f in ("do", "q", "k", "v", "o", "dq", "dk", "dv"):
            setattr(a, f"{f}_row_stride", H * D)
            setattr(a, f"{f}_head_stride", D)
        a.batch, a.nheads, a.head_dim, a.max_seqlen_q, a.max_seqlen_k = B, H, D, S, S
        a.total_q, a.lse_stride = B * S, lse.shape[2]
        a.softmax_scale, a.p_dropout, a.rng_seed, a.rng_offset = D ** -0.5, p, rng[0], rng[1]
        a.is_causal, a.dtype = int(causal), hip.FA_DTYPE_BF16
        stream = torch.cuda.current_stream().cuda_stream
        times = {n: [] for n in names}
        flops = 2.5 * 4.0 * B * H * S * S * D / (2 if causal else 1)
        for r in range(rounds):
            for n in names:
                dq, dk, dv = outs[n]
                a.dq, a.dk, a.dv = dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
                L = libs[n]
                for _ in range(2):
                    L.fa_bwd(ctypes.byref(a), stream)
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(iters):
                    rc = L.fa_bwd(ctypes.byref(a), stream)
                e.record()
                torch.cuda.synchronize()
                assert rc == 0
                times[n].append(s.elapsed_time(e) / iters)
        res = {}
        for n in names:
            ts = sorted(times[n])
            dq, dk, dv = outs[n]
            err = max((x.float() - y.float()).abs().max().item() for x, y in ((dq, dq_ref), (dk, dk_ref), (dv, dv_ref)))
            res[n] = {"ms_med": round(ts[len(ts) // 2], 4), "ms_min": round(ts[0], 4),
                      "TFLOPS_med": round(flops / ts[len(ts) // 2] / 1e9, 1), "max_diff_vs_main": err}
        results[cname] = res
        print(cname, json.dumps(res), flush=True)
    return results


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "run", "runbwd"])
    ap.add_argument("--only", default="")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    names = [n for n in VARIANTS if not args.only or n in args.only.split(",")]
    if args.mode == "build":
        build(names)
    else:
        out = run(names, args.rounds, args.iters) if args.mode == "run" else run_bwd(names, args.rounds, args.iters)
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", "variants.json"), "w") as f:
            json.dump(out, f, indent=1)
