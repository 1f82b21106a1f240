"""A/B of the rotary embedding placements in the attention forward:

  separate  : fa_rotary rotates q and k of the packed qkv in place, then fa_fwd
  fused_q   : fa_rotary rotates k only (half the bytes), fa_fwd rotates q at its fragment load
  fused_qk  : no pass; fa_fwd also rotates every K fragment it reads from LDS. That variant
              (FA_FWD_ROTK in fa_fwd_kernel.h) lost 3x and was removed; it lives in the commit
              "Rotary fused into the forward's Q load". Build var_rotk.so from that commit with
              FA_VARIANTS='{"rotk": {"FA_FWD_ROTK": 1}}' tools/fwd_variants.py build --only rotk
              to re-run the leg; without the library it is skipped.

    python tools/rotary_ab.py [--B 8 --S 2048 --H 12 --D 64]     (GPU; prints one JSON line)
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from flash_attn import flash_attn_hip as hip  # noqa: E402
from flash_attn.flash_attention import FlashAttnRotaryQKVFunc  # noqa: E402
from flash_attn.flash_attn_interface import flash_attn_unpadded_func, flash_attn_unpadded_qkvpacked_func  # noqa: E402
from flash_attn.rotary import apply_rotary_emb_qkv_  # noqa: E402
from oracle.rotary_ref import rotary_tables  # noqa: E402


def timed(fn, iters=20, reps=7):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters)
    return sorted(out)[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--D", type=int, default=64)
    args = ap.parse_args()
    B, S, H, D = args.B, args.S, args.H, args.D
    g = torch.Generator().manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, generator=g).bfloat16().cuda()
    cos, sin = (t.cuda() for t in rotary_tables(S, D, torch.bfloat16))
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device="cuda")
    # the separate leg writes rotated q, k to a scratch buffer (same bytes as in place) so both
    # legs attend over the same data: a pass repeated in place drifts it, and the kernel's
    # rescale branch makes its time data-dependent
    qk_rot = torch.empty(B, S, 2, H, D, dtype=qkv.dtype, device="cuda")
    st_x, st_y = (S * 3 * H * D, 3 * H * D, H * D, D), (S * 2 * H * D, 2 * H * D, H * D, D)
    qr, kr, vr = qk_rot[:, :, 0].view(-1, H, D), qk_rot[:, :, 1].view(-1, H, D), qkv[:, :, 2].view(-1, H, D)

    def separate():
        hip.rotary(qkv, qk_rot, cos, sin, (B, S, 2, H, D), st_x, st_y, 2, False)
        return flash_attn_unpadded_func(qr, kr, vr, cu, cu, S, S, 0.0)

    def fused_q():
        return FlashAttnRotaryQKVFunc.apply(qkv, cos, sin, 0.0, None, False)

    res = {"shape": f"B{B} S{S} H{H} D{D} bf16 non-causal forward",
           "separate_ms": round(timed(separate), 4), "fused_q_ms": round(timed(fused_q), 4),
           "attention_only_ms": round(timed(lambda: flash_attn_unpadded_qkvpacked_func(
               qkv.view(B * S, 3, H, D), cu, S, 0.0)), 4)}
    # equality of the fused-q and separate outputs (same MFMA operands)
    ref = flash_attn_unpadded_qkvpacked_func(apply_rotary_emb_qkv_(qkv.clone(), cos, sin).view(B * S, 3, H, D),
                                             cu, S, 0.0)
    res["fused_q_bitexact"] = bool(torch.equal(fused_q().reshape(B * S, H, D), ref))
    res["separate_bitexact"] = bool(torch.equal(separate(), ref))
    var = os.path.join(ROOT, "hazyresearch_flash-attention_amd", "build", "var_rotk.so")
    if os.path.exists(var):
        L = ctypes.CDLL(var)
        L.fa_fwd.argtypes = [ctypes.POINTER(hip.FaFwdArgs), ctypes.c_void_p]
        flat = qkv.view(B * S, 3, H, D)
        q, k, v = flat[:, 0], flat[:, 1], flat[:, 2]
        o = torch.empty(B * S, H, D, dtype=qkv.dtype, device="cuda")
        lse = torch.empty(B, H, S, dtype=torch.float32, device="cuda")
        a = hip.FaFwdArgs()
        a.q, a.k, a.v, a.o, a.softmax_lse = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr()
        a.cu_seqlens_q = a.cu_seqlens_k = cu.data_ptr()
        a.q_row_stride, a.q_head_stride = q.stride(0), q.stride(1)
        a.k_row_stride, a.k_head_stride = k.stride(0), k.stride(1)
        a.v_row_stride, a.v_head_stride = v.stride(0), v.stride(1)
        a.o_row_stride, a.o_head_stride = o.stride(0), o.stride(1)
        a.batch, a.nheads, a.head_dim, a.max_seqlen_q, a.max_seqlen_k, a.lse_stride = B, H, D, S, S, S
        a.softmax_scale, a.dtype = D ** -0.5, hip.FA_DTYPE_BF16
        a.rot_cos, a.rot_sin, a.rot_stride = cos.data_ptr(), sin.data_ptr(), cos.stride(0)
        stream = torch.cuda.current_stream().cuda_stream
        res["fused_qk_ms"] = round(timed(lambda: L.fa_fwd(ctypes.byref(a), stream)), 4)
        assert L.fa_fwd(ctypes.byref(a), stream) == 0
        torch.cuda.synchronize()
        res["fused_qk_max_diff"] = (o.float() - ref.float()).abs().max().item()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
