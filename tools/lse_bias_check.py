"""Forward error against an fp64 reference for the library FA_HIP_LIB names (tools only): the
signed mean and max of the LSE error and the O error, bf16 or fp16, non-causal and causal, at a few shapes.
Compares the rounding of P between library builds (e.g. PTRUNC's truncation + delta shift against the
round-to-nearest conversion).

    FA_HIP_LIB=.../libfa_hip_ptr.so python tools/lse_bias_check.py --tag ptr
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hazyresearch_flash-attention_amd"))
import torch  # noqa: E402
from flash_attn import flash_attn_hip as hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="prod")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    a = ap.parse_args()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    dev = torch.device("cuda")
    for (B, H, S, D, causal, scale_mul) in ((2, 4, 2048, 64, False, 1.0), (2, 4, 2048, 64, True, 1.0),
                                          (4, 4, 512, 32, False, 1.0), (2, 4, 1024, 64, False, 4.0),
                                          (1, 4, 8192, 64, False, 1.0), (1, 4, 8192, 64, False, 0.25)):
        g = torch.Generator(device=dev).manual_seed(1)
        q = torch.randn(B * S, H, D, generator=g, device=dev).to(dt)
        k = torch.randn(B * S, H, D, generator=g, device=dev).to(dt)
        v = torch.randn(B * S, H, D, generator=g, device=dev).to(dt)
        cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=dev)
        scale = D ** -0.5 * scale_mul
        out, lse = hip.fwd(q, k, v, cu, cu, S, S, 0.0, scale, False, causal, False, None)[:2]
        qd, kd, vd = (x.double().view(B, S, H, D).transpose(1, 2) for x in (q, k, v))
        s = torch.matmul(qd, kd.transpose(-1, -2)) * scale
        if causal:
            s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=dev), 1), float("-inf"))
        ref_lse = torch.logsumexp(s, -1)                                  # B H S
        ref_o = torch.matmul(torch.softmax(s, -1), vd).transpose(1, 2)    # B S H D
        el = lse[:, :, :S].double() - ref_lse
        eo = out.double().view(B, S, H, D) - ref_o
        print(json.dumps({"lib": a.tag, "dtype": a.dtype, "B": B, "H": H, "S": S, "D": D, "causal": causal, "scale_mul": scale_mul,
                          "lse_mean": float(el.mean()), "lse_maxabs": float(el.abs().max()),
                          "o_mean": float(eo.mean()), "o_maxabs": float(eo.abs().max()),
                          "o_rms": float(eo.pow(2).mean().sqrt())}), flush=True)


if __name__ == "__main__":
    main()
