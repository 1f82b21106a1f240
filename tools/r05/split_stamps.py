"""Per-phase shader-clock cycles of the skewed D=128 split backward kernel (tools only).

Needs a library built with -DFA_BWD_SPLIT_PROBE=6 (wrong dK / dV by design): every wave writes its
phase sums over the steps into the first key row of its output (P waves: dv, dS waves: dk).
    FA_HIP_LIB=.../libfa_hip_st.so python tools/r05/split_stamps.py [--B 16 --H 12 --S 4096 --causal 1]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "hazyresearch_flash-attention_amd"))
from flash_attn.flash_attn_interface import flash_attn_unpadded_func  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=16)
ap.add_argument("--H", type=int, default=12)
ap.add_argument("--S", type=int, default=4096)
ap.add_argument("--causal", type=int, default=1)
a = ap.parse_args()
D = 128
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
q, k, v = [torch.randn(a.B * a.S, a.H, D, generator=g, device=dev).to(torch.bfloat16).requires_grad_() for _ in range(3)]
cu = torch.arange(0, (a.B + 1) * a.S, a.S, dtype=torch.int32, device=dev)
for it in range(3):
    out = flash_attn_unpadded_func(q, k, v, cu, cu, a.S, a.S, 0.0, causal=bool(a.causal))
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), torch.ones_like(out))
torch.cuda.synchronize()
res = {}
for name, t in (("P_waves", dv), ("dS_waves", dk)):
    w = t.detach().contiguous().view(torch.int64).view(a.B * a.S, a.H, D // 4)
    rows = torch.arange(0, a.B * a.S, 32, device=dev)            # k0 + 32 kwave of every wave
    rec = w[rows][:, :, :6].reshape(-1, 6).double()
    steps = rec[:, 5].clamp(min=1)
    per = rec[:, :5] / steps[:, None]
    res[name] = {"phases_cycles_per_step": [round(x, 1) for x in per.mean(0).tolist()],
                 "total_per_step": round(per.sum(1).mean().item(), 1), "waves": rec.shape[0]}
res["phases"] = ["operand reads + S/dZ chain", "P/dS VALU + P exchange", "update MFMAs (results consumed)",
                 "staging LDS stores", "barrier"]
print(json.dumps(res))
