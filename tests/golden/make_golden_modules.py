"""Golden vectors for the §8(f) Python surface, from the REFERENCE's own modules (run here only).

    python tests/golden/make_golden_modules.py   # writes tests/golden/modules_golden.npz

flash_attn.rotary (1-D at seq_dimension -2 / -3, 2-D) and flash_attn.bert_padding
(unpad_input / pad_input) of /root/reference, imported directly (they need no CUDA). Inputs are
seeded; fp32 and bf16. tests/test_modules.py compares this build's modules against them.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")
from flash_attn.rotary import RotaryEmbedding, RotaryEmbedding2D  # noqa: E402  (the reference's)
from flash_attn.bert_padding import unpad_input, pad_input  # noqa: E402


def main():
    out = {}
    g = torch.Generator().manual_seed(0)
    for dt in (torch.float32, torch.bfloat16):
        name = str(dt).replace("torch.", "")
        q = torch.randn(2, 3, 16, 32, generator=g).to(dt)   # (b, h, s, d)
        k = torch.randn(2, 3, 16, 32, generator=g).to(dt)
        r1 = RotaryEmbedding(32)
        qa, ka = r1(q, k, seq_dimension=-2)
        qs = q.transpose(1, 2).contiguous()                  # (b, s, h, d)
        ks = k.transpose(1, 2).contiguous()
        qb, kb = RotaryEmbedding(32)(qs, ks, seq_dimension=-3)
        qc, kc = RotaryEmbedding2D(32)(q, k, seq_dimension=-2)
        qd, kd = RotaryEmbedding2D(32)(qs, ks, seq_dimension=-3)
        for key, t in dict(q=q, k=k, qa=qa, ka=ka, qb=qb, kb=kb, qc=qc, kc=kc, qd=qd, kd=kd).items():
            out[f"rotary_{name}/{key}"] = t.float().numpy()
    x = torch.randn(3, 7, 5, generator=g)
    mask = torch.tensor([[1, 1, 1, 0, 0, 0, 0], [1, 1, 1, 1, 1, 1, 1], [1, 0, 1, 1, 0, 0, 1]], dtype=torch.bool)
    xu, idx, cu, mx = unpad_input(x, mask)
    xp = pad_input(xu, idx, 3, 7)
    out.update({"pad/x": x.numpy(), "pad/mask": mask.numpy(), "pad/x_unpad": xu.numpy(), "pad/indices": idx.numpy(),
                "pad/cu_seqlens": cu.numpy(), "pad/max_seqlen": np.array(mx), "pad/x_pad": xp.numpy()})
    path = os.path.join(HERE, "modules_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e3:.1f} kB)")


if __name__ == "__main__":
    main()
