"""Golden vectors for the block-sparse path, from the REFERENCE's own code (build container only).

    python tests/golden/make_golden_blocksparse.py   # writes tests/golden/blocksparse_golden.npz

Imports /root/reference/flash_attn/flash_blocksparse_attn_interface.py (convert_blockmask; an
empty `flash_attn_cuda` stub satisfies its import) and /root/reference/tests/test_flash_attn.py
(attention_blocksparse_ref; patched torch.cuda.get_device_capability), and records:
  - convert_blockmask outputs for seeded random layouts, including empty rows and columns;
  - attention_blocksparse_ref outputs and fp32 autograd gradients for small seeded cases, with
    the keep mask of this build's RNG (oracle/philox.py, regenerated from the stored seed and
    offset) in the dropout case.
tests/test_oracle.py compares the product's convert_blockmask and oracle/attention_ref.py's
restatement against these vectors without reading /root/reference.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

# name, B, S, H, D, dtype, dropout_p, padded
ATTN_CASES = [
    ("fp16_s512", 2, 512, 1, 16, torch.float16, 0.0, False),
    ("bf16_s300_pad", 2, 300, 2, 16, torch.bfloat16, 0.0, True),
    ("fp16_s512_dropout", 1, 512, 2, 16, torch.float16, 0.15, False),
]
MASK_SHAPES = [(4, 1), (16, 2), (32, 2), (64, 4), (128, 8), (7, 3)]


def import_reference():
    sys.modules.setdefault("flash_attn_cuda", types.ModuleType("flash_attn_cuda"))
    torch.cuda.get_device_capability = lambda *a, **k: (8, 0)
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "tests"))
    import test_flash_attn as ref_tests  # noqa: E402
    from flash_attn import flash_blocksparse_attn_interface as ref_bs  # noqa: E402
    return ref_tests, ref_bs


def main():
    ref, ref_bs = import_reference()
    sys.path.insert(0, ROOT)
    from oracle.philox import dropout_keep_mask
    out = {}
    g = torch.Generator().manual_seed(0)
    for i, (nr, nc) in enumerate(MASK_SHAPES):
        m = torch.rand(nr, nc, generator=g) < 0.5
        if i % 2 == 0:
            m[0] = False          # an empty row
        if nc > 1 and i % 3 == 0:
            m[:, -1] = False      # an empty column
        out[f"mask{i}/layout"] = m.numpy()
        out[f"mask{i}/converted"] = ref_bs.convert_blockmask(m, causal=False).numpy()
    for (name, B, S, H, D, dtype, p, padded) in ATTN_CASES:
        torch.manual_seed(len(name))
        nr, nc = (S + 255) // 256 * 16, (S + 255) // 256
        layout = torch.rand(nr, nc) < 0.6
        layout[3] = False                         # rows 48..63 see nothing -> output 0
        qkv = torch.randn(B, S, 3, H, D).to(dtype)
        attn_mask = (ref.generate_random_padding_mask(S, B, "cpu", "random") if padded
                     else torch.ones(B, S, dtype=torch.bool))
        if p > 0:
            seed, offset = 99, 4
            keep = torch.from_numpy(dropout_keep_mask(seed, offset, p, B, H, S, S))
        else:
            seed, offset = 0, 0
            keep = torch.ones(B, H, S, S, dtype=torch.bool)
        q32 = qkv.float().requires_grad_()
        o32, a32 = ref.attention_blocksparse_ref(q32, layout, attn_mask, p, keep)
        go = torch.randn(o32.shape, generator=torch.Generator().manual_seed(3))
        o32 = torch.nan_to_num(o32)
        (dqkv,) = torch.autograd.grad(o32, (q32,), go)
        o_lp, a_lp = ref.attention_blocksparse_ref(qkv, layout, attn_mask, p, keep)
        rec = dict(qkv=qkv.float(), layout=layout, attn_mask=attn_mask, out32=o32.detach(), go=go, dqkv32=dqkv,
                   out_lp=torch.nan_to_num(o_lp.float()))
        for key, val in rec.items():
            out[f"{name}/{key}"] = val.numpy()
        out[f"{name}/meta"] = np.array([B, S, H, D, seed, offset], dtype=np.int64)
        out[f"{name}/fparams"] = np.array([p], dtype=np.float64)
        out[f"{name}/dtype"] = np.array(str(dtype).replace("torch.", ""))
    np.savez_compressed(os.path.join(HERE, "blocksparse_golden.npz"), **out)


if __name__ == "__main__":
    main()
