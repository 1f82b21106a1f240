"""Generate golden vectors from the REFERENCE's own oracle (run in the build container only).

    python tests/golden/make_golden.py            # writes tests/golden/attention_ref_golden.npz

It imports /root/reference/tests/test_flash_attn.py (with an empty `flash_attn_cuda` stub and a
patched torch.cuda.get_device_capability, both needed only to import it on a CPU-only torch),
draws seeded inputs, and records the reference's attention_ref outputs (fp32 upcast oracle and
the reordered low-precision baseline), its get_dropout_fraction, and the autograd gradients of
the fp32 oracle. Dropout cases use the keep mask of this build's RNG (oracle/philox.py), so the
fixture also pins that mask. The tests (tests/test_oracle.py) never read /root/reference: they
compare oracle/attention_ref.py against these stored vectors.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

CASES = [
    # name, B, Sq, Sk, H, D, dtype, causal, dropout_p, masks(q,k), grads
    ("c1_fp32_full", 2, 128, 128, 2, 16, torch.float32, False, 0.0, ("full", "full"), True),
    ("fp16_pad_97", 2, 97, 97, 2, 32, torch.float16, False, 0.0, ("random", "random"), True),
    ("bf16_pad_causal_128", 2, 128, 128, 2, 32, torch.bfloat16, True, 0.0, ("random", "random"), True),
    ("bf16_cross_64x100_causal", 2, 64, 100, 2, 32, torch.bfloat16, True, 0.0, ("random", "random"), True),
    ("fp16_dropout_causal_80", 2, 80, 80, 2, 32, torch.float16, True, 0.17, ("random", "random"), True),
    ("bf16_dropout_cross_48x96", 2, 48, 96, 2, 64, torch.bfloat16, False, 0.1, ("third", "random"), True),
]


def import_reference():
    sys.modules.setdefault("flash_attn_cuda", types.ModuleType("flash_attn_cuda"))
    torch.cuda.get_device_capability = lambda *a, **k: (8, 0)
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "tests"))
    import test_flash_attn as ref_tests  # noqa: E402
    return ref_tests


def main():
    ref = import_reference()
    sys.path.insert(0, ROOT)
    from oracle.philox import dropout_keep_mask
    out = {}
    for (name, B, Sq, Sk, H, D, dtype, causal, p, (mq, mk), grads) in CASES:
        torch.manual_seed(len(name))
        q = torch.randn(B, Sq, H, D).to(dtype).requires_grad_()
        k = torch.randn(B, Sk, H, D).to(dtype).requires_grad_()
        v = torch.randn(B, Sk, H, D).to(dtype).requires_grad_()
        qmask = ref.generate_random_padding_mask(Sq, B, "cpu", mq)
        kmask = ref.generate_random_padding_mask(Sk, B, "cpu", mk)
        if p > 0:
            seed, offset = 1234 + len(name), 8
            keep = torch.from_numpy(dropout_keep_mask(seed, offset, p, B, H, Sq, Sk))
        else:
            seed, offset = 0, 0
            keep = torch.ones(B, H, Sq, Sk, dtype=torch.bool)
        o_ref, a_ref = ref.attention_ref(q, k, v, qmask, kmask, p, keep, causal=causal)
        o_pt, a_pt = ref.attention_ref(q, k, v, qmask, kmask, p, keep, causal=causal, upcast=False, reorder_ops=True)
        frac = ref.get_dropout_fraction(keep, qmask, kmask, causal=causal).item()
        rec = dict(q=q, k=k, v=v, qmask=qmask, kmask=kmask, keep=keep, out_ref=o_ref, attn_ref=a_ref,
                   out_pt=o_pt, attn_pt=a_pt)
        if grads:
            g = torch.randn(o_ref.shape, generator=torch.Generator().manual_seed(7)).to(dtype)
            dq, dk, dv = torch.autograd.grad(o_ref, (q, k, v), g)
            rec.update(g=g, dq_ref=dq, dk_ref=dk, dv_ref=dv)
        for key, val in rec.items():
            t = val.detach()
            if t.dtype in (torch.float16, torch.bfloat16):
                t = t.float()  # exact: every 16-bit value is representable in fp32
            out[f"{name}/{key}"] = t.numpy()
        out[f"{name}/meta"] = np.array([B, Sq, Sk, H, D, int(causal), seed, offset], dtype=np.int64)
        out[f"{name}/fparams"] = np.array([p, frac], dtype=np.float64)
        out[f"{name}/dtype"] = np.array(str(dtype).replace("torch.", ""))
    path = os.path.join(HERE, "attention_ref_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(CASES)} cases)")


if __name__ == "__main__":
    main()
