"""Shared helpers for the parity tests (test infrastructure)."""
import math

import torch

from oracle.attention_ref import generate_random_padding_mask, unpad, pad


def make_inputs(batch, seqlen_q, seqlen_k, nheads, d, dtype, device, mode_q="random", mode_k="random",
                layout="separate", seed=0, scale_in=1.0):
    """Random q/k/v (B,S,H,D) with padding masks and their unpadded forms.
    layout: 'separate' | 'kvpacked' | 'qkvpacked' (qkvpacked requires seqlen_q == seqlen_k and
    shares the key mask, like tests/test_flash_attn.py:357-362)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    q = (torch.randn(batch, seqlen_q, nheads, d, generator=g) * scale_in).to(dtype).to(device)
    k = (torch.randn(batch, seqlen_k, nheads, d, generator=g) * scale_in).to(dtype).to(device)
    v = torch.randn(batch, seqlen_k, nheads, d, generator=g).to(dtype).to(device)
    kmask = generate_random_padding_mask(seqlen_k, batch, "cpu", mode_k, generator=g).to(device)
    if layout == "qkvpacked":
        qmask = kmask
    else:
        qmask = generate_random_padding_mask(seqlen_q, batch, "cpu", mode_q, generator=g).to(device)
    q_unpad, idx_q, cu_q, max_q = unpad(q, qmask)
    k_unpad, idx_k, cu_k, max_k = unpad(k, kmask)
    v_unpad, _, _, _ = unpad(v, kmask)
    return dict(q=q, k=k, v=v, qmask=qmask, kmask=kmask, q_unpad=q_unpad, k_unpad=k_unpad, v_unpad=v_unpad,
                idx_q=idx_q, idx_k=idx_k, cu_q=cu_q, cu_k=cu_k, max_q=max_q, max_k=max_k)


def convert_s_dmask(S, seqlen_q, seqlen_k, qmask, kmask, causal):
    """Decode this build's S_dmask (row-major (B,H,Sq_r,Sk_r), local coordinates) into the padded
    (B,H,seqlen_q,seqlen_k) grid of the reference test (the role of
    convert_flash_attn_S_to_softmax, tests/test_flash_attn.py:218-262)."""
    B, H = S.shape[:2]
    out = torch.zeros(B, H, seqlen_q, seqlen_k, dtype=S.dtype, device=S.device)
    rq = min(seqlen_q, S.shape[2])
    rk = min(seqlen_k, S.shape[3])
    out[:, :, :rq, :rk] = S[:, :, :rq, :rk]
    out = out.masked_fill(~qmask[:, None, :, None], 0.0)
    out = out.masked_fill(~kmask[:, None, None, :], 0.0)
    if causal:
        cm = torch.triu(torch.ones(seqlen_q, seqlen_k, dtype=torch.bool, device=S.device), 1)
        out = out.masked_fill(cm, 0.0)
    return out
