"""The §8(f) Python surface: rotary embeddings and var-len padding restated in this build,
pinned bit-exactly against golden vectors from the reference's own modules
(tests/golden/make_golden_modules.py); FlashAttention / FlashMHA modules on the GPU against the
oracle under the 2x rule (rows f1, f2 of SURVEY.md §8)."""
import math
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "modules_golden.npz")


def _z():
    return np.load(GOLD, allow_pickle=False)


@pytest.mark.parametrize("dt", ["float32", "bfloat16"])
def test_rotary_matches_reference_golden(dt):
    from flash_attn.rotary import RotaryEmbedding, RotaryEmbedding2D
    z = _z()
    t = lambda k: torch.from_numpy(z[f"rotary_{dt}/{k}"]).to(getattr(torch, dt))
    q, k = t("q"), t("k")
    qs, ks = q.transpose(1, 2).contiguous(), k.transpose(1, 2).contiguous()
    got = {}
    got["qa"], got["ka"] = RotaryEmbedding(32)(q, k, seq_dimension=-2)
    got["qb"], got["kb"] = RotaryEmbedding(32)(qs, ks, seq_dimension=-3)
    got["qc"], got["kc"] = RotaryEmbedding2D(32)(q, k, seq_dimension=-2)
    got["qd"], got["kd"] = RotaryEmbedding2D(32)(qs, ks, seq_dimension=-3)
    for key, val in got.items():
        assert torch.equal(val.float(), t(key).float()), key


def test_padding_matches_reference_golden():
    from flash_attn.bert_padding import pad_input, unpad_input
    z = _z()
    x = torch.from_numpy(z["pad/x"])
    mask = torch.from_numpy(z["pad/mask"])
    xu, idx, cu, mx = unpad_input(x, mask)
    assert torch.equal(xu, torch.from_numpy(z["pad/x_unpad"]))
    assert torch.equal(idx, torch.from_numpy(z["pad/indices"]))
    assert torch.equal(cu, torch.from_numpy(z["pad/cu_seqlens"]))
    assert mx == int(z["pad/max_seqlen"])
    assert torch.equal(pad_input(xu, idx, 3, 7), torch.from_numpy(z["pad/x_pad"]))


def test_padding_autograd_roundtrip():
    from flash_attn.bert_padding import pad_input, unpad_input
    x = torch.randn(2, 5, 3, requires_grad=True)
    mask = torch.tensor([[1, 1, 0, 0, 0], [1, 1, 1, 1, 0]], dtype=torch.bool)
    xu, idx, cu, mx = unpad_input(x, mask)
    y = pad_input(xu * 2, idx, 2, 5)
    y.sum().backward()
    assert torch.equal(x.grad, mask[..., None].float().expand_as(x) * 2)


def _mha_ref(mha, x, key_padding_mask, causal):
    """The same block with the oracle attention (fp32 upcast / native low precision)."""
    from oracle.attention_ref import attention_ref
    qkv = mha.Wqkv(x).reshape(x.shape[0], x.shape[1], 3, mha.num_heads, mha.head_dim)
    q, k, v = qkv.unbind(dim=2)
    if mha.use_rotary_emb:   # the torch expression on the host (fresh module, same tables)
        from flash_attn.rotary import RotaryEmbedding, RotaryEmbedding2D
        emb = (RotaryEmbedding if mha.use_rotary_emb == "1d" else RotaryEmbedding2D)(mha.head_dim)
        qc, kc = emb(q.detach().cpu(), k.detach().cpu(), seq_dimension=-3)
        q, k = qc.to(q.device), kc.to(k.device)
    outs = []
    for up in (True, False):
        o, _ = attention_ref(q, k, v, key_padding_mask, key_padding_mask, causal=causal, upcast=up, reorder_ops=not up)
        outs.append(mha.out_proj(o.reshape(x.shape[0], x.shape[1], -1)))
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("rotary", [None, "1d", "2d"])
@pytest.mark.parametrize("padded", [False, True])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_flash_mha_module(rotary, padded, dtype):
    from flash_attn.flash_attention import FlashMHA
    from oracle.attention_ref import generate_random_padding_mask
    torch.manual_seed(0)
    B, S, E, H = 4, 256, 256, 4
    mha = FlashMHA(E, H, causal=True, use_rotary_emb=rotary, device="cuda", dtype=dtype).eval()
    x = torch.randn(B, S, E, device="cuda", dtype=dtype)
    mask = generate_random_padding_mask(S, B, "cuda", "random") if padded else None
    out, _ = mha(x, key_padding_mask=mask)
    ref, pt = _mha_ref(mha, x, mask, True)
    if mask is not None:  # padded query rows are garbage-in/zero-out; compare valid rows
        m = mask[..., None]
        out, ref, pt = out * m, ref * m, pt * m
    err = (out.float() - ref.float()).abs().max().item()
    bound = 2 * (pt.float() - ref.float()).abs().max().item()
    assert err <= max(bound, 1e-2), (err, bound)
    out.float().sum().backward()   # the module trains: backward runs through the HIP kernels
    assert mha.Wqkv.weight.grad is not None and torch.isfinite(mha.Wqkv.weight.grad).all()
