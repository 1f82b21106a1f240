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


@pytest.mark.parametrize("dt", ["float32", "bfloat16"])
def test_rotary_oracle_matches_reference_golden(dt):
    """The oracle's rotary restatement (oracle/rotary_ref.py) against the reference's outputs."""
    from oracle.rotary_ref import rotary_1d_ref, rotary_2d_ref
    z = _z()
    t = lambda k: torch.from_numpy(z[f"rotary_{dt}/{k}"]).to(getattr(torch, dt))
    q, k = t("q"), t("k")
    qs, ks = q.transpose(1, 2).contiguous(), k.transpose(1, 2).contiguous()
    got = {}
    got["qa"], got["ka"] = rotary_1d_ref(q, k, -2)
    got["qb"], got["kb"] = rotary_1d_ref(qs, ks, -3)
    got["qc"], got["kc"] = rotary_2d_ref(q, k, -2)
    got["qd"], got["kd"] = rotary_2d_ref(qs, ks, -3)
    for key, val in got.items():
        assert torch.equal(val.float(), t(key).float()), key


def test_rotary_2d_token_tables_equal_grid_form():
    from oracle.rotary_ref import apply_rotary_ref, rotary_2d_ref, rotary_token_tables_2d
    g = torch.Generator().manual_seed(3)
    q = torch.randn(2, 3, 64, 16, generator=g).bfloat16()
    k = torch.randn(2, 3, 64, 16, generator=g).bfloat16()
    cos, sin = rotary_token_tables_2d(64, 16, torch.bfloat16)
    qr, kr = rotary_2d_ref(q, k, -2)
    assert torch.equal(apply_rotary_ref(q, cos, sin, -2), qr) and torch.equal(apply_rotary_ref(k, cos, sin, -2), kr)


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
    if mha.use_rotary_emb:   # the oracle's restatement of the reference rotary, on the host
        from oracle.rotary_ref import rotary_1d_ref, rotary_2d_ref
        fn = rotary_1d_ref if mha.use_rotary_emb == "1d" else rotary_2d_ref
        qc, kc = fn(q.detach().cpu(), k.detach().cpu(), -3)
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
    from oracle.attention_ref import ulp_floor
    assert err <= max(bound, ulp_floor(ref, dtype)), (err, bound)
    out.float().sum().backward()   # the module trains: backward runs through the HIP kernels
    assert mha.Wqkv.weight.grad is not None and torch.isfinite(mha.Wqkv.weight.grad).all()


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["auto", "hip"])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D", [32, 64, 128])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_fused_rotary_equals_separate_pass(route, causal, D, dtype):
    """FlashAttnRotaryQKVFunc gives the same output bits as rotating q and k first (fa_rotary) and
    running the plain forward, whichever route it takes: AUTO (assembly forward at D = 32 / 64 / 128)
    rotates q and k in one fa_rotary pass; under force_impl(FA_IMPL_HIP) the route follows the HIP
    forward, which rotates q at its Q load (the route decision sees the forced impl); its
    backward gives the same dk/dv bits and dq up to the order of the fp32 dQ atomics (D <= 64)."""
    import contextlib
    from flash_attn import flash_attn_hip as hip
    ctx = hip.force_impl(hip.FA_IMPL_HIP) if route == "hip" else contextlib.nullcontext()
    with ctx:
        _fused_rotary_case(causal, D, dtype, route)


def _fused_rotary_case(causal, D, dtype, route):
    from flash_attn.flash_attention import FlashAttnRotaryQKVFunc
    from flash_attn.flash_attn_interface import flash_attn_unpadded_qkvpacked_func
    from flash_attn.rotary import apply_rotary_emb_qkv_
    from oracle.rotary_ref import rotary_tables
    g = torch.Generator().manual_seed(D)
    B, S, H = 2, 333, 3
    qkv = torch.randn(B, S, 3, H, D, generator=g).to(dtype).cuda()
    cos, sin = (t.cuda() for t in rotary_tables(S, D, dtype))
    dout = torch.randn(B, S, H, D, generator=g).to(dtype).cuda()
    a = qkv.clone().requires_grad_()
    out_f = FlashAttnRotaryQKVFunc.apply(a, cos, sin, 0.0, None, causal)
    b = qkv.clone().requires_grad_()
    rot = apply_rotary_emb_qkv_(b.clone(), cos, sin)
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device="cuda")
    from flash_attn import flash_attn_hip as hip
    name = hip.fwd_kernel_name(B, H, D, S, S, dtype, causal, row_elems=3 * H * D, impl=hip._impl())
    assert name.endswith("_asm") == (route == "auto"), name
    out_s = flash_attn_unpadded_qkvpacked_func(rot.reshape(B * S, 3, H, D), cu, S, 0.0, causal=causal)
    assert torch.equal(out_f.reshape(B * S, H, D), out_s)
    ga, = torch.autograd.grad(out_f, a, dout)
    gb, = torch.autograd.grad(out_s, b, dout.reshape(B * S, H, D))
    assert torch.equal(ga[:, :, 1:], gb[:, :, 1:])                # dk, dv
    torch.testing.assert_close(ga[:, :, 0], gb[:, :, 0], rtol=0, atol=2e-2 if dtype == torch.bfloat16 else 4e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("rotary", ["1d", "2d"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_fused_rotary_against_oracle(rotary, dtype):
    """FlashMHA's fused-rotary path (no key padding mask) against oracle rotary + oracle
    attention, output and input gradients, under the reference's 2x rule."""
    from flash_attn.flash_attention import FlashAttnRotaryQKVFunc
    from oracle.attention_ref import attention_ref, max_err_bound
    from oracle.rotary_ref import rotary_1d_ref, rotary_2d_ref, rotary_tables, rotary_token_tables_2d
    g = torch.Generator().manual_seed(7)
    B, S, H, D = 2, 256, 4, 64
    qkv = torch.randn(B, S, 3, H, D, generator=g).to(dtype)
    dout = torch.randn(B, S, H, D, generator=g).to(dtype)
    cos, sin = (rotary_tables(S, D, dtype) if rotary == "1d" else rotary_token_tables_2d(S, D, dtype))
    a = qkv.cuda().requires_grad_()
    out = FlashAttnRotaryQKVFunc.apply(a, cos.cuda(), sin.cuda(), 0.0, None, True)
    grad, = torch.autograd.grad(out, a, dout.cuda())
    x = qkv.clone().requires_grad_()
    q, k, v = x.unbind(dim=2)
    q_r, k_r = (rotary_1d_ref if rotary == "1d" else rotary_2d_ref)(q, k, -3)
    refs = []
    for up in (True, False):
        o, _ = attention_ref(q_r.cuda(), k_r.cuda(), v.cuda(), causal=True, upcast=up, reorder_ops=not up)
        refs.append((o, torch.autograd.grad(o, x, dout.cuda(), retain_graph=True)[0]))
    (ref, gref), (pt, gpt) = refs
    err = (out.float() - ref.float()).abs().max().item()
    assert err <= max_err_bound(pt, ref), err
    for i in range(3):
        e = (grad[:, :, i].float() - gref[:, :, i].float().cuda()).abs().max().item()
        assert e <= max_err_bound(gpt[:, :, i].cuda(), gref[:, :, i].cuda()), (i, e)
