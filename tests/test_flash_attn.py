"""GPU parity tests of the HIP path against the oracle (the port of /root/reference/tests/test_flash_attn.py).

Same structure as the reference tests (:332-607): random padded batches, the unpadded
qkv-packed / kv-packed / separate layouts, return_attn_probs=True, and the "2x baseline" rule
(:407-409): max|out - ref_fp32| <= 2 * max|out_pt - ref_fp32|, where out_pt is the PyTorch
computation in the input dtype with reordered ops. The gradient checks the reference left
commented out (:390-403, :416-418, :575-607) are enabled here against autograd of the fp32
oracle with the kernel's own dropout mask. Dropout fraction within +-1 % relative of p
(:411-414). Everything goes through the C ABI (libfa_hip.so).
"""
import math

import numpy as np
import pytest
import torch

from fa_testutil import convert_s_dmask, make_inputs
from oracle.attention_ref import attention_ref, get_dropout_fraction, max_err_bound, pad, ulp_floor
from oracle.philox import dropout_keep_mask

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _fa():
    from flash_attn import flash_attn_interface as fi
    return fi


def run_case(layout, batch, seqlen_q, seqlen_k, nheads, d, dtype, causal, dropout_p, grad=True, seed=0,
             mode="random"):
    fi = _fa()
    torch.manual_seed(seed)
    x = make_inputs(batch, seqlen_q, seqlen_k, nheads, d, dtype, DEV, mode_q=mode, mode_k=mode,
                    layout=layout, seed=seed)
    qmask, kmask = x["qmask"], x["kmask"]
    q_u = x["q_unpad"].detach().requires_grad_()
    k_u = x["k_unpad"].detach().requires_grad_()
    v_u = x["v_unpad"].detach().requires_grad_()
    if layout == "qkvpacked":
        qkv_u = torch.stack([x["q_unpad"], x["k_unpad"], x["v_unpad"]], dim=1).detach().requires_grad_()
        out_u, lse, S = fi.flash_attn_unpadded_qkvpacked_func(qkv_u, x["cu_q"], x["max_q"], dropout_p,
                                                              causal=causal, return_attn_probs=True)
        inputs = (qkv_u,)
    elif layout == "kvpacked":
        kv_u = torch.stack([x["k_unpad"], x["v_unpad"]], dim=1).detach().requires_grad_()
        out_u, lse, S = fi.flash_attn_unpadded_kvpacked_func(q_u, kv_u, x["cu_q"], x["cu_k"], x["max_q"],
                                                             x["max_k"], dropout_p, causal=causal,
                                                             return_attn_probs=True)
        inputs = (q_u, kv_u)
    else:
        out_u, lse, S = fi.flash_attn_unpadded_func(q_u, k_u, v_u, x["cu_q"], x["cu_k"], x["max_q"], x["max_k"],
                                                    dropout_p, causal=causal, return_attn_probs=True)
        inputs = (q_u, k_u, v_u)
    out = pad(out_u, x["idx_q"], batch, seqlen_q)
    S_conv = convert_s_dmask(S, seqlen_q, seqlen_k, qmask, kmask, causal)
    dropout_mask = S_conv >= 0
    attn = S_conv.abs()
    q = x["q"].detach().requires_grad_()
    k = x["k"].detach().requires_grad_()
    v = x["v"].detach().requires_grad_()
    out_ref, attn_ref = attention_ref(q, k, v, qmask, kmask, dropout_p, dropout_mask, causal=causal)
    out_pt, attn_pt = attention_ref(q, k, v, qmask, kmask, dropout_p, dropout_mask, causal=causal,
                                    upcast=False, reorder_ops=True)
    err = (out - out_ref).abs().max().item()
    bound = max_err_bound(out_pt, out_ref)
    assert err <= bound, f"output max err {err} > {bound}"
    aerr = (attn - attn_ref).abs().max().item()
    abound = max_err_bound(attn_pt, attn_ref)
    assert aerr <= abound, f"attention max err {aerr} > {abound}"
    if dropout_p == 0.0:
        assert dropout_mask.all()
    else:
        frac = get_dropout_fraction(dropout_mask, qmask, kmask, causal=causal).item()
        assert 0.99 <= frac / dropout_p <= 1.01, f"dropout fraction {frac}"
    # LSE: natural log-sum-exp of the scaled scores on valid rows
    scores = torch.einsum("bthd,bshd->bhts", q.float(), k.float()) / math.sqrt(d)
    scores = scores.masked_fill(~kmask[:, None, None, :], float("-inf"))
    if causal:
        scores = scores.masked_fill(torch.triu(torch.ones(seqlen_q, seqlen_k, dtype=torch.bool, device=DEV), 1),
                                    float("-inf"))
    lse_ref = torch.logsumexp(scores, dim=-1)  # (B, H, Sq)
    valid = qmask[:, None, :].expand_as(lse_ref) & torch.isfinite(lse_ref)
    lse_k = lse[:, :, :seqlen_q] if lse.shape[2] >= seqlen_q else torch.nn.functional.pad(lse, (0, seqlen_q - lse.shape[2]))
    assert torch.allclose(lse_k[valid], lse_ref[valid], atol=2e-3, rtol=1e-3)
    if grad:
        g = torch.randn(out_u.shape, generator=torch.Generator().manual_seed(seed + 1)).to(dtype).to(DEV)
        grads = torch.autograd.grad(out_u, inputs, g)
        gpad = pad(g, x["idx_q"], batch, seqlen_q)
        dq_ref, dk_ref, dv_ref = torch.autograd.grad(out_ref, (q, k, v), gpad)
        dq_pt, dk_pt, dv_pt = torch.autograd.grad(out_pt, (q, k, v), gpad)
        if layout == "qkvpacked":
            dqkv = grads[0]
            dq_u, dk_u, dv_u = dqkv[:, 0], dqkv[:, 1], dqkv[:, 2]
        elif layout == "kvpacked":
            dq_u, dkv = grads
            dk_u, dv_u = dkv[:, 0], dkv[:, 1]
        else:
            dq_u, dk_u, dv_u = grads
        dq = pad(dq_u, x["idx_q"], batch, seqlen_q)
        dk = pad(dk_u, x["idx_k"], batch, seqlen_k)
        dv = pad(dv_u, x["idx_k"], batch, seqlen_k)
        for name, a, r, p in (("dq", dq, dq_ref, dq_pt), ("dk", dk, dk_ref, dk_pt), ("dv", dv, dv_ref, dv_pt)):
            e = (a.float() - r.float()).abs().max().item()
            bnd = max_err_bound(p, r)
            assert e <= bnd, f"{name} max err {e} > {bnd}"
    return out_u, lse, S


# The reference grid (:332-342) is 528 cases per layout; the default run samples it, the
# `slow` sweep covers all of it.
SEQLENS = [97, 128, 200, 256, 257, 384, 512, 768, 1024, 1025, 2048]
DIMS = [32, 56, 64, 80, 96, 128]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [32, 64, 80, 128])
@pytest.mark.parametrize("seqlen", [97, 128, 257, 512])
@pytest.mark.parametrize("dropout_p", [0.0, 0.17])
def test_flash_attn_unpadded(seqlen, d, dropout_p, causal, dtype):
    run_case("separate", 32, seqlen, seqlen, 4, d, dtype, causal, dropout_p)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [56, 64, 96])
@pytest.mark.parametrize("seqlen", [200, 384, 1025])
@pytest.mark.parametrize("dropout_p", [0.0, 0.17])
def test_flash_attn_unpadded_qkvpacked(seqlen, d, dropout_p, causal, dtype):
    run_case("qkvpacked", 32, seqlen, seqlen, 4, d, dtype, causal, dropout_p)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("seqlen_q,seqlen_k", [(128, 512), (512, 128), (257, 1025), (1024, 4096)])
@pytest.mark.parametrize("dropout_p", [0.0, 0.17])
def test_flash_attn_unpadded_kvpacked_cross(seqlen_q, seqlen_k, d, dropout_p, causal, dtype):
    # cross attention Sq != Sk (config 5 uses the kv-packed entry point); causal is top-left aligned
    run_case("kvpacked", 4, seqlen_q, seqlen_k, 4, d, dtype, causal, dropout_p)


@pytest.mark.slow
@pytest.mark.parametrize("layout", ["qkvpacked", "kvpacked", "separate"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", DIMS)
@pytest.mark.parametrize("seqlen", SEQLENS)
@pytest.mark.parametrize("dropout_p", [0.0, 0.17])
def test_flash_attn_reference_grid(layout, seqlen, d, dropout_p, causal, dtype):
    run_case(layout, 32, seqlen, seqlen, 4, d, dtype, causal, dropout_p)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [16, 32, 64, 128])
@pytest.mark.parametrize("seqlen", [97, 257, 1025])
@pytest.mark.parametrize("dropout_p", [0.0, 0.17])
def test_flash_attn_race_condition(seqlen, d, dropout_p, causal, dtype):
    """Determinism (tests/test_flash_attn.py:610-671): 10 reruns with the same seed give bit-identical
    outputs, probabilities and (here enabled) gradients. dQ is bitwise too where the query-major dQ
    pass writes it (D=128, no dropout); the atomic-dQ kernels sum it with fp32 atomics in a varying
    order, so there it may differ by one unit in the last place of the output dtype."""
    fi = _fa()
    from flash_attn import flash_attn_hip as hip
    atomic_dq = hip._bwd_needs_workspace(d, dropout_p > 0, False)
    x = make_inputs(8, seqlen, seqlen, 4, d, dtype, DEV, seed=0)
    q_u = x["q_unpad"].detach().requires_grad_()
    k_u = x["k_unpad"].detach().requires_grad_()
    v_u = x["v_unpad"].detach().requires_grad_()
    g = None
    ref = None
    for _ in range(10):
        torch.manual_seed(0)
        out, lse, S = fi.flash_attn_unpadded_func(q_u, k_u, v_u, x["cu_q"], x["cu_k"], x["max_q"], x["max_k"],
                                                  dropout_p, causal=causal, return_attn_probs=True)
        if g is None:
            g = torch.randn_like(out)
        dq, dk, dv = torch.autograd.grad(out, (q_u, k_u, v_u), g)
        if ref is None:
            ref = (out, S, dq, dk, dv)
            continue
        assert torch.equal(out, ref[0])
        assert torch.equal(S, ref[1])
        assert torch.equal(dk, ref[3])
        assert torch.equal(dv, ref[4])
        if atomic_dq:
            # fp32 atomics: the summation order of dQ varies, so the bf16/fp16 output may round to
            # the neighbouring value: at most one unit in the last place of the output dtype
            eps = torch.finfo(dtype).eps
            torch.testing.assert_close(dq.float(), ref[2].float(), rtol=eps, atol=eps * 1e-3)
        else:
            assert torch.equal(dq, ref[2])   # query-major dQ pass writes dq directly: bitwise


@pytest.mark.parametrize("causal", [False, True])
def test_dropout_mask_matches_oracle_rng(causal):
    """Bit-exact dropout pattern: the kernel's sign-encoded S_dmask equals the oracle's Philox mask."""
    fi = _fa()
    B, H, S, d, p = 2, 3, 200, 64, 0.17
    x = make_inputs(B, S, S, H, d, torch.bfloat16, DEV, mode_q="full", mode_k="full", seed=3)
    torch.manual_seed(123)
    from flash_attn import flash_attn_hip as hip
    seed, offset, _ = hip.reserve_rng(torch.device(DEV))
    out, lse, Sd = hip.fwd(x["q_unpad"], x["k_unpad"], x["v_unpad"], x["cu_q"], x["cu_k"], S, S, p, d ** -0.5,
                           False, causal, True, None, rng_state=(seed, offset))
    keep = torch.from_numpy(dropout_keep_mask(seed, offset, p, B, H, S, S)).to(DEV)
    Sd = Sd[:, :, :S, :S].float()
    valid = Sd != 0
    if causal:
        valid &= ~torch.triu(torch.ones(S, S, dtype=torch.bool, device=DEV), 1)
    assert valid.float().mean() > 0.4
    assert torch.equal((Sd >= 0)[valid], keep[valid])


def test_forced_max_rescale():
    """Rule 26 of the MI355X guide: force the online-softmax rescale branch (a spike key that a
    row only meets in a later tile) and compare against fp32."""
    fi = _fa()
    B, H, S, d = 2, 2, 512, 64
    x = make_inputs(B, S, S, H, d, torch.bfloat16, DEV, mode_q="full", mode_k="full", seed=5)
    q, k = x["q_unpad"].clone(), x["k_unpad"].clone()
    k[300] = q[7] * 3.0  # row 7 meets a huge score at key 300 (tile 4)
    k[450] = q[7] * 4.0
    out = fi.flash_attn_unpadded_func(q, k, x["v_unpad"], x["cu_q"], x["cu_k"], S, S, 0.0)
    ref, _ = attention_ref(q.view(B, S, H, d), k.view(B, S, H, d), x["v_unpad"].view(B, S, H, d))
    pt, _ = attention_ref(q.view(B, S, H, d), k.view(B, S, H, d), x["v_unpad"].view(B, S, H, d),
                          upcast=False, reorder_ops=True)
    err = (out.view(B, S, H, d).float() - ref.float()).abs().max().item()
    assert err <= max_err_bound(pt, ref)


def test_empty_and_ragged_sequences():
    """Zero-length and 1-token sequences: output 0 and lse -inf for empty key sets
    (fmha_fprop_kernel_1xN.h:617,645), correct values elsewhere."""
    fi = _fa()
    H, d = 2, 64
    lens_q = [5, 0, 1, 130, 64]
    lens_k = [7, 3, 0, 129, 1]
    cu_q = torch.tensor([0] + list(np.cumsum(lens_q)), dtype=torch.int32, device=DEV)
    cu_k = torch.tensor([0] + list(np.cumsum(lens_k)), dtype=torch.int32, device=DEV)
    g = torch.Generator().manual_seed(0)
    q = torch.randn(sum(lens_q), H, d, generator=g).bfloat16().to(DEV)
    k = torch.randn(sum(lens_k), H, d, generator=g).bfloat16().to(DEV)
    v = torch.randn(sum(lens_k), H, d, generator=g).bfloat16().to(DEV)
    out, lse, _ = fi.flash_attn_unpadded_func(q, k, v, cu_q, cu_k, max(lens_q), max(lens_k), 0.0,
                                              return_attn_probs=True)
    for b in range(len(lens_q)):
        qs, ks = slice(int(cu_q[b]), int(cu_q[b + 1])), slice(int(cu_k[b]), int(cu_k[b + 1]))
        if lens_q[b] == 0:
            continue
        if lens_k[b] == 0:
            assert (out[qs] == 0).all()
            assert torch.isinf(lse[b, :, :lens_q[b]]).all()
            continue
        ref, _ = attention_ref(q[qs][None], k[ks][None], v[ks][None])
        pt, _ = attention_ref(q[qs][None], k[ks][None], v[ks][None], upcast=False, reorder_ops=True)
        err = (out[qs].float() - ref[0].float()).abs().max().item()
        assert err <= max_err_bound(pt, ref, floor=ulp_floor(ref)), (b, err)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("d", [64, 128])
def test_empty_and_ragged_sequences_backward(d, causal):
    """Backward on zero-length and 1-token sequences: zero dQ for empty key sets, zero dK/dV for
    empty query sets, the 2x rule elsewhere. d=128 runs the P/dS split kernel plus the query-major
    dQ pass (no dq workspace, no convert pass), d=64 the atomic-dQ kernel."""
    fi = _fa()
    H = 2
    lens_q = [5, 0, 1, 130, 64, 3]
    lens_k = [7, 3, 0, 129, 1, 300]
    cu_q = torch.tensor([0] + list(np.cumsum(lens_q)), dtype=torch.int32, device=DEV)
    cu_k = torch.tensor([0] + list(np.cumsum(lens_k)), dtype=torch.int32, device=DEV)
    g = torch.Generator().manual_seed(1)
    q = torch.randn(sum(lens_q), H, d, generator=g).bfloat16().to(DEV).requires_grad_()
    k = torch.randn(sum(lens_k), H, d, generator=g).bfloat16().to(DEV).requires_grad_()
    v = torch.randn(sum(lens_k), H, d, generator=g).bfloat16().to(DEV).requires_grad_()
    out = fi.flash_attn_unpadded_func(q, k, v, cu_q, cu_k, max(lens_q), max(lens_k), 0.0, causal=causal)
    gout = torch.randn(out.shape, generator=g).bfloat16().to(DEV)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), gout)
    for b in range(len(lens_q)):
        qs, ks = slice(int(cu_q[b]), int(cu_q[b + 1])), slice(int(cu_k[b]), int(cu_k[b + 1]))
        if lens_q[b] == 0:
            assert (dk[ks] == 0).all() and (dv[ks] == 0).all()
            continue
        if lens_k[b] == 0:
            assert (dq[qs] == 0).all()
            continue
        qb, kb, vb = [t.detach()[sl][None].requires_grad_() for t, sl in ((q, qs), (k, ks), (v, ks))]
        ref, _ = attention_ref(qb, kb, vb, causal=causal)
        pt, _ = attention_ref(qb, kb, vb, causal=causal, upcast=False, reorder_ops=True)
        refs = torch.autograd.grad(ref, (qb, kb, vb), gout[qs][None])
        pts = torch.autograd.grad(pt, (qb, kb, vb), gout[qs][None])
        for name, a, r, lo in zip(("dq", "dk", "dv"), (dq[qs], dk[ks], dv[ks]), refs, pts):
            err = (a.float() - r[0].float()).abs().max().item()
            # a 1-key row has dq = 0 exactly in fp32, while the kernel's dP - delta cancels to
            # fp32 rounding residue (~1e-6): the floor is one output ulp, at least 1e-5
            assert err <= max_err_bound(lo, r, floor=max(ulp_floor(r), 1e-5)), (b, name, err)


def test_invalid_arguments_raise():
    fi = _fa()
    q = torch.randn(16, 2, 60, device=DEV, dtype=torch.float16)
    cu = torch.tensor([0, 16], dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError):
        fi.flash_attn_unpadded_func(q, q, q, cu, cu, 16, 16, 0.0)
    q = torch.randn(16, 2, 64, device=DEV, dtype=torch.float32)
    with pytest.raises(RuntimeError):
        fi.flash_attn_unpadded_func(q, q, q, cu, cu, 16, 16, 0.0)
