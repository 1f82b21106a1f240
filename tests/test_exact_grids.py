"""GPU parity at the exact BASELINE.json grids, through the product path (no return_attn_probs):

  C2  B=8  H=12 S=512         D=64  fp16 non-causal, forward (+ LSE)
  C3  B=8  H=12 S=2048        D=64  bf16 causal, dropout 0.1, forward + backward
  C4  B=16 H=12 S=4096        D=128 bf16 causal, forward (+ LSE)
  C5  B=4  H=16 Sq=1024 Sk=4096 D=64 bf16 cross-attention via flash_attn_unpadded_kvpacked_func,
      forward + backward

Each is checked against the fp32 oracle (oracle/attention_ref.py, the reference's attention_ref,
tests/test_flash_attn.py:115-159) with the reference's 2x rule (:407-409): max|out - ref| <=
2 max|out_pt - ref|, out_pt = the same computation in the input dtype with reordered ops; the
gradients with the same rule against autograd of both. C3's dropout mask is the oracle's Philox
stream (oracle/philox.py) at the (seed, offset) the forward reserved from the torch generator
(its bit-exactness against the kernels is test_flash_attn.py::test_dropout_mask_matches_oracle_rng).
The oracle runs on the GPU in fp32 (seconds at these sizes); C4's in batch chunks.
"""
import math

import pytest
import torch

from oracle.attention_ref import attention_ref, max_err_bound
from oracle.philox import dropout_keep_mask_torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _fi():
    from flash_attn import flash_attn_interface as fi
    return fi


def _inputs(B, Sq, Sk, H, D, dtype, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    q = torch.randn(B * Sq, H, D, generator=g, device=DEV).to(dtype)
    k = torch.randn(B * Sk, H, D, generator=g, device=DEV).to(dtype)
    v = torch.randn(B * Sk, H, D, generator=g, device=DEV).to(dtype)
    cu_q = torch.arange(0, (B + 1) * Sq, Sq, dtype=torch.int32, device=DEV)
    cu_k = torch.arange(0, (B + 1) * Sk, Sk, dtype=torch.int32, device=DEV)
    return q, k, v, cu_q, cu_k


def _lse_ref(q4, k4, causal):
    d = q4.shape[-1]
    s = torch.einsum("bthd,bshd->bhts", q4.float(), k4.float()) / math.sqrt(d)
    if causal:
        Sq, Sk = s.shape[-2:]
        s.masked_fill_(torch.triu(torch.ones(Sq, Sk, dtype=torch.bool, device=DEV), 1), float("-inf"))
    return torch.logsumexp(s, dim=-1)


def _check_lse(q, k, v, cu_q, cu_k, B, Sq, Sk, H, D, causal, chunk=None):
    from flash_attn import flash_attn_hip as hip
    _, lse = hip.fwd(q, k, v, cu_q, cu_k, Sq, Sk, 0.0, D ** -0.5, False, causal, False, None)
    chunk = chunk or B
    for b0 in range(0, B, chunk):
        b1 = min(B, b0 + chunk)
        ref = _lse_ref(q[b0 * Sq:b1 * Sq].view(b1 - b0, Sq, H, D), k[b0 * Sk:b1 * Sk].view(b1 - b0, Sk, H, D), causal)
        torch.testing.assert_close(lse[b0:b1, :, :Sq], ref, atol=2e-3, rtol=1e-3)


def _check_fwd(out, q, k, v, B, Sq, Sk, H, D, causal, chunk=None):
    chunk = chunk or B
    with torch.no_grad():
        for b0 in range(0, B, chunk):
            b1 = min(B, b0 + chunk)
            q4 = q[b0 * Sq:b1 * Sq].view(b1 - b0, Sq, H, D)
            k4 = k[b0 * Sk:b1 * Sk].view(b1 - b0, Sk, H, D)
            v4 = v[b0 * Sk:b1 * Sk].view(b1 - b0, Sk, H, D)
            ref, _ = attention_ref(q4, k4, v4, causal=causal)
            pt, _ = attention_ref(q4, k4, v4, causal=causal, upcast=False, reorder_ops=True)
            err = (out[b0 * Sq:b1 * Sq].view(b1 - b0, Sq, H, D).float() - ref.float()).abs().max().item()
            bound = max_err_bound(pt, ref)
            assert err <= bound, f"batches {b0}:{b1}: output max err {err} > {bound}"


def _check_fwd_bwd(fn, inputs, unpack, q, k, v, B, Sq, Sk, H, D, causal, p=0.0, keep=None, seed=0):
    """fn(*inputs) -> out (product path); unpack(grads) -> (dq, dk, dv) unpadded."""
    out = fn(*inputs)
    g = torch.randn(out.shape, generator=torch.Generator(device=DEV).manual_seed(seed + 1), device=DEV).to(out.dtype)
    dq, dk, dv = unpack(torch.autograd.grad(out, inputs, g))
    q4 = q.detach().view(B, Sq, H, D).requires_grad_()
    k4 = k.detach().view(B, Sk, H, D).requires_grad_()
    v4 = v.detach().view(B, Sk, H, D).requires_grad_()
    ref, _ = attention_ref(q4, k4, v4, dropout_p=p, dropout_mask=keep, causal=causal)
    pt, _ = attention_ref(q4, k4, v4, dropout_p=p, dropout_mask=keep, causal=causal, upcast=False, reorder_ops=True)
    err = (out.view(B, Sq, H, D).float() - ref.float()).abs().max().item()
    bound = max_err_bound(pt, ref)
    assert err <= bound, f"output max err {err} > {bound}"
    g4 = g.view(B, Sq, H, D)
    r = torch.autograd.grad(ref, (q4, k4, v4), g4)
    pg = torch.autograd.grad(pt, (q4, k4, v4), g4)
    for name, a, rr, pp, S in (("dq", dq, r[0], pg[0], Sq), ("dk", dk, r[1], pg[1], Sk), ("dv", dv, r[2], pg[2], Sk)):
        e = (a.view(B, S, H, D).float() - rr.float()).abs().max().item()
        bnd = max_err_bound(pp, rr)
        assert e <= bnd, f"{name} max err {e} > {bnd}"


def test_c2_exact_grid_fp16_forward():
    B, S, H, D = 8, 512, 12, 64
    q, k, v, cu, _ = _inputs(B, S, S, H, D, torch.float16, seed=21)
    out = _fi().flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0)
    _check_fwd(out, q, k, v, B, S, S, H, D, causal=False)
    _check_lse(q, k, v, cu, cu, B, S, S, H, D, causal=False)


def test_c3_exact_grid_bf16_causal_dropout_fwd_bwd():
    B, S, H, D, p = 8, 2048, 12, 64, 0.1
    q, k, v, cu, _ = _inputs(B, S, S, H, D, torch.bfloat16, seed=31)
    q, k, v = (t.requires_grad_() for t in (q, k, v))
    gen = torch.cuda.default_generators[torch.cuda.current_device()]
    torch.cuda.manual_seed(1234)
    seed, offset = gen.initial_seed(), gen.get_offset()      # what the forward reserves next
    keep = dropout_keep_mask_torch(seed, offset, p, B, H, S, S, DEV)
    fi = _fi()
    _check_fwd_bwd(lambda a, b, c: fi.flash_attn_unpadded_func(a, b, c, cu, cu, S, S, p, causal=True),
                   (q, k, v), lambda gr: gr, q, k, v, B, S, S, H, D, causal=True, p=p, keep=keep)
    assert gen.get_offset() == offset + 4, "the forward must have drawn exactly one Philox reservation"


def test_c4_exact_grid_d128_causal_forward():
    B, S, H, D = 16, 4096, 12, 128
    q, k, v, cu, _ = _inputs(B, S, S, H, D, torch.bfloat16, seed=41)
    out = _fi().flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0, causal=True)
    _check_fwd(out, q, k, v, B, S, S, H, D, causal=True, chunk=2)
    _check_lse(q, k, v, cu, cu, B, S, S, H, D, causal=True, chunk=2)


def test_c5_exact_grid_kvpacked_cross_fwd_bwd():
    B, Sq, Sk, H, D = 4, 1024, 4096, 16, 64
    q, k, v, cu_q, cu_k = _inputs(B, Sq, Sk, H, D, torch.bfloat16, seed=51)
    kv = torch.stack([k, v], dim=1).requires_grad_()
    q = q.requires_grad_()
    fi = _fi()
    _check_fwd_bwd(lambda a, b: fi.flash_attn_unpadded_kvpacked_func(a, b, cu_q, cu_k, Sq, Sk, 0.0),
                   (q, kv), lambda gr: (gr[0], gr[1][:, 0], gr[1][:, 1]), q, k, v, B, Sq, Sk, H, D, causal=False)
    _check_lse(q.detach(), k, v, cu_q, cu_k, B, Sq, Sk, H, D, causal=False)


def _check_fwd_bwd_chunked(out, g, grads, q, k, v, B, Sq, Sk, H, D, causal, chunk):
    """The 2x rule over the whole grid with the oracle run in batch chunks (attention is per sequence,
    so every chunk's fp32 and low-precision autograd is exact for its rows): the maximum error over
    all chunks against twice the maximum baseline error over all chunks, for out, dq, dk, dv."""
    worst = {n: [0.0, 0.0] for n in ("out", "dq", "dk", "dv")}
    for b0 in range(0, B, chunk):
        b1 = min(B, b0 + chunk)
        n = b1 - b0
        q4 = q[b0 * Sq:b1 * Sq].detach().view(n, Sq, H, D).requires_grad_()
        k4 = k[b0 * Sk:b1 * Sk].detach().view(n, Sk, H, D).requires_grad_()
        v4 = v[b0 * Sk:b1 * Sk].detach().view(n, Sk, H, D).requires_grad_()
        g4 = g[b0 * Sq:b1 * Sq].view(n, Sq, H, D)
        for upcast in (True, False):
            o, _ = attention_ref(q4, k4, v4, causal=causal, upcast=upcast, reorder_ops=not upcast)
            gr = torch.autograd.grad(o, (q4, k4, v4), g4)
            if upcast:
                ref, rgr = o.detach(), gr
            else:
                pt, pgr = o.detach(), gr
        mine = (out[b0 * Sq:b1 * Sq].view(n, Sq, H, D),) + tuple(
            t[r0:r1].view(n, S, H, D) for t, (r0, r1, S) in
            zip(grads, ((b0 * Sq, b1 * Sq, Sq), (b0 * Sk, b1 * Sk, Sk), (b0 * Sk, b1 * Sk, Sk))))
        for name, a, rr, pp in zip(("out", "dq", "dk", "dv"), mine, (ref,) + tuple(rgr), (pt,) + tuple(pgr)):
            worst[name][0] = max(worst[name][0], (a.float() - rr.float()).abs().max().item())
            worst[name][1] = max(worst[name][1], max_err_bound(pp, rr))
        del ref, pt, rgr, pgr, q4, k4, v4
    for name, (e, bnd) in worst.items():
        assert e <= bnd, f"{name}: max err {e} > {bnd} (2x rule over the whole grid)"


def test_c4_exact_grid_d128_causal_backward():
    """C4 (B16 H12 S4096 D128 causal) forward + backward at the exact grid, the
    gradients under the 2x rule against autograd of the oracle run in 2-batch chunks."""
    B, S, H, D = 16, 4096, 12, 128
    q, k, v, cu, _ = _inputs(B, S, S, H, D, torch.bfloat16, seed=42)
    q, k, v = (t.requires_grad_() for t in (q, k, v))
    out = _fi().flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0, causal=True)
    g = torch.randn(out.shape, generator=torch.Generator(device=DEV).manual_seed(43), device=DEV).to(out.dtype)
    grads = torch.autograd.grad(out, (q, k, v), g)
    _check_fwd_bwd_chunked(out.detach(), g, grads, q, k, v, B, S, S, H, D, causal=True, chunk=2)


def test_north_star_grid_all_heads_persistent_forward():
    """the bench workload (B8 H12 S2048 D64 bf16, 768 blocks, the persistent asm form
    FA_IMPL_AUTO picks) against the fp32 oracle on all 96 heads under the 2x rule, with the LSE."""
    from flash_attn import flash_attn_hip as hip
    B, S, H, D = 8, 2048, 12, 64
    assert hip.fwd_kernel_name(B, H, D, S, S, torch.bfloat16) == "fa_fwd_d64p_bf16_asm"
    q, k, v, cu, _ = _inputs(B, S, S, H, D, torch.bfloat16, seed=61)
    out = _fi().flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0)
    worst = [0.0, 0.0]
    with torch.no_grad():
        for b0 in range(0, B, 2):
            q4, k4, v4 = (t[b0 * S:(b0 + 2) * S].view(2, S, H, D) for t in (q, k, v))
            ref, _ = attention_ref(q4, k4, v4)
            pt, _ = attention_ref(q4, k4, v4, upcast=False, reorder_ops=True)
            worst[0] = max(worst[0], (out[b0 * S:(b0 + 2) * S].view(2, S, H, D).float() - ref.float()).abs().max().item())
            worst[1] = max(worst[1], max_err_bound(pt, ref))
    assert worst[0] <= worst[1], f"max err {worst[0]} > {worst[1]}"
    _check_lse(q, k, v, cu, cu, B, S, S, H, D, causal=False, chunk=2)
