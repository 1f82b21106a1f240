"""Parity of the assembly forward on the inputs where round 4's pre-scaled persistent form was weakest
(VERDICT r4 "Next round" 1): a ragged batch whose key lengths include 1, 2, 17, 64 and 300
next to sequences of >= 1024 keys, through AUTO dispatch (no force_impl; 240 blocks: the one-block
form on parts with at least 240 CUs, the persistent form below that) and the persistent form forced (FA_IMPL_ASM4P, the north star's kernel), separate and kv-packed
layouts, forward + backward. On this batch the pre-scaled scores (Q rounded after the multiply by
softmax_scale * log2(e)) broke the LSE tolerance and, at softmax_scale 1.0, the 2x rule on dV
(tools/r05/prescale_diag.py); every shipped form now computes fp32-exact scores. Checks, unchanged from the rest of
the suite: the reference's 2x rule (/root/reference/tests/test_flash_attn.py:407-409) on out, dq, dk,
dv against autograd of the fp32 oracle (the reference's attention_ref, :115-159), and the LSE within
2e-3 / 1e-3 of fp32 logsumexp. Non-default softmax_scale (1.0 and 1/d) is checked the same way: at
D = 64 both are exact power-of-two multiples of d^-0.5, so the oracle sees q rescaled exactly."""
import math

import pytest
import torch

from oracle.attention_ref import attention_ref, max_err_bound, pad

pytestmark = pytest.mark.gpu

DEV = "cuda"
LENS_K = [1, 2, 17, 64, 300, 1024, 1100, 5, 33, 129, 700, 3]
LENS_Q = [300, 64, 1, 128, 257, 1030, 1024, 200, 17, 5, 700, 1050]


def _batch(lens_q, lens_k, H, d, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    B, Sq, Sk = len(lens_q), max(lens_q), max(lens_k)
    q = torch.randn(B, Sq, H, d, generator=g).to(dtype).to(DEV)
    k = torch.randn(B, Sk, H, d, generator=g).to(dtype).to(DEV)
    v = torch.randn(B, Sk, H, d, generator=g).to(dtype).to(DEV)
    qmask = torch.arange(Sq, device=DEV)[None, :] < torch.tensor(lens_q, device=DEV)[:, None]
    kmask = torch.arange(Sk, device=DEV)[None, :] < torch.tensor(lens_k, device=DEV)[:, None]
    idx_q = torch.nonzero(qmask.reshape(-1)).reshape(-1)
    idx_k = torch.nonzero(kmask.reshape(-1)).reshape(-1)
    cu = lambda lens: torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    return q, k, v, qmask, kmask, idx_q, idx_k, cu(lens_q), cu(lens_k)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("layout", ["separate", "kvpacked"])
@pytest.mark.parametrize("scale_mul", [1.0, 8.0, 0.125])
@pytest.mark.parametrize("impl", ["AUTO", "ASM4P"])
def test_asm_forward_ragged_short_and_long_keys(impl, layout, dtype, scale_mul):
    """scale_mul multiplies the default d^-0.5 = 1/8: 8 gives softmax_scale 1.0, 1/8 gives 1/d."""
    _ragged_case(impl, layout, dtype, scale_mul, 64)


@pytest.mark.parametrize("d", [32, 96, 128])
@pytest.mark.parametrize("scale_mul", [4.0, 0.25])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_non_default_scale_other_head_dims(d, scale_mul, dtype):
    """a non-default softmax_scale at the other head-dim tiles (the assembly D = 32,
    96 and 128 tiles), the same ragged batch, forward and backward. scale_mul is a power of two, so the oracle sees q rescaled exactly."""
    _ragged_case("AUTO", "separate", dtype, scale_mul, d)


def _ragged_case(impl, layout, dtype, scale_mul, d):
    import contextlib
    from flash_attn import flash_attn_hip as hip
    from flash_attn import flash_attn_interface as fi
    H = 4
    B, Sq, Sk = len(LENS_Q), max(LENS_Q), max(LENS_K)
    q, k, v, qmask, kmask, idx_q, idx_k, cu_q, cu_k = _batch(LENS_Q, LENS_K, H, d, dtype, seed=int(scale_mul * 8))
    tag = "bf16" if dtype == torch.bfloat16 else "f16"
    code = getattr(hip, f"FA_IMPL_{impl}")
    # AUTO takes the persistent form when the grid has more blocks than the CUs (rounded down to whole
    # XCDs: fa_asm.cpp persist_grid); this batch's 240 blocks decide by the part's CU count
    nwg = (Sq + 255) // 256 * H * B
    ncu = torch.cuda.get_device_properties(DEV).multi_processor_count // 8 * 8
    persistent = impl == "ASM4P" or nwg > ncu
    want = f"fa_fwd_d{d}p_{tag}_asm" if persistent else f"fa_fwd_d{d}_{tag}_asm"
    assert hip.fwd_kernel_name(B, H, d, Sq, Sk, dtype, impl=code) == want
    ctx = hip.force_impl(code) if impl != "AUTO" else contextlib.nullcontext()
    scale = d ** -0.5 * scale_mul
    q_u = q.reshape(-1, H, d)[idx_q].detach().requires_grad_()
    k_u = k.reshape(-1, H, d)[idx_k]
    v_u = v.reshape(-1, H, d)[idx_k]
    if layout == "kvpacked":
        kv_u = torch.stack([k_u, v_u], dim=1).detach().requires_grad_()
        with ctx:
            out_u, lse, _ = fi.flash_attn_unpadded_kvpacked_func(q_u, kv_u, cu_q, cu_k, Sq, Sk, 0.0,
                                                                 softmax_scale=scale, return_attn_probs=True)
        inputs = (q_u, kv_u)
    else:
        k_u, v_u = k_u.detach().requires_grad_(), v_u.detach().requires_grad_()
        with ctx:
            out_u, lse, _ = fi.flash_attn_unpadded_func(q_u, k_u, v_u, cu_q, cu_k, Sq, Sk, 0.0, softmax_scale=scale,
                                                        return_attn_probs=True)
        inputs = (q_u, k_u, v_u)
    # the oracle scales by d^-0.5: q times scale_mul (a power of two) is exact in the input dtype
    qs = (q.float() * scale_mul).to(dtype).detach().requires_grad_()
    kr, vr = k.detach().requires_grad_(), v.detach().requires_grad_()
    ref, _ = attention_ref(qs, kr, vr, qmask, kmask)
    pt, _ = attention_ref(qs, kr, vr, qmask, kmask, upcast=False, reorder_ops=True)
    out = pad(out_u, idx_q, B, Sq)
    err = (out.float() - ref.float()).abs().max().item()
    assert err <= max_err_bound(pt, ref), f"out max err {err} > {max_err_bound(pt, ref)}"
    # LSE: the suite's tolerance (tests/test_flash_attn.py::run_case), on every valid row
    s = torch.einsum("bthd,bshd->bhts", q.float(), k.float()) * scale
    s = s.masked_fill(~kmask[:, None, None, :], float("-inf"))
    lse_ref = torch.logsumexp(s, -1)
    valid = qmask[:, None, :].expand_as(lse_ref)
    torch.testing.assert_close(lse[:, :, :Sq][valid], lse_ref[valid], atol=2e-3, rtol=1e-3)
    # backward: 2x rule on dq, dk, dv (dq of the oracle through the exact rescaling of q)
    gout = torch.randn(out_u.shape, generator=torch.Generator().manual_seed(7)).to(dtype).to(DEV)
    grads = torch.autograd.grad(out_u, inputs, gout)
    gpad = pad(gout, idx_q, B, Sq)
    dref = torch.autograd.grad(ref, (qs, kr, vr), gpad)
    dpt = torch.autograd.grad(pt, (qs, kr, vr), gpad)
    if layout == "kvpacked":
        dq_u, dk_u, dv_u = grads[0], grads[1][:, 0], grads[1][:, 1]
    else:
        dq_u, dk_u, dv_u = grads
    got = (pad(dq_u, idx_q, B, Sq).float() / scale_mul, pad(dk_u, idx_k, B, Sk), pad(dv_u, idx_k, B, Sk))
    for name, a, r, p in zip(("dq", "dk", "dv"), got, dref, dpt):
        e = (a.float() - r.float()).abs().max().item()
        bnd = max_err_bound(p, r)
        assert e <= bnd, f"{name} max err {e} > {bnd}"
