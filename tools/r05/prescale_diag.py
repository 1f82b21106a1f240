"""Diagnostic (round 5): LSE and gradient errors of the pre-scaled persistent forward (AUTO) against the
fp32-exact one-block form (FA_IMPL_ASM4) on the ragged short/long-key batch of
tests/test_prescale_dispatch.py, per softmax scale and dtype; errors in units of the 2x-rule bound."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "..", "hazyresearch_flash-attention_amd")]
import torch
from test_auto_dispatch_numerics import _batch, LENS_Q, LENS_K
from oracle.attention_ref import attention_ref, max_err_bound, pad
from flash_attn import flash_attn_interface as fi, flash_attn_hip as hip

H, d = 4, 64
B, Sq, Sk = len(LENS_Q), max(LENS_Q), max(LENS_K)
for dtype in (torch.bfloat16, torch.float16):
    for mul in (1.0, 8.0, 0.125):
        q, k, v, qm, km, iq, ik, cq, ck = _batch(LENS_Q, LENS_K, H, d, dtype, seed=int(mul * 8))
        qs = (q.float() * mul).to(dtype).requires_grad_()
        kr, vr = k.clone().requires_grad_(), v.clone().requires_grad_()
        ref, _ = attention_ref(qs, kr, vr, qm, km)
        pt, _ = attention_ref(qs, kr, vr, qm, km, upcast=False, reorder_ops=True)
        gout = torch.randn(int(cq[-1]), H, d, generator=torch.Generator().manual_seed(7)).to(dtype).cuda()
        gp = pad(gout, iq, B, Sq)
        dref = torch.autograd.grad(ref, (qs, kr, vr), gp, retain_graph=True)
        dpt = torch.autograd.grad(pt, (qs, kr, vr), gp)
        s = torch.einsum("bthd,bshd->bhts", q.float(), k.float()) * d ** -0.5 * mul
        s = s.masked_fill(~km[:, None, None, :], float("-inf"))
        lref = torch.logsumexp(s, -1)
        valid = qm[:, None, :].expand_as(lref)
        for impl in (hip.FA_IMPL_AUTO, hip.FA_IMPL_ASM4):
            qu = q.reshape(-1, H, d)[iq].clone().requires_grad_()
            ku = k.reshape(-1, H, d)[ik].clone().requires_grad_()
            vu = v.reshape(-1, H, d)[ik].clone().requires_grad_()
            with hip.force_impl(impl):
                o, lse, _ = fi.flash_attn_unpadded_func(qu, ku, vu, cq, ck, Sq, Sk, 0.0, softmax_scale=d ** -0.5 * mul,
                                                        return_attn_probs=True)
            g = torch.autograd.grad(o, (qu, ku, vu), gout)
            r = {"out": (pad(o, iq, B, Sq).float() - ref.float()).abs().max().item() / max_err_bound(pt, ref)}
            got = (pad(g[0], iq, B, Sq).float() / mul, pad(g[1], ik, B, Sk), pad(g[2], ik, B, Sk))
            for n, a, rr, p in zip(("dq", "dk", "dv"), got, dref, dpt):
                r[n] = (a.float() - rr.float()).abs().max().item() / max_err_bound(p, rr)
            dl = (lse[:, :, :Sq] - lref).abs()
            tol = 2e-3 + 1e-3 * lref.abs()
            r["lse_over_tol_max"] = (dl / tol)[valid].max().item()
            r["lse_fail_frac"] = (dl > tol)[valid].float().mean().item()
            per_b = [round((dl / tol)[b][valid[b]].max().item(), 2) for b in range(B)]
            print(dtype, "scale*", mul, "impl", impl, {k_: round(v_, 3) for k_, v_ in r.items()}, "lse/tol by seq", per_b, flush=True)
