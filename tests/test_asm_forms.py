"""GPU parity of each hand-scheduled assembly forward form, forced through FaFwdArgs.impl
(include/fa_hip.h): FA_IMPL_ASM4 (one wave per SIMD, two 32-row blocks per wave, one workgroup per
block) and FA_IMPL_ASM4P (the same body in the persistent form), against the fp32 oracle under the
reference's 2x rule (/root/reference/tests/test_flash_attn.py:407-409) and the LSE tolerance of
tests/test_flash_attn.py, so both forms stay green whichever one FA_IMPL_AUTO picks."""
import pytest
import torch

from fa_testutil import make_inputs
from oracle.attention_ref import attention_ref, max_err_bound, ulp_floor
from test_flash_attn import run_case

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _hip():
    from flash_attn import flash_attn_hip as hip
    return hip


@pytest.mark.parametrize("form", ["ASM4", "ASM4P"])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("seqlen_q,seqlen_k", [(97, 97), (257, 513), (512, 512), (1025, 300), (2048, 2048)])
def test_asm_form_forward(form, dtype, causal, seqlen_q, seqlen_k):
    hip = _hip()
    with hip.force_impl(getattr(hip, f"FA_IMPL_{form}")):
        run_case("separate", 3, seqlen_q, seqlen_k, 4, 64, dtype, causal, 0.0, grad=False, seed=seqlen_q)


@pytest.mark.parametrize("form", ["ASM4", "ASM4P"])
def test_asm_form_forced_rescale(form):
    """A spike key that row 7 meets only in a later tile: the out-of-line rescale block."""
    from flash_attn import flash_attn_interface as fi
    hip = _hip()
    B, H, S, d = 2, 2, 512, 64
    x = make_inputs(B, S, S, H, d, torch.bfloat16, DEV, mode_q="full", mode_k="full", seed=5)
    q, k = x["q_unpad"].clone(), x["k_unpad"].clone()
    k[300] = q[7] * 3.0
    k[450] = q[7] * 4.0
    with hip.force_impl(getattr(hip, f"FA_IMPL_{form}")):
        out = fi.flash_attn_unpadded_func(q, k, x["v_unpad"], x["cu_q"], x["cu_k"], S, S, 0.0)
    ref, _ = attention_ref(q.view(B, S, H, d), k.view(B, S, H, d), x["v_unpad"].view(B, S, H, d))
    pt, _ = attention_ref(q.view(B, S, H, d), k.view(B, S, H, d), x["v_unpad"].view(B, S, H, d),
                          upcast=False, reorder_ops=True)
    err = (out.view(B, S, H, d).float() - ref.float()).abs().max().item()
    assert err <= max_err_bound(pt, ref)


def test_asm_forms_agree_at_north_star_grid():
    """B=8 H=12 S=2048 D=64 bf16 (the bench workload, 768 blocks: three per CU in the persistent
    form): the two forms compute the same fp32-exact scores and sums in the same order, so their
    outputs are bitwise equal, and every form matches fp32."""
    from flash_attn import flash_attn_interface as fi
    hip = _hip()
    B, H, S, d = 8, 12, 2048, 64
    g = torch.Generator(device="cpu").manual_seed(0)
    q, k, v = (torch.randn(B * S, H, d, generator=g).bfloat16().to(DEV) for _ in range(3))
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=DEV)
    outs = {}
    for form in ("ASM4", "ASM4P"):
        with hip.force_impl(getattr(hip, f"FA_IMPL_{form}")):
            outs[form] = fi.flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0, return_attn_probs=False)
    assert torch.equal(outs["ASM4"], outs["ASM4P"])
    # against fp32 on two heads of the first sequence
    qf, kf, vf = (x[:S, :2].float().transpose(0, 1) for x in (q, k, v))
    ref = torch.matmul(torch.softmax(torch.matmul(qf, kf.transpose(1, 2)) * d ** -0.5, -1), vf).transpose(0, 1)
    for form, o in outs.items():
        assert (o[:S, :2].float() - ref).abs().max().item() <= 1e-2, form


@pytest.mark.parametrize("form", ["ASM4", "ASM4P"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("seqlen_k", [1, 2, 17, 300])
@pytest.mark.parametrize("amp", [1.0, 2.5])
def test_asm_short_key_sets_exact_lse(form, seqlen_k, amp, dtype):
    """Short key sets (one key: the LSE is that one score) and amplified inputs, one-block and
    persistent: fp32-exact scores keep the output under the 2x rule and the LSE within
    tests/test_flash_attn.py's tolerance (2e-3 + 1e-3 |lse|) on every row. (Round 4's pre-scaled
    persistent form needed an extra 2^-9 softmax_scale sum_d |q_d k_d| here)"""
    from flash_attn import flash_attn_interface as fi
    hip = _hip()
    B, H, Sq, d = 3, 4, 300, 64
    g = torch.Generator().manual_seed(seqlen_k)
    q, k, v = ((torch.randn(B * n, H, d, generator=g) * s).to(dtype).to(DEV)
               for n, s in ((Sq, amp), (seqlen_k, amp), (seqlen_k, 1.0)))
    cu_q = torch.arange(0, (B + 1) * Sq, Sq, dtype=torch.int32, device=DEV)
    cu_k = torch.arange(0, (B + 1) * seqlen_k, seqlen_k, dtype=torch.int32, device=DEV)
    tag = "bf16" if dtype == torch.bfloat16 else "f16"
    code = getattr(hip, f"FA_IMPL_{form}")
    assert hip.fwd_kernel_name(B, H, d, Sq, seqlen_k, dtype, impl=code) == \
        f"fa_fwd_d64{'p' if form == 'ASM4P' else ''}_{tag}_asm"
    with hip.force_impl(code):
        out, lse, _ = fi.flash_attn_unpadded_func(q, k, v, cu_q, cu_k, Sq, seqlen_k, 0.0, return_attn_probs=True)
    qb, kb, vb = (x.view(B, -1, H, d) for x in (q, k, v))
    ref, _ = attention_ref(qb, kb, vb)
    pt, _ = attention_ref(qb, kb, vb, upcast=False, reorder_ops=True)
    err = (out.view(B, Sq, H, d).float() - ref.float()).abs().max().item()
    assert err <= max_err_bound(pt, ref, floor=ulp_floor(ref, dtype)), err
    s = torch.einsum("bthd,bshd->bhts", qb.float(), kb.float()) * d ** -0.5
    lse_ref = torch.logsumexp(s, -1)
    torch.testing.assert_close(lse[:, :, :Sq], lse_ref, atol=2e-3, rtol=1e-3)


def test_asm_persistent_var_len_many_blocks():
    """Persistent form over more blocks than CUs with ragged sequences (tails into blocks of other
    lengths, empty q-blocks, key counts with and without the K/V tail) against the oracle."""
    hip = _hip()
    with hip.force_impl(hip.FA_IMPL_ASM4P):
        run_case("separate", 40, 600, 1100, 8, 64, torch.bfloat16, False, 0.0, grad=False, seed=11)


@pytest.mark.parametrize("form", ["ASM4", "ASM4P"])
@pytest.mark.parametrize("seqlen_q,seqlen_k", [(257, 513), (1025, 1100), (2048, 2048)])
def test_asm_form_forward_d128(form, seqlen_q, seqlen_k):
    """The head_dim = 128 tile in its one-block and persistent forms (grids of 72-384 blocks)."""
    hip = _hip()
    with hip.force_impl(getattr(hip, f"FA_IMPL_{form}")):
        run_case("separate", 6, seqlen_q, seqlen_k, 8, 128, torch.bfloat16, False, 0.0, grad=False, seed=seqlen_k)


@pytest.mark.parametrize("form", ["ASM4", "ASM4P"])
@pytest.mark.parametrize("d", [80, 96])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("seqlen_q,seqlen_k", [(257, 513), (1025, 1100)])
def test_asm_form_forward_d96(form, d, causal, seqlen_q, seqlen_k):
    """The D = 96 tile (D = 128 layout computing 96 columns) at head_dim 96 and 80 (Q's k-step 5
    loaded as zeros, O columns 80..95 never stored), one-block and persistent."""
    hip = _hip()
    assert hip.fwd_kernel_name(6, 8, d, seqlen_q, seqlen_k, torch.bfloat16,
                               impl=getattr(hip, f"FA_IMPL_{form}")).startswith("fa_fwd_d96")
    with hip.force_impl(getattr(hip, f"FA_IMPL_{form}")):
        run_case("separate", 6, seqlen_q, seqlen_k, 8, d, torch.bfloat16, causal, 0.0, grad=False, seed=seqlen_k + d)


@pytest.mark.parametrize("form", ["ASM4", "ASM4P"])
@pytest.mark.parametrize("d", [8, 16, 24, 32])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("seqlen_q,seqlen_k", [(97, 97), (257, 513), (1025, 1100)])
def test_asm_form_forward_d32(form, d, dtype, causal, seqlen_q, seqlen_k):
    """The D = 32 tile (round 6: head_dim <= 32, zero-padded; one O d-block, 4-KiB K / V tiles, two
    16-deep QK k-steps), one-block and persistent, against the fp32 oracle under the 2x rule."""
    hip = _hip()
    code = getattr(hip, f"FA_IMPL_{form}")
    name = hip.fwd_kernel_name(6, 8, d, seqlen_q, seqlen_k, dtype, causal, impl=code)
    assert name.startswith("fa_fwd_d32"), name
    with hip.force_impl(code):
        run_case("separate", 6, seqlen_q, seqlen_k, 8, d, dtype, causal, 0.0, grad=False, seed=seqlen_k + d)


def test_d32_asm_and_hip_agree_at_the_d32_roofline_shape():
    """B=8 H=12 S=2048 D=32 (the per-tile roofline shape): AUTO takes the assembly D = 32 tile
    (persistent: 768 blocks), and its output is within one bf16 ulp-scale of the HIP forward's."""
    from flash_attn import flash_attn_interface as fi
    hip = _hip()
    B, H, S, d = 8, 12, 2048, 32
    assert hip.fwd_kernel_name(B, H, d, S, S, torch.bfloat16) == "fa_fwd_d32p_bf16_asm"
    g = torch.Generator(device="cpu").manual_seed(1)
    q, k, v = (torch.randn(B * S, H, d, generator=g).bfloat16().to(DEV) for _ in range(3))
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=DEV)
    out = fi.flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0)
    with hip.force_impl(hip.FA_IMPL_HIP):
        ref = fi.flash_attn_unpadded_func(q, k, v, cu, cu, S, S, 0.0)
    assert (out.float() - ref.float()).abs().max().item() <= 1e-2


@pytest.mark.parametrize("d", [64, 128])
def test_asm_persistent_empty_key_set_after_tail(d):
    """the persistent form's .Lempty path right after a block that took the K/V tail
    (key counts that are multiples of 4 tiles alternate with empty key sets), with more blocks than
    CUs: empty rows give out == 0 and lse == -inf, every other row matches the oracle."""
    import numpy as np
    from flash_attn import flash_attn_interface as fi
    from oracle.attention_ref import ulp_floor
    hip = _hip()
    B, H = 48, 8
    lens_q = [300] * B
    lens_k = [1024 if b % 2 == 0 else 0 for b in range(B)]
    cu_q = torch.tensor([0] + list(np.cumsum(lens_q)), dtype=torch.int32, device=DEV)
    cu_k = torch.tensor([0] + list(np.cumsum(lens_k)), dtype=torch.int32, device=DEV)
    g = torch.Generator().manual_seed(d)
    q = torch.randn(sum(lens_q), H, d, generator=g).bfloat16().to(DEV)
    k = torch.randn(sum(lens_k), H, d, generator=g).bfloat16().to(DEV)
    v = torch.randn(sum(lens_k), H, d, generator=g).bfloat16().to(DEV)
    with hip.force_impl(hip.FA_IMPL_ASM4P):
        out, lse, _ = fi.flash_attn_unpadded_func(q, k, v, cu_q, cu_k, max(lens_q), max(lens_k), 0.0,
                                                  return_attn_probs=True)
    torch.cuda.synchronize()
    for b in range(B):
        qs, ks = slice(int(cu_q[b]), int(cu_q[b + 1])), slice(int(cu_k[b]), int(cu_k[b + 1]))
        if lens_k[b] == 0:
            assert (out[qs] == 0).all(), b
            assert torch.isinf(lse[b, :, :lens_q[b]]).all() and (lse[b, :, :lens_q[b]] < 0).all(), b
            continue
        if b % 8:     # the oracle on a sample of the non-empty sequences
            continue
        ref, _ = attention_ref(q[qs][None], k[ks][None], v[ks][None])
        pt, _ = attention_ref(q[qs][None], k[ks][None], v[ks][None], upcast=False, reorder_ops=True)
        err = (out[qs].float() - ref[0].float()).abs().max().item()
        assert err <= max_err_bound(pt, ref, floor=ulp_floor(ref)), (b, err)


@pytest.mark.parametrize("form", ["ASM4", "ASM4P"])
@pytest.mark.parametrize("d", [32, 64])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("spike", [False, True])
def test_asm_forward_probabilities_through_one_hot_v(form, d, causal, spike):
    """the assembly forward's own P, observed directly. With V's rows one-hot
    (key k of chunk j -> column k - d j, zero rows outside the chunk), O = P V / l is the normalised
    probability of every key of chunk j, computed by the kernel's exps, its rounded P and its MFMA row
    sums; compared with softmax(scale Q K^T) in fp32 over every chunk, within the rounding of P to
    bf16 and of O to bf16 (2^-7 relative + 1e-3). spike: a key that passes the running max in a later
    tile (the out-of-line rescale path)."""
    from flash_attn import flash_attn_interface as fi
    hip = _hip()
    B, H, Sq, Sk = 2, 2, 300, 200
    g = torch.Generator(device="cpu").manual_seed(d + 7 * causal + 3 * spike)
    q = torch.randn(B * Sq, H, d, generator=g).bfloat16()
    k = torch.randn(B * Sk, H, d, generator=g).bfloat16()
    if spike:
        k[150] = (q[7].float() * 3.0).bfloat16()        # sequence 0, tile 2, strong for query 7
    q, k = q.to(DEV), k.to(DEV)
    cu_q = torch.arange(0, (B + 1) * Sq, Sq, dtype=torch.int32, device=DEV)
    cu_k = torch.arange(0, (B + 1) * Sk, Sk, dtype=torch.int32, device=DEV)
    code = getattr(hip, f"FA_IMPL_{form}")
    assert hip.fwd_kernel_name(B, H, d, Sq, Sk, torch.bfloat16, causal, impl=code).endswith("_asm")
    qf, kf = q.float().view(B, Sq, H, d), k.float().view(B, Sk, H, d)
    s = torch.einsum("bqhd,bkhd->bhqk", qf, kf) * d ** -0.5
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(Sq, Sk, dtype=torch.bool, device=DEV), 1), float("-inf"))
    p_ref = torch.softmax(s, -1)                                   # (B, H, Sq, Sk)
    for j in range((Sk + d - 1) // d):
        keys = torch.arange(Sk, device=DEV)
        v = torch.zeros(B, Sk, H, d, device=DEV)
        inc = (keys >= j * d) & (keys < (j + 1) * d)
        v[:, inc, :, :] = torch.eye(d, device=DEV)[keys[inc] - j * d][None, :, None, :]
        v = v.bfloat16().view(B * Sk, H, d)
        with hip.force_impl(code):
            out = fi.flash_attn_unpadded_func(q, k, v, cu_q, cu_k, Sq, Sk, 0.0, causal=causal)
        got = out.float().view(B, Sq, H, d).permute(0, 2, 1, 3)[..., :int(inc.sum())]
        want = p_ref[..., j * d:j * d + int(inc.sum())]
        bad = (got - want).abs() > 2 ** -7 * want.abs() + 1e-3
        assert not bad.any(), (j, (got - want).abs().max().item())
