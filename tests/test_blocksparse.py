"""Block-sparse attention: flash_blocksparse_attn_func / fa_fwd_block / fa_bwd_block.

CPU: the product's convert_blockmask and its inverse against golden vectors made by the
reference's own convert_blockmask, and oracle/attention_ref.attention_blocksparse_ref against
the reference's attention_blocksparse_ref (tests/golden/make_golden_blocksparse.py).
GPU: the HIP path against that oracle with the 2x rule of tests/test_flash_attn.py:407-409 on
outputs, probabilities and gradients; layouts with empty rows/columns, causal, dropout, padding.
"""
import os

import numpy as np
import pytest
import torch

from fa_testutil import convert_s_dmask
from oracle.attention_ref import (attention_blocksparse_ref, attention_ref, generate_random_padding_mask, max_err_bound,
                                  pad, unpad)
from oracle.philox import dropout_keep_mask

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "blocksparse_golden.npz")


def _bsi():
    from flash_attn import flash_blocksparse_attn_interface as bsi
    return bsi


# ---------------------------------------------------------------------------------- CPU
def test_convert_blockmask_golden():
    bsi = _bsi()
    from flash_attn.flash_attn_hip import decode_blockmask
    z = np.load(GOLDEN)
    n = 0
    for key in z.files:
        if key.endswith("/layout") and key.startswith("mask"):
            name = key.split("/")[0]
            layout = torch.from_numpy(z[key])
            conv = bsi.convert_blockmask(layout, causal=False)
            assert np.array_equal(conv.numpy(), z[f"{name}/converted"]), name
            assert torch.equal(decode_blockmask(conv), layout.to(torch.uint8)), name
            n += 1
    assert n >= 5


@pytest.mark.parametrize("name", ["fp16_s512", "bf16_s300_pad", "fp16_s512_dropout"])
def test_blocksparse_oracle_golden(name):
    z = np.load(GOLDEN)
    B, S, H, D, seed, offset = (int(x) for x in z[f"{name}/meta"])
    p = float(z[f"{name}/fparams"][0])
    dtype = getattr(torch, str(z[f"{name}/dtype"]))
    qkv = torch.from_numpy(z[f"{name}/qkv"]).to(dtype)
    layout = torch.from_numpy(z[f"{name}/layout"])
    attn_mask = torch.from_numpy(z[f"{name}/attn_mask"])
    keep = (torch.from_numpy(dropout_keep_mask(seed, offset, p, B, H, S, S)) if p > 0
            else torch.ones(B, H, S, S, dtype=torch.bool))
    q32 = qkv.float().requires_grad_()
    o32, _ = attention_blocksparse_ref(q32, layout, attn_mask, p, keep)
    (dqkv,) = torch.autograd.grad(o32, (q32,), torch.from_numpy(z[f"{name}/go"]))
    assert torch.allclose(o32.detach(), torch.from_numpy(z[f"{name}/out32"]), atol=1e-5, rtol=1e-5)
    assert torch.allclose(dqkv, torch.from_numpy(z[f"{name}/dqkv32"]), atol=1e-4, rtol=1e-4)
    o_lp, _ = attention_blocksparse_ref(qkv, layout, attn_mask, p, keep, upcast=False)
    ref_lp = torch.from_numpy(z[f"{name}/out_lp"])
    assert (o_lp.float() - ref_lp).abs().max().item() <= 2 * (ref_lp - torch.from_numpy(z[f"{name}/out32"])).abs().max().item() + 1e-3
    # rows of a dead 16-row block attend nothing -> output 0
    assert o32[:, 48:64].abs().max().item() == 0.0


# ---------------------------------------------------------------------------------- GPU
DEV = "cuda"


def _layout(S, density, seed, empty_row=True, empty_col=False):
    g = torch.Generator().manual_seed(seed)
    nr, nc = (S + 15) // 16, (S + 255) // 256
    m = torch.rand(nr, nc, generator=g) < density
    if empty_row and nr > 3:
        m[3] = False
    if empty_col and nc > 1:
        m[:, 0] = False
    return m


def run_bs_case(B, S, H, D, dtype, causal, p, density, seed=0, padded=True, convert_mask=True, grad=True):
    bsi = _bsi()
    g = torch.Generator().manual_seed(seed)
    qkv = torch.randn(B, S, 3, H, D, generator=g).to(dtype).to(DEV)
    mask = (generate_random_padding_mask(S, B, "cpu", "random", generator=g) if padded
            else torch.ones(B, S, dtype=torch.bool)).to(DEV)
    layout = _layout(S, density, seed, empty_col=seed % 2 == 1)
    qkv_u, idx, cu, max_s = unpad(qkv, mask)
    qkv_u = qkv_u.detach().requires_grad_()
    bm = layout if convert_mask else bsi.convert_blockmask(layout, causal=False)
    out_u, S_dmask, lse = bsi.flash_blocksparse_attn_func(qkv_u, cu, bm.to(DEV), p, max_s, causal=causal,
                                                          return_attn_probs=True, convert_mask=convert_mask)
    out = pad(out_u, idx, B, S)
    S_conv = convert_s_dmask(S_dmask, S, S, mask, mask, causal)
    keep = S_conv >= 0   # the kernel's own dropout mask (sign of S_dmask), as in test_flash_attn.run_case
    q = qkv.detach().float().requires_grad_()
    out_ref, attn_ref = attention_blocksparse_ref(q, layout, mask, p, keep, causal=causal)
    q_lp = qkv.detach().requires_grad_()
    out_pt, attn_pt = attention_blocksparse_ref(q_lp, layout, mask, p, keep, causal=causal, upcast=False,
                                                reorder_ops=True)
    err = (out.float() - out_ref.float()).abs().max().item()
    bound = max_err_bound(out_pt, out_ref, floor=1e-3)
    assert err <= bound, f"output max err {err} > {bound}"
    attn = S_conv.abs()
    aerr = (attn.float() - attn_ref.float()).abs().max().item()
    assert aerr <= max_err_bound(attn_pt, attn_ref, floor=1e-3), f"attention err {aerr}"
    # dead blocks: zero probability everywhere they apply
    live = layout.to(DEV).repeat_interleave(16, 0).repeat_interleave(256, 1)[:S, :S]
    assert attn[:, :, ~live].abs().max().item() == 0.0
    if grad:
        go = torch.randn(out_u.shape, generator=torch.Generator().manual_seed(seed + 1)).to(dtype).to(DEV)
        (dqkv_u,) = torch.autograd.grad(out_u, (qkv_u,), go)
        gpad = pad(go, idx, B, S)
        (d_ref,) = torch.autograd.grad(out_ref, (q,), gpad.float())
        (d_pt,) = torch.autograd.grad(out_pt, (q_lp,), gpad)
        dqkv = pad(dqkv_u, idx, B, S)
        for i, name in enumerate(("dq", "dk", "dv")):
            e = (dqkv[:, :, i].float() - d_ref[:, :, i]).abs().max().item()
            bnd = max_err_bound(d_pt[:, :, i], d_ref[:, :, i], floor=1e-3)
            assert e <= bnd, f"{name} max err {e} > {bnd}"
    return out_u, lse


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D", [32, 64, 128])
@pytest.mark.parametrize("S", [256, 513, 1024])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_blocksparse_parity(S, D, p, causal, dtype):
    run_bs_case(4, S, 2, D, dtype, causal, p, density=0.5, seed=S + D)


@pytest.mark.gpu
@pytest.mark.parametrize("density", [0.0, 0.2, 1.0])
def test_blocksparse_density_extremes(density):
    # 0.0: every row attends nothing (output 0, lse -inf); 1.0: equals dense attention
    out_u, lse = run_bs_case(2, 600, 2, 64, torch.bfloat16, False, 0.0, density, seed=5, padded=False)
    if density == 0.0:
        assert out_u.abs().max().item() == 0.0
        assert torch.isinf(lse[:, :, :600]).all()


@pytest.mark.gpu
def test_blocksparse_converted_mask_same_result():
    a, _ = run_bs_case(2, 1024, 2, 64, torch.float16, False, 0.0, 0.5, seed=7, grad=False)
    b, _ = run_bs_case(2, 1024, 2, 64, torch.float16, False, 0.0, 0.5, seed=7, grad=False, convert_mask=False)
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_blocksparse_long_sequence():
    # 16 column blocks, skipped tiles in both kernels' walks
    run_bs_case(1, 4096, 2, 64, torch.bfloat16, False, 0.0, 0.25, seed=11, padded=False)


@pytest.mark.gpu
def test_blocksparse_full_layout_matches_dense():
    bsi = _bsi()
    from flash_attn.flash_attn_interface import flash_attn_unpadded_qkvpacked_func
    g = torch.Generator().manual_seed(3)
    # H=24: 144 eight-wave workgroups, so the dense forward takes its plain 8-wave kernel (the same
    # loop body as the block-sparse one; smaller grids take the split-K kernel, whose merge rounds
    # differently)
    B, S, H, D = 2, 768, 24, 64
    qkv = torch.randn(B * S, 3, H, D, generator=g).to(torch.float16).to(DEV)
    cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=DEV)
    layout = torch.ones((S + 15) // 16, (S + 255) // 256, dtype=torch.bool, device=DEV)
    o_bs = bsi.flash_blocksparse_attn_func(qkv, cu, layout, 0.0, S)
    # bitwise against the HIP dense kernel (impl=FA_IMPL_HIP); the default dense path for this shape
    # is the assembly forward, which sums rows in another order: within the 2x rule of the oracle
    from flash_attn import flash_attn_hip as hip
    o_d = hip.fwd(qkv[:, 0], qkv[:, 1], qkv[:, 2], cu, cu, S, S, 0.0, D ** -0.5, False, False, False, None,
                  impl=hip.FA_IMPL_HIP)[0]
    assert torch.equal(o_bs, o_d)
    o_auto = flash_attn_unpadded_qkvpacked_func(qkv, cu, S, 0.0)
    q4, k4, v4 = (qkv[:, i].view(B, S, H, D) for i in range(3))
    ref, _ = attention_ref(q4, k4, v4)
    pt, _ = attention_ref(q4, k4, v4, upcast=False, reorder_ops=True)
    assert (o_auto.view(B, S, H, D).float() - ref.float()).abs().max().item() <= max_err_bound(pt, ref)


@pytest.mark.gpu
def test_blocksparse_module():
    from flash_attn.flash_blocksparse_attention import FlashBlocksparseAttention, FlashBlocksparseMHA
    S = 512
    layout = _layout(2048, 0.5, 1)
    attn = FlashBlocksparseAttention(layout, max_seq_length=2048).to(DEV)
    qkv = torch.randn(2, S, 3, 2, 32, device=DEV, dtype=torch.float16)
    out, _ = attn(qkv)
    ref, _ = attention_blocksparse_ref(qkv.float(), layout[:S // 16, :S // 256], None, 0.0, None)
    pt, _ = attention_blocksparse_ref(qkv, layout[:S // 16, :S // 256], None, 0.0, None, upcast=False,
                                      reorder_ops=True)
    assert (out.float() - ref).abs().max().item() <= max_err_bound(pt, ref, floor=1e-3)
    mha = FlashBlocksparseMHA(64, 2, layout, max_seq_length=2048, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(2, S, 64, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y, _ = mha(x, None, None)
    y.sum().backward()
    assert torch.isfinite(x.grad).all()


@pytest.mark.gpu
def test_blocksparse_invalid_layouts():
    bsi = _bsi()
    qkv = torch.randn(2 * 512, 3, 2, 64, device=DEV, dtype=torch.float16)
    cu = torch.tensor([0, 512, 1024], dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError, match="does not cover"):
        bsi.flash_blocksparse_attn_func(qkv, cu, torch.ones(16, 1, dtype=torch.bool), 0.0, 512)
    big = torch.randn(20000, 3, 1, 64, device=DEV, dtype=torch.float16)
    cu2 = torch.tensor([0, 20000], dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError, match="columns"):
        bsi.flash_blocksparse_attn_func(big, cu2, torch.ones(1250, 79, dtype=torch.bool), 0.0, 20000)
