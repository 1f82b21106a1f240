"""GPU parity of the HIP var-len packing (csrc/fa_padding.hip) against torch
indexing, the reference's own algorithm (flash_attn/bert_padding.py:11-134): bit-exact, for
16-, 4- and 2-byte row paths, strided sources, empty inputs, and the autograd functions."""
import pytest
import torch

from oracle.attention_ref import generate_random_padding_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bp():
    from flash_attn import bert_padding
    return bert_padding


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(8, 300, 12, 64), (3, 97, 3, 5), (2, 64, 7), (1, 3, 8)])
@pytest.mark.parametrize("mode", ["random", "third", "full"])
def test_unpad_pad_roundtrip(shape, dtype, mode):
    bp = _bp()
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(*shape, generator=g).to(dtype).to(DEV)
    mask = generate_random_padding_mask(shape[1], shape[0], "cpu", mode, generator=g).to(DEV)
    xu, idx, cu, mx = bp.unpad_input(x, mask)
    flat = x.reshape(shape[0] * shape[1], *shape[2:])
    assert torch.equal(xu, flat.index_select(0, idx))
    assert cu.dtype == torch.int32 and cu[-1].item() == int(mask.sum())
    back = bp.pad_input(xu, idx, shape[0], shape[1])
    ref = torch.zeros_like(flat)
    ref.index_copy_(0, idx, xu)
    assert torch.equal(back, ref.reshape(x.shape))


def test_strided_source_rows():
    bp = _bp()
    base = torch.randn(500, 2, 48, device=DEV, dtype=torch.bfloat16)
    src = base[:, 1]                      # row stride 96 elements, rows of 48
    idx = torch.randperm(500, device=DEV)[:321]
    assert torch.equal(bp.index_first_axis(src, idx), src[idx])
    out = bp.index_put_first_axis(src[:321], idx, 500)
    ref = torch.zeros(500, 48, device=DEV, dtype=torch.bfloat16)
    ref[idx] = src[:321]
    assert torch.equal(out, ref)


def test_empty_and_all_padding():
    bp = _bp()
    x = torch.randn(4, 16, device=DEV)
    idx = torch.zeros(0, dtype=torch.int64, device=DEV)
    assert bp.index_first_axis(x, idx).shape == (0, 16)
    assert torch.equal(bp.index_put_first_axis(x[:0], idx, 4), torch.zeros(4, 16, device=DEV))


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_autograd_matches_torch(dtype):
    bp = _bp()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(6, 50, 4, 8, generator=g).to(dtype).to(DEV).requires_grad_()
    mask = generate_random_padding_mask(50, 6, "cpu", "random", generator=g).to(DEV)
    xu, idx, _, _ = bp.unpad_input(x, mask)
    go = torch.randn(xu.shape, generator=g).to(dtype).to(DEV)
    (gx,) = torch.autograd.grad(xu, (x,), go)
    ref = torch.zeros(300, 4, 8, dtype=dtype, device=DEV)
    ref[idx] = go
    assert torch.equal(gx, ref.reshape(x.shape))
    v = xu.detach().requires_grad_()
    out = bp.pad_input(v, idx, 6, 50)
    gp = torch.randn(out.shape, generator=g).to(dtype).to(DEV)
    (gv,) = torch.autograd.grad(out, (v,), gp)
    assert torch.equal(gv, gp.reshape(300, 4, 8)[idx])


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_index_first_axis_residual(dtype):
    bp = _bp()
    g = torch.Generator().manual_seed(2)
    x = torch.randn(200, 3, 16, generator=g).to(dtype).to(DEV).requires_grad_()
    idx = torch.randperm(200, generator=g)[:120].to(DEV)
    out, res = bp.index_first_axis_residual(x, idx)
    go = torch.randn(out.shape, generator=g).to(dtype).to(DEV)
    gr = torch.randn(res.shape, generator=g).to(dtype).to(DEV)
    ref = gr.clone()   # the backward adds into grad_residual in place, like the reference's scatter_add_
    ref.index_add_(0, idx, go)
    (gx,) = torch.autograd.grad((out, res), (x,), (go, gr))
    assert torch.equal(gx, ref)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_compiled_and_ctypes_routes_agree(dtype):
    """index_first_axis / index_put_first_axis take the compiled binding (_fa_C) on CUDA tensors; the
    ctypes autograd functions (IndexFirstAxis / IndexPutFirstAxis) are the same operations: bitwise
    equal outputs and gradients, strided sources included."""
    bp = _bp()
    from flash_attn import flash_attn_hip as hip
    if hip._C is None:
        pytest.skip("compiled binding not loaded (FA_HIP_LIB variant)")
    g = torch.Generator().manual_seed(7)
    base = torch.randn(400, 2, 6, 16, generator=g).to(dtype).to(DEV)
    src = base[:, 1]                                           # strided rows
    idx = torch.randperm(400, generator=g)[:257].to(DEV)
    assert torch.equal(bp.index_first_axis(src, idx), bp.IndexFirstAxis.apply(src, idx))
    vals = torch.randn(257, 6, 16, generator=g).to(dtype).to(DEV)
    assert torch.equal(bp.index_put_first_axis(vals, idx, 400), bp.IndexPutFirstAxis.apply(vals, idx, 400))
    x = src.detach().clone().requires_grad_()
    go = torch.randn(257, 6, 16, generator=g).to(dtype).to(DEV)
    (g_c,) = torch.autograd.grad(bp.index_first_axis(x, idx), (x,), go)
    (g_p,) = torch.autograd.grad(bp.IndexFirstAxis.apply(x, idx), (x,), go)
    assert torch.equal(g_c, g_p)
    v = vals.clone().requires_grad_()
    gp = torch.randn(400, 6, 16, generator=g).to(dtype).to(DEV)
    (gv_c,) = torch.autograd.grad(bp.index_put_first_axis(v, idx, 400), (v,), gp)
    (gv_p,) = torch.autograd.grad(bp.IndexPutFirstAxis.apply(v, idx, 400), (v,), gp)
    assert torch.equal(gv_c, gv_p)
    with pytest.raises(RuntimeError):
        bp.index_first_axis(src, idx.cpu())                    # indices on another device


def test_odd_byte_rows():
    """1-byte dtypes with an odd row size (the C ABI moves 2-byte words) keep the reference's torch
    indexing semantics on the device."""
    bp = _bp()
    x = torch.randint(0, 255, (50, 3), dtype=torch.uint8, device=DEV)
    idx = torch.randperm(50, device=DEV)[:17]
    assert torch.equal(bp.index_first_axis(x, idx), x[idx])
    ref = torch.zeros(50, 3, dtype=torch.uint8, device=DEV)
    ref[idx] = x[:17]
    assert torch.equal(bp.index_put_first_axis(x[:17], idx, 50), ref)
    assert torch.equal(bp.IndexFirstAxis.apply(x, idx), x[idx])
