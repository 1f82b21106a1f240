"""Var-len packing helpers with the reference's API (flash_attn/bert_padding.py:11-134).

unpad_input turns (batch, seqlen, ...) + a key-padding mask into the "unpadded" (total, ...)
layout with int32 cu_seqlens; pad_input scatters it back. index_first_axis /
index_put_first_axis / index_first_axis_residual are gather/scatter autograd functions on the
first axis.

On GPU tensors the row moves run in HIP (libfa_hip.so: fa_index_first_axis,
fa_index_put_first_axis, fa_index_add_first_axis; csrc/fa_padding.hip), which raise if the
library is missing. index_first_axis and index_put_first_axis go through the compiled binding
(_fa_C: checks, allocation, launch and the autograd node in C++; the ctypes path below cost about
twice the kernel's time per call on the host) when it is loaded; the autograd functions below
are the same operations over ctypes. Host tensors use torch indexing, as the reference does on any
device.
"""
import ctypes

import torch
import torch.nn.functional as F

_DTYPE = {torch.float16: 0, torch.bfloat16: 1, torch.float32: 2}


def _rows(x):
    """(x with contiguous rows, row stride in bytes, row bytes)."""
    inner = x.shape[1:]
    want = 1
    ok = True
    for size, st in zip(reversed(inner), reversed(x.stride()[1:])):
        if size != 1 and st != want:
            ok = False
            break
        want *= size
    row_elems = 1
    for size in inner:
        row_elems *= size
    # rows that overlap or are broadcast (stride(0) < row, e.g. an expand along dim 0) cannot be
    # addressed as row_stride-spaced rows: copy them out instead of clamping the stride
    if ok and x.shape[0] > 1 and x.stride(0) < row_elems:
        ok = False
    if not ok:
        x = x.contiguous()
    es = x.element_size()
    stride = x.stride(0) * es if x.shape[0] > 1 else row_elems * es
    return x, stride, row_elems * es


def _hip():
    from flash_attn import flash_attn_hip
    return flash_attn_hip


def _idx64(indices):
    return indices if indices.dtype == torch.int64 else indices.to(torch.int64)


def _gather(src, indices):
    """src[indices] along dim 0."""
    if not src.is_cuda:
        return src.index_select(0, indices)
    hip = _hip()
    src, sstride, row_bytes = _rows(src)
    indices = _idx64(indices).contiguous()
    if row_bytes % 2:      # odd-byte rows (1-byte dtypes): the C ABI moves 2-byte words
        return src.index_select(0, indices)
    out = torch.empty((indices.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    if out.numel() == 0:
        return out
    with hip._on_device(src.device):
        rc = hip.lib().fa_index_first_axis(ctypes.c_void_p(src.data_ptr()), src.shape[0], sstride,
                                           ctypes.c_void_p(indices.data_ptr()), indices.shape[0],
                                           ctypes.c_void_p(out.data_ptr()), row_bytes, row_bytes,
                                           ctypes.c_void_p(hip._stream_ptr(src.device)))
    if rc != 0:
        hip._raise(rc, "fa_index_first_axis")
    return out


def _pad(values, indices, first_axis_dim):
    """zeros(first_axis_dim, ...) with rows `indices` set to `values`."""
    if not values.is_cuda:
        out = values.new_zeros((first_axis_dim,) + tuple(values.shape[1:]))
        out.index_copy_(0, indices, values)
        return out
    hip = _hip()
    values, vstride, row_bytes = _rows(values)
    indices = _idx64(indices).contiguous()
    if row_bytes % 2:      # odd-byte rows (1-byte dtypes)
        out = values.new_zeros((first_axis_dim,) + tuple(values.shape[1:]))
        return out.index_copy_(0, indices, values)
    out = torch.empty((first_axis_dim,) + tuple(values.shape[1:]), dtype=values.dtype, device=values.device)
    if out.numel() == 0:
        return out
    ws = torch.empty(first_axis_dim, dtype=torch.int32, device=values.device)
    with hip._on_device(values.device):
        rc = hip.lib().fa_index_put_first_axis(ctypes.c_void_p(values.data_ptr()), vstride,
                                               ctypes.c_void_p(indices.data_ptr()), indices.shape[0],
                                               ctypes.c_void_p(out.data_ptr()), first_axis_dim, row_bytes,
                                               row_bytes, ctypes.c_void_p(ws.data_ptr()),
                                               ctypes.c_void_p(hip._stream_ptr(values.device)))
    if rc != 0:
        hip._raise(rc, "fa_index_put_first_axis")
    return out


def _index_add_(dst, indices, src):
    """dst[indices] += src (indices unique); dst has contiguous rows."""
    if not dst.is_cuda or src.dtype not in _DTYPE:
        dst.index_add_(0, indices, src)
        return dst
    hip = _hip()
    src, sstride, row_bytes = _rows(src.to(dst.dtype))
    dst_c, dstride, _ = _rows(dst)
    assert dst_c.data_ptr() == dst.data_ptr(), "destination rows must be contiguous"
    indices = _idx64(indices).contiguous()
    if src.numel() == 0:
        return dst
    with hip._on_device(dst.device):
        rc = hip.lib().fa_index_add_first_axis(ctypes.c_void_p(src.data_ptr()), sstride,
                                               ctypes.c_void_p(indices.data_ptr()), indices.shape[0],
                                               ctypes.c_void_p(dst.data_ptr()), dst.shape[0], dstride,
                                               row_bytes // src.element_size(), _DTYPE[src.dtype],
                                               ctypes.c_void_p(hip._stream_ptr(dst.device)))
    if rc != 0:
        hip._raise(rc, "fa_index_add_first_axis")
    return dst


class IndexFirstAxis(torch.autograd.Function):
    """out = input[indices] along dim 0; backward scatters into zeros (reference :11-38)."""

    @staticmethod
    def forward(ctx, input, indices):
        assert input.ndim >= 2
        ctx.save_for_backward(indices)
        ctx.first_axis_dim = input.shape[0]
        return _gather(input, indices)

    @staticmethod
    def backward(ctx, grad_output):
        indices, = ctx.saved_tensors
        return _pad(grad_output, indices, ctx.first_axis_dim), None


def _compiled():
    from flash_attn import flash_attn_hip
    return flash_attn_hip._C


def index_first_axis(input, indices):
    """input[indices] along dim 0 (IndexFirstAxis, reference :11-38); CUDA tensors through _fa_C."""
    C = _compiled()
    if C is not None and input.is_cuda:
        return C.index_first_axis(input, indices)
    return IndexFirstAxis.apply(input, indices)


class IndexPutFirstAxis(torch.autograd.Function):
    """out = zeros(first_axis_dim, ...); out[indices] = values; backward gathers (reference :41-64)."""

    @staticmethod
    def forward(ctx, values, indices, first_axis_dim):
        assert indices.ndim == 1 and values.ndim >= 2
        ctx.save_for_backward(indices)
        return _pad(values, indices, first_axis_dim)

    @staticmethod
    def backward(ctx, grad_output):
        indices, = ctx.saved_tensors
        return _gather(grad_output, indices), None, None


def index_put_first_axis(values, indices, first_axis_dim):
    """zeros(first_axis_dim, ...) with rows `indices` = values (IndexPutFirstAxis, reference :41-64);
    CUDA tensors through _fa_C."""
    C = _compiled()
    if C is not None and values.is_cuda:
        return C.index_put_first_axis(values, indices, first_axis_dim)
    return IndexPutFirstAxis.apply(values, indices, first_axis_dim)


class IndexFirstAxisResidual(torch.autograd.Function):
    """(input[indices], input) where the second output carries a residual gradient; backward adds
    grad_output into grad_residual at `indices` (reference :67-94)."""

    @staticmethod
    def forward(ctx, input, indices):
        ctx.save_for_backward(indices)
        assert input.ndim >= 2
        ctx.first_axis_dim, ctx.other_shape = input.shape[0], input.shape[1:]
        return _gather(input, indices), input.detach()

    @staticmethod
    def backward(ctx, grad_output, grad_residual):
        indices, = ctx.saved_tensors
        assert grad_output.ndim >= 2
        assert grad_residual.shape[1:] == grad_output.shape[1:]
        grad_input = grad_residual.contiguous()   # updated in place, as the reference's scatter_add_
        _index_add_(grad_input, indices, grad_output)
        return grad_input.reshape(ctx.first_axis_dim, *ctx.other_shape), None


index_first_axis_residual = IndexFirstAxisResidual.apply


def unpad_input(hidden_states, attention_mask):
    """hidden_states (batch, seqlen, ...), attention_mask (batch, seqlen) bool/int (1 = keep).
    Returns (hidden (total, ...), indices (total,), cu_seqlens (batch+1,) int32, max_seqlen int)."""
    seqlens = attention_mask.sum(dim=-1, dtype=torch.int32)
    indices = torch.nonzero(attention_mask.reshape(-1), as_tuple=False).reshape(-1)
    max_seqlen = int(seqlens.max().item())
    cu_seqlens = F.pad(torch.cumsum(seqlens, dim=0, dtype=torch.int32), (1, 0))
    flat = hidden_states.reshape((-1,) + tuple(hidden_states.shape[2:]))
    return index_first_axis(flat, indices), indices, cu_seqlens, max_seqlen


def pad_input(hidden_states, indices, batch, seqlen):
    """hidden_states (total, ...) -> (batch, seqlen, ...), zeros at padded positions."""
    out = index_put_first_axis(hidden_states, indices, batch * seqlen)
    return out.reshape((batch, seqlen) + tuple(hidden_states.shape[1:]))
