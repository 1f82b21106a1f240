"""Var-len packing helpers with the reference's API (flash_attn/bert_padding.py:11-134).

unpad_input turns (batch, seqlen, ...) + a key-padding mask into the "unpadded" (total, ...)
layout with int32 cu_seqlens; pad_input scatters it back. index_first_axis /
index_put_first_axis are gather/scatter autograd functions on the first axis.
"""
import torch
import torch.nn.functional as F


class IndexFirstAxis(torch.autograd.Function):
    """out = input[indices] along dim 0; backward scatters into zeros."""

    @staticmethod
    def forward(ctx, input, indices):
        assert input.ndim >= 2
        ctx.save_for_backward(indices)
        ctx.first_axis_dim = input.shape[0]
        return input.index_select(0, indices)

    @staticmethod
    def backward(ctx, grad_output):
        indices, = ctx.saved_tensors
        grad_input = grad_output.new_zeros((ctx.first_axis_dim,) + tuple(grad_output.shape[1:]))
        grad_input.index_copy_(0, indices, grad_output)
        return grad_input, None


index_first_axis = IndexFirstAxis.apply


class IndexPutFirstAxis(torch.autograd.Function):
    """out = zeros(first_axis_dim, ...); out[indices] = values; backward gathers."""

    @staticmethod
    def forward(ctx, values, indices, first_axis_dim):
        assert indices.ndim == 1 and values.ndim >= 2
        ctx.save_for_backward(indices)
        out = values.new_zeros((first_axis_dim,) + tuple(values.shape[1:]))
        out.index_copy_(0, indices, values)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        indices, = ctx.saved_tensors
        return grad_output.index_select(0, indices), None, None


index_put_first_axis = IndexPutFirstAxis.apply


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
