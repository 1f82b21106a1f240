"""Block-sparse attention interface, drop-in for the reference's
flash_attn/flash_blocksparse_attn_interface.py (same names, arguments and return values).

The reference declares `flash_attn_cuda.fwd_block` / `bwd_block` but never binds them; here
they are `fa_fwd_block` / `fa_bwd_block` of libfa_hip.so (include/fa_hip.h). The kernels take
the 0/1 layout directly (16-query x 256-key blocks, semantics of the reference's
tests/test_flash_attn.py:189-215), so `convert_mask=True` passes the layout straight through and
`convert_mask=False` decodes a pre-converted mask (convert_blockmask's format) back to it.
Differences from the reference: the dropout replay saves (seed, offset) instead of the whole
CUDA RNG state, and `causal=True` is supported (the causal mask is applied on top of the layout).
"""
import torch

from flash_attn import flash_attn_hip as _hip


def convert_blockmask(blockmask, causal):
    """0/1 (row, col) layout -> the reference's converted format
    (flash_attn/flash_blocksparse_attn_interface.py:8-40): for each column, the row indices of
    its nonzero blocks in increasing order, times 4, +1 on a row's first nonzero column, +2 on
    its last, padded with -1 to `row` entries; shape (col, row), int32."""
    assert not causal
    nrow, ncol = blockmask.shape
    live = blockmask.to(torch.bool)
    dev = blockmask.device
    rows = torch.arange(nrow, device=dev).unsqueeze(1)
    cols = torch.arange(ncol, device=dev).unsqueeze(0)
    first = torch.where(live, cols, ncol).amin(dim=1, keepdim=True)
    last = torch.where(live, cols, -1).amax(dim=1, keepdim=True)
    code = rows * 4 + (cols == first).long() + 2 * (cols == last).long()
    code = torch.where(live, code, torch.full_like(code, -1))
    # per column: live rows first, in increasing row order (stable sort on "is dead")
    order = torch.sort((~live).to(torch.uint8), dim=0, stable=True).indices
    return torch.gather(code, 0, order).T.contiguous().to(torch.int32)


def _layout(blockmask, convert_mask, device):
    blockmask = blockmask.to(device)
    return blockmask if convert_mask else _hip.decode_blockmask(blockmask)


def _flash_blocksparse_attn_forward(qkv, cu_seqlens, layout, dropout_p, max_s, softmax_scale, causal,
                                     return_softmax, rng_state=None):
    context, softmax_lse, *rest = _hip.fwd(qkv[:, 0], qkv[:, 1], qkv[:, 2], cu_seqlens, cu_seqlens, max_s, max_s,
                                           dropout_p, softmax_scale, False, causal, return_softmax, None,
                                           rng_state=rng_state, layout=layout)
    S_dmask = rest[0] if return_softmax else None
    return context, softmax_lse, S_dmask


def _flash_blocksparse_attn_backward(dout, qkv, out, softmax_lse, cu_seqlens, layout, dropout_p, max_s,
                                      softmax_scale, causal, rng_state=None):
    dqkv = torch.empty_like(qkv)
    _hip.bwd(dout, qkv[:, 0], qkv[:, 1], qkv[:, 2], out, softmax_lse, dqkv[:, 0], dqkv[:, 1], dqkv[:, 2],
             cu_seqlens, cu_seqlens, max_s, max_s, dropout_p, softmax_scale, False, causal, None,
             rng_state=rng_state, layout=layout)
    return dqkv


class FlashBlocksparseAttnFun(torch.autograd.Function):

    @staticmethod
    def forward(ctx, qkv, cu_seqlens, layout, dropout_p, max_s, softmax_scale, causal):
        rng_state = _hip.reserve_rng(qkv.device) if dropout_p > 0 else None
        if softmax_scale is None:
            softmax_scale = qkv.shape[-1] ** (-0.5)
        context, softmax_lse, _ = _flash_blocksparse_attn_forward(
            qkv, cu_seqlens, layout, dropout_p, max_s, softmax_scale, causal, False, rng_state)
        ctx.save_for_backward(qkv, context, softmax_lse, cu_seqlens, layout)
        ctx.rng_state = rng_state
        ctx.dropout_p = dropout_p
        ctx.max_s = max_s
        ctx.softmax_scale = softmax_scale
        ctx.causal = causal
        return context

    @staticmethod
    def backward(ctx, dout):
        qkv, context, softmax_lse, cu_seqlens, layout = ctx.saved_tensors
        dqkv = _flash_blocksparse_attn_backward(dout, qkv, context, softmax_lse, cu_seqlens, layout, ctx.dropout_p,
                                                ctx.max_s, ctx.softmax_scale, ctx.causal, ctx.rng_state)
        return dqkv, None, None, None, None, None, None


class FlashBlocksparseAttnFunWithS(torch.autograd.Function):
    """Also returns the attention probabilities and the LSE (test path, reference :107-142)."""

    @staticmethod
    def forward(ctx, qkv, cu_seqlens, layout, dropout_p, max_s, softmax_scale, causal):
        rng_state = _hip.reserve_rng(qkv.device) if dropout_p > 0 else None
        if softmax_scale is None:
            softmax_scale = qkv.shape[-1] ** (-0.5)
        context, softmax_lse, S_dmask = _flash_blocksparse_attn_forward(
            qkv, cu_seqlens, layout, dropout_p, max_s, softmax_scale, causal, True, rng_state)
        ctx.save_for_backward(qkv, context, softmax_lse, cu_seqlens, layout)
        ctx.rng_state = rng_state
        ctx.dropout_p = dropout_p
        ctx.max_s = max_s
        ctx.softmax_scale = softmax_scale
        ctx.causal = causal
        return context, S_dmask, softmax_lse

    @staticmethod
    def backward(ctx, dout, _dS_dmask_ignored, _dsoftmax_sum_ignored):
        qkv, context, softmax_lse, cu_seqlens, layout = ctx.saved_tensors
        dqkv = _flash_blocksparse_attn_backward(dout, qkv, context, softmax_lse, cu_seqlens, layout, ctx.dropout_p,
                                                ctx.max_s, ctx.softmax_scale, ctx.causal, ctx.rng_state)
        return dqkv, None, None, None, None, None, None


def flash_blocksparse_attn_func(qkv, cu_seqlens, blockmask, dropout_p, max_s, softmax_scale=None,
                                causal=False, return_attn_probs=False, convert_mask=True):
    """dropout_p should be set to 0.0 during evaluation.

    qkv: (total, 3, nheads, headdim) fp16/bf16; cu_seqlens: (batch+1) int32; blockmask: the 0/1
    layout (seqlen/16, seqlen/256) when convert_mask, else convert_blockmask's output."""
    func = FlashBlocksparseAttnFun if not return_attn_probs else FlashBlocksparseAttnFunWithS
    layout = _layout(blockmask, convert_mask, qkv.device)
    return func.apply(qkv, cu_seqlens, layout, dropout_p, max_s, softmax_scale, causal)
