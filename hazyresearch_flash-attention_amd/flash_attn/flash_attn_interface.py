"""Drop-in `flash_attn.flash_attn_interface` for MI355X.

Same public names, argument order, defaults and return values as the reference module
(flash_attn/flash_attn_interface.py:39-252). Differences, all behind the same surface:

* the compute goes to libfa_hip.so (hand-written gfx950 kernels) through `flash_attn_hip`;
* backward exists (the reference branch never bound `flash_attn_cuda.bwd`, :31-33);
* for dropout the forward reserves a Philox (seed, offset) from the torch generator and saves
  that pair in ctx, instead of snapshotting the whole RNG state (:44, :60-63, :70-71);
* `S_dmask` (return_attn_probs=True) is row-major (B, H, round16(max_q), round16(max_k)),
  holds softmax probabilities already normalised, negated where dropout dropped the entry,
  and 0 outside the valid (and causal) region;
* the three autograd functions run in C++ (csrc/fa_torch.cpp, module _fa_C) when the compiled
  binding is built and the inputs are on the GPU: one pybind11 call per forward, a C++ backward
  node. The Python classes below are the same computation and serve return_attn_probs=True.
"""
import torch

from flash_attn import flash_attn_hip as _hip


def _get_block_size(device, head_dim, is_dropout):
    """Key-block size of the forward kernel (reference: flash_attn_interface.py:8-14). On gfx950
    the forward always walks K/V in 64-key tiles; kept for callers that query it."""
    assert head_dim % 8 == 0 and head_dim <= 128
    return 64


def _flash_attn_forward(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p,
                        softmax_scale, causal, return_softmax, rng_state=None):
    out, softmax_lse, *rest = _hip.fwd(
        q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p, softmax_scale,
        False, causal, return_softmax, None, rng_state=rng_state)
    S_dmask = rest[0] if return_softmax else None
    return out, softmax_lse, S_dmask


def _flash_attn_backward(dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_seqlens_q, cu_seqlens_k,
                         max_seqlen_q, max_seqlen_k, dropout_p, softmax_scale, causal, rng_state=None):
    softmax_d = _hip.bwd(
        dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_seqlens_q, cu_seqlens_k,
        max_seqlen_q, max_seqlen_k, dropout_p, softmax_scale, False, causal, None, rng_state=rng_state)
    return dq, dk, dv, softmax_d


_NO_RNG = (0, 0, None)


def _reserve(dropout_p, device):
    return _hip.reserve_rng(device) if dropout_p > 0 else None


class FlashAttnQKVPackedFunc(torch.autograd.Function):

    @staticmethod
    def forward(ctx, qkv, cu_seqlens, max_seqlen, dropout_p, softmax_scale, causal, return_softmax):
        rng_state = _reserve(dropout_p, qkv.device)
        if softmax_scale is None:
            softmax_scale = qkv.shape[-1] ** (-0.5)
        out, softmax_lse, S_dmask = _flash_attn_forward(
            qkv[:, 0], qkv[:, 1], qkv[:, 2], cu_seqlens, cu_seqlens, max_seqlen, max_seqlen,
            dropout_p, softmax_scale, causal=causal, return_softmax=return_softmax, rng_state=rng_state)
        ctx.save_for_backward(qkv, out, softmax_lse, cu_seqlens)
        ctx.rng_state = rng_state
        ctx.dropout_p = dropout_p
        ctx.max_seqlen = max_seqlen
        ctx.softmax_scale = softmax_scale
        ctx.causal = causal
        return out if not return_softmax else (out, softmax_lse, S_dmask)

    @staticmethod
    def backward(ctx, dout, *args):
        qkv, out, softmax_lse, cu_seqlens = ctx.saved_tensors
        dqkv = torch.empty_like(qkv)
        _flash_attn_backward(
            dout, qkv[:, 0], qkv[:, 1], qkv[:, 2], out, softmax_lse,
            dqkv[:, 0], dqkv[:, 1], dqkv[:, 2], cu_seqlens, cu_seqlens,
            ctx.max_seqlen, ctx.max_seqlen, ctx.dropout_p, ctx.softmax_scale, ctx.causal,
            rng_state=ctx.rng_state)
        return dqkv, None, None, None, None, None, None


class FlashAttnKVPackedFunc(torch.autograd.Function):

    @staticmethod
    def forward(ctx, q, kv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p,
                softmax_scale, causal, return_softmax):
        rng_state = _reserve(dropout_p, q.device)
        if softmax_scale is None:
            softmax_scale = q.shape[-1] ** (-0.5)
        out, softmax_lse, S_dmask = _flash_attn_forward(
            q, kv[:, 0], kv[:, 1], cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
            dropout_p, softmax_scale, causal=causal, return_softmax=return_softmax, rng_state=rng_state)
        ctx.save_for_backward(q, kv, out, softmax_lse, cu_seqlens_q, cu_seqlens_k)
        ctx.rng_state = rng_state
        ctx.dropout_p = dropout_p
        ctx.max_seqlen_q = max_seqlen_q
        ctx.max_seqlen_k = max_seqlen_k
        ctx.softmax_scale = softmax_scale
        ctx.causal = causal
        return out if not return_softmax else (out, softmax_lse, S_dmask)

    @staticmethod
    def backward(ctx, dout, *args):
        q, kv, out, softmax_lse, cu_seqlens_q, cu_seqlens_k = ctx.saved_tensors
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        _flash_attn_backward(
            dout, q, kv[:, 0], kv[:, 1], out, softmax_lse, dq, dkv[:, 0], dkv[:, 1],
            cu_seqlens_q, cu_seqlens_k, ctx.max_seqlen_q, ctx.max_seqlen_k, ctx.dropout_p,
            ctx.softmax_scale, ctx.causal, rng_state=ctx.rng_state)
        return dq, dkv, None, None, None, None, None, None, None, None


class FlashAttnFunc(torch.autograd.Function):

    @staticmethod
    def forward(ctx, q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p,
                softmax_scale, causal, return_softmax):
        rng_state = _reserve(dropout_p, q.device)
        if softmax_scale is None:
            softmax_scale = q.shape[-1] ** (-0.5)
        out, softmax_lse, S_dmask = _flash_attn_forward(
            q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
            dropout_p, softmax_scale, causal=causal, return_softmax=return_softmax, rng_state=rng_state)
        ctx.save_for_backward(q, k, v, out, softmax_lse, cu_seqlens_q, cu_seqlens_k)
        ctx.rng_state = rng_state
        ctx.dropout_p = dropout_p
        ctx.max_seqlen_q = max_seqlen_q
        ctx.max_seqlen_k = max_seqlen_k
        ctx.softmax_scale = softmax_scale
        ctx.causal = causal
        return out if not return_softmax else (out, softmax_lse, S_dmask)

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, softmax_lse, cu_seqlens_q, cu_seqlens_k = ctx.saved_tensors
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _flash_attn_backward(
            dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_seqlens_q, cu_seqlens_k,
            ctx.max_seqlen_q, ctx.max_seqlen_k, ctx.dropout_p, ctx.softmax_scale, ctx.causal,
            rng_state=ctx.rng_state)
        return dq, dk, dv, None, None, None, None, None, None, None, None


def flash_attn_unpadded_qkvpacked_func(qkv, cu_seqlens, max_seqlen, dropout_p, softmax_scale=None,
                                       causal=False, return_attn_probs=False):
    """Attention over packed qkv (total, 3, nheads, headdim); cu_seqlens (batch+1,) int32.
    Returns out (total, nheads, headdim), or (out, softmax_lse, S_dmask) with return_attn_probs.
    softmax_scale defaults to headdim**-0.5. Set dropout_p to 0.0 for evaluation."""
    C = _hip._C
    if C is not None and not return_attn_probs and qkv.is_cuda:
        seed, offset, od = _hip._rng_args(dropout_p, qkv.device) if dropout_p > 0 else _NO_RNG
        return C.flash_attn_unpadded_qkvpacked_func(qkv, cu_seqlens, max_seqlen, dropout_p, softmax_scale, causal,
                                                    seed, offset, od, _hip._impl())
    return FlashAttnQKVPackedFunc.apply(qkv, cu_seqlens, max_seqlen, dropout_p, softmax_scale,
                                        causal, return_attn_probs)


def flash_attn_unpadded_kvpacked_func(q, kv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                                      dropout_p, softmax_scale=None, causal=False,
                                      return_attn_probs=False):
    """Attention with q (total_q, nheads, headdim) and packed kv (total_k, 2, nheads, headdim)."""
    C = _hip._C
    if C is not None and not return_attn_probs and q.is_cuda:
        seed, offset, od = _hip._rng_args(dropout_p, q.device) if dropout_p > 0 else _NO_RNG
        return C.flash_attn_unpadded_kvpacked_func(q, kv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                                                   dropout_p, softmax_scale, causal, seed, offset, od, _hip._impl())
    return FlashAttnKVPackedFunc.apply(q, kv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                                       dropout_p, softmax_scale, causal, return_attn_probs)


def flash_attn_unpadded_func(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                             dropout_p, softmax_scale=None, causal=False, return_attn_probs=False):
    """Attention with separate q (total_q, nheads, headdim), k and v (total_k, nheads, headdim)."""
    C = _hip._C
    if C is not None and not return_attn_probs and q.is_cuda:
        seed, offset, od = _hip._rng_args(dropout_p, q.device) if dropout_p > 0 else _NO_RNG
        return C.flash_attn_unpadded_func(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, dropout_p,
                                          softmax_scale, causal, seed, offset, od, _hip._impl())
    return FlashAttnFunc.apply(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
                               dropout_p, softmax_scale, causal, return_attn_probs)


def flash_attn_func(qkv, cu_seqlens, dropout_p, max_s, softmax_scale=None, causal=False,
                    return_attn_probs=False):
    """Legacy argument order (qkv, cu_seqlens, dropout_p, max_s), kept for compatibility."""
    return flash_attn_unpadded_qkvpacked_func(qkv, cu_seqlens, max_s, dropout_p, softmax_scale,
                                              causal, return_attn_probs)
