"""Restatement of the reference's correctness oracle and test-input helpers.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows /root/reference/tests/test_flash_attn.py:
  generate_random_padding_mask  :17-26
  generate_qkv                  :29-112  (inputs built directly, no nn.Linear)
  attention_ref                 :115-159 (fp32 upcast oracle; upcast=False + reorder_ops is the
                                          "PyTorch baseline error" estimator of the 2x rule :407-409)
  get_dropout_fraction          :300-329
  attention_blocksparse_ref     :189-215 (plus causal / upcast / reorder_ops, and fully masked rows
                                          give 0 instead of NaN, as the kernels do)
The reference's attention_ref raises UnboundLocalError when dropout_mask is None (:153-155);
here a missing mask means "keep everything".

And /root/reference/benchmarks/benchmark_flash_attention.py:
  attention_pytorch_bench       :14-36   (the benchmark's naive PyTorch attention on packed qkv: the
                                          CPU baseline bench.py times, torch.utils.benchmark.Timer as
                                          benchmarks/utils.py:8-20 does)
"""
import math

import torch


def generate_random_padding_mask(max_seqlen, batch_size, device, mode="random", generator=None):
    assert mode in ("full", "random", "third")
    if mode == "full":
        lengths = torch.full((batch_size, 1), max_seqlen, device=device, dtype=torch.int32)
    elif mode == "random":
        lengths = torch.randint(max(1, max_seqlen - 20), max_seqlen, (batch_size, 1), device=device,
                                generator=generator)
    else:
        lengths = torch.randint(max_seqlen // 3, max_seqlen, (batch_size, 1), device=device, generator=generator)
    return torch.arange(max_seqlen, device=device)[None, :] < lengths


def unpad(x, mask):
    """x (B, S, ...) + mask (B, S) -> (x_unpad (total, ...), indices, cu_seqlens int32, max_seqlen)."""
    seqlens = mask.sum(dim=-1, dtype=torch.int32)
    indices = torch.nonzero(mask.reshape(-1), as_tuple=False).reshape(-1)
    cu = torch.zeros(mask.shape[0] + 1, dtype=torch.int32, device=mask.device)
    cu[1:] = torch.cumsum(seqlens, 0)
    flat = x.reshape((-1,) + tuple(x.shape[2:]))
    return flat.index_select(0, indices), indices, cu, int(seqlens.max().item())


def pad(x_unpad, indices, batch, seqlen):
    out = x_unpad.new_zeros((batch * seqlen,) + tuple(x_unpad.shape[1:]))
    out.index_copy_(0, indices, x_unpad)
    return out.reshape((batch, seqlen) + tuple(x_unpad.shape[1:]))


def attention_ref(q, k, v, query_padding_mask=None, key_padding_mask=None, dropout_p=0.0,
                  dropout_mask=None, causal=False, upcast=True, reorder_ops=False):
    """q (B, Sq, H, D), k/v (B, Sk, H, D); masks (B, S) bool (True = valid);
    dropout_mask (B, H, Sq, Sk) bool (True = keep). Returns (output (B,Sq,H,D), attention (B,H,Sq,Sk))."""
    dtype_og = q.dtype
    if upcast:
        q, k, v = q.float(), k.float(), v.float()
    seqlen_q, seqlen_k = q.shape[1], k.shape[1]
    d = q.shape[-1]
    if not reorder_ops:
        scores = torch.einsum("bthd,bshd->bhts", q / math.sqrt(d), k)
    else:
        scores = torch.einsum("bthd,bshd->bhts", q, k / math.sqrt(d))
    if key_padding_mask is not None:
        scores.masked_fill_(~key_padding_mask[:, None, None, :], float("-inf"))
    if causal:
        cm = torch.triu(torch.ones(seqlen_q, seqlen_k, dtype=torch.bool, device=q.device), 1)
        scores.masked_fill_(cm, float("-inf"))
    attention = torch.softmax(scores, dim=-1)
    dropout_scaling = 1.0 / (1 - dropout_p)
    attention_drop = attention if dropout_mask is None else attention.masked_fill(~dropout_mask, 0.0)
    output = torch.einsum("bhts,bshd->bthd", attention_drop, v * dropout_scaling)
    if query_padding_mask is not None:
        output.masked_fill_(~query_padding_mask[:, :, None, None], 0.0)
        attention = attention.masked_fill(~query_padding_mask[:, None, :, None], 0.0)
    return output.to(dtype=dtype_og), attention.to(dtype=dtype_og)


def get_dropout_fraction(dropout_mask, query_padding_mask=None, key_padding_mask=None, causal=False):
    batch_size, nheads, seqlen_q, seqlen_k = dropout_mask.shape
    dropped = ~dropout_mask
    if query_padding_mask is not None:
        dropped = dropped.masked_fill(~query_padding_mask[:, None, :, None], False)
    if key_padding_mask is not None:
        dropped = dropped.masked_fill(~key_padding_mask[:, None, None, :], False)
    if causal:
        cm = torch.triu(torch.ones(seqlen_q, seqlen_k, dtype=torch.bool, device=dropout_mask.device), 1)
        dropped = dropped.masked_fill(cm, False)
    dropped_total = dropped.sum()
    ql = (query_padding_mask.sum(dim=-1) if query_padding_mask is not None
          else torch.full((batch_size,), seqlen_q, device=dropout_mask.device))
    kl = (key_padding_mask.sum(dim=-1) if key_padding_mask is not None
          else torch.full((batch_size,), seqlen_k, device=dropout_mask.device))
    if not causal:
        numel = ql * kl
    else:
        numel = torch.where(ql <= kl, ql * (ql + 1) / 2, ql * kl - (kl * (kl - 1) / 2))
    return dropped_total / (numel.sum() * nheads)


def max_err_bound(out_pt, out_ref, floor=0.0):
    """The reference's 2x rule (tests/test_flash_attn.py:407-409): allowed max |out - ref|.
    `floor` covers fp32 inputs, where the PyTorch baseline error can be exactly 0."""
    return max(2 * (out_pt.float() - out_ref.float()).abs().max().item(), floor)


def ulp_floor(ref, dtype=torch.bfloat16):
    """One unit of the output dtype's last place at the reference's magnitude: the floor of the
    2x rule where the low-precision baseline happens to be exact (1-key rows, tiny sequences)."""
    eps = torch.finfo(dtype).eps
    return float(ref.float().abs().max().item()) * eps


def attention_blocksparse_ref(qkv, blockmask, attn_mask=None, dropout_p=0.0, dropout_mask=None, causal=False,
                              upcast=True, reorder_ops=False):
    """qkv (B, S, 3, H, D); blockmask (S/16 rounded up, S/256 rounded up) 0/1, entry [r][c] lets
    query rows 16r..16r+15 see keys 256c..256c+255; attn_mask (B, S) bool key/query padding
    (True = valid); dropout_mask (B, H, S, S) bool (True = keep).
    Returns (output (B, S, H, D), attention (B, H, S, S)) in qkv's dtype."""
    dtype_og = qkv.dtype
    q, k, v = qkv.unbind(dim=2)
    if upcast:
        q, k, v = q.float(), k.float(), v.float()
    seqlen, d = qkv.shape[1], qkv.shape[-1]
    if not reorder_ops:
        scores = torch.einsum("bthd,bshd->bhts", q / math.sqrt(d), k)
    else:
        scores = torch.einsum("bthd,bshd->bhts", q, k / math.sqrt(d))
    if attn_mask is not None:
        scores.masked_fill_(~attn_mask[:, None, None, :], float("-inf"))
    live = blockmask.to(torch.bool).repeat_interleave(16, dim=0).repeat_interleave(256, dim=1)[:seqlen, :seqlen]
    live = live.to(scores.device)
    scores.masked_fill_(~live[None, None], float("-inf"))
    if causal:
        cm = torch.triu(torch.ones(seqlen, seqlen, dtype=torch.bool, device=scores.device), 1)
        scores.masked_fill_(cm, float("-inf"))
    attention = torch.softmax(scores, dim=-1).nan_to_num(0.0)   # rows with no live key -> 0
    if attn_mask is not None:
        attention = attention.masked_fill(~attn_mask[:, None, :, None], 0.0)
    attention = attention.masked_fill(~live[None, None], 0.0)
    attention_drop = attention if dropout_mask is None else attention.masked_fill(~dropout_mask, 0.0)
    output = torch.einsum("bhts,bshd->bthd", attention_drop / (1 - dropout_p), v)
    if attn_mask is not None:
        output.masked_fill_(~attn_mask[:, :, None, None], 0.0)
    return output.to(dtype=dtype_og), attention.to(dtype=dtype_og)


def attention_pytorch_bench(qkv, attn_mask=None, dropout_p=0.0, upcast=False, causal=False):
    """The reference benchmark's naive attention (benchmarks/benchmark_flash_attention.py:14-36):
    qkv (B, S, 3, H, D), attn_mask (B, S) bool (True = valid, None = all valid). Scores are
    q . (k / sqrt(d)), masked keys and (causal) the upper triangle get -inf, softmax, dropout by
    F.dropout, then P V; the output comes back in qkv's dtype."""
    import torch.nn.functional as F
    q, k, v = (qkv.float() if upcast else qkv).unbind(dim=2)
    seqlen, d = qkv.shape[1], qkv.shape[-1]
    scores = torch.einsum("bthd,bshd->bhts", q, k / math.sqrt(d))
    if attn_mask is not None:
        scores.masked_fill_(~attn_mask[:, None, None, :], float("-inf"))
    if causal:
        cm = torch.triu(torch.ones(seqlen, seqlen, dtype=torch.bool, device=qkv.device), 1)
        scores.masked_fill_(cm, float("-inf"))
    attention = torch.softmax(scores, dim=-1)
    attention_drop = F.dropout(attention, dropout_p)
    output = torch.einsum("bhts,bshd->bthd", attention_drop, v)
    return output.to(dtype=qkv.dtype)
