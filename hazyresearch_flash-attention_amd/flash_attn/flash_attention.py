"""nn.Module surface above the path (reference flash_attn/flash_attention.py:12-115).

FlashAttention(qkv, key_padding_mask, causal, cu_seqlens, max_s) and FlashMHA(x) keep the
reference's constructor and forward signatures. Differences: bf16 is accepted as well as fp16
(the reference asserts fp16, :37), and the backward works.
"""
import torch
import torch.nn as nn

from flash_attn.bert_padding import pad_input, unpad_input
from flash_attn.flash_attn_interface import flash_attn_unpadded_qkvpacked_func
from flash_attn.rotary import RotaryEmbedding, RotaryEmbedding2D, apply_rotary_emb_qkv_


class FlashAttention(nn.Module):
    """Scaled dot-product attention with softmax over packed qkv.

    softmax_scale: temperature (default 1/sqrt(headdim)); attention_dropout: dropout rate in
    training mode."""

    def __init__(self, softmax_scale=None, attention_dropout=0.0, device=None, dtype=None):
        super().__init__()
        self.softmax_scale = softmax_scale
        self.dropout_p = attention_dropout

    def forward(self, qkv, key_padding_mask=None, causal=False, cu_seqlens=None, max_s=None,
                need_weights=False):
        """qkv: (B, S, 3, H, D), or (nnz, 3, H, D) when cu_seqlens is given.
        key_padding_mask: (B, S) bool, True = keep. Returns (output, None)."""
        assert not need_weights
        assert qkv.dtype in (torch.float16, torch.bfloat16)
        assert qkv.is_cuda
        dropout_p = self.dropout_p if self.training else 0.0
        if cu_seqlens is not None:
            assert max_s is not None
            out = flash_attn_unpadded_qkvpacked_func(qkv, cu_seqlens, max_s, dropout_p,
                                                     softmax_scale=self.softmax_scale, causal=causal)
            return out, None
        batch, seqlen = qkv.shape[0], qkv.shape[1]
        if key_padding_mask is None:
            qkv_u = qkv.reshape(batch * seqlen, *qkv.shape[2:])
            cu = torch.arange(0, (batch + 1) * seqlen, seqlen, dtype=torch.int32, device=qkv.device)
            out = flash_attn_unpadded_qkvpacked_func(qkv_u, cu, seqlen, dropout_p,
                                                     softmax_scale=self.softmax_scale, causal=causal)
            return out.reshape(batch, seqlen, *out.shape[1:]), None
        nheads = qkv.shape[-2]
        x = qkv.reshape(batch, seqlen, -1)
        x_u, indices, cu, max_s = unpad_input(x, key_padding_mask)
        x_u = x_u.reshape(x_u.shape[0], 3, nheads, -1)
        out_u = flash_attn_unpadded_qkvpacked_func(x_u, cu, max_s, dropout_p,
                                                   softmax_scale=self.softmax_scale, causal=causal)
        out = pad_input(out_u.reshape(out_u.shape[0], -1), indices, batch, seqlen)
        return out.reshape(batch, seqlen, nheads, -1), None


class FlashMHA(nn.Module):
    """Multi-head attention block: Wqkv -> optional rotary -> FlashAttention -> out_proj."""

    def __init__(self, embed_dim, num_heads, bias=True, batch_first=True, attention_dropout=0.0,
                 causal=False, use_rotary_emb=None, device=None, dtype=None, **kwargs) -> None:
        assert batch_first
        factory_kwargs = {"device": device, "dtype": dtype}
        super().__init__()
        self.embed_dim = embed_dim
        self.causal = causal
        self.num_heads = num_heads
        assert self.embed_dim % num_heads == 0, "self.kdim must be divisible by num_heads"
        self.head_dim = self.embed_dim // num_heads
        assert self.head_dim in (16, 32, 64, 128), "Only support head_dim == 16, 32, 64, or 128"
        assert use_rotary_emb in (None, "1d", "2d")
        self.use_rotary_emb = use_rotary_emb
        if use_rotary_emb == "1d":
            self.rotary_emb = RotaryEmbedding(self.head_dim)
        elif use_rotary_emb == "2d":
            self.rotary_emb = RotaryEmbedding2D(self.head_dim)
        self.Wqkv = nn.Linear(embed_dim, 3 * embed_dim, bias=bias, **factory_kwargs)
        self.inner_attn = FlashAttention(attention_dropout=attention_dropout, **factory_kwargs)
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=bias, **factory_kwargs)

    def forward(self, x, key_padding_mask=None, need_weights=False):
        """x: (batch, seqlen, embed_dim); key_padding_mask: (batch, seqlen) bool."""
        qkv = self.Wqkv(x)
        b, s = qkv.shape[0], qkv.shape[1]
        if self.use_rotary_emb and qkv.is_cuda and qkv.is_contiguous():
            # q and k rotated in place in the packed projection (fa_rotary): no unbind/stack copies
            cos, sin = self.rotary_emb.cos_sin_tables(s, qkv.device, qkv.dtype)
            qkv = apply_rotary_emb_qkv_(qkv, cos, sin, self.num_heads, self.head_dim)
        qkv = qkv.reshape(b, s, 3, self.num_heads, self.head_dim)
        if self.use_rotary_emb and not qkv.is_cuda:
            q, k, v = qkv.unbind(dim=2)
            q, k = self.rotary_emb(q, k, seq_dimension=-3)
            qkv = torch.stack([q, k, v], dim=2)
        context, attn_weights = self.inner_attn(qkv, key_padding_mask=key_padding_mask,
                                                need_weights=need_weights, causal=self.causal)
        return self.out_proj(context.reshape(b, s, -1)), attn_weights
