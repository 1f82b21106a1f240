"""Block-sparse attention modules (reference flash_attn/flash_blocksparse_attention.py:12-150).

FlashBlocksparseAttention and FlashBlocksparseMHA keep the reference's constructor and forward
signatures. The reference builds its sparsity config with `hydra.utils.instantiate`; hydra is
not part of this build, so `sparsity_config` is used as given: an object with
`make_layout(max_seq_length)`, a callable `f(max_seq_length) -> layout`, or the 0/1 layout
tensor itself, shape (max_seq_length/16, max_seq_length/256). bf16 is accepted as well as fp16
(the reference asserts fp16, :51).
"""
import torch
import torch.nn as nn

from flash_attn.bert_padding import pad_input, unpad_input
from flash_attn.flash_blocksparse_attn_interface import convert_blockmask, flash_blocksparse_attn_func


def _make_layout(sparsity_config, max_seq_length):
    if isinstance(sparsity_config, torch.Tensor):
        return sparsity_config
    if hasattr(sparsity_config, "make_layout"):
        return sparsity_config.make_layout(max_seq_length)
    return sparsity_config(max_seq_length)


class FlashBlocksparseAttention(nn.Module):
    """Scaled dot-product attention with softmax under a block-sparse layout.

    softmax_temp: temperature (default 1/sqrt(headdim)); attention_dropout: dropout rate in
    training mode."""

    def __init__(self, sparsity_config, softmax_temp=None, attention_dropout=0.0, max_seq_length=2048,
                 device=None, dtype=None):
        super().__init__()
        self.sparsity_config = sparsity_config
        self.softmax_temp = softmax_temp
        self.dropout_p = attention_dropout
        max_seq_length = ((max_seq_length + 256 - 1) // 256) * 256
        layout = _make_layout(sparsity_config, max_seq_length)
        self.register_buffer("layout", layout)
        self.register_buffer("blockmask_converted", convert_blockmask(self.layout, causal=False))

    def forward(self, qkv, attn_mask=None, key_padding_mask=None, causal=False, cu_seqlens=None, max_s=None,
                need_weights=False, convert_mask=True):
        """qkv: (B, S, 3, H, D), or (nnz, 3, H, D) when cu_seqlens is given.
        key_padding_mask: (B, S) bool, True = keep (the reference takes a mask object with
        `.bool_matrix`; both are accepted). Returns (output, None)."""
        assert not need_weights
        assert attn_mask is None
        assert qkv.dtype in (torch.float16, torch.bfloat16)
        assert qkv.is_cuda
        dropout_p = self.dropout_p if self.training else 0.0
        if cu_seqlens is None:
            batch_size, seqlen = qkv.shape[0], qkv.shape[1]
            seqlen_rounded = ((seqlen + 256 - 1) // 256) * 256
            assert seqlen_rounded // 16 <= self.layout.shape[0], seqlen_rounded // 256 <= self.layout.shape[1]
            blockmask = self.layout[:seqlen_rounded // 16, :seqlen_rounded // 256]
            if key_padding_mask is None:
                qkv_u = qkv.reshape(batch_size * seqlen, *qkv.shape[2:])
                cu = torch.arange(0, (batch_size + 1) * seqlen, seqlen, dtype=torch.int32, device=qkv.device)
                out = flash_blocksparse_attn_func(qkv_u, cu, blockmask, dropout_p, seqlen,
                                                  softmax_scale=self.softmax_temp, causal=causal)
                return out.reshape(batch_size, seqlen, *out.shape[1:]), None
            kpm = getattr(key_padding_mask, "bool_matrix", key_padding_mask)
            nheads = qkv.shape[-2]
            x = qkv.reshape(batch_size, seqlen, -1)
            x_u, indices, cu, max_s = unpad_input(x, kpm)
            x_u = x_u.reshape(x_u.shape[0], 3, nheads, -1)
            out_u = flash_blocksparse_attn_func(x_u, cu, blockmask, dropout_p, max_s,
                                                softmax_scale=self.softmax_temp, causal=causal)
            out = pad_input(out_u.reshape(out_u.shape[0], -1), indices, batch_size, seqlen)
            return out.reshape(batch_size, seqlen, nheads, -1), None
        assert max_s is not None
        seqlen_rounded = ((max_s + 256 - 1) // 256) * 256
        assert seqlen_rounded // 16 <= self.layout.shape[0], seqlen_rounded // 256 <= self.layout.shape[1]
        if convert_mask:
            blockmask = self.layout[:seqlen_rounded // 16, :seqlen_rounded // 256]
            out = flash_blocksparse_attn_func(qkv, cu_seqlens, blockmask, dropout_p, max_s,
                                              softmax_scale=self.softmax_temp, causal=causal)
        else:
            out = flash_blocksparse_attn_func(qkv, cu_seqlens, self.blockmask_converted, dropout_p, max_s,
                                              softmax_scale=self.softmax_temp, causal=causal, convert_mask=False)
        return out, None


class FlashBlocksparseMHA(nn.Module):
    """Wqkv -> FlashBlocksparseAttention -> out_proj (reference :118-150)."""

    def __init__(self, embed_dim, num_heads, sparsity_config, bias=True, batch_first=True, attention_dropout=0.0,
                 causal=False, max_seq_length=2048, device=None, dtype=None, **kwargs) -> None:
        assert batch_first
        factory_kwargs = {"device": device, "dtype": dtype}
        super().__init__()
        self.embed_dim = embed_dim
        self.causal = causal
        self.num_heads = num_heads
        assert self.embed_dim % num_heads == 0, "self.kdim must be divisible by num_heads"
        self.head_dim = self.embed_dim // num_heads
        assert self.head_dim % 8 == 0 and self.head_dim <= 128, "head_dim must be a multiple of 8 and <= 128"
        self.Wqkv = nn.Linear(embed_dim, 3 * embed_dim, bias=bias, **factory_kwargs)
        self.inner_attn = FlashBlocksparseAttention(sparsity_config, attention_dropout=attention_dropout,
                                                    max_seq_length=max_seq_length, **factory_kwargs)
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=bias, **factory_kwargs)

    def forward(self, x, x_ignored_, x_ignored_1_, attn_mask=None, key_padding_mask=None, need_weights=False):
        qkv = self.Wqkv(x)
        b, s = qkv.shape[0], qkv.shape[1]
        qkv = qkv.reshape(b, s, 3, self.num_heads, self.head_dim)
        context, attn_weights = self.inner_attn(qkv, key_padding_mask=key_padding_mask, need_weights=need_weights,
                                                causal=self.causal)
        return self.out_proj(context.reshape(b, s, -1)), attn_weights
