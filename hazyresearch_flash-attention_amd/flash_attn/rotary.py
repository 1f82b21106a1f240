"""Rotary position embeddings with the reference's API and numerics (flash_attn/rotary.py:22-135).

Pairs are interleaved ((d 2) -> d 2, the reference's split): x' = x*cos + rotate_half(x)*sin with
rotate_half(x0, x1) = (-x1, x0), cos/sin computed in fp32 from inv_freq = 10000^(-2i/d), cast to x's
dtype and repeated per pair, all products in x's dtype, exactly as the reference does.
"""
import math
from typing import Tuple

import torch


def rotate_half(x):
    x = x.unflatten(dim=-1, sizes=(-1, 2))
    x1, x2 = x.unbind(dim=-1)
    return torch.stack((-x2, x1), dim=-1).flatten(start_dim=-2)


def apply_rotary_pos_emb(x, cos, sin, seq_dimension: int = -2):
    cos = cos[:x.shape[seq_dimension], :]
    sin = sin[:x.shape[seq_dimension], :]
    if seq_dimension == -3:
        cos = cos[:, None, :]
        sin = sin[:, None, :]
    return (x * cos) + (rotate_half(x) * sin)


class RotaryEmbedding(torch.nn.Module):
    """1-D RoPE (RoFormer, Su et al.) for q, k laid out (b, h, s, d) (seq_dimension=-2) or
    (b, s, h, d) (seq_dimension=-3). cos/sin tables are cached per (length, device, dtype)."""

    def __init__(self, dim_model: int, *_, **__):
        super().__init__()
        inv_freq = 1.0 / (10000 ** (torch.arange(0, dim_model, 2).float() / dim_model))
        self.register_buffer("inv_freq", inv_freq)
        self._seq_len_cached = None
        self._cos_cached = None
        self._sin_cached = None

    def _update_cos_sin_tables(self, x, seq_dimension=-2):
        seq_len = x.shape[seq_dimension]
        if (seq_len != self._seq_len_cached or self._cos_cached.device != x.device
                or self._cos_cached.dtype != x.dtype):
            self._seq_len_cached = seq_len
            inv_freq = self.inv_freq.to(x.device)   # FlashMHA(device=...) leaves the buffer on cpu
            t = torch.arange(seq_len, device=x.device, dtype=inv_freq.dtype)
            freqs = torch.outer(t, inv_freq)
            self._cos_cached = torch.cos(freqs).to(x.dtype).repeat_interleave(2, dim=-1)
            self._sin_cached = torch.sin(freqs).to(x.dtype).repeat_interleave(2, dim=-1)
        return self._cos_cached, self._sin_cached

    def forward(self, q: torch.Tensor, k: torch.Tensor, seq_dimension=-2) -> Tuple[torch.Tensor, torch.Tensor]:
        assert seq_dimension in (-2, -3)
        cos, sin = self._update_cos_sin_tables(k, seq_dimension=seq_dimension)
        return (apply_rotary_pos_emb(q, cos, sin, seq_dimension),
                apply_rotary_pos_emb(k, cos, sin, seq_dimension))


class RotaryEmbedding2D(torch.nn.Module):
    """2-D RoPE over a square (h w) token grid: the first half of d rotates along w, the
    second along h (reference rotary.py:103-135)."""

    def __init__(self, dim: int):
        super().__init__()
        assert dim % 4 == 0
        self.rotary_emb1d = RotaryEmbedding(dim // 2)

    def forward(self, q: torch.Tensor, k: torch.Tensor, seq_dimension=-2):
        assert seq_dimension in (-2, -3)
        seqlen = q.shape[seq_dimension]
        side = int(math.sqrt(seqlen))
        assert seqlen == side ** 2
        if seq_dimension == -3:  # (b, s, h, d) -> (b, h, s, d)
            q, k = q.transpose(1, 2), k.transpose(1, 2)
        q0, q1 = q.chunk(2, dim=-1)
        k0, k1 = k.chunk(2, dim=-1)
        grid = lambda t: t.reshape(t.shape[0], t.shape[1], side, side, t.shape[-1])
        flat = lambda t: t.reshape(t.shape[0], t.shape[1], side * side, t.shape[-1])
        q0e, k0e = self.rotary_emb1d(grid(q0), grid(k0), seq_dimension=-2)
        q1e, k1e = self.rotary_emb1d(grid(q1), grid(k1), seq_dimension=-3)
        q_emb = torch.cat([flat(q0e), flat(q1e)], dim=-1)
        k_emb = torch.cat([flat(k0e), flat(k1e)], dim=-1)
        if seq_dimension == -3:
            q_emb, k_emb = q_emb.transpose(1, 2), k_emb.transpose(1, 2)
        return q_emb, k_emb
