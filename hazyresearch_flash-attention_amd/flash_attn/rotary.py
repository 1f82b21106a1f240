"""Rotary position embeddings with the reference's API and numerics (flash_attn/rotary.py:22-135).

Pairs are interleaved ((d 2) -> d 2, the reference's split): x' = x*cos + rotate_half(x)*sin with
rotate_half(x0, x1) = (-x1, x0), cos/sin computed in fp32 from inv_freq = 10000^(-2i/d), cast to x's
dtype and repeated per pair, all products in x's dtype, exactly as the reference does.

On GPU tensors the element-wise chain runs in one HIP kernel (fa_rotary, csrc/fa_rotary.hip) that
reproduces torch's rounding bit for bit, forward and backward. `apply_rotary_emb_qkv_` rotates
q and k of a packed (B, S, 3, H, D) qkv in place, so FlashMHA needs no unbind/stack copies:
one read and one write of q and k. Host tensors use the torch expression, as the reference.
"""
import math
from typing import Tuple

import torch


def rotate_half(x):
    x = x.unflatten(dim=-1, sizes=(-1, 2))
    x1, x2 = x.unbind(dim=-1)
    return torch.stack((-x2, x1), dim=-1).flatten(start_dim=-2)


def _apply_rotary_torch(x, cos, sin, seq_dimension: int = -2):
    cos = cos[:x.shape[seq_dimension], :]
    sin = sin[:x.shape[seq_dimension], :]
    if seq_dimension == -3:
        cos = cos[:, None, :]
        sin = sin[:, None, :]
    return (x * cos) + (rotate_half(x) * sin)


def _view4(x, seq_dimension):
    """(shape (B, S, 1, H, D), strides (batch, seq, slot, head)) of a (b,h,s,d) / (b,s,h,d) tensor."""
    if seq_dimension == -2:
        b, h, s, d = x.shape
        return (b, s, 1, h, d), (x.stride(0), x.stride(2), 0, x.stride(1))
    b, s, h, d = x.shape
    return (b, s, 1, h, d), (x.stride(0), x.stride(1), 0, x.stride(2))


def _hip_ok(x, cos):
    return (x.is_cuda and x.dtype in (torch.float16, torch.bfloat16) and x.dim() == 4 and x.stride(-1) == 1
            and x.shape[-1] % 8 == 0 and cos.shape[-1] == x.shape[-1])


class ApplyRotaryEmb(torch.autograd.Function):
    """y = x*cos + rotate_half(x)*sin on the GPU (fa_rotary), backward = the autograd transpose."""

    @staticmethod
    def forward(ctx, x, cos, sin, seq_dimension):
        from flash_attn import flash_attn_hip as hip
        if x.data_ptr() % 16 or any(st % 8 for st in x.stride()[:-1]):
            x = x.contiguous()
        cos, sin = cos.contiguous(), sin.contiguous()
        y = torch.empty_like(x)
        shape, xs = _view4(x, seq_dimension)
        _, ys = _view4(y, seq_dimension)
        hip.rotary(x, y, cos, sin, shape, xs, ys, 1, False)
        ctx.save_for_backward(cos, sin)
        ctx.seq_dimension = seq_dimension
        return y

    @staticmethod
    def backward(ctx, grad):
        from flash_attn import flash_attn_hip as hip
        cos, sin = ctx.saved_tensors
        g = grad.contiguous()
        dx = torch.empty_like(g)
        shape, gs = _view4(g, ctx.seq_dimension)
        _, ds = _view4(dx, ctx.seq_dimension)
        hip.rotary(g, dx, cos, sin, shape, gs, ds, 1, True)
        return dx, None, None, None


def apply_rotary_pos_emb(x, cos, sin, seq_dimension: int = -2):
    """Reference :31-41. cos/sin: (>= seqlen, d) tables in x's dtype."""
    if _hip_ok(x, cos):
        s = x.shape[seq_dimension]
        return ApplyRotaryEmb.apply(x, cos[:s], sin[:s], seq_dimension)
    return _apply_rotary_torch(x, cos, sin, seq_dimension)


class ApplyRotaryEmbQKV_(torch.autograd.Function):
    """In place on packed qkv (B, S, 3, H, D) (any tensor whose memory is that layout, e.g. the
    (B, S, 3*H*D) output of Wqkv): q and k rotated, v untouched. Backward writes a fresh gradient
    with the q/k parts rotated back and the v part copied, in one launch."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, nheads, head_dim):
        from flash_attn import flash_attn_hip as hip
        B, S = qkv.shape[0], qkv.shape[1]
        assert qkv.is_contiguous() and qkv.numel() == B * S * 3 * nheads * head_dim
        cos, sin = cos.contiguous(), sin.contiguous()
        st = (S * 3 * nheads * head_dim, 3 * nheads * head_dim, nheads * head_dim, head_dim)
        hip.rotary(qkv, qkv, cos, sin, (B, S, 3, nheads, head_dim), st, st, 2, False)
        ctx.mark_dirty(qkv)
        ctx.save_for_backward(cos, sin)
        ctx.dims = (B, S, nheads, head_dim, st)
        return qkv

    @staticmethod
    def backward(ctx, grad):
        from flash_attn import flash_attn_hip as hip
        cos, sin = ctx.saved_tensors
        B, S, H, D, st = ctx.dims
        g = grad.contiguous()
        dx = torch.empty_like(g)
        hip.rotary(g, dx, cos, sin, (B, S, 3, H, D), st, st, 2, True)
        return dx, None, None, None, None


def apply_rotary_emb_qkv_(qkv, cos, sin, nheads=None, head_dim=None):
    """Rotate q and k of a packed qkv in place; qkv (B, S, 3, H, D) or its (B, S, 3*H*D) storage."""
    if nheads is None:
        nheads, head_dim = qkv.shape[-2], qkv.shape[-1]
    return ApplyRotaryEmbQKV_.apply(qkv, cos[:qkv.shape[1]], sin[:qkv.shape[1]], nheads, head_dim)


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

    def _tables(self, seq_len, device, dtype):
        if (seq_len != self._seq_len_cached or self._cos_cached.device != device
                or self._cos_cached.dtype != dtype):
            self._seq_len_cached = seq_len
            inv_freq = self.inv_freq.to(device)   # FlashMHA(device=...) leaves the buffer on cpu
            t = torch.arange(seq_len, device=device, dtype=inv_freq.dtype)
            freqs = torch.outer(t, inv_freq)
            self._cos_cached = torch.cos(freqs).to(dtype).repeat_interleave(2, dim=-1)
            self._sin_cached = torch.sin(freqs).to(dtype).repeat_interleave(2, dim=-1)
        return self._cos_cached, self._sin_cached

    def _update_cos_sin_tables(self, x, seq_dimension=-2):
        return self._tables(x.shape[seq_dimension], x.device, x.dtype)

    def cos_sin_tables(self, seqlen, device, dtype):
        """(seqlen, dim) cos/sin per token position (for apply_rotary_emb_qkv_)."""
        return self._tables(seqlen, device, dtype)

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

    def cos_sin_tables(self, seqlen, device, dtype):
        """Per-token (seqlen, dim) tables: token s = (s // side, s % side) takes the 1-D tables of
        its w index in the first half of d and of its h index in the second."""
        side = int(math.sqrt(seqlen))
        assert seqlen == side ** 2
        c1, s1 = self.rotary_emb1d.cos_sin_tables(side, device, dtype)
        pos = torch.arange(seqlen, device=device)
        cos = torch.cat([c1[pos % side], c1[pos // side]], dim=-1)
        sin = torch.cat([s1[pos % side], s1[pos // side]], dim=-1)
        return cos, sin

    def forward(self, q: torch.Tensor, k: torch.Tensor, seq_dimension=-2):
        assert seq_dimension in (-2, -3)
        seqlen = q.shape[seq_dimension]
        side = int(math.sqrt(seqlen))
        assert seqlen == side ** 2
        if q.is_cuda:
            cos, sin = self.cos_sin_tables(seqlen, q.device, q.dtype)
            return apply_rotary_pos_emb(q, cos, sin, seq_dimension), apply_rotary_pos_emb(k, cos, sin, seq_dimension)
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
