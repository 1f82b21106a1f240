"""Restatement of the reference's rotary embeddings (flash_attn/rotary.py) for checking.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): tests compare the HIP rotary pass and the
rotary fused into the forward with these functions; the product never imports them.

Follows /root/reference/flash_attn/rotary.py:
  rotate_half               :22-29   pairs (2i, 2i+1) -> (-x[2i+1], x[2i])
  apply_rotary_pos_emb      :32-42   x*cos + rotate_half(x)*sin, tables cut to the sequence length
  RotaryEmbedding tables    :65-86   inv_freq = 10000^(-2i/d), cos/sin of t*inv_freq in fp32, cast to
                                     x's dtype, each value repeated for its pair
  RotaryEmbedding2D         :103-135 first half of d rotated along the row index w of an (h w) grid,
                                     the second half along h
Every operation runs in x's dtype in torch's eager order, so results are bit-exact references.
Pinned against the reference's own outputs in tests/golden/modules_golden.npz (test_modules.py).
"""
import math

import torch


def _rotate_pairs(x):
    even, odd = x[..., 0::2], x[..., 1::2]
    return torch.stack((-odd, even), dim=-1).reshape(x.shape)


def rotary_tables(seqlen, dim, dtype, device="cpu"):
    """(seqlen, dim) cos and sin tables of a 1-D rotary embedding over `dim` features."""
    inv_freq = 1.0 / (10000 ** (torch.arange(0, dim, 2, device=device).float() / dim))
    ang = torch.arange(seqlen, device=device, dtype=torch.float32)[:, None] * inv_freq[None, :]
    cos = torch.cos(ang).to(dtype)
    sin = torch.sin(ang).to(dtype)
    return cos.repeat_interleave(2, dim=-1), sin.repeat_interleave(2, dim=-1)


def apply_rotary_ref(x, cos, sin, seq_dimension=-2):
    """x * cos + rotate_half(x) * sin with the tables indexed by position along seq_dimension."""
    n = x.shape[seq_dimension]
    c, s = cos[:n], sin[:n]
    if seq_dimension == -3:
        c, s = c[:, None, :], s[:, None, :]
    return x * c + _rotate_pairs(x) * s


def rotary_1d_ref(q, k, seq_dimension=-2):
    cos, sin = rotary_tables(k.shape[seq_dimension], k.shape[-1], k.dtype, k.device)
    return apply_rotary_ref(q, cos, sin, seq_dimension), apply_rotary_ref(k, cos, sin, seq_dimension)


def rotary_2d_ref(q, k, seq_dimension=-2):
    """2-D form: q, k (b, h, s, d) or (b, s, h, d) with s a square number of tokens."""
    if seq_dimension == -3:
        q, k = q.transpose(1, 2), k.transpose(1, 2)
    b, h, s, d = q.shape
    side = int(math.sqrt(s))
    assert side * side == s
    cos, sin = rotary_tables(side, d // 2, q.dtype, q.device)
    outs = []
    for x in (q, k):
        lo, hi = x[..., : d // 2], x[..., d // 2:]
        grid_lo = lo.reshape(b, h, side, side, d // 2)
        grid_hi = hi.reshape(b, h, side, side, d // 2)
        rot_lo = apply_rotary_ref(grid_lo, cos, sin, -2)      # along w
        rot_hi = apply_rotary_ref(grid_hi, cos, sin, -3)      # along h
        outs.append(torch.cat([rot_lo.reshape(b, h, s, d // 2), rot_hi.reshape(b, h, s, d // 2)], dim=-1))
    if seq_dimension == -3:
        outs = [o.transpose(1, 2) for o in outs]
    return outs[0], outs[1]


def rotary_token_tables_2d(seqlen, dim, dtype, device="cpu"):
    """Per-token (seqlen, dim) tables equivalent to rotary_2d_ref for a flattened (h w) grid:
    token t = (t // side, t % side) uses the 1-D tables of w in the first half of d and of h in
    the second."""
    side = int(math.sqrt(seqlen))
    assert side * side == seqlen
    c1, s1 = rotary_tables(side, dim // 2, dtype, device)
    t = torch.arange(seqlen, device=device)
    return (torch.cat([c1[t % side], c1[t // side]], dim=-1), torch.cat([s1[t % side], s1[t // side]], dim=-1))
