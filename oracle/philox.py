"""Counter-based dropout RNG restated in numpy — TEST INFRASTRUCTURE ONLY.

Philox-4x32 (Salmon et al., SC'11; the generator of the reference,
/root/reference/csrc/flash_attn/src/philox.cuh:30-59,121-136: multipliers 0xD2511F53/0xCD9E8D57,
Weyl key bumps 0x9E3779B9/0xBB67AE85, 7 rounds = 6 keyed rounds + a final one). rounds=10 is the
standard Philox-4x32-10 checked against the Random123 known-answer vectors in
tests/test_oracle.py.

Element mapping (this build's definition; the reference's per-thread stream is tied to its
sm80 MMA layout, tests/test_flash_attn.py:232-235, and does not carry over):
    g    = (row >> 5) << 2 | ((row >> 4) & 1) << 1 | ((row >> 2) & 1)
    slot = (row & 3) | ((row >> 3) & 1) << 2
    out  = Philox7(key=(seed_lo, seed_hi), ctr=(g, col, b*H + h, offset >> 2))
    rnd16 = 16-bit word `slot` of out;  keep = rnd16 <= floor((1-p) * 65535)
(keep rule: fmha_api.cpp:104 and softmax.h:256-296). The same function is in
hazyresearch_flash-attention_amd/csrc/fa_common.h.
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32(ctr, key, rounds=7):
    """ctr: (4, ...) uint32 array-like; key: (k0, k1) ints or (2, ...) arrays. Returns (4, ...) uint32."""
    c = [np.asarray(x, dtype=np.uint64) for x in ctr]
    k0 = np.asarray(key[0], dtype=np.uint64) & MASK32
    k1 = np.asarray(key[1], dtype=np.uint64) & MASK32
    for _ in range(rounds):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        n0 = (p1 >> np.uint64(32)) ^ c[1] ^ k0
        n1 = p1 & MASK32
        n2 = (p0 >> np.uint64(32)) ^ c[3] ^ k1
        n3 = p0 & MASK32
        c = [n0 & MASK32, n1, n2 & MASK32, n3]
        k0 = (k0 + np.uint64(W0)) & MASK32
        k1 = (k1 + np.uint64(W1)) & MASK32
    return np.stack([x.astype(np.uint32) for x in c])


def keep_threshold(p_dropout):
    return int(np.floor(np.float32(1.0 - np.float32(p_dropout)) * np.float32(65535.0)))


def rnd16(seed, offset, bh, rows, cols):
    """16-bit randoms for the (rows x cols) grid of one (batch, head): returns (len(rows), len(cols)) uint16."""
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    g = ((rows >> 5) << 2) | (((rows >> 4) & 1) << 1) | ((rows >> 2) & 1)
    slot = (rows & 3) | (((rows >> 3) & 1) << 2)
    G, C = np.meshgrid(g, cols, indexing="ij")
    ctr = (G.astype(np.uint64), C.astype(np.uint64),
           np.full(G.shape, bh, dtype=np.uint64), np.full(G.shape, (offset >> 2) & 0xFFFFFFFF, dtype=np.uint64))
    out = philox4x32(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF), rounds=7)  # (4, R, C)
    word = out[(slot >> 1)[:, None], np.arange(len(rows))[:, None], np.arange(len(cols))[None, :]]
    half = (slot & 1)[:, None]
    return ((word >> (16 * half).astype(np.uint32)) & 0xFFFF).astype(np.uint16)


def dropout_keep_mask(seed, offset, p_dropout, batch, nheads, seqlen_q, seqlen_k):
    """(batch, nheads, seqlen_q, seqlen_k) bool keep mask, rows/cols local to each sequence."""
    thr = keep_threshold(p_dropout)
    rows = np.arange(seqlen_q)
    cols = np.arange(seqlen_k)
    m = np.empty((batch, nheads, seqlen_q, seqlen_k), dtype=bool)
    for b in range(batch):
        for h in range(nheads):
            m[b, h] = rnd16(seed, offset, b * nheads + h, rows, cols) <= thr
    return m


def philox4x32_torch(c0, c1, c2, c3, k0, k1, rounds=7):
    """philox4x32 on int64 torch tensors holding uint32 values (any device): the same rounds as
    philox4x32 above; products wrap modulo 2^64 and the & masks recover the 32-bit halves."""
    m = 0xFFFFFFFF
    for _ in range(rounds):
        p0 = c0 * int(M0)
        p1 = c2 * int(M1)
        c0, c1, c2, c3 = ((p1 >> 32) & m) ^ c1 ^ k0, p1 & m, ((p0 >> 32) & m) ^ c3 ^ k1, p0 & m
        k0 = (k0 + W0) & m
        k1 = (k1 + W1) & m
    return c0, c1, c2, c3


def dropout_keep_mask_torch(seed, offset, p_dropout, batch, nheads, seqlen_q, seqlen_k, device):
    """dropout_keep_mask evaluated with torch on `device` (the exact-grid GPU tests need the
    8x12x2048x2048 mask in seconds): one Philox call per (b*H + h, g, col) covers the 8 rows of
    group g, word slot >> 1, half slot & 1, exactly as rnd16 maps them."""
    import torch
    thr = keep_threshold(p_dropout)
    rows = torch.arange(seqlen_q, device=device)
    g = ((rows >> 5) << 2) | (((rows >> 4) & 1) << 1) | ((rows >> 2) & 1)
    slot = (rows & 3) | (((rows >> 3) & 1) << 2)
    ng = int(g.max().item()) + 1
    gg = torch.arange(ng, device=device, dtype=torch.int64)[:, None].expand(ng, seqlen_k)
    cc = torch.arange(seqlen_k, device=device, dtype=torch.int64)[None, :].expand(ng, seqlen_k)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    c3 = torch.full_like(gg, (offset >> 2) & 0xFFFFFFFF)
    out = torch.empty((batch, nheads, seqlen_q, seqlen_k), dtype=torch.bool, device=device)
    for bh in range(batch * nheads):
        w = torch.stack(philox4x32_torch(gg, cc, torch.full_like(gg, bh), c3, k0, k1))   # (4, ng, Sk)
        word = w[(slot >> 1), g]                                                     # (Sq, Sk)
        r16 = (word >> (16 * (slot & 1))[:, None]) & 0xFFFF
        out[bh // nheads, bh % nheads] = r16 <= thr
    return out
