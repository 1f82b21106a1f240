"""CPU tests: pin the oracle before trusting it (no GPU needed).

* Philox-4x32-10 against the Random123 known-answer vectors (numpy and C restatements);
  the 7-round stream used for dropout against itself across numpy / C.
* oracle/attention_ref.py against golden vectors produced by the REFERENCE's own
  attention_ref / get_dropout_fraction (tests/golden/make_golden.py), outputs, attention
  probabilities and fp32 gradients.
* the C tiled online-softmax restatement (oracle/fa_tiled.c) against attention_ref, including
  dropout, causal, var-len and empty sequences.
* the dropout fraction of the RNG over a large grid is within the reference's +-1 % band.
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle import philox, tiled
from oracle.attention_ref import attention_ref, get_dropout_fraction, max_err_bound, pad, unpad

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "attention_ref_golden.npz")

# Random123 kat_vectors for philox4x32_10 (ctr, key, expected)
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_philox_kat_numpy(ctr, key, expect):
    got = philox.philox4x32([[c] for c in ctr], key, rounds=10)[:, 0]
    assert tuple(int(x) for x in got) == expect


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_philox_kat_c(ctr, key, expect):
    assert tuple(tiled.philox(ctr, key, 10)) == expect


def test_rng_numpy_matches_c():
    rng = np.random.default_rng(0)
    for _ in range(50):
        seed = int(rng.integers(0, 2 ** 63))
        offset = int(rng.integers(0, 2 ** 20)) * 4
        bh = int(rng.integers(0, 1000))
        row, col = int(rng.integers(0, 5000)), int(rng.integers(0, 5000))
        assert int(philox.rnd16(seed, offset, bh, [row], [col])[0, 0]) == tiled.rnd16(seed, offset, bh, row, col)


@pytest.mark.parametrize("seed,offset,Sq,Sk", [(0x1234567890ABCDEF, 8, 200, 130), (2 ** 63 - 25, 4 * 77777, 97, 257)])
def test_torch_keep_mask_matches_numpy(seed, offset, Sq, Sk):
    """The torch restatement used by the exact-grid GPU tests equals the numpy oracle bit for bit."""
    ref = philox.dropout_keep_mask(seed, offset, 0.1, 2, 3, Sq, Sk)
    got = philox.dropout_keep_mask_torch(seed, offset, 0.1, 2, 3, Sq, Sk, "cpu").numpy()
    assert np.array_equal(ref, got)


def test_rng_element_map_is_bijective_per_call():
    """Each Philox call feeds 8 distinct rows of one column; all rows of a 32-block are covered."""
    rows = np.arange(64)
    g = ((rows >> 5) << 2) | (((rows >> 4) & 1) << 1) | ((rows >> 2) & 1)
    slot = (rows & 3) | (((rows >> 3) & 1) << 2)
    pairs = set(zip(g.tolist(), slot.tolist()))
    assert len(pairs) == 64


def test_dropout_fraction_band():
    p = 0.1
    keep = philox.dropout_keep_mask(42, 0, p, 2, 3, 512, 512)
    frac = 1.0 - keep.mean()
    assert 0.99 <= frac / p <= 1.01
    # different offsets give different streams
    keep2 = philox.dropout_keep_mask(42, 4, p, 1, 1, 64, 64)
    assert (keep2 != keep[0, 0, :64, :64]).any()


def _golden():
    if not os.path.exists(GOLDEN):
        pytest.skip("golden fixture missing (run tests/golden/make_golden.py)")
    return np.load(GOLDEN, allow_pickle=False)


def _case_names():
    if not os.path.exists(GOLDEN):
        return []
    z = np.load(GOLDEN, allow_pickle=False)
    return sorted({k.split("/")[0] for k in z.files})


@pytest.mark.parametrize("name", _case_names())
def test_attention_ref_matches_reference_golden(name):
    z = _golden()
    dt = getattr(torch, str(z[f"{name}/dtype"]))
    B, Sq, Sk, H, D, causal, seed, offset = [int(x) for x in z[f"{name}/meta"]]
    p, frac_ref = [float(x) for x in z[f"{name}/fparams"]]
    t = lambda key: torch.from_numpy(z[f"{name}/{key}"])
    q, k, v = (t("q").to(dt).requires_grad_(), t("k").to(dt).requires_grad_(), t("v").to(dt).requires_grad_())
    qmask, kmask, keep = t("qmask"), t("kmask"), t("keep")
    if p > 0:  # the stored keep mask was drawn from this build's RNG: it must reproduce exactly
        assert np.array_equal(philox.dropout_keep_mask(seed, offset, p, B, H, Sq, Sk), keep.numpy())
    o_ref, a_ref = attention_ref(q, k, v, qmask, kmask, p, keep, causal=bool(causal))
    o_pt, a_pt = attention_ref(q, k, v, qmask, kmask, p, keep, causal=bool(causal), upcast=False, reorder_ops=True)
    # the restatement must reproduce the reference oracle bit for bit (same ops, same order)
    assert torch.equal(o_ref.float(), t("out_ref"))
    assert torch.equal(a_ref.float(), t("attn_ref"))
    assert torch.equal(o_pt.float(), t("out_pt"))
    assert torch.equal(a_pt.float(), t("attn_pt"))
    assert get_dropout_fraction(keep, qmask, kmask, causal=bool(causal)).item() == pytest.approx(frac_ref, abs=1e-7)
    g = t("g").to(dt)
    dq, dk, dv = torch.autograd.grad(o_ref, (q, k, v), g)
    assert torch.equal(dq.float(), t("dq_ref"))
    assert torch.equal(dk.float(), t("dk_ref"))
    assert torch.equal(dv.float(), t("dv_ref"))


def _tiled_vs_ref(B, Sq, Sk, H, D, causal, p, mode="random", seed=0, round_p=0):
    gen = torch.Generator().manual_seed(seed)
    q = torch.randn(B, Sq, H, D, generator=gen)
    k = torch.randn(B, Sk, H, D, generator=gen)
    v = torch.randn(B, Sk, H, D, generator=gen)
    from oracle.attention_ref import generate_random_padding_mask
    qmask = generate_random_padding_mask(Sq, B, "cpu", mode, generator=gen)
    kmask = generate_random_padding_mask(Sk, B, "cpu", mode, generator=gen)
    qu, iq, cuq, mq = unpad(q, qmask)
    ku, ik, cuk, mk = unpad(k, kmask)
    vu, _, _, _ = unpad(v, kmask)
    rng_seed, rng_off = 777, 12
    out_u, lse = tiled.fwd(qu.numpy(), ku.numpy(), vu.numpy(), cuq.numpy(), cuk.numpy(), D ** -0.5, p, rng_seed,
                           rng_off, causal, round_p)
    keep = None
    if p > 0:
        keep = torch.ones(B, H, Sq, Sk, dtype=torch.bool)
        km = philox.dropout_keep_mask(rng_seed, rng_off, p, B, H, max(mq, 1), max(mk, 1))
        keep[:, :, :km.shape[2], :km.shape[3]] = torch.from_numpy(km)
    o_ref, _ = attention_ref(q, k, v, qmask, kmask, p, keep, causal=causal)
    out = pad(torch.from_numpy(out_u), iq, B, Sq)
    return out, o_ref


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("p", [0.0, 0.17])
@pytest.mark.parametrize("Sq,Sk", [(97, 97), (130, 200), (200, 70)])
def test_tiled_c_oracle_matches_attention_ref(Sq, Sk, p, causal):
    out, ref = _tiled_vs_ref(2, Sq, Sk, 2, 32, causal, p)
    assert (out - ref).abs().max().item() < 2e-5


def test_tiled_c_oracle_empty_key_set():
    q = np.random.default_rng(0).standard_normal((3, 1, 16)).astype(np.float32)
    k = np.zeros((0, 1, 16), np.float32)
    out, lse = tiled.fwd(q, k, k, np.array([0, 3], np.int32), np.array([0, 0], np.int32), 0.25)
    assert (out == 0).all() and np.isneginf(lse[0, 0, :3]).all()


def test_tiled_c_oracle_lse():
    gen = torch.Generator().manual_seed(1)
    q, k, v = (torch.randn(150, 2, 64, generator=gen) for _ in range(3))
    cu = np.array([0, 150], np.int32)
    out, lse = tiled.fwd(q.numpy(), k.numpy(), v.numpy(), cu, cu, 0.125)
    s = torch.einsum("thd,shd->hts", q, k) * 0.125
    assert np.allclose(lse[0], torch.logsumexp(s, -1).numpy(), atol=1e-5)


def test_max_err_bound_floor():
    a = torch.zeros(3)
    assert max_err_bound(a, a) == 0.0
    assert max_err_bound(a, a, floor=1e-5) == 1e-5


def test_benchmark_attention_restatement_matches_attention_ref():
    """oracle.attention_pytorch_bench (the reference benchmark's naive attention, bench.py's CPU
    baseline: benchmarks/benchmark_flash_attention.py:14-36) computes what the pinned attention_ref
    computes with the scale on k (reorder_ops), bit for bit at fp32, with a key mask and causal."""
    from oracle.attention_ref import attention_pytorch_bench, attention_ref
    g = torch.Generator().manual_seed(3)
    B, S, H, D = 2, 96, 3, 32
    qkv = torch.randn(B, S, 3, H, D, generator=g)
    mask = torch.arange(S)[None, :] < torch.tensor([[S], [S - 17]])
    for causal in (False, True):
        out = attention_pytorch_bench(qkv, mask, 0.0, upcast=True, causal=causal)
        q, k, v = qkv.unbind(2)
        ref, _ = attention_ref(q, k, v, key_padding_mask=mask, causal=causal, reorder_ops=True)
        assert torch.equal(out, ref)
