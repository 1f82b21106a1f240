"""GPU parity of the HIP rotary embedding (csrc/fa_rotary.hip) with the
oracle's restatement of the reference rotary (oracle/rotary_ref.py of flash_attn/rotary.py:22-41, 86-135): bit-exact forward and
backward (same rounding sequence), 1-D and 2-D tables, both sequence layouts, and the in-place
packed-qkv form used by FlashMHA."""
import pytest
import torch

from oracle.rotary_ref import apply_rotary_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rot():
    from flash_attn import rotary
    return rotary


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("seq_dimension", [-2, -3])
@pytest.mark.parametrize("D", [16, 64, 128])
def test_rotary_1d_bitexact(D, seq_dimension, dtype):
    rot = _rot()
    g = torch.Generator().manual_seed(D)
    B, H, S = 3, 4, 200
    shape = (B, H, S, D) if seq_dimension == -2 else (B, S, H, D)
    q = torch.randn(*shape, generator=g).to(dtype).to(DEV).requires_grad_()
    k = torch.randn(*shape, generator=g).to(dtype).to(DEV).requires_grad_()
    emb = rot.RotaryEmbedding(D).to(DEV)
    qh, kh = emb(q, k, seq_dimension=seq_dimension)
    cos, sin = emb.cos_sin_tables(S, DEV, dtype)
    qt = apply_rotary_ref(q, cos, sin, seq_dimension)
    kt = apply_rotary_ref(k, cos, sin, seq_dimension)
    assert torch.equal(qh, qt) and torch.equal(kh, kt)
    go = torch.randn(qh.shape, generator=g).to(dtype).to(DEV)
    (gq_h,) = torch.autograd.grad(qh, (q,), go)
    (gq_t,) = torch.autograd.grad(qt, (q,), go)
    assert torch.equal(gq_h, gq_t)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("seq_dimension", [-2, -3])
def test_rotary_2d_bitexact(seq_dimension, dtype):
    rot = _rot()
    g = torch.Generator().manual_seed(1)
    B, H, S, D = 2, 3, 16 * 16, 32
    shape = (B, H, S, D) if seq_dimension == -2 else (B, S, H, D)
    q = torch.randn(*shape, generator=g).to(dtype).to(DEV).requires_grad_()
    k = torch.randn(*shape, generator=g).to(dtype).to(DEV)
    emb = rot.RotaryEmbedding2D(D).to(DEV)
    qh, kh = emb(q, k, seq_dimension=seq_dimension)
    # the reference's grid-based expression, on the same device (so the same cos/sin tables)
    side = 16
    qq, kk = (q, k) if seq_dimension == -2 else (q.transpose(1, 2), k.transpose(1, 2))
    grid = lambda t: t.reshape(t.shape[0], t.shape[1], side, side, t.shape[-1])
    flat = lambda t: t.reshape(t.shape[0], t.shape[1], side * side, t.shape[-1])
    c1, s1 = emb.rotary_emb1d.cos_sin_tables(side, DEV, dtype)
    q0, q1 = qq.chunk(2, dim=-1)
    k0, k1 = kk.chunk(2, dim=-1)
    qt = torch.cat([flat(apply_rotary_ref(grid(q0), c1, s1, -2)),
                    flat(apply_rotary_ref(grid(q1), c1, s1, -3))], dim=-1)
    kt = torch.cat([flat(apply_rotary_ref(grid(k0), c1, s1, -2)),
                    flat(apply_rotary_ref(grid(k1), c1, s1, -3))], dim=-1)
    if seq_dimension == -3:
        qt, kt = qt.transpose(1, 2), kt.transpose(1, 2)
    assert torch.equal(qh, qt) and torch.equal(kh, kt)
    go = torch.randn(qh.shape, generator=g).to(dtype).to(DEV)
    assert torch.equal(torch.autograd.grad(qh, (q,), go)[0], torch.autograd.grad(qt, (q,), go)[0])


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("kind", ["1d", "2d"])
def test_rotary_qkv_inplace(kind, dtype):
    rot = _rot()
    g = torch.Generator().manual_seed(2)
    B, S, H, D = 2, 144, 3, 64
    w = torch.randn(B, S, 3 * H * D, generator=g).to(dtype).to(DEV).requires_grad_()
    emb = (rot.RotaryEmbedding(D) if kind == "1d" else rot.RotaryEmbedding2D(D)).to(DEV)
    cos, sin = emb.cos_sin_tables(S, DEV, dtype)
    base = w * 1.0                       # a non-leaf tensor, like the Wqkv output
    out = rot.apply_rotary_emb_qkv_(base, cos, sin, H, D).reshape(B, S, 3, H, D)
    ref_in = (w * 1.0).reshape(B, S, 3, H, D)
    q, k, v = ref_in.unbind(dim=2)
    ref = torch.stack([apply_rotary_ref(q, cos, sin, -3), apply_rotary_ref(k, cos, sin, -3), v], dim=2)
    assert torch.equal(out, ref)
    go = torch.randn(out.shape, generator=g).to(dtype).to(DEV)
    assert torch.equal(torch.autograd.grad(out, (w,), go)[0], torch.autograd.grad(ref, (w,), go)[0])


def test_rotary_invalid_args():
    from flash_attn import flash_attn_hip as hip
    x = torch.randn(1, 4, 1, 2, 12, device=DEV, dtype=torch.float16)
    cos = torch.ones(4, 12, device=DEV, dtype=torch.float16)
    with pytest.raises(RuntimeError, match="multiple of 8"):
        hip.rotary(x, x, cos, cos, (1, 4, 1, 2, 12), (96, 24, 24, 12), (96, 24, 24, 12), 1, False)
