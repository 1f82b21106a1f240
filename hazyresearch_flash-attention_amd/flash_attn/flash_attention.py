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


class FlashAttnRotaryQKVFunc:
    """Entry point of the fused-rotary attention: `apply(qkv, cos, sin, dropout_p, softmax_scale,
    causal)` runs the compiled autograd function (csrc/fa_torch.cpp FlashAttnRotaryQKVFn, one
    pybind11 call) when the binding is built and qkv is on the GPU, else the Python one below
    (same kernels, same results)."""

    @staticmethod
    def apply(qkv, cos, sin, dropout_p, softmax_scale, causal):
        from flash_attn import flash_attn_hip as hip
        C = hip._C
        if C is None or not qkv.is_cuda:
            return _FlashAttnRotaryQKVFuncPy.apply(qkv, cos, sin, dropout_p, softmax_scale, causal)
        B, S, _, H, D = qkv.shape
        seed, offset, od = hip._rng_args(dropout_p, qkv.device)
        return C.flash_attn_rotary_qkv_func(qkv, cos, sin, _uniform_cu_seqlens(B, S, qkv.device), dropout_p,
                                            D ** -0.5 if softmax_scale is None else softmax_scale, causal,
                                            seed, offset, od, hip._impl())


class _FlashAttnRotaryQKVFuncPy(torch.autograd.Function):
    """Attention over a padded, contiguous qkv (B, S, 3, H, D) with rotary embeddings fused into
    the forward (README.md:56 "Fuse rotary embedding"; rotation = rotary.py:31-41):
    * forward: where fa_fwd takes an assembly kernel (no dropout, head_dim <= 64, 80, 96, 128)
      one fa_rotary pass rotates q and k into a (B, S, 2, H, D) buffer and the assembly forward reads
      it (measured faster than the HIP forward rotating q at its load); otherwise k
      is rotated by one fa_rotary pass into a (B, S, H, D) buffer (the backward needs it anyway) and
      q by the HIP fa_fwd at its one-time fragment load, never written to HBM. The operands are
      bit-identical to rotating q and k first (same rounding, fa_common.h rotary8).
    * backward: q is rotated once more (fa_rotary), the attention backward runs on (q_rot, k_rot,
      v), and dq, dk are rotated back in place (the autograd transpose, fa_rotary inverse)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, dropout_p, softmax_scale, causal):
        from flash_attn import flash_attn_hip as hip
        from flash_attn.flash_attn_interface import _reserve
        B, S, _, H, D = qkv.shape
        assert qkv.is_contiguous()
        cos, sin = cos[:S].contiguous(), sin[:S].contiguous()
        if softmax_scale is None:
            softmax_scale = D ** (-0.5)
        rng_state = _reserve(dropout_p, qkv.device)
        flat = qkv.view(B * S, 3, H, D)
        cu = _uniform_cu_seqlens(B, S, qkv.device)
        # the route follows the kernel this call will really take: the thread's force_impl applies
        # to the route decision and to the forward alike
        impl = hip._impl()
        name = hip.fwd_kernel_name(B, H, D, S, S, qkv.dtype, causal, dropout_p, row_elems=3 * H * D, impl=impl)
        if name is not None and name.endswith("_asm"):
            # the Q rotation at the Q load exists in the HIP forward only: where fa_fwd takes an
            # assembly kernel, one fa_rotary pass rotates q and k (B, S, 2, H, D) and the assembly
            # forward reads them (the backward reuses both: no second q pass)
            qk_rot = torch.empty((B, S, 2, H, D), dtype=qkv.dtype, device=qkv.device)
            hip.rotary(qkv, qk_rot, cos, sin, (B, S, 2, H, D), (S * 3 * H * D, 3 * H * D, H * D, D),
                       (S * 2 * H * D, 2 * H * D, H * D, D), 2, False)
            qk = qk_rot.view(B * S, 2, H, D)
            out, lse = hip.fwd(qk[:, 0], qk[:, 1], flat[:, 2], cu, cu, S, S, dropout_p, softmax_scale,
                               False, causal, False, None, rng_state=rng_state, impl=impl)
            k_rot = qk_rot
        else:
            st = (S * 3 * H * D, 3 * H * D, 0, D)
            k_rot = torch.empty((B, S, H, D), dtype=qkv.dtype, device=qkv.device)
            hip.rotary(qkv[:, :, 1], k_rot, cos, sin, (B, S, 1, H, D), st, (S * H * D, H * D, 0, D), 1, False)
            out, lse = hip.fwd(flat[:, 0], k_rot.view(B * S, H, D), flat[:, 2], cu, cu, S, S, dropout_p,
                               softmax_scale, False, causal, False, None, rng_state=rng_state, rotary=(cos, sin),
                               impl=impl)
        ctx.save_for_backward(qkv, k_rot, out, lse, cos, sin, cu)
        ctx.rng_state, ctx.dropout_p, ctx.softmax_scale, ctx.causal = rng_state, dropout_p, softmax_scale, causal
        return out.view(B, S, H, D)

    @staticmethod
    def backward(ctx, dout):
        from flash_attn import flash_attn_hip as hip
        qkv, k_rot, out, lse, cos, sin, cu = ctx.saved_tensors
        B, S, _, H, D = qkv.shape
        if k_rot.dim() == 5:     # (B, S, 2, H, D): q and k rotated by the forward (assembly forward)
            qk = k_rot.view(B * S, 2, H, D)
            q_rot, k_rot = qk[:, 0], qk[:, 1]
        else:
            st = (S * 3 * H * D, 3 * H * D, 0, D)
            q_rot = torch.empty((B, S, H, D), dtype=qkv.dtype, device=qkv.device)
            hip.rotary(qkv[:, :, 0], q_rot, cos, sin, (B, S, 1, H, D), st, (S * H * D, H * D, 0, D), 1, False)
            q_rot, k_rot = q_rot.view(B * S, H, D), k_rot.view(B * S, H, D)
        dqkv = torch.empty_like(qkv)
        d = dqkv.view(B * S, 3, H, D)
        hip.bwd(dout.reshape(B * S, H, D), q_rot, k_rot,
                qkv.view(B * S, 3, H, D)[:, 2], out, lse, d[:, 0], d[:, 1], d[:, 2], cu, cu, S, S, ctx.dropout_p,
                ctx.softmax_scale, False, ctx.causal, None, rng_state=ctx.rng_state)
        st3 = (S * 3 * H * D, 3 * H * D, H * D, D)
        hip.rotary(dqkv, dqkv, cos, sin, (B, S, 3, H, D), st3, st3, 2, True)   # dq, dk back; dv as is
        return dqkv, None, None, None, None, None


_cu_cache = {}
_CU_CACHE_MAX = 256


def _uniform_cu_seqlens(B, S, device):
    """cu_seqlens of B sequences of length S (cached per shape and device: one arange launch per
    shape instead of one per call; the tensor is only read by the kernels).

    Graph safety: entries are never evicted (a captured graph may hold the address of a cached
    tensor; freeing it would let replays read reused memory as sequence bounds), past the cap new
    shapes simply get a fresh tensor; and while the current stream is capturing, the tensor is made
    fresh inside the capture (its arange is replayed with the graph) and not cached, so an eager
    call never sees graph-pool memory that only a replay initialises."""
    capturing = device.type == "cuda" and torch.cuda.is_current_stream_capturing()
    key = (B, S, device)
    cu = None if capturing else _cu_cache.get(key)
    if cu is None:
        cu = torch.arange(0, (B + 1) * S, S, dtype=torch.int32, device=device)
        if not capturing and len(_cu_cache) < _CU_CACHE_MAX:
            _cu_cache[key] = cu
    return cu


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
        fused = (self.use_rotary_emb and qkv.is_cuda and qkv.is_contiguous() and key_padding_mask is None
                 and qkv.dtype in (torch.float16, torch.bfloat16) and self.head_dim % 8 == 0)
        if fused:
            cos, sin = self.rotary_emb.cos_sin_tables(s, qkv.device, qkv.dtype)
            # the kernel's Q load rotates all head_dim features: tables narrower than the head go
            # through the separate pass below
            fused = cos.shape[-1] >= self.head_dim and cos.shape[0] >= s
        if fused:
            # fused rotary: q rotated inside the attention kernel, k by one half-size pass
            dropout_p = self.inner_attn.dropout_p if self.inner_attn.training else 0.0
            context = FlashAttnRotaryQKVFunc.apply(qkv.view(b, s, 3, self.num_heads, self.head_dim), cos, sin,
                                                   dropout_p, self.inner_attn.softmax_scale, self.causal)
            return self.out_proj(context.reshape(b, s, -1)), None
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
