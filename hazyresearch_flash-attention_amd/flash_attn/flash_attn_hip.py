"""Host binding of libfa_hip.so — the MI355X replacement of the reference's `flash_attn_cuda`.

`fwd` keeps the exact signature and return value of the reference's pybind11 `fwd`
(csrc/flash_attn/fmha_api.cpp:112-125, 239-241): ``[out, softmax_lse, (S_dmask)]``, and `bwd`
the signature the reference interface calls but never bound (flash_attn/flash_attn_interface.py:31-33),
returning ``softmax_d``. Both accept one extra keyword, ``rng_state=(seed, offset)``, so that
the autograd layer can replay a forward's dropout mask without saving the whole RNG state
(a third element, a device word, carries the offset advance of a captured hipGraph replay).

Dense `fwd` / `bwd` calls go through the compiled module `_fa_C` (csrc/fa_torch.cpp: checks,
allocation and launch in C++, as the reference's pybind11 binding does); block-sparse layouts,
fused rotary and the helpers load the library with ctypes (plain C ABI, include/fa_hip.h). Both
drive the same libfa_hip.so. There is no CPU fallback: if the shared object is missing every
call raises.
"""
import contextlib
import ctypes
import math
import os
import struct
import threading

import torch

_LIB_PATH = os.environ.get("FA_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfa_hip.so"))

# compiled fwd/bwd binding (links the in-tree libfa_hip.so; not used when FA_HIP_LIB points elsewhere)
_C = None
if "FA_HIP_LIB" not in os.environ:
    try:
        from . import _fa_C as _C
    except ImportError:
        _C = None

FA_DTYPE_FP16 = 0
FA_DTYPE_BF16 = 1
FA_QUERY_BWD_WORKSPACE = 1
FA_QUERY_MAX_HEAD_DIM = 2
FA_QUERY_RNG_INCREMENT = 3
FA_QUERY_FWD_ARGS_SIZE = 4
FA_QUERY_BWD_ARGS_SIZE = 5
FA_QUERY_MASK_ARGS_SIZE = 6
FA_QUERY_PAD_WORKSPACE = 7
FA_QUERY_ROTARY_ARGS_SIZE = 8
FA_QUERY_BWD_WORKSPACE_NEEDED = 9
FA_QUERY_ASM_LAUNCHES = 10

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_u64 = ctypes.c_uint64
_f32 = ctypes.c_float


class FaFwdArgs(ctypes.Structure):
    """ctypes mirror of FaFwdArgs (include/fa_hip.h)."""
    _fields_ = [
        ("q", _vp), ("k", _vp), ("v", _vp), ("o", _vp), ("softmax_lse", _vp), ("s_dmask", _vp),
        ("cu_seqlens_q", _vp), ("cu_seqlens_k", _vp),
        ("q_row_stride", _i64), ("q_head_stride", _i64),
        ("k_row_stride", _i64), ("k_head_stride", _i64),
        ("v_row_stride", _i64), ("v_head_stride", _i64),
        ("o_row_stride", _i64), ("o_head_stride", _i64),
        ("batch", _i32), ("nheads", _i32), ("head_dim", _i32),
        ("max_seqlen_q", _i32), ("max_seqlen_k", _i32), ("lse_stride", _i32),
        ("s_rows", _i32), ("s_cols", _i32),
        ("softmax_scale", _f32), ("p_dropout", _f32),
        ("rng_seed", _u64), ("rng_offset", _u64), ("rng_offset_dev", _vp),
        ("is_causal", _i32), ("dtype", _i32),
        ("rot_cos", _vp), ("rot_sin", _vp), ("rot_stride", _i64),
        ("impl", _i32), ("reserved", _i32),
    ]


FA_IMPL_AUTO = 0
FA_IMPL_HIP = 1
FA_IMPL_ASM4 = 2    # the one-wave-per-SIMD assembly forward where eligible (tests, A/B)
FA_IMPL_ASM8 = 3    # reserved: the two-waves-per-SIMD form is an A/B generator build, not in the library
FA_IMPL_ASM4P = 4   # the persistent one-wave-per-SIMD assembly forward where eligible (non-causal)


class FaBwdArgs(ctypes.Structure):
    """ctypes mirror of FaBwdArgs (include/fa_hip.h)."""
    _fields_ = [
        ("dout", _vp), ("q", _vp), ("k", _vp), ("v", _vp), ("out", _vp), ("softmax_lse", _vp),
        ("dq", _vp), ("dk", _vp), ("dv", _vp), ("softmax_d", _vp), ("dq_accum", _vp),
        ("cu_seqlens_q", _vp), ("cu_seqlens_k", _vp),
        ("do_row_stride", _i64), ("do_head_stride", _i64),
        ("q_row_stride", _i64), ("q_head_stride", _i64),
        ("k_row_stride", _i64), ("k_head_stride", _i64),
        ("v_row_stride", _i64), ("v_head_stride", _i64),
        ("o_row_stride", _i64), ("o_head_stride", _i64),
        ("dq_row_stride", _i64), ("dq_head_stride", _i64),
        ("dk_row_stride", _i64), ("dk_head_stride", _i64),
        ("dv_row_stride", _i64), ("dv_head_stride", _i64),
        ("batch", _i32), ("nheads", _i32), ("head_dim", _i32),
        ("max_seqlen_q", _i32), ("max_seqlen_k", _i32),
        ("total_q", _i32), ("lse_stride", _i32),
        ("softmax_scale", _f32), ("p_dropout", _f32),
        ("rng_seed", _u64), ("rng_offset", _u64), ("rng_offset_dev", _vp),
        ("is_causal", _i32), ("dtype", _i32),
    ]


class FaBlockMask(ctypes.Structure):
    """ctypes mirror of FaBlockMask (include/fa_hip.h): 0/1 bytes, 16-query x 256-key blocks."""
    _fields_ = [("mask", _vp), ("row_stride", _i64), ("rows", _i32), ("cols", _i32)]


class FaRotaryArgs(ctypes.Structure):
    """ctypes mirror of FaRotaryArgs (include/fa_hip.h)."""
    _fields_ = [("x", _vp), ("y", _vp), ("cos", _vp), ("sin", _vp),
                ("x_strides", _i64 * 4), ("y_strides", _i64 * 4), ("table_stride", _i64),
                ("batch", _i32), ("seqlen", _i32), ("nslot", _i32), ("nheads", _i32), ("head_dim", _i32),
                ("nrot", _i32), ("inverse", _i32), ("dtype", _i32)]


_lib_handle = None


def lib():
    """Load libfa_hip.so (once). Raises if it is missing: there is no fallback path."""
    global _lib_handle
    if _lib_handle is None:
        if not os.path.exists(_LIB_PATH):
            raise ImportError(
                f"libfa_hip.so not found at {_LIB_PATH}; build it with "
                f"`python hazyresearch_flash-attention_amd/build.py`")
        h = ctypes.CDLL(_LIB_PATH)
        h.fa_fwd.argtypes = [ctypes.POINTER(FaFwdArgs), _vp]
        h.fa_fwd.restype = ctypes.c_int
        h.fa_bwd.argtypes = [ctypes.POINTER(FaBwdArgs), _vp]
        h.fa_bwd.restype = ctypes.c_int
        h.fa_fwd_block.argtypes = [ctypes.POINTER(FaFwdArgs), ctypes.POINTER(FaBlockMask), _vp]
        h.fa_fwd_block.restype = ctypes.c_int
        h.fa_bwd_block.argtypes = [ctypes.POINTER(FaBwdArgs), ctypes.POINTER(FaBlockMask), _vp]
        h.fa_bwd_block.restype = ctypes.c_int
        h.fa_index_first_axis.argtypes = [_vp, _i64, _i64, _vp, _i64, _vp, _i64, _i64, _vp]
        h.fa_index_first_axis.restype = ctypes.c_int
        h.fa_index_put_first_axis.argtypes = [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp]
        h.fa_index_put_first_axis.restype = ctypes.c_int
        h.fa_index_add_first_axis.argtypes = [_vp, _i64, _vp, _i64, _vp, _i64, _i64, _i64, _i32, _vp]
        h.fa_index_add_first_axis.restype = ctypes.c_int
        h.fa_rotary.argtypes = [ctypes.POINTER(FaRotaryArgs), _vp]
        h.fa_rotary.restype = ctypes.c_int
        h.fa_query.argtypes = [ctypes.c_int, _i64, _i64, _i64]
        h.fa_query.restype = _i64
        h.fa_last_error.argtypes = []
        h.fa_last_error.restype = ctypes.c_char_p
        h.fa_version.argtypes = []
        h.fa_version.restype = ctypes.c_char_p
        h.fa_fwd_kernel_name.argtypes = [ctypes.POINTER(FaFwdArgs)]
        h.fa_fwd_kernel_name.restype = ctypes.c_char_p
        if h.fa_query(FA_QUERY_FWD_ARGS_SIZE, 0, 0, 0) != ctypes.sizeof(FaFwdArgs):
            raise ImportError("FaFwdArgs layout mismatch between fa_hip.h and flash_attn_hip.py")
        if h.fa_query(FA_QUERY_BWD_ARGS_SIZE, 0, 0, 0) != ctypes.sizeof(FaBwdArgs):
            raise ImportError("FaBwdArgs layout mismatch between fa_hip.h and flash_attn_hip.py")
        if h.fa_query(FA_QUERY_ROTARY_ARGS_SIZE, 0, 0, 0) != ctypes.sizeof(FaRotaryArgs):
            raise ImportError("FaRotaryArgs layout mismatch between fa_hip.h and flash_attn_hip.py")
        if h.fa_query(FA_QUERY_MASK_ARGS_SIZE, 0, 0, 0) != ctypes.sizeof(FaBlockMask):
            raise ImportError("FaBlockMask layout mismatch between fa_hip.h and flash_attn_hip.py")
        _lib_handle = h
    return _lib_handle


def _check(cond, msg):
    # TORCH_CHECK raises RuntimeError (fmha_api.cpp:131-170); keep that error type.
    if not cond:
        raise RuntimeError(msg)


def _dtype_code(t):
    if t == torch.float16:
        return FA_DTYPE_FP16
    if t == torch.bfloat16:
        return FA_DTYPE_BF16
    raise RuntimeError(f"FlashAttention only supports fp16 and bf16, got {t}")


def _round16(x):
    return (x + 15) // 16 * 16


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream_ptr(device):
    if _raw_stream is not None:
        return _raw_stream(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def _packer(cls):
    """A struct.Struct whose layout equals the ctypes mirror `cls` (explicit padding), so a call
    fills the whole argument block with one pack_into instead of one ctypes setattr per field."""
    codes = {_vp: "Q", _i64: "q", _i32: "i", _u64: "Q", _f32: "f"}
    fmt, off = "<", 0
    for name, typ in cls._fields_:
        o = getattr(cls, name).offset
        if o > off:
            fmt += f"{o - off}x"
        if issubclass(typ, ctypes.Array):
            fmt += f"{typ._length_}{codes[typ._type_]}"
        else:
            fmt += codes[typ]
        off = o + ctypes.sizeof(typ)
    if ctypes.sizeof(cls) > off:
        fmt += f"{ctypes.sizeof(cls) - off}x"
    st = struct.Struct(fmt)
    assert st.size == ctypes.sizeof(cls)
    return st


_packers = {}


def _raw_call(cls, symbol, nargs=2):
    """(packer, per-thread argument buffer, its address, raw `symbol` taking the address and
    nargs-1 further pointers) for the argument struct `cls`."""
    key = (cls, symbol)
    c = getattr(_tls, "raw", {}).get(key)
    if c is None:
        st = _packers.get(cls)
        if st is None:
            st = _packers[cls] = _packer(cls)
        buf = ctypes.create_string_buffer(st.size)
        fn = lib()[symbol]              # a second prototype of the same symbol, taking the address
        fn.argtypes = [_vp] * nargs
        fn.restype = ctypes.c_int
        c = (st, buf, ctypes.addressof(buf), fn)
        if not hasattr(_tls, "raw"):
            _tls.raw = {}
        _tls.raw[key] = c
    return c


def _fwd_call():
    return _raw_call(FaFwdArgs, "fa_fwd")


_tls = threading.local()


@contextlib.contextmanager
def force_impl(impl):
    """Within the block, forward calls of this thread that leave `impl` at FA_IMPL_AUTO use `impl`
    instead (e.g. FA_IMPL_HIP: the HIP kernels for every shape, so that a result can be compared
    bit for bit with a path the assembly forward does not serve, such as fused rotary)."""
    prev = getattr(_tls, "impl", FA_IMPL_AUTO)
    _tls.impl = impl
    try:
        yield
    finally:
        _tls.impl = prev


def _on_device(dev):
    # the reference runs under a CUDAGuard for q's device (fmha_api.cpp:184)
    if dev.index is None or dev.index == torch.cuda.current_device():
        return contextlib.nullcontext()
    return torch.cuda.device(dev)


_rng_lock = threading.Lock()
_graph_ctr = {}   # device index -> int64 (1,) device counter advanced by captured graphs
GRAPH_RNG_BASE = 1 << 33   # Philox offset of captured launches (the kernels use offset >> 2 as a 32-bit counter)


def _dev_index(device):
    return device.index if device.index is not None else torch.cuda.current_device()


def _graph_counter(device):
    """The per-device counter word that captured dropout launches advance (allocated eagerly: an
    allocation made during capture would be re-initialised by every replay)."""
    idx = _dev_index(device)
    c = _graph_ctr.get(idx)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(
                "flash_attn: dropout inside hipGraph capture needs one eager (warm-up) call of the "
                "attention on this device before capture, as torch.cuda.graph recommends")
        c = torch.zeros(1, dtype=torch.int64, device=torch.device("cuda", idx))
        _graph_ctr[idx] = c
    return c


def reserve_rng(device, gen=None, increment=None):
    """Reserve a Philox (seed, offset) pair from the torch generator, like
    `gen->philox_cuda_state(counter_offset)` under the generator mutex (fmha_api.cpp:228-235).

    Returns (seed, offset, offset_dev). offset_dev is None in eager mode. Under hipGraph capture
    (where the reference's PhiloxCudaState reads its offset from device memory) it is a fresh
    one-word device tensor that the captured graph sets, on every replay, from a per-device
    counter advanced by `increment`; the kernels add it to `offset`, so each replay draws a new
    dropout mask and the backward (which gets the same word) replays its forward's mask."""
    if increment is None:
        increment = 4
    if gen is None:
        gen = torch.cuda.default_generators[_dev_index(device)]
    capturing = torch.cuda.is_current_stream_capturing()
    ctr = _graph_counter(device) if capturing or _dev_index(device) not in _graph_ctr else None
    offset_dev = None
    if capturing:
        # the generator's offset cannot be read or advanced during capture: captured launches
        # draw from their own Philox sub-stream (offset GRAPH_RNG_BASE + the device counter),
        # disjoint from the eager offsets below 2^33
        seed = gen.initial_seed()
        offset = GRAPH_RNG_BASE
        ctr.add_(increment)                       # captured: runs on every replay
        offset_dev = torch.empty_like(ctr)        # graph-pool word owned by this call
        offset_dev.copy_(ctr)
    else:
        with _rng_lock:
            seed = gen.initial_seed()
            offset = gen.get_offset()
            gen.set_offset(offset + increment)
        if offset + increment > GRAPH_RNG_BASE:
            # eager offsets must stay below the captured sub-stream (and offset >> 2 within the
            # kernels' 32-bit counter word), or eager and replayed dropout masks could repeat
            raise RuntimeError("flash_attn: the CUDA generator's Philox offset passed 2^33; "
                               "re-seed the generator (torch.cuda.manual_seed) to continue with dropout")
    return int(seed) & 0xFFFFFFFFFFFFFFFF, int(offset), offset_dev


def _rng_args(p_dropout, device):
    """(seed, offset, device word or None) for one dropout call (reserve_rng), zeros without dropout:
    the arguments the compiled autograd functions (_fa_C) take and save for their backward."""
    if p_dropout > 0.0:
        return reserve_rng(device)
    return 0, 0, None


def _impl():
    return getattr(_tls, "impl", FA_IMPL_AUTO)


def _unpack_rng(rng_state):
    seed, offset = rng_state[0], rng_state[1]
    dev_word = rng_state[2] if len(rng_state) > 2 else None
    return seed, offset, (dev_word.data_ptr() if dev_word is not None else None)


def _rows_ok(t):
    """True when every (row, head) slice of a (rows, H, D) tensor is its own contiguous D-run and
    rows do not overlap: the kernels address rows through buffer descriptors sized
    seqlen * row_stride, which a broadcast (stride 0) or overlapping row stride breaks."""
    if t.stride(-1) != 1:
        return False
    n, h, d = t.shape
    row_extent = (h - 1) * t.stride(1) + d if h > 0 else d
    return t.stride(0) >= max(row_extent, d) and (h <= 1 or t.stride(1) >= d)


def _rows_input(t):
    return t if _rows_ok(t) else t.contiguous()


_ws_needed = {}


def _bwd_needs_workspace(head_dim, dropout, sparse):
    key = (head_dim, bool(dropout), bool(sparse))
    v = _ws_needed.get(key)
    if v is None:
        v = bool(lib().fa_query(FA_QUERY_BWD_WORKSPACE_NEEDED, head_dim, int(dropout), int(sparse)))
        _ws_needed[key] = v
    return v


def _raise(rc, what):
    msg = lib().fa_last_error().decode()
    raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def _mask_struct(layout, dev):
    """FaBlockMask for a 0/1 layout tensor (rows = 16-query blocks, cols = 256-key blocks)."""
    _check(layout.dim() == 2, "blockmask layout must be 2-D (seqlen/16, seqlen/256)")
    _check(layout.device == dev, "blockmask must be on the device of q")
    if layout.dtype != torch.uint8 or layout.stride(-1) != 1:
        layout = layout.to(torch.uint8).contiguous()
    m = FaBlockMask()
    m.mask, m.row_stride, m.rows, m.cols = layout.data_ptr(), layout.stride(0), layout.shape[0], layout.shape[1]
    return m, layout


def fwd(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, p_dropout, softmax_scale,
        zero_tensors, is_causal, return_softmax, gen, rng_state=None, layout=None, rotary=None, impl=FA_IMPL_AUTO):
    """Forward pass; same arguments and result as the reference's `flash_attn_cuda.fwd`.
    `layout` (optional, 0/1 (seqlen/16, seqlen/256) on the device) selects the block-sparse kernel.
    `rotary` (optional (cos, sin) tables, (>= max_seqlen_q, >= D) in q's dtype) rotates q inside
    the kernel at its load (fused rotary, rotary.py:31-41); k must come rotated already.
    `impl` (FA_IMPL_AUTO / FA_IMPL_HIP) picks the kernel family (include/fa_hip.h)."""
    if impl == FA_IMPL_AUTO:
        impl = getattr(_tls, "impl", FA_IMPL_AUTO)
    if _C is not None and layout is None and rotary is None and q.is_cuda:
        if p_dropout > 0.0:
            seed, offset, offset_dev = _unpack_rng(rng_state if rng_state is not None else reserve_rng(q.device, gen))
        else:
            seed, offset, offset_dev = 0, 0, None
        return _C.fwd(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, p_dropout, softmax_scale,
                      zero_tensors, is_causal, return_softmax, seed, offset, offset_dev or 0, impl)
    qdt = q.dtype
    dt = _dtype_code(qdt)
    _check(k.dtype == qdt and v.dtype == qdt, "q, k, v must have the same dtype")
    _check(cu_seqlens_q.dtype == torch.int32 and cu_seqlens_k.dtype == torch.int32, "cu_seqlens must be int32")
    _check(q.is_cuda and k.is_cuda and v.is_cuda and cu_seqlens_q.is_cuda and cu_seqlens_k.is_cuda,
           "all tensors must be on the GPU")
    _check(q.dim() == 3 and k.dim() == 3 and v.dim() == 3, "q, k, v must be (total, nheads, headdim)")
    qs, ks, vs = q.stride(), k.stride(), v.stride()
    _check(qs[2] == 1 and ks[2] == 1 and vs[2] == 1, "last dimension must be contiguous")
    _check(cu_seqlens_q.is_contiguous() and cu_seqlens_k.is_contiguous(), "cu_seqlens must be contiguous")
    if not _rows_ok(q):
        q = q.contiguous()
        qs = q.stride()
    if not _rows_ok(k):
        k = k.contiguous()
        ks = k.stride()
    if not _rows_ok(v):
        v = v.contiguous()
        vs = v.stride()
    batch = cu_seqlens_q.numel() - 1
    total_q, nheads, head_dim = q.shape
    kshape = k.shape
    total_k = kshape[0]
    _check(batch > 0, "batch_size must be positive")
    _check(head_dim % 8 == 0 and head_dim <= 128, "head_size must be a multiple of 8 and <= 128")
    _check(tuple(kshape) == (total_k, nheads, head_dim) and tuple(v.shape) == (total_k, nheads, head_dim),
           "k, v must have shape (total_k, nheads, headdim)")
    _check(cu_seqlens_k.numel() == batch + 1, "cu_seqlens_k must have shape (batch_size + 1)")
    _check(0.0 <= p_dropout < 1.0, "dropout_p must be in [0, 1)")
    max_seqlen_q = int(max_seqlen_q)
    max_seqlen_k = int(max_seqlen_k)
    dev = q.device

    with _on_device(dev):
        o = torch.empty((total_q, nheads, head_dim), dtype=qdt, device=dev)
        lse_stride = max(_round16(max_seqlen_q), 16)
        lse = torch.empty((batch, nheads, lse_stride), dtype=torch.float32, device=dev)
        s = None
        if return_softmax:
            s = torch.empty((batch, nheads, lse_stride, max(_round16(max_seqlen_k), 16)), dtype=qdt, device=dev)
        if zero_tensors:
            o.zero_()
            lse.fill_(-math.inf)
            if s is not None:
                s.zero_()
        if p_dropout > 0.0:
            seed, offset, offset_dev = _unpack_rng(rng_state if rng_state is not None else reserve_rng(dev, gen))
        else:
            seed, offset, offset_dev = 0, 0, None
        rot_cos = rot_sin = 0
        rot_stride = 0
        if rotary is not None:
            cos, sin = rotary
            _check(cos.dtype == qdt and sin.dtype == qdt and cos.is_cuda and sin.is_cuda,
                   "rotary tables must be on the GPU in q's dtype")
            _check(cos.dim() == 2 and cos.stride(-1) == 1 and cos.stride() == sin.stride() and cos.shape == sin.shape
                   and cos.shape[0] >= max_seqlen_q and cos.shape[1] >= head_dim,
                   "rotary tables must be (>= max_seqlen_q, >= head_dim) with one row stride")
            rot_cos, rot_sin, rot_stride = cos.data_ptr(), sin.data_ptr(), cos.stride(0)
        # FaFwdArgs field order (include/fa_hip.h), packed in one call
        packer, buf, addr, raw_fwd = _fwd_call()
        nh_d = nheads * head_dim
        packer.pack_into(
            buf, 0, q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
            s.data_ptr() if s is not None else 0, cu_seqlens_q.data_ptr(), cu_seqlens_k.data_ptr(),
            qs[0], qs[1], ks[0], ks[1], vs[0], vs[1], nh_d, head_dim,
            batch, nheads, head_dim, max_seqlen_q, max_seqlen_k, lse_stride,
            s.shape[2] if s is not None else 0, s.shape[3] if s is not None else 0,
            float(softmax_scale), float(p_dropout), seed, offset, offset_dev or 0,
            1 if is_causal else 0, dt, rot_cos, rot_sin, rot_stride, int(impl), 0)
        if layout is None:
            rc = raw_fwd(addr, _stream_ptr(dev))
        else:
            a = FaFwdArgs.from_buffer_copy(buf)
            m, _keep = _mask_struct(layout, dev)
            rc = lib().fa_fwd_block(ctypes.byref(a), ctypes.byref(m), _stream_ptr(dev))
        if rc != 0:
            _raise(rc, "fa_fwd")
    result = [o, lse]
    if return_softmax:
        result.append(s)
    return result


def bwd(dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k,
        p_dropout, softmax_scale, zero_tensors, is_causal, gen, rng_state=None, layout=None):
    """Backward pass with the signature flash_attn_interface.py:31-33 expects. Writes dq, dk, dv
    in place (strided views allowed) and returns softmax_d = rowsum(dout * out), (B, H, lse_stride)."""
    if _C is not None and layout is None and q.is_cuda:
        if p_dropout > 0.0:
            seed, offset, offset_dev = _unpack_rng(rng_state if rng_state is not None else reserve_rng(q.device, gen))
        else:
            seed, offset, offset_dev = 0, 0, None
        return _C.bwd(dout, q, k, v, out, softmax_lse, dq, dk, dv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
                      max_seqlen_k, p_dropout, softmax_scale, zero_tensors, is_causal, seed, offset, offset_dev or 0)
    dt = _dtype_code(q.dtype)
    for t, n in ((dout, "dout"), (k, "k"), (v, "v"), (out, "out"), (dq, "dq"), (dk, "dk"), (dv, "dv")):
        _check(t.dtype == q.dtype, f"{n} must have the dtype of q")
        _check(t.is_cuda, f"{n} must be on the GPU")
    # inputs with broadcast or overlapping rows (e.g. the dout of out.sum(0)) are made contiguous
    dout, q, k, v, out = (_rows_input(t) for t in (dout, q, k, v, out))
    for t, n in ((dq, "dq"), (dk, "dk"), (dv, "dv")):
        _check(_rows_ok(t), f"{n} must have contiguous last dimension and non-overlapping rows")
    _check(softmax_lse.dtype == torch.float32 and softmax_lse.is_contiguous(), "softmax_lse must be fp32 contiguous")
    _check(softmax_lse.is_cuda and q.is_cuda, "softmax_lse and q must be on the GPU")
    _check(cu_seqlens_q.dtype == torch.int32 and cu_seqlens_k.dtype == torch.int32, "cu_seqlens must be int32")
    _check(cu_seqlens_q.is_cuda and cu_seqlens_k.is_cuda, "cu_seqlens must be on the GPU")
    _check(cu_seqlens_q.is_contiguous() and cu_seqlens_k.is_contiguous(), "cu_seqlens must be contiguous")
    _check(cu_seqlens_k.numel() == cu_seqlens_q.numel(), "cu_seqlens_k must have shape (batch_size + 1)")
    batch = cu_seqlens_q.numel() - 1
    total_q, nheads, head_dim = q.shape
    _check(head_dim % 8 == 0 and head_dim <= 128, "head_size must be a multiple of 8 and <= 128")
    _check(tuple(dq.shape) == tuple(q.shape) and tuple(dout.shape) == tuple(q.shape) and tuple(out.shape) == tuple(q.shape),
           "dq/dout/out must have the shape of q")
    _check(tuple(dk.shape) == tuple(k.shape) and tuple(dv.shape) == tuple(v.shape), "dk/dv must match k/v")
    lse_stride = softmax_lse.shape[-1]
    dev = q.device
    with _on_device(dev):
        if zero_tensors:
            dq.zero_()
            dk.zero_()
            dv.zero_()
        softmax_d = torch.empty((batch, nheads, lse_stride), dtype=torch.float32, device=dev)
        # the fp32 dQ workspace only exists for the atomic-dQ kernels (fa_query says which)
        dq_accum = None
        if _bwd_needs_workspace(head_dim, p_dropout > 0.0, layout is not None):
            dq_accum = torch.empty((total_q, nheads, head_dim), dtype=torch.float32, device=dev)
        if p_dropout > 0.0:
            # Without rng_state, draw from the generator like the reference protocol does: the
            # caller restored the forward's RNG state (flash_attn_interface.py:60-63), so the
            # same (seed, offset) comes out again.
            seed, offset, offset_dev = _unpack_rng(rng_state if rng_state is not None else reserve_rng(dev, gen))
        else:
            seed, offset, offset_dev = 0, 0, None
        # FaBwdArgs field order (include/fa_hip.h), packed in one call
        if layout is None:
            packer, buf, addr, raw_bwd = _raw_call(FaBwdArgs, "fa_bwd")
        else:
            packer, buf, addr, raw_bwd = _raw_call(FaBwdArgs, "fa_bwd_block", 3)
        dos, qs, ks, vs, os_ = dout.stride(), q.stride(), k.stride(), v.stride(), out.stride()
        dqs, dks, dvs = dq.stride(), dk.stride(), dv.stride()
        packer.pack_into(
            buf, 0, dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(),
            softmax_lse.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), softmax_d.data_ptr(),
            dq_accum.data_ptr() if dq_accum is not None else 0,
            cu_seqlens_q.data_ptr(), cu_seqlens_k.data_ptr(),
            dos[0], dos[1], qs[0], qs[1], ks[0], ks[1], vs[0], vs[1], os_[0], os_[1],
            dqs[0], dqs[1], dks[0], dks[1], dvs[0], dvs[1],
            batch, nheads, head_dim, int(max_seqlen_q), int(max_seqlen_k), total_q, lse_stride,
            float(softmax_scale), float(p_dropout), seed, offset, offset_dev or 0,
            1 if is_causal else 0, dt)
        if layout is None:
            rc = raw_bwd(addr, _stream_ptr(dev))
        else:
            m, _keep = _mask_struct(layout, dev)
            rc = raw_bwd(addr, ctypes.addressof(m), _stream_ptr(dev))
        if rc != 0:
            _raise(rc, "fa_bwd")
    return softmax_d


def decode_blockmask(blockmask, nrow=None):
    """Inverse of convert_blockmask (flash_attn/flash_blocksparse_attn_interface.py:8-40): the
    (col, row) int32 list of row indices x4 (+flags, -1 padded) back to the 0/1 (row, col) layout."""
    ncol, nr = blockmask.shape
    nrow = nr if nrow is None else nrow
    bm = blockmask.to(torch.int64)
    valid = bm >= 0
    rows = torch.div(bm.clamp(min=0), 4, rounding_mode="floor")
    cols = torch.arange(ncol, device=bm.device).unsqueeze(1).expand_as(bm)
    layout = torch.zeros((nrow, ncol), dtype=torch.uint8, device=bm.device)
    layout[rows[valid], cols[valid]] = 1
    return layout


def fwd_block(qkv, cu_seqlens, blockmask, p_dropout, max_s, softmax_scale, is_causal, return_softmax, gen,
              rng_state=None):
    """`flash_attn_cuda.fwd_block` as called at flash_blocksparse_attn_interface.py:46-48: packed
    qkv (total, 3, H, D) and the CONVERTED blockmask (convert_blockmask's int32 (col, row) list).
    Returns [context, softmax_lse, (S_dmask)]."""
    _check(qkv.dim() == 4 and qkv.shape[1] == 3, "qkv must be (total, 3, nheads, headdim)")
    layout = decode_blockmask(blockmask)
    return fwd(qkv[:, 0], qkv[:, 1], qkv[:, 2], cu_seqlens, cu_seqlens, max_s, max_s, p_dropout, softmax_scale,
               False, is_causal, return_softmax, gen, rng_state=rng_state, layout=layout)


def bwd_block(dout, qkv, out, S_dmask, softmax_lse, cu_seqlens, blockmask, p_dropout, softmax_scale, max_s,
              is_causal, gen, rng_state=None):
    """`flash_attn_cuda.bwd_block` as called at flash_blocksparse_attn_interface.py:55-58.
    Returns (dqkv, None, softmax_d); S_dmask is not needed (the mask is replayed from Philox)."""
    layout = decode_blockmask(blockmask)
    dqkv = torch.empty_like(qkv)
    softmax_d = bwd(dout, qkv[:, 0], qkv[:, 1], qkv[:, 2], out, softmax_lse, dqkv[:, 0], dqkv[:, 1], dqkv[:, 2],
                    cu_seqlens, cu_seqlens, max_s, max_s, p_dropout, softmax_scale, False, is_causal, gen,
                    rng_state=rng_state, layout=layout)
    return dqkv, None, softmax_d


def rotary(x, y, cos, sin, shape, x_strides, y_strides, nrot, inverse):
    """fa_rotary over the (B, S, NSLOT, H, D) views of x and y given by `shape` and element
    strides (batch, seq, slot, head); y may be x (in place)."""
    B, S, NS, H, D = shape
    _check(cos.stride(0) == sin.stride(0), "cos and sin tables must share a row stride")
    packer, buf, addr, raw = _raw_call(FaRotaryArgs, "fa_rotary")
    xs, ys = x_strides, y_strides
    packer.pack_into(buf, 0, x.data_ptr(), y.data_ptr(), cos.data_ptr(), sin.data_ptr(),
                     int(xs[0]), int(xs[1]), int(xs[2]), int(xs[3]), int(ys[0]), int(ys[1]), int(ys[2]), int(ys[3]),
                     cos.stride(0), B, S, NS, H, D, nrot, 1 if inverse else 0, _dtype_code(x.dtype))
    with _on_device(x.device):
        rc = raw(addr, _stream_ptr(x.device))
    if rc != 0:
        _raise(rc, "fa_rotary")
    return y


def asm_launch_count():
    """Assembly-forward launches this process has enqueued or captured (fa_query FA_QUERY_ASM_LAUNCHES):
    diagnostics of which kernel family a call or a graph capture took."""
    return int(lib().fa_query(FA_QUERY_ASM_LAUNCHES, 0, 0, 0))


def fwd_kernel_name(batch, nheads, head_dim, max_seqlen_q, max_seqlen_k, dtype=torch.bfloat16, causal=False,
                    p_dropout=0.0, row_elems=None, impl=FA_IMPL_AUTO):
    """Name of the GPU kernel fa_fwd launches for a dense forward of this shape (as rocprofv3 shows it;
    include/fa_hip.h fa_fwd_kernel_name). row_elems: the q/k/v/o row stride in elements (default
    nheads * head_dim, the unpadded layout)."""
    a = FaFwdArgs()
    rs = nheads * head_dim if row_elems is None else row_elems
    a.q_row_stride = a.k_row_stride = a.v_row_stride = a.o_row_stride = rs
    a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = head_dim
    a.batch, a.nheads, a.head_dim = batch, nheads, head_dim
    a.max_seqlen_q, a.max_seqlen_k = max_seqlen_q, max_seqlen_k
    a.lse_stride = max((max_seqlen_q + 15) // 16 * 16, 16)
    a.softmax_scale, a.p_dropout = head_dim ** -0.5, p_dropout
    a.is_causal, a.dtype, a.impl = int(causal), _dtype_code(dtype), impl
    name = lib().fa_fwd_kernel_name(ctypes.byref(a))
    return None if name is None else name.decode()
