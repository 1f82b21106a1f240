"""CPU tests of the drop-in boundary: libfa_hip.so loads, exports every symbol include/fa_hip.h
declares, the ctypes struct layouts match the C ones, argument validation fails with error codes
(no GPU call is made on those paths), and the Python surface mirrors the reference's names and
signatures (flash_attn/flash_attn_interface.py:39-252)."""
import ctypes
import inspect
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "fa_hip.h")


def _declared_functions():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char \*)\s*(fa_\w+)\s*\(", src, re.M)))


def test_header_declares_the_entry_points():
    assert _declared_functions() == ["fa_bwd", "fa_bwd_block", "fa_fwd", "fa_fwd_block", "fa_fwd_kernel_name",
                                     "fa_index_add_first_axis", "fa_index_first_axis", "fa_index_put_first_axis", "fa_last_error",
                                     "fa_query", "fa_rotary", "fa_version"]


def test_library_exports_every_declared_symbol():
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    for name in _declared_functions():
        assert hasattr(L, name), name


def test_struct_layouts_match():
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    assert L.fa_query(hip.FA_QUERY_FWD_ARGS_SIZE, 0, 0, 0) == ctypes.sizeof(hip.FaFwdArgs)
    assert L.fa_query(hip.FA_QUERY_BWD_ARGS_SIZE, 0, 0, 0) == ctypes.sizeof(hip.FaBwdArgs)
    assert L.fa_query(hip.FA_QUERY_MASK_ARGS_SIZE, 0, 0, 0) == ctypes.sizeof(hip.FaBlockMask)
    assert L.fa_query(hip.FA_QUERY_ROTARY_ARGS_SIZE, 0, 0, 0) == ctypes.sizeof(hip.FaRotaryArgs)
    assert L.fa_query(hip.FA_QUERY_MAX_HEAD_DIM, 0, 0, 0) == 128
    assert L.fa_query(hip.FA_QUERY_BWD_WORKSPACE, 10, 2, 64) == 10 * 2 * 64 * 4
    assert L.fa_query(999, 0, 0, 0) == -1
    assert L.fa_query(hip.FA_QUERY_ASM_LAUNCHES, 0, 0, 0) == hip.asm_launch_count() >= 0
    assert b"gfx950" in L.fa_version()


def _valid_fwd_args(hip):
    a = hip.FaFwdArgs()
    a.q = a.k = a.v = a.o = a.softmax_lse = 4096
    a.cu_seqlens_q = a.cu_seqlens_k = 4096
    a.q_row_stride = a.k_row_stride = a.v_row_stride = a.o_row_stride = 128
    a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = 64
    a.batch, a.nheads, a.head_dim = 1, 2, 64
    a.max_seqlen_q = a.max_seqlen_k = 0   # zero-size: returns before any launch
    a.lse_stride = 16
    a.softmax_scale = 0.125
    a.dtype = hip.FA_DTYPE_BF16
    return a


@pytest.mark.parametrize("field,value,code", [
    ("head_dim", 60, 2), ("head_dim", 136, 2), ("batch", 0, 1), ("nheads", 0, 1), ("dtype", 7, 1),
    ("p_dropout", 1.0, 1), ("p_dropout", -0.1, 1), ("lse_stride", -1, 1), ("cu_seqlens_q", None, 1),
    ("q_row_stride", 129, 1), ("softmax_scale", float("inf"), 1),
    ("q_row_stride", 0, 1), ("k_row_stride", 8, 1),      # broadcast / overlapping rows
    ("impl", 3, 1), ("impl", 5, 1), ("impl", -1, 1),     # FA_IMPL_ASM8 is reserved (not in the library)
])
def test_fwd_argument_validation(field, value, code):
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    a = _valid_fwd_args(hip)
    assert L.fa_fwd(ctypes.byref(a), None) == 0  # the valid zero-size call succeeds without a GPU
    setattr(a, field, value)
    rc = L.fa_fwd(ctypes.byref(a), None)
    assert rc == code
    assert len(L.fa_last_error()) > 0


def _valid_bwd_args(hip):
    a = hip.FaBwdArgs()
    for f in ("dout", "q", "k", "v", "out", "softmax_lse", "dq", "dk", "dv", "softmax_d", "cu_seqlens_q",
              "cu_seqlens_k"):
        setattr(a, f, 4096)
    for f in ("do", "q", "k", "v", "o", "dq", "dk", "dv"):
        setattr(a, f + "_row_stride", 256)
        setattr(a, f + "_head_stride", 128)
    a.batch, a.nheads, a.head_dim = 1, 2, 128
    a.max_seqlen_q = 0                      # no query rows and no keys: returns before any launch
    a.max_seqlen_k = 0                      # (with keys, dk/dv are zeroed: a launch, GPU tests)
    a.lse_stride = 16
    a.softmax_scale = 0.125
    a.dtype = hip.FA_DTYPE_BF16
    return a


def test_bwd_workspace_query_and_validation():
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    W = hip.FA_QUERY_BWD_WORKSPACE_NEEDED
    # D=128 dense: dq written directly (no fp32 workspace); dropout / block-sparse / D<=64: atomics
    assert L.fa_query(W, 128, 0, 0) == 0 and L.fa_query(W, 96, 0, 0) == 0
    assert L.fa_query(W, 128, 1, 0) == 1 and L.fa_query(W, 128, 0, 1) == 1 and L.fa_query(W, 64, 0, 0) == 1
    assert hip._bwd_needs_workspace(128, False, False) is False
    a = _valid_bwd_args(hip)
    assert L.fa_bwd(ctypes.byref(a), None) == 0          # max_seqlen_q = 0: nothing to launch (no grid 0)
    a.head_dim = 64
    a.max_seqlen_q = 4
    a.max_seqlen_k = 16
    assert L.fa_bwd(ctypes.byref(a), None) == 1          # D=64 with query rows and keys needs dq_accum
    a.max_seqlen_k = 0
    a.max_seqlen_q = 0
    assert L.fa_bwd(ctypes.byref(a), None) == 0          # ... but not without any
    a.dq_accum = 4096
    assert L.fa_bwd(ctypes.byref(a), None) == 0
    a.do_row_stride = 0                                   # broadcast dO rows are rejected
    assert L.fa_bwd(ctypes.byref(a), None) == 1
    a.do_row_stride = 256
    a.max_seqlen_k = 1 << 23                              # 2^23 rows x 256 x 2 B >= 2 GiB
    assert L.fa_bwd(ctypes.byref(a), None) == 2
    assert b"2 GiB" in L.fa_last_error()


def test_rows_normalisation():
    import torch
    from flash_attn import flash_attn_hip as hip
    x = torch.randn(1, 2, 64).expand(5, 2, 64)            # stride(0) == 0
    assert not hip._rows_ok(x) and hip._rows_ok(hip._rows_input(x))
    y = torch.randn(5, 3, 2, 64)[:, 1]                    # packed view: stride(0) = 3*2*64
    assert hip._rows_ok(y) and hip._rows_input(y) is y
    from flash_attn.bert_padding import _rows
    z = torch.randn(1, 4, 8).expand(6, 4, 8)
    zc, stride, row = _rows(z)
    assert zc.is_contiguous() and stride == row == 4 * 8 * 4


@pytest.mark.parametrize("rows,cols,stride,code", [
    (0, 0, 0, 1),          # NULL mask pointer (set below only when rows > 0)
    (16, 65, 65, 2),       # more than 64 column blocks
    (16, 1, 1, 1),         # 256 rows < max_seqlen_q = 300
    (19, 2, 1, 1),         # row_stride < cols
])
def test_block_mask_validation(rows, cols, stride, code):
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    a = _valid_fwd_args(hip)
    a.max_seqlen_q = a.max_seqlen_k = 300
    m = hip.FaBlockMask()
    m.mask = 4096 if rows else None
    m.rows, m.cols, m.row_stride = rows, cols, stride
    assert L.fa_fwd_block(ctypes.byref(a), ctypes.byref(m), None) == code
    assert len(L.fa_last_error()) > 0
    b = hip.FaBwdArgs()
    b.max_seqlen_q = b.max_seqlen_k = 300
    assert L.fa_bwd_block(ctypes.byref(b), ctypes.byref(m), None) == code


def test_blocksparse_interface_mirrors_reference():
    from flash_attn import flash_blocksparse_attn_interface as bsi
    sig = lambda f: list(inspect.signature(f).parameters)
    assert sig(bsi.flash_blocksparse_attn_func) == ["qkv", "cu_seqlens", "blockmask", "dropout_p", "max_s",
                                                    "softmax_scale", "causal", "return_attn_probs", "convert_mask"]
    assert sig(bsi.convert_blockmask) == ["blockmask", "causal"]
    for cls in ("FlashBlocksparseAttnFun", "FlashBlocksparseAttnFunWithS"):
        assert hasattr(bsi, cls)


def test_padding_entry_validation():
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    # zero-size calls succeed without touching a GPU; bad sizes/strides are rejected
    assert L.fa_index_first_axis(None, 0, 128, None, 0, None, 128, 128, None) == 0
    assert L.fa_index_first_axis(4096, 10, 64, 4096, 5, 4096, 128, 128, None) == 1       # src stride < row
    assert L.fa_index_first_axis(4096, 10, 128, 4096, 5, 4096, 128, 127, None) == 1     # odd row bytes
    assert L.fa_index_put_first_axis(None, 128, None, 0, None, 0, 128, 128, None, None) == 0
    assert L.fa_index_put_first_axis(4096, 128, 4096, 5, 4096, 10, 128, 128, None, None) == 1   # no workspace
    assert L.fa_index_add_first_axis(4096, 128, 4096, 5, 4096, 10, 128, 64, 3, None) == 1        # bad dtype
    assert L.fa_query(hip.FA_QUERY_PAD_WORKSPACE, 100, 0, 0) == 400


def test_bert_padding_host_path_matches_reference_semantics():
    import torch
    from flash_attn.bert_padding import index_first_axis_residual, pad_input, unpad_input
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 7, 4, generator=g, requires_grad=True)
    mask = torch.arange(7)[None, :] < torch.tensor([[7], [3], [5]])
    xu, idx, cu, mx = unpad_input(x, mask)
    assert cu.tolist() == [0, 7, 10, 15] and mx == 7 and xu.shape == (15, 4)
    back = pad_input(xu, idx, 3, 7)
    assert torch.equal(back, x.detach() * mask[..., None])
    out, res = index_first_axis_residual(x.reshape(21, 4), idx)
    (out.sum() + 2 * res.sum()).backward()
    assert torch.equal(x.grad.reshape(21, 4)[idx], torch.full((15, 4), 3.0))


@pytest.mark.parametrize("cls_name", ["FaFwdArgs", "FaBwdArgs", "FaRotaryArgs"])
def test_packer_matches_ctypes_layout(cls_name):
    """The one-call struct.pack_into image of an argument struct (flash_attn_hip._raw_call) is
    byte-identical to the ctypes mirror filled field by field (whose size fa_query checks against
    the C header)."""
    import random
    from flash_attn import flash_attn_hip as hip
    cls = getattr(hip, cls_name)
    packer = hip._packer(cls)
    rnd = random.Random(1)
    a = cls()

    def draw(typ):
        if typ is ctypes.c_float:
            return ctypes.c_float(rnd.random()).value
        if typ is ctypes.c_int32:
            return rnd.randint(-2 ** 31, 2 ** 31 - 1)
        if typ is ctypes.c_int64:
            return rnd.randint(-2 ** 63, 2 ** 63 - 1)
        return rnd.randint(0, 2 ** 64 - 1)

    vals = []
    for name, typ in cls._fields_:
        if issubclass(typ, ctypes.Array):
            arr = getattr(a, name)
            for i in range(typ._length_):
                arr[i] = draw(typ._type_)
                vals.append(arr[i])
        else:
            v = draw(typ)
            setattr(a, name, v)
            vals.append(v)
    buf = ctypes.create_string_buffer(packer.size)
    packer.pack_into(buf, 0, *vals)
    assert bytes(buf) == bytes(a)


def test_empty_tensors_may_have_null_data():
    """torch.empty(0, ...) has a NULL data pointer: a call with no query rows (or no keys) must
    not reject it (the reference's zero-size calls succeed)."""
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    a = _valid_fwd_args(hip)
    a.q = a.o = a.softmax_lse = a.k = a.v = None
    assert L.fa_fwd(ctypes.byref(a), None) == 0
    a.max_seqlen_q = 4
    assert L.fa_fwd(ctypes.byref(a), None) == 1     # query rows need q/o/lse
    assert b"NULL" in L.fa_last_error()


def test_null_args_pointer():
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    assert L.fa_fwd(None, None) == 1
    assert L.fa_bwd(None, None) == 1
    assert b"NULL" in L.fa_last_error()


def test_last_error_is_thread_local():
    import threading
    from flash_attn import flash_attn_hip as hip
    L = hip.lib()
    L.fa_fwd(None, None)
    seen = []
    t = threading.Thread(target=lambda: seen.append(L.fa_last_error()))
    t.start()
    t.join()
    assert seen == [b""]
    assert L.fa_last_error() != b""


def test_interface_mirrors_reference_signatures():
    from flash_attn import flash_attn_interface as fi
    sig = lambda f: list(inspect.signature(f).parameters)
    assert sig(fi.flash_attn_unpadded_qkvpacked_func) == [
        "qkv", "cu_seqlens", "max_seqlen", "dropout_p", "softmax_scale", "causal", "return_attn_probs"]
    assert sig(fi.flash_attn_unpadded_kvpacked_func) == [
        "q", "kv", "cu_seqlens_q", "cu_seqlens_k", "max_seqlen_q", "max_seqlen_k", "dropout_p", "softmax_scale",
        "causal", "return_attn_probs"]
    assert sig(fi.flash_attn_unpadded_func) == [
        "q", "k", "v", "cu_seqlens_q", "cu_seqlens_k", "max_seqlen_q", "max_seqlen_k", "dropout_p", "softmax_scale",
        "causal", "return_attn_probs"]
    assert sig(fi.flash_attn_func) == ["qkv", "cu_seqlens", "dropout_p", "max_s", "softmax_scale", "causal",
                                       "return_attn_probs"]
    for cls in ("FlashAttnQKVPackedFunc", "FlashAttnKVPackedFunc", "FlashAttnFunc"):
        assert hasattr(fi, cls)
    from flash_attn import flash_attn_hip as hip
    assert sig(hip.fwd)[:13] == ["q", "k", "v", "cu_seqlens_q", "cu_seqlens_k", "max_seqlen_q", "max_seqlen_k",
                                 "p_dropout", "softmax_scale", "zero_tensors", "is_causal", "return_softmax", "gen"]


def test_python_checks_raise_runtime_error_on_cpu_tensors():
    import torch
    from flash_attn import flash_attn_interface as fi
    q = torch.randn(16, 2, 64, dtype=torch.float16)
    cu = torch.tensor([0, 16], dtype=torch.int32)
    with pytest.raises(RuntimeError):
        fi.flash_attn_unpadded_func(q, q, q, cu, cu, 16, 16, 0.0)


def test_compiled_binding_loads_and_checks():
    """flash_attn._fa_C (csrc/fa_torch.cpp) is built next to libfa_hip.so, exposes fwd/bwd with the
    binding's argument lists and raises the binding's RuntimeErrors before any GPU call."""
    import torch
    from flash_attn import flash_attn_hip as hip
    assert hip._C is not None, "flash_attn/_fa_C.so missing: run hazyresearch_flash-attention_amd/build.py"
    assert hip._C.version() == hip.lib().fa_version().decode()
    q = torch.zeros(16, 2, 64, dtype=torch.bfloat16)
    cu = torch.tensor([0, 16], dtype=torch.int32)
    with pytest.raises(RuntimeError, match="all tensors must be on the GPU"):
        hip._C.fwd(q, q, q, cu, cu, 16, 16, 0.0, 0.125, False, False, False, 0, 0, 0, 0)
    with pytest.raises(RuntimeError, match="FlashAttention only supports fp16 and bf16"):
        hip._C.fwd(q.float(), q, q, cu, cu, 16, 16, 0.0, 0.125, False, False, False, 0, 0, 0, 0)
    with pytest.raises(RuntimeError, match="dout must be on the GPU"):
        hip._C.bwd(q, q, q, q, q, torch.zeros(1, 2, 16), q, q, q, cu, cu, 16, 16, 0.0, 0.125, False, False, 0, 0, 0)
