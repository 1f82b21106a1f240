// fa_api.cpp — the C ABI of libfa_hip.so (declared in include/fa_hip.h).
//
// Replaces the reference's pybind11 host layer (csrc/flash_attn/fmha_api.cpp:112-247):
// argument validation (fmha_api.cpp:131-170, same rules, reported as error codes instead of
// TORCH_CHECK/exit(1)), head-dim tile selection (fmha_fprop_kernel_dispatch.cu:90-134, here
// 32/64/128 tiles instead of CUTLASS traits), and the launches. Dropout seed/offset arrive
// from the caller (the Python layer reserves them from the torch generator), so the library
// holds no generator state.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <string>

#include "fa_launch.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(FA_ERR_LAUNCH, "%s: HIP error %d (%s)", what, (int)e, hipGetErrorString(e));
}

int pick_tile(int head_dim) {
    if (head_dim <= 32) return 32;
    if (head_dim <= 64) return 64;
    return 128;
}

template <typename Args>
int check_common(const Args *a, const char *fn) {
    if (a == nullptr) return fail(FA_ERR_INVALID_ARGUMENT, "%s: args is NULL", fn);
    if (a->dtype != FA_DTYPE_FP16 && a->dtype != FA_DTYPE_BF16)
        return fail(FA_ERR_INVALID_ARGUMENT, "%s: dtype must be fp16 or bf16", fn);
    if (a->batch <= 0) return fail(FA_ERR_INVALID_ARGUMENT, "%s: batch_size must be > 0", fn);
    if (a->nheads <= 0) return fail(FA_ERR_INVALID_ARGUMENT, "%s: num_heads must be > 0", fn);
    if (a->head_dim <= 0 || a->head_dim % 8 != 0 || a->head_dim > 128)
        return fail(FA_ERR_UNSUPPORTED, "%s: head_size must be a multiple of 8 and <= 128 (got %d)", fn,
                    a->head_dim);
    if (a->max_seqlen_q < 0 || a->max_seqlen_k < 0)
        return fail(FA_ERR_INVALID_ARGUMENT, "%s: max_seqlen must be >= 0", fn);
    if (!(a->p_dropout >= 0.f && a->p_dropout < 1.f))
        return fail(FA_ERR_INVALID_ARGUMENT, "%s: p_dropout must be in [0, 1)", fn);
    if (!std::isfinite(a->softmax_scale)) return fail(FA_ERR_INVALID_ARGUMENT, "%s: softmax_scale must be finite", fn);
    if (a->lse_stride < a->max_seqlen_q) return fail(FA_ERR_INVALID_ARGUMENT, "%s: lse_stride < max_seqlen_q", fn);
    // empty tensors may come with NULL data: q/lse matter only with query rows, k/v only with keys too
    const bool has_q = a->max_seqlen_q > 0, has_k = has_q && a->max_seqlen_k > 0;
    if (!a->cu_seqlens_q || !a->cu_seqlens_k || (has_q && (!a->q || !a->softmax_lse)) || (has_k && (!a->k || !a->v)))
        return fail(FA_ERR_INVALID_ARGUMENT, "%s: NULL tensor pointer", fn);
    return FA_OK;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

const char *fa_last_error(void) { return g_last_error.c_str(); }

const char *fa_version(void) { return "fa_hip 0.1.0 (gfx950)"; }

const char *fa_fwd_kernel_name(const FaFwdArgs *a) {
    // the checks fwd_impl makes before it launches anything (NULL: fa_fwd would fail or launch nothing)
    if (a == nullptr || a->head_dim <= 0 || a->head_dim > 128 || a->head_dim % 8 != 0 || a->batch <= 0 ||
        a->nheads <= 0 || a->max_seqlen_q <= 0 || a->max_seqlen_k < 0 ||
        (a->dtype != FA_DTYPE_FP16 && a->dtype != FA_DTYPE_BF16) || a->impl < FA_IMPL_AUTO || a->impl > FA_IMPL_ASM4P ||
        a->impl == FA_IMPL_ASM8 ||
        a->p_dropout < 0.f || a->p_dropout >= 1.f)
        return nullptr;
    if (fa::fwd_asm_eligible(*a, FaBlockMask{nullptr, 0, 0, 0})) return fa::asm_kernel_name(*a);
    // HIP family: the prefix of the demangled template name a rocprofv3 trace shows
    // ("void fa::fa_fwd_kernel<64, fa::Bf16, ...>(FaFwdArgs, FaBlockMask, int)")
    const int t = pick_tile(a->head_dim);
    return t == 32 ? "fa::fa_fwd_kernel<32," : t == 64 ? "fa::fa_fwd_kernel<64," : "fa::fa_fwd_kernel<128,";
}

int64_t fa_query(int what, int64_t a, int64_t b, int64_t c) {
    switch (what) {
        case FA_QUERY_BWD_WORKSPACE: return a * b * c * (int64_t)sizeof(float);
        case FA_QUERY_MAX_HEAD_DIM: return 128;
        case FA_QUERY_RNG_INCREMENT: return 4;
        case FA_QUERY_FWD_ARGS_SIZE: return (int64_t)sizeof(FaFwdArgs);
        case FA_QUERY_BWD_ARGS_SIZE: return (int64_t)sizeof(FaBwdArgs);
        case FA_QUERY_MASK_ARGS_SIZE: return (int64_t)sizeof(FaBlockMask);
        case FA_QUERY_PAD_WORKSPACE: return a * (int64_t)sizeof(int32_t);
        case FA_QUERY_ROTARY_ARGS_SIZE: return (int64_t)sizeof(FaRotaryArgs);
        case FA_QUERY_ASM_LAUNCHES: return fa::asm_launch_count();
        case FA_QUERY_BWD_WORKSPACE_NEEDED: {
            // a = head_dim, b = p_dropout > 0, c = block-sparse: 1 if fa_bwd needs dq_accum
            FaBwdArgs t{};
            t.head_dim = (int32_t)a;
            t.p_dropout = b ? 0.5f : 0.f;
            const FaBlockMask m = {c ? (const uint8_t *)1 : nullptr, 0, 0, 0};
            return fa::bwd_dq_direct(t, m) ? 0 : 1;
        }
        default: return -1;
    }
}

}  // extern "C"

namespace {

// Block-sparse layout checks (fa_fwd_block / fa_bwd_block).
int check_mask(const FaBlockMask *m, int max_q, int max_k, const char *fn) {
    if (m == nullptr || m->mask == nullptr) return fail(FA_ERR_INVALID_ARGUMENT, "%s: blockmask is NULL", fn);
    if (m->cols <= 0 || m->cols > 64)
        return fail(FA_ERR_UNSUPPORTED, "%s: blockmask columns must be in [1, 64] (max_seqlen_k <= 16384)", fn);
    if (m->row_stride < m->cols) return fail(FA_ERR_INVALID_ARGUMENT, "%s: blockmask row_stride < cols", fn);
    if ((int64_t)m->rows * 16 < max_q || (int64_t)m->cols * 256 < max_k)
        return fail(FA_ERR_INVALID_ARGUMENT,
                    "%s: blockmask (%d x %d) does not cover max_seqlen_q=%d / max_seqlen_k=%d (16 x 256 blocks)", fn,
                    m->rows, m->cols, max_q, max_k);
    if (max_q > 32768) return fail(FA_ERR_UNSUPPORTED, "%s: block-sparse max_seqlen_q must be <= 32768", fn);
    return FA_OK;
}

const FaBlockMask kDense = {nullptr, 0, 0, 0};

int fwd_impl(const FaFwdArgs *a, const FaBlockMask &bm, void *stream) {
    int rc = check_common(a, "fa_fwd");
    if (rc) return rc;
    if (!a->o && a->max_seqlen_q > 0) return fail(FA_ERR_INVALID_ARGUMENT, "fa_fwd: o is NULL");
    if (!aligned16(a->q) || !aligned16(a->k) || !aligned16(a->v) || !aligned16(a->o) ||
        (a->q_row_stride | a->k_row_stride | a->v_row_stride | a->o_row_stride | a->q_head_stride |
         a->k_head_stride | a->v_head_stride | a->o_head_stride) % 8 != 0)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_fwd: q/k/v/o must be 16-byte aligned with strides multiple of 8");
    if (a->q_row_stride < a->head_dim || a->k_row_stride < a->head_dim || a->v_row_stride < a->head_dim ||
        a->o_row_stride < a->head_dim)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_fwd: row strides must be >= head_dim (no overlapping/broadcast rows)");
    if (a->s_dmask && (a->s_rows < a->max_seqlen_q || a->s_cols < a->max_seqlen_k))
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_fwd: s_dmask extents smaller than max_seqlen");
    if (a->rot_cos || a->rot_sin) {
        if (!a->rot_cos || !a->rot_sin || !aligned16(a->rot_cos) || !aligned16(a->rot_sin) || a->rot_stride % 8 != 0 ||
            a->rot_stride < a->head_dim)
            return fail(FA_ERR_INVALID_ARGUMENT,
                        "fa_fwd: rotary tables must both be set, 16-byte aligned, rot_stride >= head_dim and a multiple of 8");
        if (a->s_dmask) return fail(FA_ERR_UNSUPPORTED, "fa_fwd: fused rotary cannot return the attention probabilities");
        if ((int64_t)a->max_seqlen_q * a->rot_stride * 2 >= ((int64_t)1 << 31))
            return fail(FA_ERR_UNSUPPORTED, "fa_fwd: rotary tables span more than 2 GiB");
    }
    // the forward addresses each sequence through 32-bit buffer offsets
    const int64_t lim = (int64_t)1 << 31;
    if ((int64_t)a->max_seqlen_q * a->q_row_stride * 2 >= lim || (int64_t)a->max_seqlen_k * a->k_row_stride * 2 >= lim ||
        (int64_t)a->max_seqlen_k * a->v_row_stride * 2 >= lim)
        return fail(FA_ERR_UNSUPPORTED, "fa_fwd: a sequence spans more than 2 GiB (seqlen * row_stride)");
    if (a->impl < FA_IMPL_AUTO || a->impl > FA_IMPL_ASM4P || a->impl == FA_IMPL_ASM8)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_fwd: impl must be one of FA_IMPL_AUTO / HIP / ASM4 / ASM4P "
                                             "(FA_IMPL_ASM8 is not in this library)");
    if (a->max_seqlen_q == 0) return FA_OK;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipSuccess;
    bool asm_unavailable = false;
    if (fa::fwd_asm_eligible(*a, bm)) e = fa::launch_fwd_asm(*a, s, &asm_unavailable);
    // FA_IMPL_AUTO falls back to the HIP kernels when the code objects cannot be loaded (first call
    // of a device inside a capture that refuses module loads); a forced asm form reports it
    if (asm_unavailable && a->impl != FA_IMPL_AUTO)
        return fail(FA_ERR_UNSUPPORTED, "fa_fwd: the assembly kernels could not be loaded on this device");
    if (!fa::fwd_asm_eligible(*a, bm) || asm_unavailable) switch (pick_tile(a->head_dim)) {
        case 32: e = fa::launch_fwd<32>(*a, bm, s); break;
        case 64: e = fa::launch_fwd<64>(*a, bm, s); break;
        default: e = fa::launch_fwd<128>(*a, bm, s); break;
    }
    if (e != hipSuccess) return hip_fail(e, "fa_fwd launch");
    if (a->s_dmask) {
        e = fa::launch_probs(*a, bm, s);
        if (e != hipSuccess) return hip_fail(e, "fa_fwd probs launch");
    }
    return FA_OK;
}

int bwd_impl(const FaBwdArgs *a, const FaBlockMask &bm, void *stream) {
    int rc = check_common(a, "fa_bwd");
    if (rc) return rc;
    if (a->max_seqlen_q > 0 && (!a->dout || !a->out || !a->dq || !a->softmax_d ||
                                (a->max_seqlen_k > 0 && (!a->dk || !a->dv))))
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_bwd: NULL tensor pointer");
    // the fp32 dQ workspace is only touched when dq is not written directly
    const bool direct = fa::bwd_dq_direct(*a, bm);
    if (!direct && !a->dq_accum && a->max_seqlen_q > 0 && a->max_seqlen_k > 0)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_bwd: dq_accum is NULL (required unless fa_query(FA_QUERY_BWD_WORKSPACE_NEEDED) is 0)");
    if (!aligned16(a->q) || !aligned16(a->k) || !aligned16(a->v) || !aligned16(a->dout) || !aligned16(a->out) ||
        !aligned16(a->dq) || !aligned16(a->dk) || !aligned16(a->dv) || (a->dq_accum && !aligned16(a->dq_accum)) ||
        (a->q_row_stride | a->k_row_stride | a->v_row_stride | a->o_row_stride | a->do_row_stride |
         a->dq_row_stride | a->dk_row_stride | a->dv_row_stride | a->q_head_stride | a->k_head_stride |
         a->v_head_stride | a->o_head_stride | a->do_head_stride | a->dq_head_stride | a->dk_head_stride |
         a->dv_head_stride) % 8 != 0)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_bwd: tensors must be 16-byte aligned with strides multiple of 8");
    if (a->total_q < 0) return fail(FA_ERR_INVALID_ARGUMENT, "fa_bwd: total_q < 0");
    if (a->q_row_stride < a->head_dim || a->k_row_stride < a->head_dim || a->v_row_stride < a->head_dim ||
        a->o_row_stride < a->head_dim || a->do_row_stride < a->head_dim || a->dq_row_stride < a->head_dim ||
        a->dk_row_stride < a->head_dim || a->dv_row_stride < a->head_dim)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_bwd: row strides must be >= head_dim (no overlapping/broadcast rows)");
    // the backward kernels address each sequence through 32-bit buffer offsets, like the forward
    const int64_t lim = (int64_t)1 << 31;
    const int64_t q_span = (int64_t)a->max_seqlen_q * 2, k_span = (int64_t)a->max_seqlen_k * 2;   // bytes per unit stride
    if (q_span * a->q_row_stride >= lim || q_span * a->do_row_stride >= lim ||
        q_span * a->dq_row_stride >= lim || q_span * a->o_row_stride >= lim ||
        k_span * a->k_row_stride >= lim || k_span * a->v_row_stride >= lim ||
        k_span * a->dk_row_stride >= lim || k_span * a->dv_row_stride >= lim)
        return fail(FA_ERR_UNSUPPORTED, "fa_bwd: a sequence spans more than 2 GiB (seqlen * row_stride)");
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    // no query rows: no output depends on k or v, so dk = dv = 0 (softmax_d has no rows)
    if (a->max_seqlen_q == 0) {
        e = fa::launch_zero_seq_rows(a->dk, a->cu_seqlens_k, a->dk_row_stride, a->dk_head_stride, a->batch, a->nheads,
                                     a->head_dim, a->max_seqlen_k, s);
        if (e == hipSuccess)
            e = fa::launch_zero_seq_rows(a->dv, a->cu_seqlens_k, a->dv_row_stride, a->dv_head_stride, a->batch,
                                         a->nheads, a->head_dim, a->max_seqlen_k, s);
        return e == hipSuccess ? FA_OK : hip_fail(e, "fa_bwd zero dk/dv launch");
    }
    e = fa::launch_bwd_pre(*a, s);
    if (e != hipSuccess) return hip_fail(e, "fa_bwd pre launch");
    // no keys anywhere: the output is 0 and does not depend on q, so dq = 0 (softmax_d = 0 above)
    if (a->max_seqlen_k == 0) {
        e = fa::launch_zero_seq_rows(a->dq, a->cu_seqlens_q, a->dq_row_stride, a->dq_head_stride, a->batch, a->nheads,
                                     a->head_dim, a->max_seqlen_q, s);
        return e == hipSuccess ? FA_OK : hip_fail(e, "fa_bwd zero dq launch");
    }
    switch (pick_tile(a->head_dim)) {
        case 32: e = fa::launch_bwd<32>(*a, bm, s); break;
        case 64: e = fa::launch_bwd<64>(*a, bm, s); break;
        default: e = fa::launch_bwd<128>(*a, bm, s); break;
    }
    if (e != hipSuccess) return hip_fail(e, "fa_bwd launch");
    if (!direct) {
        e = fa::launch_bwd_post(*a, s);
        if (e != hipSuccess) return hip_fail(e, "fa_bwd post launch");
    }
    return FA_OK;
}

}  // namespace

extern "C" {

int fa_fwd(const FaFwdArgs *a, void *stream) {
    g_last_error.clear();
    return fwd_impl(a, kDense, stream);
}

int fa_bwd(const FaBwdArgs *a, void *stream) {
    g_last_error.clear();
    return bwd_impl(a, kDense, stream);
}

int fa_fwd_block(const FaFwdArgs *a, const FaBlockMask *m, void *stream) {
    g_last_error.clear();
    if (a == nullptr) return fail(FA_ERR_INVALID_ARGUMENT, "fa_fwd_block: args is NULL");
    int rc = check_mask(m, a->max_seqlen_q, a->max_seqlen_k, "fa_fwd_block");
    if (rc) return rc;
    return fwd_impl(a, *m, stream);
}

int fa_bwd_block(const FaBwdArgs *a, const FaBlockMask *m, void *stream) {
    g_last_error.clear();
    if (a == nullptr) return fail(FA_ERR_INVALID_ARGUMENT, "fa_bwd_block: args is NULL");
    int rc = check_mask(m, a->max_seqlen_q, a->max_seqlen_k, "fa_bwd_block");
    if (rc) return rc;
    return bwd_impl(a, *m, stream);
}

// ---- var-len packing (bert_padding)
int fa_index_first_axis(const void *src, int64_t src_rows, int64_t src_row_stride, const int64_t *indices, int64_t n,
                        void *dst, int64_t dst_row_stride, int64_t row_bytes, void *stream) {
    g_last_error.clear();
    if (n < 0 || src_rows < 0 || row_bytes < 0 || row_bytes % 2 != 0)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_first_axis: negative size or odd row_bytes");
    if (n > 0 && row_bytes > 0 && (!src || !dst || !indices))
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_first_axis: NULL pointer");
    if (src_row_stride < row_bytes || dst_row_stride < row_bytes || src_row_stride % 2 || dst_row_stride % 2)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_first_axis: row stride smaller than the row or odd");
    hipError_t e = fa::launch_gather_rows(src, src_rows, src_row_stride, indices, n, dst, dst_row_stride, row_bytes,
                                          (hipStream_t)stream);
    return e == hipSuccess ? FA_OK : hip_fail(e, "fa_index_first_axis launch");
}

int fa_index_put_first_axis(const void *src, int64_t src_row_stride, const int64_t *indices, int64_t n, void *dst,
                            int64_t dst_rows, int64_t dst_row_stride, int64_t row_bytes, int32_t *workspace,
                            void *stream) {
    g_last_error.clear();
    if (n < 0 || dst_rows < 0 || row_bytes < 0 || row_bytes % 2 != 0)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_put_first_axis: negative size or odd row_bytes");
    if (dst_rows > 0 && row_bytes > 0 && (!dst || !workspace || (n > 0 && (!src || !indices))))
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_put_first_axis: NULL pointer");
    if (dst_rows > INT32_MAX || n > INT32_MAX)
        return fail(FA_ERR_UNSUPPORTED, "fa_index_put_first_axis: more than 2^31 rows");
    if (src_row_stride < row_bytes || dst_row_stride < row_bytes || src_row_stride % 2 || dst_row_stride % 2)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_put_first_axis: row stride smaller than the row or odd");
    hipError_t e = fa::launch_pad_rows(src, src_row_stride, indices, n, dst, dst_rows, dst_row_stride, row_bytes,
                                       workspace, (hipStream_t)stream);
    return e == hipSuccess ? FA_OK : hip_fail(e, "fa_index_put_first_axis launch");
}

int fa_index_add_first_axis(const void *src, int64_t src_row_stride, const int64_t *indices, int64_t n, void *dst,
                            int64_t dst_rows, int64_t dst_row_stride, int64_t row_elems, int32_t dtype,
                            void *stream) {
    g_last_error.clear();
    if (dtype != FA_DTYPE_FP16 && dtype != FA_DTYPE_BF16 && dtype != FA_DTYPE_FP32)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_add_first_axis: dtype must be fp16, bf16 or fp32");
    const int64_t esz = dtype == FA_DTYPE_FP32 ? 4 : 2;
    if (n < 0 || dst_rows < 0 || row_elems < 0)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_add_first_axis: negative size");
    if (n > 0 && row_elems > 0 && (!src || !dst || !indices))
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_add_first_axis: NULL pointer");
    if (src_row_stride < row_elems * esz || dst_row_stride < row_elems * esz || src_row_stride % esz ||
        dst_row_stride % esz)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_index_add_first_axis: bad row stride");
    hipError_t e = fa::launch_scatter_add_rows(src, src_row_stride, indices, n, dst, dst_rows, dst_row_stride,
                                               row_elems, dtype, (hipStream_t)stream);
    return e == hipSuccess ? FA_OK : hip_fail(e, "fa_index_add_first_axis launch");
}

// ---- rotary embedding
int fa_rotary(const FaRotaryArgs *a, void *stream) {
    g_last_error.clear();
    if (a == nullptr) return fail(FA_ERR_INVALID_ARGUMENT, "fa_rotary: args is NULL");
    if (a->dtype != FA_DTYPE_FP16 && a->dtype != FA_DTYPE_BF16)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_rotary: dtype must be fp16 or bf16");
    if (a->batch < 0 || a->seqlen < 0 || a->nslot < 0 || a->nheads < 0 || a->nrot < 0 || a->nrot > a->nslot)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_rotary: negative size or nrot > nslot");
    if (a->head_dim <= 0 || a->head_dim % 8 != 0)
        return fail(FA_ERR_UNSUPPORTED, "fa_rotary: head_dim must be a positive multiple of 8 (got %d)", a->head_dim);
    if ((int64_t)a->batch * a->seqlen * a->nslot * a->nheads == 0) return FA_OK;
    if (!a->x || !a->y || (a->nrot > 0 && (!a->cos || !a->sin)))
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_rotary: NULL pointer");
    int64_t m = a->table_stride;
    for (int i = 0; i < 4; ++i) m |= a->x_strides[i] | a->y_strides[i];
    if (m % 8 != 0 || !aligned16(a->x) || !aligned16(a->y) || (a->nrot > 0 && (!aligned16(a->cos) || !aligned16(a->sin))))
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_rotary: tensors must be 16-byte aligned with strides multiple of 8");
    if (a->nrot > 0 && a->table_stride < a->head_dim)
        return fail(FA_ERR_INVALID_ARGUMENT, "fa_rotary: table_stride < head_dim");
    hipError_t e = fa::launch_rotary(*a, (hipStream_t)stream);
    return e == hipSuccess ? FA_OK : hip_fail(e, "fa_rotary launch");
}

}  // extern "C"
