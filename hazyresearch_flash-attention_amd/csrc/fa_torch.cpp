// fa_torch.cpp — compiled Python binding of libfa_hip.so (module flash_attn._fa_C).
//
// The reference binds its kernels as the pybind11 module `flash_attn_cuda` (fmha_api.cpp:244-247):
// argument checks, output allocation and the launch all run in C++. This module does the same
// over the C ABI (include/fa_hip.h) for the two calls on the training path, `fwd` and `bwd`, so
// the per-call host cost is one pybind11 dispatch, the at::empty allocations and the launch.
// flash_attn_hip.py routes its dense calls here (block-sparse layouts and fused rotary keep the
// ctypes path) and keeps the dropout RNG reservation in Python (reserve_rng), passing the
// reserved (seed, offset, device word) in.
//
// Checks and error messages are the ones flash_attn_hip.py raises (RuntimeError through
// TORCH_CHECK, as fmha_api.cpp:131-170 does).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/utils/pybind.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "fa_hip.h"

namespace {

int dtype_code(at::ScalarType t) {
    if (t == at::kHalf) return FA_DTYPE_FP16;
    if (t == at::kBFloat16) return FA_DTYPE_BF16;
    TORCH_CHECK(false, "FlashAttention only supports fp16 and bf16, got ", t);
    return -1;
}

// every (row, head) slice of a (rows, H, D) tensor is its own contiguous D-run and rows do not
// overlap (flash_attn_hip._rows_ok): the kernels address rows through buffer descriptors
bool rows_ok(const at::Tensor &t) {
    if (t.stride(2) != 1) return false;
    const int64_t h = t.size(1), d = t.size(2);
    const int64_t row_extent = h > 0 ? (h - 1) * t.stride(1) + d : d;
    return t.stride(0) >= std::max(row_extent, d) && (h <= 1 || t.stride(1) >= d);
}

at::Tensor rows_input(const at::Tensor &t) { return rows_ok(t) ? t : t.contiguous(); }

int64_t round16(int64_t x) { return (x + 15) / 16 * 16; }

[[noreturn]] void raise_rc(int rc, const char *what) {
    TORCH_CHECK(false, what, " failed (code ", rc, "): ", fa_last_error());
    throw;  // unreachable
}

hipStream_t current_stream(const at::Device &dev) {
    return c10::hip::getCurrentHIPStream(dev.index()).stream();
}

// fa_query(FA_QUERY_BWD_WORKSPACE_NEEDED, ...) per (head_dim, dropout): a pure function of its
// arguments, cached
bool bwd_needs_workspace(int64_t head_dim, bool dropout) {
    static std::mutex mu;
    static int8_t cache[129][2];
    static bool init = false;
    std::lock_guard<std::mutex> lk(mu);
    if (!init) {
        for (auto &r : cache) r[0] = r[1] = -1;
        init = true;
    }
    int8_t &v = cache[head_dim][dropout ? 1 : 0];
    if (v < 0) v = fa_query(FA_QUERY_BWD_WORKSPACE_NEEDED, head_dim, dropout ? 1 : 0, 0) ? 1 : 0;
    return v == 1;
}

// fa_fwd with the signature of flash_attn_hip.fwd minus gen/layout/rotary (the Python layer
// reserves the Philox pair for dropout and passes it in)
std::vector<at::Tensor> fwd(at::Tensor q, at::Tensor k, at::Tensor v, const at::Tensor &cu_q, const at::Tensor &cu_k,
                            int64_t max_seqlen_q, int64_t max_seqlen_k, double p_dropout, double softmax_scale,
                            bool zero_tensors, bool is_causal, bool return_softmax, uint64_t seed, uint64_t offset,
                            int64_t offset_dev, int64_t impl) {
    const auto qdt = q.scalar_type();
    const int dt = dtype_code(qdt);
    TORCH_CHECK(k.scalar_type() == qdt && v.scalar_type() == qdt, "q, k, v must have the same dtype");
    TORCH_CHECK(cu_q.scalar_type() == at::kInt && cu_k.scalar_type() == at::kInt, "cu_seqlens must be int32");
    TORCH_CHECK(q.is_cuda() && k.is_cuda() && v.is_cuda() && cu_q.is_cuda() && cu_k.is_cuda(),
                "all tensors must be on the GPU");
    TORCH_CHECK(q.dim() == 3 && k.dim() == 3 && v.dim() == 3, "q, k, v must be (total, nheads, headdim)");
    TORCH_CHECK(q.stride(2) == 1 && k.stride(2) == 1 && v.stride(2) == 1, "last dimension must be contiguous");
    TORCH_CHECK(cu_q.is_contiguous() && cu_k.is_contiguous(), "cu_seqlens must be contiguous");
    q = rows_input(q);
    k = rows_input(k);
    v = rows_input(v);
    const int64_t batch = cu_q.numel() - 1;
    const int64_t total_q = q.size(0), nheads = q.size(1), head_dim = q.size(2);
    const int64_t total_k = k.size(0);
    TORCH_CHECK(batch > 0, "batch_size must be positive");
    TORCH_CHECK(head_dim % 8 == 0 && head_dim <= 128, "head_size must be a multiple of 8 and <= 128");
    TORCH_CHECK(k.size(1) == nheads && k.size(2) == head_dim && v.size(0) == total_k && v.size(1) == nheads &&
                    v.size(2) == head_dim,
                "k, v must have shape (total_k, nheads, headdim)");
    TORCH_CHECK(cu_k.numel() == batch + 1, "cu_seqlens_k must have shape (batch_size + 1)");
    TORCH_CHECK(0.0 <= p_dropout && p_dropout < 1.0, "dropout_p must be in [0, 1)");

    const at::Device dev = q.device();
    c10::DeviceGuard guard(dev);
    at::Tensor o = at::empty({total_q, nheads, head_dim}, q.options());
    const int64_t lse_stride = std::max<int64_t>(round16(max_seqlen_q), 16);
    at::Tensor lse = at::empty({batch, nheads, lse_stride}, q.options().dtype(at::kFloat));
    at::Tensor s;
    if (return_softmax)
        s = at::empty({batch, nheads, lse_stride, std::max<int64_t>(round16(max_seqlen_k), 16)}, q.options());
    if (zero_tensors) {
        o.zero_();
        lse.fill_(-INFINITY);
        if (s.defined()) s.zero_();
    }
    FaFwdArgs a{};
    a.q = q.data_ptr();
    a.k = k.data_ptr();
    a.v = v.data_ptr();
    a.o = o.data_ptr();
    a.softmax_lse = lse.data_ptr<float>();
    a.s_dmask = s.defined() ? s.data_ptr() : nullptr;
    a.cu_seqlens_q = cu_q.data_ptr<int32_t>();
    a.cu_seqlens_k = cu_k.data_ptr<int32_t>();
    a.q_row_stride = q.stride(0);
    a.q_head_stride = q.stride(1);
    a.k_row_stride = k.stride(0);
    a.k_head_stride = k.stride(1);
    a.v_row_stride = v.stride(0);
    a.v_head_stride = v.stride(1);
    a.o_row_stride = nheads * head_dim;
    a.o_head_stride = head_dim;
    a.batch = (int32_t)batch;
    a.nheads = (int32_t)nheads;
    a.head_dim = (int32_t)head_dim;
    a.max_seqlen_q = (int32_t)max_seqlen_q;
    a.max_seqlen_k = (int32_t)max_seqlen_k;
    a.lse_stride = (int32_t)lse_stride;
    a.s_rows = s.defined() ? (int32_t)s.size(2) : 0;
    a.s_cols = s.defined() ? (int32_t)s.size(3) : 0;
    a.softmax_scale = (float)softmax_scale;
    a.p_dropout = (float)p_dropout;
    a.rng_seed = seed;
    a.rng_offset = offset;
    a.rng_offset_dev = reinterpret_cast<const uint64_t *>(offset_dev);
    a.is_causal = is_causal ? 1 : 0;
    a.dtype = dt;
    a.impl = (int32_t)impl;
    const int rc = fa_fwd(&a, current_stream(dev));
    if (rc != 0) raise_rc(rc, "fa_fwd");
    std::vector<at::Tensor> res{o, lse};
    if (return_softmax) res.push_back(s);
    return res;
}

at::Tensor bwd(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor out, const at::Tensor &lse,
               at::Tensor dq, at::Tensor dk, at::Tensor dv, const at::Tensor &cu_q, const at::Tensor &cu_k,
               int64_t max_seqlen_q, int64_t max_seqlen_k, double p_dropout, double softmax_scale, bool zero_tensors,
               bool is_causal, uint64_t seed, uint64_t offset, int64_t offset_dev) {
    const auto qdt = q.scalar_type();
    const int dt = dtype_code(qdt);
    const std::pair<const at::Tensor *, const char *> same[] = {{&dout, "dout"}, {&k, "k"},   {&v, "v"}, {&out, "out"},
                                                                 {&dq, "dq"},     {&dk, "dk"}, {&dv, "dv"}};
    for (const auto &tn : same) {
        TORCH_CHECK(tn.first->scalar_type() == qdt, tn.second, " must have the dtype of q");
        TORCH_CHECK(tn.first->is_cuda(), tn.second, " must be on the GPU");
    }
    dout = rows_input(dout);
    q = rows_input(q);
    k = rows_input(k);
    v = rows_input(v);
    out = rows_input(out);
    TORCH_CHECK(rows_ok(dq), "dq must have contiguous last dimension and non-overlapping rows");
    TORCH_CHECK(rows_ok(dk), "dk must have contiguous last dimension and non-overlapping rows");
    TORCH_CHECK(rows_ok(dv), "dv must have contiguous last dimension and non-overlapping rows");
    TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous(), "softmax_lse must be fp32 contiguous");
    const int64_t batch = cu_q.numel() - 1;
    const int64_t total_q = q.size(0), nheads = q.size(1), head_dim = q.size(2);
    TORCH_CHECK(head_dim % 8 == 0 && head_dim <= 128, "head_size must be a multiple of 8 and <= 128");
    TORCH_CHECK(dq.sizes() == q.sizes() && dout.sizes() == q.sizes() && out.sizes() == q.sizes(),
                "dq/dout/out must have the shape of q");
    TORCH_CHECK(dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "dk/dv must match k/v");
    const int64_t lse_stride = lse.size(-1);
    const at::Device dev = q.device();
    c10::DeviceGuard guard(dev);
    if (zero_tensors) {
        dq.zero_();
        dk.zero_();
        dv.zero_();
    }
    at::Tensor softmax_d = at::empty({batch, nheads, lse_stride}, q.options().dtype(at::kFloat));
    at::Tensor dq_accum;
    if (bwd_needs_workspace(head_dim, p_dropout > 0.0))
        dq_accum = at::empty({total_q, nheads, head_dim}, q.options().dtype(at::kFloat));
    FaBwdArgs a{};
    a.dout = dout.data_ptr();
    a.q = q.data_ptr();
    a.k = k.data_ptr();
    a.v = v.data_ptr();
    a.out = out.data_ptr();
    a.softmax_lse = lse.data_ptr<float>();
    a.dq = dq.data_ptr();
    a.dk = dk.data_ptr();
    a.dv = dv.data_ptr();
    a.softmax_d = softmax_d.data_ptr<float>();
    a.dq_accum = dq_accum.defined() ? dq_accum.data_ptr<float>() : nullptr;
    a.cu_seqlens_q = cu_q.data_ptr<int32_t>();
    a.cu_seqlens_k = cu_k.data_ptr<int32_t>();
    a.do_row_stride = dout.stride(0);
    a.do_head_stride = dout.stride(1);
    a.q_row_stride = q.stride(0);
    a.q_head_stride = q.stride(1);
    a.k_row_stride = k.stride(0);
    a.k_head_stride = k.stride(1);
    a.v_row_stride = v.stride(0);
    a.v_head_stride = v.stride(1);
    a.o_row_stride = out.stride(0);
    a.o_head_stride = out.stride(1);
    a.dq_row_stride = dq.stride(0);
    a.dq_head_stride = dq.stride(1);
    a.dk_row_stride = dk.stride(0);
    a.dk_head_stride = dk.stride(1);
    a.dv_row_stride = dv.stride(0);
    a.dv_head_stride = dv.stride(1);
    a.batch = (int32_t)batch;
    a.nheads = (int32_t)nheads;
    a.head_dim = (int32_t)head_dim;
    a.max_seqlen_q = (int32_t)max_seqlen_q;
    a.max_seqlen_k = (int32_t)max_seqlen_k;
    a.total_q = (int32_t)total_q;
    a.lse_stride = (int32_t)lse_stride;
    a.softmax_scale = (float)softmax_scale;
    a.p_dropout = (float)p_dropout;
    a.rng_seed = seed;
    a.rng_offset = offset;
    a.rng_offset_dev = reinterpret_cast<const uint64_t *>(offset_dev);
    a.is_causal = is_causal ? 1 : 0;
    a.dtype = dt;
    const int rc = fa_bwd(&a, current_stream(dev));
    if (rc != 0) raise_rc(rc, "fa_bwd");
    return softmax_d;
}

}  // namespace

PYBIND11_MODULE(_fa_C, m) {
    m.doc() = "compiled binding of libfa_hip.so (fwd / bwd over include/fa_hip.h)";
    m.def("fwd", &fwd);
    m.def("bwd", &bwd);
    m.def("version", [] { return std::string(fa_version()); });
}
