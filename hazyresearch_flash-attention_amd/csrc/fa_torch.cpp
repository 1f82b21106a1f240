// fa_torch.cpp — compiled Python binding of libfa_hip.so (module flash_attn._fa_C).
//
// The reference binds its kernels as the pybind11 module `flash_attn_cuda` (fmha_api.cpp:244-247):
// argument checks, output allocation and the launch all run in C++. This module does the same
// over the C ABI (include/fa_hip.h) for the calls on the training path: `fwd` and `bwd`, and the
// autograd functions of flash_attn_interface / flash_attention (below), so the per-call host cost
// is one pybind11 dispatch, the at::empty allocations and the launch. flash_attn_hip.py routes its
// dense calls here (block-sparse layouts keep the ctypes path) and keeps the dropout RNG
// reservation in Python (reserve_rng), passing the reserved (seed, offset, device word) in.
//
// Checks and error messages are the ones flash_attn_hip.py raises (RuntimeError through
// TORCH_CHECK, as fmha_api.cpp:131-170 does).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/custom_function.h>
#include <torch/csrc/utils/pybind.h>

#include <cmath>
#include <cstring>
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
                            int64_t offset_dev, int64_t impl, const c10::optional<at::Tensor> &rot_cos = c10::nullopt,
                            const c10::optional<at::Tensor> &rot_sin = c10::nullopt) {
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
    if (rot_cos && rot_cos->defined()) {
        // flash_attn_hip.fwd(rotary=(cos, sin)): q rotated at the kernel's Q load
        TORCH_CHECK(rot_sin && rot_sin->defined(), "rotary needs both cos and sin tables");
        const at::Tensor &c = *rot_cos, &sn = *rot_sin;
        TORCH_CHECK(c.scalar_type() == qdt && sn.scalar_type() == qdt && c.is_cuda() && sn.is_cuda(),
                    "rotary tables must be on the GPU in q's dtype");
        TORCH_CHECK(c.dim() == 2 && c.stride(-1) == 1 && c.strides() == sn.strides() && c.sizes() == sn.sizes() &&
                        c.size(0) >= max_seqlen_q && c.size(1) >= head_dim,
                    "rotary tables must be (>= max_seqlen_q, >= head_dim) with one row stride");
        a.rot_cos = c.data_ptr();
        a.rot_sin = sn.data_ptr();
        a.rot_stride = c.stride(0);
    }
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
    TORCH_CHECK(lse.is_cuda() && q.is_cuda(), "softmax_lse and q must be on the GPU");
    TORCH_CHECK(cu_q.scalar_type() == at::kInt && cu_k.scalar_type() == at::kInt, "cu_seqlens must be int32");
    TORCH_CHECK(cu_q.is_cuda() && cu_k.is_cuda(), "cu_seqlens must be on the GPU");
    TORCH_CHECK(cu_q.is_contiguous() && cu_k.is_contiguous(), "cu_seqlens must be contiguous");
    TORCH_CHECK(cu_k.numel() == cu_q.numel(), "cu_seqlens_k must have shape (batch_size + 1)");
    const int64_t batch = cu_q.numel() - 1;
    TORCH_CHECK(batch > 0, "batch_size must be positive");
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

// ---------------------------------------------------------------------------------------------
// Autograd functions of flash_attn_interface (FlashAttnFunc / FlashAttnKVPackedFunc /
// FlashAttnQKVPackedFunc, reference flash_attn_interface.py:39-252) and of the fused-rotary
// FlashAttnRotaryQKVFunc (flash_attention.py), in C++: one pybind11 call per forward, the
// backward node runs without Python. The Python classes stay for return_attn_probs=True.
// Dropout: the caller reserves (seed, offset[, device word]) from the torch generator exactly as
// the Python functions do (flash_attn_hip.reserve_rng) and passes them in; they are saved for the
// backward (the device word as a tensor, so a captured graph's word outlives the forward).
// ---------------------------------------------------------------------------------------------
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

struct Saved {
    int64_t max_q, max_k;
    double p, scale;
    bool causal;
    uint64_t seed, offset;
    at::Tensor od;
};

void save_cfg(AutogradContext *ctx, int64_t max_q, int64_t max_k, double p, double scale, bool causal, uint64_t seed,
              uint64_t offset, const c10::optional<at::Tensor> &od) {
    ctx->saved_data["mq"] = max_q;
    ctx->saved_data["mk"] = max_k;
    ctx->saved_data["p"] = p;
    ctx->saved_data["sc"] = scale;
    ctx->saved_data["ca"] = causal;
    ctx->saved_data["se"] = (int64_t)seed;
    ctx->saved_data["of"] = (int64_t)offset;
    if (od && od->defined()) ctx->saved_data["od"] = *od;
}

Saved load_cfg(AutogradContext *ctx) {
    Saved s;
    s.max_q = ctx->saved_data["mq"].toInt();
    s.max_k = ctx->saved_data["mk"].toInt();
    s.p = ctx->saved_data["p"].toDouble();
    s.scale = ctx->saved_data["sc"].toDouble();
    s.causal = ctx->saved_data["ca"].toBool();
    s.seed = (uint64_t)ctx->saved_data["se"].toInt();
    s.offset = (uint64_t)ctx->saved_data["of"].toInt();
    auto it = ctx->saved_data.find("od");
    if (it != ctx->saved_data.end() && it->second.isTensor()) s.od = it->second.toTensor();
    return s;
}

int64_t od_ptr(const c10::optional<at::Tensor> &od) {
    return od && od->defined() ? reinterpret_cast<int64_t>(od->data_ptr()) : 0;
}

int64_t od_ptr(const at::Tensor &od) { return od.defined() ? reinterpret_cast<int64_t>(od.data_ptr()) : 0; }

// true when autograd would record a node (grad mode on and some input requires grad); otherwise
// the entry points call the forward directly, which is what apply would run
bool needs_grad(std::initializer_list<const at::Tensor *> ts) {
    if (!at::GradMode::is_enabled()) return false;
    for (const at::Tensor *t : ts)
        if (t->requires_grad()) return true;
    return false;
}

struct FlashAttnFn : public torch::autograd::Function<FlashAttnFn> {
    static variable_list forward(AutogradContext *ctx, const at::Tensor &q, const at::Tensor &k, const at::Tensor &v,
                                 const at::Tensor &cu_q, const at::Tensor &cu_k, int64_t max_q, int64_t max_k, double p,
                                 double scale, bool causal, uint64_t seed, uint64_t offset,
                                 const c10::optional<at::Tensor> &od, int64_t impl) {
        auto r = fwd(q, k, v, cu_q, cu_k, max_q, max_k, p, scale, false, causal, false, seed, offset, od_ptr(od), impl);
        ctx->save_for_backward({q, k, v, r[0], r[1], cu_q, cu_k});
        save_cfg(ctx, max_q, max_k, p, scale, causal, seed, offset, od);
        return {r[0]};
    }
    static variable_list backward(AutogradContext *ctx, variable_list g) {
        auto t = ctx->get_saved_variables();
        Saved s = load_cfg(ctx);
        at::Tensor dq = at::empty_like(t[0]), dk = at::empty_like(t[1]), dv = at::empty_like(t[2]);
        bwd(g[0], t[0], t[1], t[2], t[3], t[4], dq, dk, dv, t[5], t[6], s.max_q, s.max_k, s.p, s.scale, false,
            s.causal, s.seed, s.offset, od_ptr(s.od));
        at::Tensor n;
        return {dq, dk, dv, n, n, n, n, n, n, n, n, n, n, n};
    }
};

struct FlashAttnKVPackedFn : public torch::autograd::Function<FlashAttnKVPackedFn> {
    static variable_list forward(AutogradContext *ctx, const at::Tensor &q, const at::Tensor &kv,
                                 const at::Tensor &cu_q, const at::Tensor &cu_k, int64_t max_q, int64_t max_k, double p,
                                 double scale, bool causal, uint64_t seed, uint64_t offset,
                                 const c10::optional<at::Tensor> &od, int64_t impl) {
        TORCH_CHECK(kv.dim() == 4 && kv.size(1) == 2, "kv must be (total_k, 2, nheads, headdim)");
        auto r = fwd(q, kv.select(1, 0), kv.select(1, 1), cu_q, cu_k, max_q, max_k, p, scale, false, causal, false,
                     seed, offset, od_ptr(od), impl);
        ctx->save_for_backward({q, kv, r[0], r[1], cu_q, cu_k});
        save_cfg(ctx, max_q, max_k, p, scale, causal, seed, offset, od);
        return {r[0]};
    }
    static variable_list backward(AutogradContext *ctx, variable_list g) {
        auto t = ctx->get_saved_variables();
        Saved s = load_cfg(ctx);
        at::Tensor dq = at::empty_like(t[0]), dkv = at::empty_like(t[1]);
        bwd(g[0], t[0], t[1].select(1, 0), t[1].select(1, 1), t[2], t[3], dq, dkv.select(1, 0), dkv.select(1, 1),
            t[4], t[5], s.max_q, s.max_k, s.p, s.scale, false, s.causal, s.seed, s.offset, od_ptr(s.od));
        at::Tensor n;
        return {dq, dkv, n, n, n, n, n, n, n, n, n, n, n};
    }
};

struct FlashAttnQKVPackedFn : public torch::autograd::Function<FlashAttnQKVPackedFn> {
    static variable_list forward(AutogradContext *ctx, const at::Tensor &qkv, const at::Tensor &cu, int64_t max_s,
                                 double p, double scale, bool causal, uint64_t seed, uint64_t offset,
                                 const c10::optional<at::Tensor> &od, int64_t impl) {
        TORCH_CHECK(qkv.dim() == 4 && qkv.size(1) == 3, "qkv must be (total, 3, nheads, headdim)");
        auto r = fwd(qkv.select(1, 0), qkv.select(1, 1), qkv.select(1, 2), cu, cu, max_s, max_s, p, scale, false,
                     causal, false, seed, offset, od_ptr(od), impl);
        ctx->save_for_backward({qkv, r[0], r[1], cu});
        save_cfg(ctx, max_s, max_s, p, scale, causal, seed, offset, od);
        return {r[0]};
    }
    static variable_list backward(AutogradContext *ctx, variable_list g) {
        auto t = ctx->get_saved_variables();
        Saved s = load_cfg(ctx);
        at::Tensor dqkv = at::empty_like(t[0]);
        bwd(g[0], t[0].select(1, 0), t[0].select(1, 1), t[0].select(1, 2), t[1], t[2], dqkv.select(1, 0),
            dqkv.select(1, 1), dqkv.select(1, 2), t[3], t[3], s.max_q, s.max_k, s.p, s.scale, false, s.causal, s.seed,
            s.offset, od_ptr(s.od));
        at::Tensor n;
        return {dqkv, n, n, n, n, n, n, n, n, n};
    }
};

// fa_rotary over (B, S, NSLOT, H, D) views given by element strides (flash_attn_hip.rotary)
void rotary_call(const at::Tensor &x, const at::Tensor &y, const at::Tensor &cos, const at::Tensor &sin,
                 std::array<int64_t, 5> shape, std::array<int64_t, 4> xs, std::array<int64_t, 4> ys, int nrot,
                 bool inverse) {
    TORCH_CHECK(cos.stride(0) == sin.stride(0), "cos and sin tables must share a row stride");
    FaRotaryArgs r{};
    r.x = x.data_ptr();
    r.y = y.data_ptr();
    r.cos = cos.data_ptr();
    r.sin = sin.data_ptr();
    for (int i = 0; i < 4; ++i) {
        r.x_strides[i] = xs[i];
        r.y_strides[i] = ys[i];
    }
    r.table_stride = cos.stride(0);
    r.batch = (int32_t)shape[0];
    r.seqlen = (int32_t)shape[1];
    r.nslot = (int32_t)shape[2];
    r.nheads = (int32_t)shape[3];
    r.head_dim = (int32_t)shape[4];
    r.nrot = nrot;
    r.inverse = inverse ? 1 : 0;
    r.dtype = dtype_code(x.scalar_type());
    const int rc = fa_rotary(&r, current_stream(x.device()));
    if (rc != 0) raise_rc(rc, "fa_rotary");
}

// True when fa_fwd takes an assembly kernel for the unrotated dense call of this shape
// (include/fa_hip.h fa_fwd_kernel_name).
bool asm_forward_for(int64_t B, int64_t S, int64_t H, int64_t D, double p, bool causal, double scale,
                     at::ScalarType t, int64_t impl) {
    FaFwdArgs a{};
    a.q_row_stride = a.k_row_stride = a.v_row_stride = 3 * H * D;
    a.o_row_stride = H * D;
    a.q_head_stride = a.k_head_stride = a.v_head_stride = a.o_head_stride = D;
    a.batch = (int32_t)B;
    a.nheads = (int32_t)H;
    a.head_dim = (int32_t)D;
    a.max_seqlen_q = a.max_seqlen_k = (int32_t)S;
    a.lse_stride = (int32_t)std::max<int64_t>(round16(S), 16);
    a.softmax_scale = (float)scale;
    a.p_dropout = (float)p;
    a.is_causal = causal ? 1 : 0;
    a.dtype = dtype_code(t);
    a.impl = (int32_t)impl;
    const char *name = fa_fwd_kernel_name(&a);
    return name != nullptr && std::strstr(name, "_asm") != nullptr;
}

// FlashAttnRotaryQKVFunc (flash_attention.py): padded contiguous qkv (B, S, 3, H, D); k rotated by
// one fa_rotary pass, q rotated inside the forward at its load; backward rotates q once more, runs
// the attention backward on (q_rot, k_rot, v) and rotates dq, dk back in place. `impl` is the
// caller's effective kernel family (flash_attn_hip.force_impl): the route (assembly forward on a
// pre-rotated q/k buffer, or the HIP forward rotating q at its load) is decided for the kernel
// that call will really take, and the forward is launched with the same impl.
// Activation memory: on the assembly route the saved tensor is the (B, S, 2, H, D) rotated q/k
// buffer (one B*S*H*D 16-bit tensor more than the HIP route's rotated k), which saves the
// backward's q rotary pass.
struct FlashAttnRotaryQKVFn : public torch::autograd::Function<FlashAttnRotaryQKVFn> {
    static variable_list forward(AutogradContext *ctx, const at::Tensor &qkv, const at::Tensor &cos_in,
                                 const at::Tensor &sin_in, const at::Tensor &cu, double p, double scale, bool causal,
                                 uint64_t seed, uint64_t offset, const c10::optional<at::Tensor> &od, int64_t impl) {
        TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.is_contiguous(), "qkv must be contiguous (B, S, 3, H, D)");
        const int64_t B = qkv.size(0), S = qkv.size(1), H = qkv.size(3), D = qkv.size(4);
        c10::DeviceGuard guard(qkv.device());
        at::Tensor cos = cos_in.slice(0, 0, S).contiguous(), sin = sin_in.slice(0, 0, S).contiguous();
        at::Tensor flat = qkv.view({B * S, 3, H, D});
        if (asm_forward_for(B, S, H, D, p, causal, scale, qkv.scalar_type(), impl)) {
            // the Q rotation at the kernel's Q load exists in the HIP forward only: where fa_fwd takes an
            // assembly kernel, one fa_rotary pass rotates q and k into (B, S, 2, H, D) and the assembly
            // forward reads them (the backward reuses both rotated tensors: no second q pass)
            at::Tensor qk_rot = at::empty({B, S, 2, H, D}, qkv.options());
            rotary_call(qkv, qk_rot, cos, sin, {B, S, 2, H, D}, {S * 3 * H * D, 3 * H * D, H * D, D},
                        {S * 2 * H * D, 2 * H * D, H * D, D}, 2, false);
            at::Tensor qk = qk_rot.view({B * S, 2, H, D});
            auto r = fwd(qk.select(1, 0), qk.select(1, 1), flat.select(1, 2), cu, cu, S, S, p, scale, false, causal,
                         false, seed, offset, od_ptr(od), impl);
            ctx->save_for_backward({qkv, qk_rot, r[0], r[1], cos, sin, cu});
            save_cfg(ctx, S, S, p, scale, causal, seed, offset, od);
            return {r[0].view({B, S, H, D})};
        }
        at::Tensor k_rot = at::empty({B, S, H, D}, qkv.options());
        rotary_call(qkv.select(2, 1), k_rot, cos, sin, {B, S, 1, H, D}, {S * 3 * H * D, 3 * H * D, 0, D},
                    {S * H * D, H * D, 0, D}, 1, false);
        auto r = fwd(flat.select(1, 0), k_rot.view({B * S, H, D}), flat.select(1, 2), cu, cu, S, S, p, scale, false,
                     causal, false, seed, offset, od_ptr(od), impl, cos, sin);
        ctx->save_for_backward({qkv, k_rot, r[0], r[1], cos, sin, cu});
        save_cfg(ctx, S, S, p, scale, causal, seed, offset, od);
        return {r[0].view({B, S, H, D})};
    }
    static variable_list backward(AutogradContext *ctx, variable_list g) {
        auto t = ctx->get_saved_variables();
        Saved s = load_cfg(ctx);
        const at::Tensor &qkv = t[0], &k_rot = t[1], &out = t[2], &lse = t[3], &cos = t[4], &sin = t[5], &cu = t[6];
        const int64_t B = qkv.size(0), S = qkv.size(1), H = qkv.size(3), D = qkv.size(4);
        c10::DeviceGuard guard(qkv.device());
        at::Tensor q_rot, kr;
        if (k_rot.dim() == 5) {     // (B, S, 2, H, D): q and k rotated by the forward (assembly forward)
            at::Tensor qk = k_rot.view({B * S, 2, H, D});
            q_rot = qk.select(1, 0);
            kr = qk.select(1, 1);
        } else {
            q_rot = at::empty({B, S, H, D}, qkv.options());
            rotary_call(qkv.select(2, 0), q_rot, cos, sin, {B, S, 1, H, D}, {S * 3 * H * D, 3 * H * D, 0, D},
                        {S * H * D, H * D, 0, D}, 1, false);
            q_rot = q_rot.view({B * S, H, D});
            kr = k_rot.view({B * S, H, D});
        }
        at::Tensor dqkv = at::empty_like(qkv);
        at::Tensor d = dqkv.view({B * S, 3, H, D});
        bwd(g[0].reshape({B * S, H, D}), q_rot, kr,
            qkv.view({B * S, 3, H, D}).select(1, 2), out, lse, d.select(1, 0), d.select(1, 1), d.select(1, 2), cu, cu,
            S, S, s.p, s.scale, false, s.causal, s.seed, s.offset, od_ptr(s.od));
        const std::array<int64_t, 4> st3{S * 3 * H * D, 3 * H * D, H * D, D};
        rotary_call(dqkv, dqkv, cos, sin, {B, S, 3, H, D}, st3, st3, 2, true);   // dq, dk back; dv as is
        at::Tensor n;
        return {dqkv, n, n, n, n, n, n, n, n, n, n};
    }
};

// ---- bert_padding row moves (flash_attn/bert_padding.py: index_first_axis / index_put_first_axis,
// the reference's flash_attn/bert_padding.py:11-64). The rows of x are made addressable as row_stride-spaced
// runs of row_bytes (the inner dimensions contiguous, rows neither overlapping nor broadcast), as
// bert_padding._rows does, else x is copied out first.
at::Tensor padding_rows(const at::Tensor &x, int64_t &row_stride, int64_t &row_bytes) {
    TORCH_CHECK(x.dim() >= 2, "row moves need at least 2 dimensions");
    int64_t want = 1, row_elems = 1;
    bool ok = true;
    for (int64_t d = x.dim() - 1; d >= 1; --d) {
        if (ok && x.size(d) != 1 && x.stride(d) != want) ok = false;
        want *= x.size(d);
        row_elems *= x.size(d);
    }
    if (ok && x.size(0) > 1 && x.stride(0) < row_elems) ok = false;
    at::Tensor y = ok ? x : x.contiguous();
    const int64_t es = y.element_size();
    row_stride = y.size(0) > 1 ? y.stride(0) * es : row_elems * es;
    row_bytes = row_elems * es;
    return y;
}

at::Tensor padding_index(const at::Tensor &indices, const at::Tensor &x) {
    TORCH_CHECK(indices.dim() == 1, "indices must be 1-D");
    TORCH_CHECK(indices.device() == x.device(), "indices must be on the tensor's device");
    return (indices.scalar_type() == at::kLong ? indices : indices.to(at::kLong)).contiguous();
}

// out[i] = src[indices[i]] along dim 0
at::Tensor gather_rows(const at::Tensor &src_in, const at::Tensor &indices) {
    c10::DeviceGuard guard(src_in.device());
    int64_t ss = 0, rb = 0;
    at::Tensor src = padding_rows(src_in, ss, rb);
    at::Tensor idx = padding_index(indices, src);
    if (rb % 2) return src.index_select(0, idx);     // odd-byte rows (1-byte dtypes): the C ABI moves 2-byte words
    std::vector<int64_t> sizes = src.sizes().vec();
    sizes[0] = idx.size(0);
    at::Tensor out = at::empty(sizes, src.options());
    if (out.numel() == 0) return out;
    const int rc = fa_index_first_axis(src.data_ptr(), src.size(0), ss, idx.data_ptr<int64_t>(), idx.size(0),
                                       out.data_ptr(), rb, rb, current_stream(src.device()));
    if (rc != 0) raise_rc(rc, "fa_index_first_axis");
    return out;
}

// out = zeros(first_axis_dim, ...); out[indices[i]] = values[i]
at::Tensor pad_rows(const at::Tensor &values_in, const at::Tensor &indices, int64_t first_axis_dim) {
    c10::DeviceGuard guard(values_in.device());
    int64_t vs = 0, rb = 0;
    at::Tensor values = padding_rows(values_in, vs, rb);
    at::Tensor idx = padding_index(indices, values);
    std::vector<int64_t> sizes = values.sizes().vec();
    sizes[0] = first_axis_dim;
    if (rb % 2) return at::zeros(sizes, values.options()).index_copy_(0, idx, values);   // odd-byte rows
    at::Tensor out = at::empty(sizes, values.options());
    if (out.numel() == 0) return out;
    at::Tensor ws = at::empty({first_axis_dim}, values.options().dtype(at::kInt));
    const int rc = fa_index_put_first_axis(values.data_ptr(), vs, idx.data_ptr<int64_t>(), idx.size(0), out.data_ptr(),
                                           first_axis_dim, rb, rb, ws.data_ptr<int32_t>(), current_stream(values.device()));
    if (rc != 0) raise_rc(rc, "fa_index_put_first_axis");
    return out;
}

struct IndexFirstAxisFn : public torch::autograd::Function<IndexFirstAxisFn> {
    static variable_list forward(AutogradContext *ctx, const at::Tensor &input, const at::Tensor &indices) {
        ctx->save_for_backward({indices});
        ctx->saved_data["n"] = input.size(0);
        return {gather_rows(input, indices)};
    }
    static variable_list backward(AutogradContext *ctx, variable_list g) {
        auto t = ctx->get_saved_variables();
        return {pad_rows(g[0], t[0], ctx->saved_data["n"].toInt()), at::Tensor()};
    }
};

struct IndexPutFirstAxisFn : public torch::autograd::Function<IndexPutFirstAxisFn> {
    static variable_list forward(AutogradContext *ctx, const at::Tensor &values, const at::Tensor &indices,
                                 int64_t first_axis_dim) {
        ctx->save_for_backward({indices});
        return {pad_rows(values, indices, first_axis_dim)};
    }
    static variable_list backward(AutogradContext *ctx, variable_list g) {
        auto t = ctx->get_saved_variables();
        return {gather_rows(g[0], t[0]), at::Tensor(), at::Tensor()};
    }
};

}  // namespace

PYBIND11_MODULE(_fa_C, m) {
    m.doc() = "compiled binding of libfa_hip.so (fwd / bwd over include/fa_hip.h)";
    m.def("fwd", &fwd, pybind11::arg("q"), pybind11::arg("k"), pybind11::arg("v"), pybind11::arg("cu_q"),
          pybind11::arg("cu_k"), pybind11::arg("max_seqlen_q"), pybind11::arg("max_seqlen_k"), pybind11::arg("p_dropout"),
          pybind11::arg("softmax_scale"), pybind11::arg("zero_tensors"), pybind11::arg("is_causal"),
          pybind11::arg("return_softmax"), pybind11::arg("seed"), pybind11::arg("offset"), pybind11::arg("offset_dev"),
          pybind11::arg("impl"), pybind11::arg("rot_cos") = pybind11::none(), pybind11::arg("rot_sin") = pybind11::none());
    m.def("bwd", &bwd);
    m.def("flash_attn_unpadded_func",
          [](const at::Tensor &q, const at::Tensor &k, const at::Tensor &v, const at::Tensor &cu_q, const at::Tensor &cu_k,
             int64_t max_q, int64_t max_k, double p, c10::optional<double> scale_opt, bool causal, uint64_t seed,
             uint64_t offset, const c10::optional<at::Tensor> &od, int64_t impl) {
              const double scale = scale_opt ? *scale_opt : 1.0 / std::sqrt((double)q.size(-1));
              if (!needs_grad({&q, &k, &v}))   // no graph to record: the forward alone, same result
                  return fwd(q, k, v, cu_q, cu_k, max_q, max_k, p, scale, false, causal, false, seed, offset, od_ptr(od),
                             impl)[0];
              return FlashAttnFn::apply(q, k, v, cu_q, cu_k, max_q, max_k, p, scale, causal, seed, offset, od, impl)[0];
          });
    m.def("flash_attn_unpadded_kvpacked_func",
          [](const at::Tensor &q, const at::Tensor &kv, const at::Tensor &cu_q, const at::Tensor &cu_k, int64_t max_q,
             int64_t max_k, double p, c10::optional<double> scale_opt, bool causal, uint64_t seed, uint64_t offset,
             const c10::optional<at::Tensor> &od, int64_t impl) {
              const double scale = scale_opt ? *scale_opt : 1.0 / std::sqrt((double)q.size(-1));
              TORCH_CHECK(kv.dim() == 4 && kv.size(1) == 2, "kv must be (total_k, 2, nheads, headdim)");
              if (!needs_grad({&q, &kv}))
                  return fwd(q, kv.select(1, 0), kv.select(1, 1), cu_q, cu_k, max_q, max_k, p, scale, false, causal,
                             false, seed, offset, od_ptr(od), impl)[0];
              return FlashAttnKVPackedFn::apply(q, kv, cu_q, cu_k, max_q, max_k, p, scale, causal, seed, offset, od,
                                                impl)[0];
          });
    m.def("flash_attn_unpadded_qkvpacked_func",
          [](const at::Tensor &qkv, const at::Tensor &cu, int64_t max_s, double p, c10::optional<double> scale_opt,
             bool causal, uint64_t seed, uint64_t offset, const c10::optional<at::Tensor> &od, int64_t impl) {
              const double scale = scale_opt ? *scale_opt : 1.0 / std::sqrt((double)qkv.size(-1));
              TORCH_CHECK(qkv.dim() == 4 && qkv.size(1) == 3, "qkv must be (total, 3, nheads, headdim)");
              if (!needs_grad({&qkv}))
                  return fwd(qkv.select(1, 0), qkv.select(1, 1), qkv.select(1, 2), cu, cu, max_s, max_s, p, scale,
                             false, causal, false, seed, offset, od_ptr(od), impl)[0];
              return FlashAttnQKVPackedFn::apply(qkv, cu, max_s, p, scale, causal, seed, offset, od, impl)[0];
          });
    m.def("flash_attn_rotary_qkv_func",
          [](const at::Tensor &qkv, const at::Tensor &cos, const at::Tensor &sin, const at::Tensor &cu, double p,
             double scale, bool causal, uint64_t seed, uint64_t offset, const c10::optional<at::Tensor> &od,
             int64_t impl) {
              return FlashAttnRotaryQKVFn::apply(qkv, cos, sin, cu, p, scale, causal, seed, offset, od, impl)[0];
          });
    m.def("index_first_axis", [](const at::Tensor &input, const at::Tensor &indices) {
        TORCH_CHECK(input.dim() >= 2, "index_first_axis: input must have at least 2 dimensions");
        if (!needs_grad({&input})) return gather_rows(input, indices);
        return IndexFirstAxisFn::apply(input, indices)[0];
    });
    m.def("index_put_first_axis", [](const at::Tensor &values, const at::Tensor &indices, int64_t first_axis_dim) {
        TORCH_CHECK(indices.dim() == 1 && values.dim() >= 2, "index_put_first_axis: 1-D indices, values of 2+ dims");
        if (!needs_grad({&values})) return pad_rows(values, indices, first_axis_dim);
        return IndexPutFirstAxisFn::apply(values, indices, first_axis_dim)[0];
    });
    m.def("version", [] { return std::string(fa_version()); });
}
