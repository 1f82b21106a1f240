// fa_aux.hip — auxiliary kernels: backward pre/post passes and the attention-probability writer.
#include "fa_launch.h"
#include "fa_bwd_kernel.h"

namespace fa {

template <typename T, bool CAUSAL, bool DROPOUT>
static hipError_t launch_probs_t(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t stream) {
    dim3 grid((a.s_rows + 31) / 32, a.nheads, a.batch);
    hipLaunchKernelGGL((fa_probs_kernel<T, CAUSAL, DROPOUT>), grid, dim3(256), 0, stream, a, bm);
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_probs_dt(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t s) {
    const bool dropout = a.p_dropout > 0.f;
    if (a.is_causal) return dropout ? launch_probs_t<T, true, true>(a, bm, s) : launch_probs_t<T, true, false>(a, bm, s);
    return dropout ? launch_probs_t<T, false, true>(a, bm, s) : launch_probs_t<T, false, false>(a, bm, s);
}

hipError_t launch_probs(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t s) {
    return a.dtype == FA_DTYPE_BF16 ? launch_probs_dt<Bf16>(a, bm, s) : launch_probs_dt<Fp16>(a, bm, s);
}

hipError_t launch_bwd_pre(const FaBwdArgs &a, hipStream_t s) {
    dim3 grid((a.max_seqlen_q + 15) / 16, a.nheads, a.batch);
    if (a.dtype == FA_DTYPE_BF16)
        hipLaunchKernelGGL(fa_bwd_dot_kernel<Bf16>, grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(fa_bwd_dot_kernel<Fp16>, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_bwd_post(const FaBwdArgs &a, hipStream_t s) {
    const int64_t total = (int64_t)a.total_q * a.nheads * (a.head_dim / 8);
    if (total == 0) return hipSuccess;
    dim3 grid((unsigned)((total + 255) / 256));
    if (a.dtype == FA_DTYPE_BF16)
        hipLaunchKernelGGL(fa_bwd_dq_convert_kernel<Bf16>, grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(fa_bwd_dq_convert_kernel<Fp16>, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace fa
