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

template <typename T, int CPR>
static void launch_dot(const FaBwdArgs &a, hipStream_t s) {
    dim3 grid((a.max_seqlen_q + 256 / CPR - 1) / (256 / CPR), a.nheads, a.batch);
    hipLaunchKernelGGL((fa_bwd_dot_kernel<T, CPR>), grid, dim3(256), 0, s, a);
}

template <typename T>
static void launch_dot_t(const FaBwdArgs &a, hipStream_t s) {
    if (a.head_dim <= 32)
        launch_dot<T, 4>(a, s);
    else if (a.head_dim <= 64)
        launch_dot<T, 8>(a, s);
    else
        launch_dot<T, 16>(a, s);
}

hipError_t launch_bwd_pre(const FaBwdArgs &a, hipStream_t s) {
    if (a.dtype == FA_DTYPE_BF16)
        launch_dot_t<Bf16>(a, s);
    else
        launch_dot_t<Fp16>(a, s);
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

// Zero the rows of every sequence of a (total, H, D) 16-bit tensor (any row / head stride):
// one thread per 16-byte chunk. Used for gradients that have no contribution at all: dk/dv when
// there are no query rows, dq when there are no keys.
__global__ __launch_bounds__(256) void zero_seq_rows_kernel(uint16_t *base, const int32_t *cu, int64_t row_stride,
                                                            int64_t head_stride, int head_dim) {
    const int b = blockIdx.z, h = blockIdx.y;
    const int start = cu[b];
    const int len = cu[b + 1] - start;
    const int nc = head_dim / 8;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    const int row = idx / nc, c = idx % nc;
    if (row >= len) return;
    const u32x4 z = {0u, 0u, 0u, 0u};
    gstore128(base + (int64_t)(start + row) * row_stride + (int64_t)h * head_stride + c * 8, z);
}

hipError_t launch_zero_seq_rows(void *base, const int32_t *cu, int64_t row_stride, int64_t head_stride, int batch,
                                int nheads, int head_dim, int max_seqlen, hipStream_t s) {
    if (max_seqlen <= 0 || batch <= 0 || nheads <= 0) return hipSuccess;
    const int64_t chunks = (int64_t)max_seqlen * (head_dim / 8);
    dim3 grid((unsigned)((chunks + 255) / 256), nheads, batch);
    hipLaunchKernelGGL(zero_seq_rows_kernel, grid, dim3(256), 0, s, (uint16_t *)base, cu, row_stride, head_stride,
                       head_dim);
    return hipGetLastError();
}

}  // namespace fa
