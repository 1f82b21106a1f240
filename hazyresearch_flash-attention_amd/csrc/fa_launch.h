// fa_launch.h — host launchers for the gfx950 kernels (one translation unit per head-dim tile).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/fa_hip.h"

namespace fa {
// D is the padded head-dim tile (32, 64 or 128); the kernels zero-fill head_dim < D.
// bm.mask == nullptr: dense; otherwise the block-sparse kernels (fa_fwd_block / fa_bwd_block).
template <int D> hipError_t launch_fwd(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t stream);
template <int D> hipError_t launch_bwd(const FaBwdArgs &a, const FaBlockMask &bm, hipStream_t stream);
hipError_t launch_probs(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t stream);
hipError_t launch_gather_rows(const void *src, int64_t src_rows, int64_t src_stride, const int64_t *idx, int64_t n,
                              void *dst, int64_t dst_stride, int64_t row_bytes, hipStream_t s);
hipError_t launch_pad_rows(const void *src, int64_t src_stride, const int64_t *idx, int64_t n, void *dst,
                           int64_t dst_rows, int64_t dst_stride, int64_t row_bytes, int32_t *inv, hipStream_t s);
hipError_t launch_scatter_add_rows(const void *src, int64_t src_stride, const int64_t *idx, int64_t n, void *dst,
                                   int64_t dst_rows, int64_t dst_stride, int64_t elems_per_row, int dtype,
                                   hipStream_t s);
hipError_t launch_rotary(const FaRotaryArgs &a, hipStream_t s);
hipError_t launch_bwd_pre(const FaBwdArgs &a, hipStream_t stream);

#ifndef FA_BWD_SPLIT128
#define FA_BWD_SPLIT128 1   // 1: D = 128 backward with the P / dS wave split (fa_bwd_split_kernel.h)
#endif
#ifndef FA_BWD_DQK
#define FA_BWD_DQK 1        // 1: D = 128 dense, no dropout: dQ by the query-major fa_bwd_dq_kernel
#endif
// true when launch_bwd writes dq itself (no fp32 accumulator, no convert pass)
#ifndef FA_BWD_DQK_MIN_D
#define FA_BWD_DQK_MIN_D 128   // smallest head-dim tile that takes the query-major dQ pass
#endif
constexpr bool bwd_dqk_tile(int D) { return FA_BWD_DQK && D >= FA_BWD_DQK_MIN_D && (D < 128 || FA_BWD_SPLIT128); }
inline bool bwd_dq_direct(const FaBwdArgs &a, const FaBlockMask &bm) {
    const int tile = a.head_dim <= 32 ? 32 : a.head_dim <= 64 ? 64 : 128;
    return bwd_dqk_tile(tile) && a.p_dropout == 0.f && bm.mask == nullptr && a.max_seqlen_k > 0;
}
hipError_t launch_bwd_post(const FaBwdArgs &a, hipStream_t stream);
}  // namespace fa
