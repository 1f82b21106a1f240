// fa_launch.h — host launchers for the gfx950 kernels (one translation unit per head-dim tile).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
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

#ifndef FA_BWD_DQK
#define FA_BWD_DQK 1        // 1: D = 128 dense, no dropout: dQ by the query-major fa_bwd_dq_kernel
#endif
// true when launch_bwd writes dq itself (no fp32 accumulator, no convert pass)
#ifndef FA_BWD_DQK_MIN_D
#define FA_BWD_DQK_MIN_D 128   // smallest head-dim tile that takes the query-major dQ pass
#endif
constexpr bool bwd_dqk_tile(int D) { return FA_BWD_DQK && D >= FA_BWD_DQK_MIN_D; }
inline bool bwd_dq_direct(const FaBwdArgs &a, const FaBlockMask &bm) {
    const int tile = a.head_dim <= 32 ? 32 : a.head_dim <= 64 ? 64 : 128;
    return bwd_dqk_tile(tile) && a.p_dropout == 0.f && bm.mask == nullptr;
}
hipError_t launch_bwd_post(const FaBwdArgs &a, hipStream_t stream);
hipError_t launch_zero_seq_rows(void *base, const int32_t *cu, int64_t row_stride, int64_t head_stride, int batch,
                                int nheads, int head_dim, int max_seqlen, hipStream_t s);
// hand-scheduled assembly forward (fa_asm.cpp, csrc/asm/gen_fwd.py)
bool fwd_asm_eligible(const FaFwdArgs &a, const FaBlockMask &bm);
// symbol name of the code object launch_fwd_asm would run for a
const char *asm_kernel_name(const FaFwdArgs &a);
// *unavailable is set (and hipSuccess returned, nothing launched) when the device's code objects
// could not be loaded: the caller then runs the HIP kernels (fa_asm.cpp load_all).
hipError_t launch_fwd_asm(const FaFwdArgs &a, hipStream_t stream, bool *unavailable);
// assembly-forward launches this process has enqueued or captured so far (fa_query)
int64_t asm_launch_count();

// Raise a kernel's dynamic-LDS limit once per (kernel, device): the attribute is per device, so
// a process that launches on several GPUs sets it on each. `done` is the call site's own bit set
// (one static per template instantiation); devices >= 64 are set on every launch.
template <typename K>
static hipError_t ensure_lds(std::atomic<uint64_t> &done, K kern, int lds) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = dev < 64 ? 1ull << dev : 0;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
    e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_release);
    return e;
}
// Compute units of the current device (cached per device; 0 if unknown).
static inline int device_cus() {
    static std::atomic<int> cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (dev < 64) {
        const int c = cus[dev].load(std::memory_order_relaxed);
        if (c) return c;
    }
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (dev < 64) cus[dev].store(n, std::memory_order_relaxed);
    return n;
}
#define FA_ENSURE_LDS(kern, lds)                                   \
    do {                                                           \
        static std::atomic<uint64_t> fa_lds_done_{0};              \
        const hipError_t fa_e_ = ensure_lds(fa_lds_done_, kern, lds); \
        if (fa_e_ != hipSuccess) return fa_e_;                     \
    } while (0)
}  // namespace fa
