// fa_kernels_impl.h — template launchers; included by fa_d{32,64,128}.hip.
#pragma once
#include "fa_launch.h"
#include "fa_fwd_kernel.h"
#include "fa_bwd_kernel.h"
#include "fa_bwd_split_kernel.h"
#include "fa_bwd_dq_kernel.h"

#ifndef FA_BWD_DQ_NW
#define FA_BWD_DQ_NW 8   // waves (32 query rows each) per dQ-pass workgroup
#endif

#include <cstdlib>

namespace fa {

// Workgroups of one kernel that run at once on one XCD (occupancy per CU x CUs / 8), the `slots`
// argument of the causal block orders (fa_common.h xcd_grouped). Called from each launcher
// template instantiation, so the cached value is per kernel.
// Measured (tools/ab_libs.sh, C3/C4 event times): groups of 2x the occupancy-derived slots run
// C4's causal forward 872 vs 891 us (x1) and 935 (global order), its backward 3375 vs 3411 /
// 3665, and C3's forward as fast as the global order (x1: +13 %)
#ifndef FA_XCD_SLOTS_MUL
#define FA_XCD_SLOTS_MUL 2
#endif
template <class K>
static int xcd_slots_of(K kern, int threads, int lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, threads, lds) != hipSuccess || n < 1) n = 1;
    const int cus = device_cus();
    return n * (cus > 0 ? cus : 256) / 8 * FA_XCD_SLOTS_MUL;
}

template <int D, typename T, bool CAUSAL, bool DROPOUT, int NW, bool SPARSE = false, bool KSPLIT = false>
static hipError_t launch_fwd_nw(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t stream) {
    using C = FwdCfg<D, NW, KSPLIT>;
    const int lds = C::lds_bytes(DROPOUT);
    auto kern = fa_fwd_kernel<D, T, CAUSAL, DROPOUT, NW, SPARSE, KSPLIT>;
    FA_ENSURE_LDS(kern, lds);
    static const int slots = xcd_slots_of(kern, C::NT, lds);
    dim3 grid((a.max_seqlen_q + C::BM - 1) / C::BM, a.nheads, a.batch);
    hipLaunchKernelGGL(kern, grid, dim3(C::NT), lds, stream, a, bm, slots);
    return hipGetLastError();
}

#ifndef FA_FWD_NW_DEFAULT
#define FA_FWD_NW_DEFAULT 8
#endif
// Waves per workgroup. 8 (256 query rows, two workgroups per CU at 128 registers) measured
// fastest without dropout on the BASELINE configs, except when the 8-wave grid fills less than
// two rounds of CU slots unevenly (fewer than 2 * CUs workgroups, not a multiple of the CU
// count): some CUs would then run two workgroups and others one, and 4-wave workgroups (four
// per CU) spread the same rows evenly. B4 H12 S2048 D64 (384 workgroups): 793 vs 728 TF/s; C5
// (256 = one per CU) and C2 (192) keep 8 (808 vs 842, 424 vs 431). With dropout the kernel
// needs ~168 registers: 8-wave workgroups then fit one per CU (two waves per SIMD), 4-wave
// ones three per CU, and C3's forward runs 457 vs 369 TF/s. The choice is made here only (no
// run-time override): 1 = split-K (below), 4 or 8 waves.
//
// Split-K (code 1, KSPLIT kernels): when the 8-wave grid has at most one workgroup per CU, each
// workgroup's latency is the whole kernel, so the two halves of a workgroup take the same 128
// query rows and half the keys each and merge at the end: twice the workgroups, half the tile
// walk per wave. Taken when the doubled grid still lands evenly (at most one workgroup per CU,
// or exactly two): C5 (256 -> 512 workgroups) 823 vs 803 TF/s; C2 (192 -> 384, half the CUs
// would run two) measured 391 vs 432 and keeps the plain kernel. Dense non-causal D <= 64
// without dropout only.
#ifndef FA_FWD_KSPLIT
#define FA_FWD_KSPLIT 1
#endif
template <int D, bool CAUSAL, bool DROPOUT>
static int pick_fwd_waves(const FaFwdArgs &a) {
    if (DROPOUT && D <= 64) return 4;
    const int64_t nwg8 = (int64_t)((a.max_seqlen_q + 255) / 256) * a.nheads * a.batch;
    const int cus = device_cus();
    if (FA_FWD_KSPLIT && !CAUSAL && D <= 64 && cus > 0 && (2 * nwg8 <= cus || 2 * nwg8 == 2 * cus)) return 1;
    if (cus > 0 && nwg8 > cus && nwg8 < 2 * cus && nwg8 % cus != 0) return 4;
    return FA_FWD_NW_DEFAULT;
}

template <int D, typename T, bool CAUSAL, bool DROPOUT>
static hipError_t launch_fwd_t(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t stream) {
    if (bm.mask) return launch_fwd_nw<D, T, CAUSAL, DROPOUT, 8, true>(a, bm, stream);
    switch (pick_fwd_waves<D, CAUSAL, DROPOUT>(a)) {
        case 1:
            if constexpr (!CAUSAL && !DROPOUT && D <= 64) return launch_fwd_nw<D, T, false, false, 8, false, true>(a, bm, stream);
            return launch_fwd_nw<D, T, CAUSAL, DROPOUT, 8>(a, bm, stream);
        case 4: return launch_fwd_nw<D, T, CAUSAL, DROPOUT, 4>(a, bm, stream);
        default: return launch_fwd_nw<D, T, CAUSAL, DROPOUT, 8>(a, bm, stream);
    }
}

template <int D, typename T, bool CAUSAL, bool DROPOUT, bool SPARSE>
static hipError_t launch_bwd_s(const FaBwdArgs &a, const FaBlockMask &bm, hipStream_t stream) {
    // D = 128: the P / dS wave split (fa_bwd_split_kernel.h); D <= 64: fa_bwd_kernel. dQ either by
    // the main kernel's atomics or by the query-major pass (bwd_dq_direct)
    if constexpr (D == 128) {
        constexpr bool DQK = bwd_dqk_tile(D) && !DROPOUT && !SPARSE;
        using C = BwdSplitCfgOf<D, CAUSAL, DROPOUT, SPARSE, !DQK>;
        auto kern = fa_bwd_split_kernel<D, T, CAUSAL, DROPOUT, SPARSE, !DQK>;
        FA_ENSURE_LDS(kern, C::LDS_BYTES);
        static const int slots = xcd_slots_of(kern, C::NT, C::LDS_BYTES);
        dim3 grid((a.max_seqlen_k + C::BKV - 1) / C::BKV, a.nheads, a.batch);
        hipLaunchKernelGGL(kern, grid, dim3(C::NT), C::LDS_BYTES, stream, a, bm, slots);
        if constexpr (DQK) {
            constexpr int NWQ = FA_BWD_DQ_NW;
            using CQ = DqCfg<D, NWQ>;
            auto kq = fa_bwd_dq_kernel<D, T, CAUSAL, NWQ>;
            FA_ENSURE_LDS(kq, CQ::LDS_BYTES);
            static const int qslots = xcd_slots_of(kq, CQ::NT, CQ::LDS_BYTES);
            dim3 gq((a.max_seqlen_q + CQ::BM - 1) / CQ::BM, a.nheads, a.batch);
            hipLaunchKernelGGL(kq, gq, dim3(CQ::NT), CQ::LDS_BYTES, stream, a, qslots);
        }
        return hipGetLastError();
    } else {
        using C = BwdCfg<D, BwdWaves<CAUSAL>::value, CAUSAL>;
        constexpr bool DQK = bwd_dqk_tile(D) && !DROPOUT && !SPARSE;
        auto kern = fa_bwd_kernel<D, T, CAUSAL, DROPOUT, SPARSE, !DQK>;
        FA_ENSURE_LDS(kern, C::LDS_BYTES);
        static const int slots = xcd_slots_of(kern, C::NT, C::LDS_BYTES);
        dim3 grid((a.max_seqlen_k + C::BKV - 1) / C::BKV, a.nheads, a.batch);
        hipLaunchKernelGGL(kern, grid, dim3(C::NT), C::LDS_BYTES, stream, a, bm, slots);
        if constexpr (DQK) {
            constexpr int NWQ = FA_BWD_DQ_NW;
            using CQ = DqCfg<D, NWQ>;
            auto kq = fa_bwd_dq_kernel<D, T, CAUSAL, NWQ>;
            FA_ENSURE_LDS(kq, CQ::LDS_BYTES);
            static const int qslots = xcd_slots_of(kq, CQ::NT, CQ::LDS_BYTES);
            dim3 gq((a.max_seqlen_q + CQ::BM - 1) / CQ::BM, a.nheads, a.batch);
            hipLaunchKernelGGL(kq, gq, dim3(CQ::NT), CQ::LDS_BYTES, stream, a, qslots);
        }
        return hipGetLastError();
    }
}

template <int D, typename T, bool CAUSAL, bool DROPOUT>
static hipError_t launch_bwd_t(const FaBwdArgs &a, const FaBlockMask &bm, hipStream_t stream) {
    return bm.mask ? launch_bwd_s<D, T, CAUSAL, DROPOUT, true>(a, bm, stream)
                   : launch_bwd_s<D, T, CAUSAL, DROPOUT, false>(a, bm, stream);
}

template <int D, typename T>
static hipError_t launch_fwd_dt(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t s) {
    const bool dropout = a.p_dropout > 0.f;
    if (a.is_causal) return dropout ? launch_fwd_t<D, T, true, true>(a, bm, s) : launch_fwd_t<D, T, true, false>(a, bm, s);
    return dropout ? launch_fwd_t<D, T, false, true>(a, bm, s) : launch_fwd_t<D, T, false, false>(a, bm, s);
}

template <int D, typename T>
static hipError_t launch_bwd_dt(const FaBwdArgs &a, const FaBlockMask &bm, hipStream_t s) {
    const bool dropout = a.p_dropout > 0.f;
    if (a.is_causal) return dropout ? launch_bwd_t<D, T, true, true>(a, bm, s) : launch_bwd_t<D, T, true, false>(a, bm, s);
    return dropout ? launch_bwd_t<D, T, false, true>(a, bm, s) : launch_bwd_t<D, T, false, false>(a, bm, s);
}

}  // namespace fa

// One translation unit per head-dim tile and direction, so each compiles in parallel and can
// take its own scheduler flags (build.py SOURCE_FLAGS)
#define FA_INSTANTIATE_FWD(D)                                                                    \
    namespace fa {                                                                               \
    template <> hipError_t launch_fwd<D>(const FaFwdArgs &a, const FaBlockMask &bm, hipStream_t s) { \
        return a.dtype == FA_DTYPE_BF16 ? launch_fwd_dt<D, Bf16>(a, bm, s) : launch_fwd_dt<D, Fp16>(a, bm, s); \
    }                                                                                            \
    }
#define FA_INSTANTIATE_BWD(D)                                                                    \
    namespace fa {                                                                               \
    template <> hipError_t launch_bwd<D>(const FaBwdArgs &a, const FaBlockMask &bm, hipStream_t s) { \
        return a.dtype == FA_DTYPE_BF16 ? launch_bwd_dt<D, Bf16>(a, bm, s) : launch_bwd_dt<D, Fp16>(a, bm, s); \
    }                                                                                            \
    }
