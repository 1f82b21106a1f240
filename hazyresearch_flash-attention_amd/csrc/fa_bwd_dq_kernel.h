// fa_bwd_dq_kernel.h — query-major dQ pass of the FlashAttention backward (gfx950).
//
// dQ = scale * dS K with dS = P * (dP - delta), P = exp(scale * Q K^T - lse), dP = dO V^T
// (the contract of fa_bwd_kernel.h, no dropout). The key-major kernels get dQ by fp32 atomics, one
// per element per key block: at D = 128 that is S/128 * S * D * 4 B per head (1.6 GB at
// B8 H12 S2048), about 1.2 ms at the device's fp32-atomic rate, several times the matrix work.
// This pass instead recomputes S and dP per query block, the forward's way round:
//   grid = (query blocks of 32*NW rows, H, B); a wave owns 32 query rows (lane = query);
//   per 64-key tile (K, V staged in LDS, double-buffered):
//     S^T = K Q^T, dP^T = V dO^T      (Q, dO rows of this lane's query as B operands in registers)
//     dS^T = P^T (dP^T - delta)      (lse and delta are per lane: no row exchange at all)
//     dQ^T += K^T dS^T               (K^T by transposed LDS reads, dS^T packed in place)
// and writes dQ (scaled, 16-bit) directly: no workspace, no atomics, no convert pass. The price is
// two extra matrix products per element (S and dP are also computed by the key-major kernel).
#pragma once

#include "fa_common.h"
#include "../../include/fa_hip.h"

namespace fa {

#ifndef FA_BWD_DQ_SEED
#define FA_BWD_DQ_SEED 1       // dP^T accumulator seeded with -delta
#endif
#ifndef FA_BWD_DQ_ENTRY_WAIT
#define FA_BWD_DQ_ENTRY_WAIT 1 // vmcnt(0) the compiler sees before the key walk
#endif
#ifndef FA_BWD_DQ_UNSWITCH
#define FA_BWD_DQ_UNSWITCH 1   // per-element mask only on the tiles that need it (uniform branch)
#endif


template <int D, int NW>
struct DqCfg {
    static constexpr int BM = 32 * NW;    // query rows per workgroup
    static constexpr int BN = 64;         // keys per tile
    static constexpr int NT = 64 * NW;
    static constexpr int NC = D / 8;
    static constexpr int TILE_BYTES = BN * D * 2;
    static constexpr int CPT = (BN * NC + NT - 1) / NT;   // 16-B chunks per thread per tile
    static constexpr int LDS_BYTES = 4 * TILE_BYTES;      // K[2], V[2]
};

template <int D, typename T, bool CAUSAL, int NW>
__global__ __launch_bounds__(64 * NW, 2) void fa_bwd_dq_kernel(const FaBwdArgs a, const int slots) {
    using C = DqCfg<D, NW>;
    using S = Swz<D>;
    constexpr float LOG2E = 1.4426950408889634f;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    // block -> (q-block, head, batch); causal: the heaviest (last) query blocks first
    const int nqb = gridDim.x;
    const int nbh = gridDim.y * gridDim.z;
    const int L = blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z);
    int qb, bh_lin;
    if (FA_BWD_XCD && CAUSAL) {
        // heaviest (last) query blocks first within XCD head groups (xcd_grouped)
        int rank;
        xcd_grouped(L, nqb, nbh, slots, rank, bh_lin);
        qb = nqb - 1 - rank;
    } else if (CAUSAL) {
        qb = nqb - 1 - L / nbh;
        bh_lin = L % nbh;
    } else {
        // XCD-aware (as the forward): blocks L and L+8 share an XCD; each XCD gets a contiguous
        // run of (head, q-block), so a head's K/V stream through one L2 (bijective for any count)
        const int nwg = nqb * nbh;
        const int xcd = L & 7, q8 = nwg >> 3, r8 = nwg & 7;
        const int Lp = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
        qb = Lp % nqb;
        bh_lin = Lp / nqb;
    }
    const int h = bh_lin % a.nheads;
    const int b = bh_lin / a.nheads;

    const int q_start = a.cu_seqlens_q[b];
    const int seqlen_q = a.cu_seqlens_q[b + 1] - q_start;
    const int k_start = a.cu_seqlens_k[b];
    const int seqlen_k = a.cu_seqlens_k[b + 1] - k_start;
    const int q0 = qb * C::BM;
    if (q0 >= seqlen_q) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31;
    const int hi = lane >> 5;
    const int qw = q0 + 32 * wave;
    const int qrow = qw + l32;
    const int head_dim = a.head_dim;

    int n_end = seqlen_k;
    if (CAUSAL) n_end = min(n_end, q0 + C::BM);
    const int nt = n_end > 0 ? (n_end + C::BN - 1) / C::BN : 0;

    const uint16_t *kbase = (const uint16_t *)a.k + (int64_t)k_start * a.k_row_stride + (int64_t)h * a.k_head_stride;
    const uint16_t *vbase = (const uint16_t *)a.v + (int64_t)k_start * a.v_row_stride + (int64_t)h * a.v_head_stride;
    const auto kr = make_rsrc_n(kbase, n_end * (int)a.k_row_stride * 2);
    const auto vr = make_rsrc_n(vbase, n_end * (int)a.v_row_stride * 2);
    const auto qr = make_rsrc((const uint16_t *)a.q + (int64_t)q_start * a.q_row_stride + (int64_t)h * a.q_head_stride);
    const auto dr = make_rsrc((const uint16_t *)a.dout + (int64_t)q_start * a.do_row_stride + (int64_t)h * a.do_head_stride);

    // ---- Q and dO rows of this lane's query (B operands of S^T = K Q^T and dP^T = V dO^T)
    typename T::frag qf[D / 16], df[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
        const int c = 2 * ks + hi;
        const bool ok = qrow < seqlen_q && c * 8 < head_dim;
        qf[ks] = as_frag<T>(bload128(qr, ok ? (qrow * (int)a.q_row_stride + c * 8) * 2 : OOB));
        df[ks] = as_frag<T>(bload128(dr, ok ? (qrow * (int)a.do_row_stride + c * 8) * 2 : OOB));
    }
    const float *lse_g = a.softmax_lse + (int64_t)(b * a.nheads + h) * a.lse_stride;
    const float *del_g = a.softmax_d + (int64_t)(b * a.nheads + h) * a.lse_stride;
    const int qc = min(qrow, seqlen_q - 1);   // rows past seqlen_q compute values nobody stores
    const float lse2 = lse_g[qc] * LOG2E;
    const float delta = del_g[qc];
    const float c_log2 = a.softmax_scale * LOG2E;

    // ---- K/V tile staging (issue early, write late); descriptors end at row n_end (zeros past it)
    int st_off_k[C::CPT], st_off_v[C::CPT], st_lds[C::CPT];
#pragma unroll
    for (int i = 0; i < C::CPT; ++i) {
        const int idx = tid + C::NT * i;
        const int row = idx / C::NC, c = idx % C::NC;
        const bool ok = idx < C::BN * C::NC && c * 8 < head_dim;
        st_off_k[i] = ok ? (row * (int)a.k_row_stride + c * 8) * 2 : OOB;
        st_off_v[i] = ok ? (row * (int)a.v_row_stride + c * 8) * 2 : OOB;
        st_lds[i] = S::off(row, c);
    }
    const int k_tile_step = C::BN * (int)a.k_row_stride * 2;
    const int v_tile_step = C::BN * (int)a.v_row_stride * 2;
    u32x4 kst[C::CPT], vst[C::CPT];
    auto gload_kv = [&](int j) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < C::CPT; ++i) {
            kst[i] = bload128s(kr, st_off_k[i], j * k_tile_step);
            vst[i] = bload128s(vr, st_off_v[i], j * v_tile_step);
        }
    };
    auto lds_store_kv = [&](char *kb, char *vb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < C::CPT; ++i)
            if ((C::BN * C::NC) % C::NT == 0 || tid + C::NT * i < C::BN * C::NC) {
                lds_write128(kb, st_lds[i], kst[i]);
                lds_write128(vb, st_lds[i], vst[i]);
            }
    };

    // lane-constant LDS offsets: row reads of K / V (S^T, dP^T) and transposed reads of K (K^T)
    const int grp = (lane >> 4) & 1;
    const int qq = (lane & 15) >> 2;
    const int pp = lane & 3;
    int k_rd[2][D / 16];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) k_rd[st][ks] = S::off(32 * st + l32, 2 * ks + hi);
    int t_rd[D / 32][2][2][2];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int rb = 32 * st + 16 * s2 + 4 * hi + qq;
                const int col = 32 * dt + 16 * grp + 4 * pp;
                t_rd[dt][st][s2][0] = S::off8(rb, col);
                t_rd[dt][st][s2][1] = S::off8(rb + 8, col);
            }

    f32x16 dq[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[dt][r] = 0.f;

    auto step = [&](auto par_tag, int j) __attribute__((always_inline)) {
        constexpr int P = decltype(par_tag)::value;
        char *kb = smem + P * C::TILE_BYTES;
        char *vb = smem + (2 + P) * C::TILE_BYTES;
        const int kv0 = j * C::BN;
        if (j + 1 < nt) gload_kv(j + 1);
        const bool need_mask = (kv0 + C::BN > seqlen_k) || (CAUSAL && kv0 + C::BN - 1 > qw);
        typename T::frag pf[2][2];
        // dP^T's accumulator starts at -delta (the lane's row constant), so dS = P dP is one
        // multiply per element; the per-element key/causal mask runs only on the tiles that need it,
        // as a second copy of the sub-tile behind one wave-uniform branch (with the test inside the
        // element loop the compiler computed the mask's compares and selects on every tile)
        auto sub_tiles = [&](auto masked_tag) __attribute__((always_inline)) {
            constexpr bool MASKED = decltype(masked_tag)::value;
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                f32x16 s, dp;
#pragma unroll
                for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = FA_BWD_DQ_SEED ? -delta : 0.f; }
#pragma unroll
                for (int ks = 0; ks < D / 16; ++ks) {
                    s = T::mfma32(as_frag<T>(lds_read128(kb, k_rd[st][ks])), qf[ks], s);
                    dp = T::mfma32(as_frag<T>(lds_read128(vb, k_rd[st][ks])), df[ks], dp);
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float p = fast_exp2(fmaf(s[r], c_log2, -lse2));
                    if constexpr (MASKED) {
                        const int kv = kv0 + 32 * st + crow(r, hi);
                        p = mask_min(p, kv >= seqlen_k || (CAUSAL && kv > qrow));
                    }
                    s[r] = FA_BWD_DQ_SEED ? p * dp[r] : p * (dp[r] - delta);
                }
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    u32x4 pk;
#pragma unroll
                    for (int e = 0; e < 4; ++e) pk[e] = T::pack2(s[8 * s2 + 2 * e], s[8 * s2 + 2 * e + 1]);
                    pf[st][s2] = as_frag<T>(pk);
                }
            }
        };
        if (!FA_BWD_DQ_UNSWITCH || __builtin_amdgcn_readfirstlane((int)need_mask))
            sub_tiles(std::true_type{});
        else
            sub_tiles(std::false_type{});
        // dQ^T += K^T dS^T
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    u32x2 lo = lds_read_tr(kb, t_rd[dt][st][s2][0]);
                    u32x2 hv = lds_read_tr(kb, t_rd[dt][st][s2][1]);
                    dq[dt] = T::mfma32(as_frag<T>(u32x4{lo[0], lo[1], hv[0], hv[1]}), pf[st][s2], dq[dt]);
                }
        if (j + 1 < nt) lds_store_kv(smem + (1 - P) * C::TILE_BYTES, smem + (3 - P) * C::TILE_BYTES);
        __syncthreads();
    };
    if (nt > 0) {
        gload_kv(0);
        lds_store_kv(smem, smem + 2 * C::TILE_BYTES);
        __syncthreads();
    }
    // Every prologue load (the Q / dO operands, lse, delta) is done before the walk, in a form the
    // compiler's wait counters see: otherwise the loop header inherits them as pending from the
    // entry edge, and every step's S / dP chain waited with vmcnt(7..1) for that step's own K/V
    // prefetch loads (issued at its top, needed only at its end)
    if (FA_BWD_DQ_ENTRY_WAIT) vmcnt0();
    for (int j = 0; j < nt; j += 2) {
        step(std::integral_constant<int, 0>(), j);
        if (j + 1 < nt) step(std::integral_constant<int, 1>(), j + 1);
    }

    // ---- epilogue: dq^T[d = 32 dt + crow(r, hi)][query = lane] -> 8-byte row stores
    if (qrow < seqlen_q) {
        uint16_t *dqp = (uint16_t *)a.dq + (int64_t)(q_start + qrow) * a.dq_row_stride + (int64_t)h * a.dq_head_stride;
        const float sc = a.softmax_scale;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = 32 * dt + 8 * g + 4 * hi;
                if (d < head_dim) {
                    u32x2 w = {T::pack2(dq[dt][4 * g + 0] * sc, dq[dt][4 * g + 1] * sc),
                               T::pack2(dq[dt][4 * g + 2] * sc, dq[dt][4 * g + 3] * sc)};
                    gstore64(dqp + d, w);
                }
            }
    }
}

}  // namespace fa
