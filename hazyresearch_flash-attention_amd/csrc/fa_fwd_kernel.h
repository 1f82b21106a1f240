// fa_fwd_kernel.h — FlashAttention forward for gfx950 (CDNA4), hand-written HIP.
//
// Reference behaviour followed (file:line in /root/reference):
//   - online softmax, exp2 with scale*log2(e) folded   csrc/flash_attn/src/fmha/softmax.h:211-226
//   - row sum taken BEFORE dropout, O scaled by 1/sum and 1/p_keep at the end
//                                                      csrc/flash_attn/src/fmha_fprop_kernel_1xN.h:522-536,637-661
//   - mask: col < seqlen_k, causal col <= row (top-left) csrc/flash_attn/src/fmha/mask.h:58-72
//   - LSE = max*scale + log(sum); empty/NaN row -> -inf and inv_sum = 1 (output 0)
//                                                      csrc/flash_attn/src/fmha_fprop_kernel_1xN.h:590-623,645
//   - var-len sequences through cu_seqlens             csrc/flash_attn/src/fmha_kernel.h:45-76
//
// MI355X-first structure (NOT the reference's FA-1 loop order): FA-2 order, grid =
// (q-blocks, H, B) remapped so that all q-blocks of one head run on one XCD (its K/V stay in
// that XCD's L2). A workgroup = 8 waves = 256 query rows, one wave = 32 rows. Q stays in VGPRs;
// K/V tiles of 64 keys go HBM -> LDS by LDS-DMA (buffer_load ... lds: each wave-instruction writes
// 1 KiB of the image, the XOR swizzle is applied on the source address; bounds-checked, so rows
// past the end and padded columns land as zeros) into a double-buffered image, one barrier per
// tile (the block-sparse walk stages through registers). The loop is unrolled by two so every LDS address is a
// lane-constant base plus an immediate. Scores are computed swapped (S^T = K Q^T,
// v_mfma_f32_32x32x16) so each lane owns one query row: the row max is a tree of v_max3 plus one
// v_permlane32_swap, the row sum stays lane-local until the epilogue, and P feeds the P·V MFMA
// straight from registers (accumulator-as-B-operand); V^T operands come from
// ds_read_b64_tr_b16. The running max is only moved when it grows by more than 2^8 (T13,
// deferred rescale): O and l are rescaled rarely, P stays <= 256. The N x N score matrix never
// leaves registers.
#pragma once

#include "fa_common.h"
#include "../../include/fa_hip.h"

namespace fa {

// Register budget of the block-sparse kernels without dropout (waves per SIMD).
#ifndef FA_FWD_SPARSE_WPE
#define FA_FWD_SPARSE_WPE 4
#endif
// 8-wave dense D<=64 kernels without dropout: minimum waves per SIMD (2 workgroups per CU).
#ifndef FA_FWD_DENSE_WPE
#define FA_FWD_DENSE_WPE 4
#endif

// NW = waves per workgroup (32 query rows each); chosen per launch (fa_kernels_impl.h).
// KSPLIT: the two halves of the workgroup share its query rows and split the key range (intra-
// workgroup split-K for short sequences, merged through LDS at the end).
template <int D, int NW_, bool KSPLIT = false>
struct FwdCfg {
    static constexpr int NW = NW_;                // waves per workgroup
    static constexpr int NT = 64 * NW;            // threads per workgroup
    static constexpr int NWR = KSPLIT ? NW / 2 : NW;   // waves per key group (distinct row blocks)
    static constexpr int BM = 32 * NWR;           // query rows per workgroup
    static constexpr int BN = 64;                 // keys per iteration
    static constexpr int NC = D / 8;              // 16-B chunks per row
    static constexpr int TILE_BYTES = BN * D * 2;
    static constexpr int CPT = (BN * NC + NT - 1) / NT;   // staged chunks per thread per tile
    static constexpr int RNG_BYTES_PER_WAVE = 2 * 32 * 32 * 2;  // two 32x32 u16 images
    static constexpr int lds_bytes(bool dropout) {
        return (KSPLIT ? 8 : 4) * TILE_BYTES + (dropout ? NW * RNG_BYTES_PER_WAVE : 0);
    }
};

// log2-domain threshold of the deferred rescale: P values stay below 2^RESCALE_THR.
constexpr float RESCALE_THR = 8.0f;


// v_max3_f32 as one instruction (plain fmaxf at -O3 adds NaN-canonicalising v_max x,x first).
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// max of 32 values: 4 independent chains of v_max3 (ILP 4), 18 instructions.
__device__ __forceinline__ float max_tree32(const f32x16 &a, const f32x16 &b) {
    float acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float x0 = a[4 * k], x1 = a[4 * k + 1], x2 = a[4 * k + 2], x3 = a[4 * k + 3];
        const float y0 = b[4 * k], y1 = b[4 * k + 1], y2 = b[4 * k + 2], y3 = b[4 * k + 3];
        float m = max3f(x0, x1, x2);
        m = max3f(m, x3, y0);
        m = max3f(m, y1, y2);
        acc[k] = max3f(m, y3, y3);
    }
    return max3f(max3f(acc[0], acc[1], acc[2]), acc[3], acc[3]);
}
// max over the lane pair (l, l^32): one v_permlane32_swap and one v_max3 (no canonicalising v_max)
__device__ __forceinline__ float pair_max3(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return max3f(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float sum_tree32(const f32x16 &a, const f32x16 &b) {
    float t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = a[i] + b[i];
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) t[i] = t[i] + t[i + w];
    return t[0];
}

// Minimum waves per SIMD the register allocation must allow (waves/SIMD = 512 / registers):
// 8-wave workgroups hold two waves per SIMD each, so 4 = two workgroups per CU (128 registers);
// 4-wave workgroups hold one, so 4 / 3 / 2 = four / three / two workgroups per CU.
constexpr int fwd_waves_per_eu(int D, int NW, bool dropout, bool sparse) {
    return sparse && !dropout && D <= 64 ? FA_FWD_SPARSE_WPE
         : NW == 8            ? (D <= 64 && !dropout ? FA_FWD_DENSE_WPE : 1)
         : NW == 4            ? (D <= 64 ? (dropout ? 3 : 4) : 2)
                              : 1;
}

#define FA_FWD_BOUNDS(NW) __launch_bounds__(64 * NW)

template <int D, typename T, bool CAUSAL, bool DROPOUT, int NW, bool SPARSE = false, bool KSPLIT = false>
__global__ FA_FWD_BOUNDS(NW) __attribute__((amdgpu_waves_per_eu(fwd_waves_per_eu(D, NW, DROPOUT, SPARSE)))) void fa_fwd_kernel(const FaFwdArgs a, const FaBlockMask bm, const int slots) {
    static_assert(!KSPLIT || (!CAUSAL && !DROPOUT && !SPARSE && NW % 2 == 0), "split-K: dense non-causal only");
    using C = FwdCfg<D, NW, KSPLIT>;
    using S = Swz<D>;
    constexpr float LOG2E = 1.4426950408889634f;
    constexpr float LN2 = 0.6931471805599453f;
    constexpr bool MTHR = !SPARSE;   // one-compare rescale test; measured slower on the block-sparse walk
    extern __shared__ __attribute__((aligned(16))) char smem[];

    // ---- block -> (q-block, head, batch)
    const int nqb = gridDim.x;
    const int nbh = gridDim.y * gridDim.z;
    const int nwg = nqb * nbh;
    const int L = blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z);
    int qb, bh_lin;
    if (CAUSAL && FA_BWD_XCD) {
        // heaviest (last) query blocks first within XCD head groups (xcd_grouped)
        int rank;
        xcd_grouped(L, nqb, nbh, slots, rank, bh_lin);
        qb = nqb - 1 - rank;
    } else if (CAUSAL) {
        // global LPT order: the heaviest (last) query blocks of every head first
        qb = nqb - 1 - L / nbh;
        bh_lin = L % nbh;
    } else {
        // XCD-aware: blocks L and L+8 share an XCD; give each XCD a contiguous run of
        // (head, q-block) so a head's K/V are fetched into one L2 (bijective for any nwg).
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
    const int kgrp = KSPLIT ? wave / C::NWR : 0;   // key group (KSPLIT: half of the key range)
    const int qw = q0 + 32 * (wave - kgrp * C::NWR);   // first query row of this wave
    const int qrow = qw + l32;           // the query row this lane owns
    const int head_dim = a.head_dim;

    const auto qr = make_rsrc((const uint16_t *)a.q + (int64_t)q_start * a.q_row_stride + (int64_t)h * a.q_head_stride);
    int n_end = seqlen_k;
    if (CAUSAL) n_end = min(n_end, q0 + C::BM);
    const int nt = (n_end + C::BN - 1) / C::BN;

    // the K/V descriptors end at row n_end, so rows past it read as zeros by themselves
    const uint16_t *kbase = (const uint16_t *)a.k + (int64_t)k_start * a.k_row_stride + (int64_t)h * a.k_head_stride;
    const uint16_t *vbase = (const uint16_t *)a.v + (int64_t)k_start * a.v_row_stride + (int64_t)h * a.v_head_stride;
    const auto kr = make_rsrc_n(kbase, n_end * (int)a.k_row_stride * 2);
    const auto vr = make_rsrc_n(vbase, n_end * (int)a.v_row_stride * 2);

    // ---- block sparsity (fa_fwd_block): this lane's live 256-key column blocks, and their union
    // over the workgroup's rows, which drives the tile walk (dead columns are never loaded)
    uint64_t lane_cols = ~0ull, wg_cols = ~0ull;
    if constexpr (SPARSE) {
        lane_cols = 0;
        const int rb = qrow >> 4;
        if (qrow < seqlen_q && rb < bm.rows) {
            const uint8_t *mr = bm.mask + (int64_t)rb * bm.row_stride;
            for (int c = 0; c < bm.cols; ++c)
                if (mr[c]) lane_cols |= 1ull << c;
        }
        uint32_t lo = (uint32_t)lane_cols, hv = (uint32_t)(lane_cols >> 32);
#pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) {
            lo |= (uint32_t)__shfl_xor((int)lo, sh);
            hv |= (uint32_t)__shfl_xor((int)hv, sh);
        }
        uint64_t *wcols = (uint64_t *)smem;
        if (lane == 0) wcols[wave] = ((uint64_t)hv << 32) | lo;
        __syncthreads();
        wg_cols = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) wg_cols |= wcols[w];
        wg_cols = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(wg_cols >> 32)) << 32) |
                  __builtin_amdgcn_readfirstlane((uint32_t)wg_cols);
        __syncthreads();   // the K image reuses these bytes
    }
    // next live 64-key tile after j (dense: j + 1; sparse: skip dead 256-key column blocks)
    auto next_tile = [&](int j) __attribute__((always_inline)) -> int {
        const int n = j + 1;
        if constexpr (!SPARSE) {
            return n;
        } else {
            const int c = n >> 2;
            if (c >= 64) return nt;
            if ((wg_cols >> c) & 1) return n;
            const uint64_t rest = c + 1 < 64 ? (wg_cols >> (c + 1)) : 0ull;
            return rest ? 4 * (c + 1 + (int)__builtin_ctzll(rest)) : nt;
        }
    };

    // ---- Q fragments (B operand of S^T = K Q^T): Q[qrow][16ks + 8hi + j]
    // With rot_cos set, the rotary embedding is applied here, once per workgroup (fused rotary:
    // rotary.py:31-41 with the rounding of fa_rotary, so the operands equal the separate pass's).
    const bool rot = a.rot_cos != nullptr;
    const auto rcos = make_rsrc(a.rot_cos), rsin = make_rsrc(a.rot_sin);
    typename T::frag qf[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
        const int c = 2 * ks + hi;
        const bool ok = qrow < seqlen_q && c * 8 < head_dim;
        u32x4 w = bload128(qr, ok ? (qrow * (int)a.q_row_stride + c * 8) * 2 : OOB);
        if (rot) {
            const int to = ok ? (qrow * (int)a.rot_stride + c * 8) * 2 : OOB;
            w = rotary8<T, false>(w, bload128(rcos, to), bload128(rsin, to));
        }
        qf[ks] = as_frag<T>(w);
    }

    // ---- register staging of K/V tiles for the block-sparse walk (issue early, write late: T14).
    // Loads are bounds-checked buffer loads: a tile past the end reads as zeros, so no branch is
    // needed around them.
    int st_off_k[C::CPT], st_off_v[C::CPT], st_lds[C::CPT];
#pragma unroll
    for (int i = 0; i < C::CPT; ++i) {
        const int idx = tid + C::NT * i;
        const int row = idx / C::NC, c = idx % C::NC;
        st_off_k[i] = (row * (int)a.k_row_stride + c * 8) * 2;
        st_off_v[i] = (row * (int)a.v_row_stride + c * 8) * 2;
        if (!(c * 8 < head_dim && idx < C::BN * C::NC)) st_off_k[i] = st_off_v[i] = OOB;   // surplus threads load nothing
        st_lds[i] = S::off(row, c);
    }
    const int k_tile_step = C::BN * (int)a.k_row_stride * 2;
    const int v_tile_step = C::BN * (int)a.v_row_stride * 2;
    u32x4 kst[C::CPT], vst[C::CPT];
    auto gload_k = [&](int j) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < C::CPT; ++i) kst[i] = bload128s(kr, st_off_k[i], j * k_tile_step);
    };
    auto gload_v = [&](int j) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < C::CPT; ++i) vst[i] = bload128s(vr, st_off_v[i], j * v_tile_step);
    };
    auto lds_store_k = [&](char *kb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < C::CPT; ++i)
            if ((C::BN * C::NC) % C::NT == 0 || tid + C::NT * i < C::BN * C::NC) lds_write128(kb, st_lds[i], kst[i]);
    };
    auto lds_store_v = [&](char *vb) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < C::CPT; ++i)
            if ((C::BN * C::NC) % C::NT == 0 || tid + C::NT * i < C::BN * C::NC) lds_write128(vb, st_lds[i], vst[i]);
    };

    f32x16 o[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_i = -INFINITY;
    float l_i = 0.f;
    const float c_log2 = a.softmax_scale * LOG2E;
    const float thr_raw = RESCALE_THR / c_log2;
    float m_thr = -INFINITY;   // MTHR: rescale when a tile max passes this (m + thr_raw)
    float mc_row = 0.f;        // MTHR: m * c_log2 (0 before the first key)

    // dropout constants
    const uint32_t keep_thr = (uint32_t)floorf((1.0f - a.p_dropout) * 65535.0f);
    const uint32_t seed_lo = (uint32_t)a.rng_seed, seed_hi = (uint32_t)(a.rng_seed >> 32);
    const uint32_t rng_ctr3 = DROPOUT ? (uint32_t)(rng_offset_of(a) >> 2) : 0u;
    const uint32_t bh = (uint32_t)(b * a.nheads + h);
    char *rng_img = smem + 4 * C::TILE_BYTES + wave * C::RNG_BYTES_PER_WAVE;

    // tr-read lane geometry (16-lane group, lane 4qq+pp supplies row qq, columns 4pp..4pp+3)
    const int grp = (lane >> 4) & 1;
    const int qq = (lane & 15) >> 2;
    const int pp = lane & 3;

    // lane-constant LDS offsets (the per-buffer base and k-step/tile parts fold into immediates)
    int k_rd[2][D / 16];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) k_rd[st][ks] = S::off(32 * st + l32, 2 * ks + hi);
    int v_rd[D / 32][2][2][2];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int rb = 32 * st + 16 * s2 + 4 * hi + qq;
                const int col = 32 * dt + 16 * grp + 4 * pp;
                v_rd[dt][st][s2][0] = S::off8(rb, col);
                v_rd[dt][st][s2][1] = S::off8(rb + 8, col);
            }

    // S^T = K Q^T for one 64-key tile: two 32x32 sub-tiles, lane = query row, registers = keys
    auto qk = [&](const char *kb, f32x16 (&s)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[st][r] = 0.f;
#pragma unroll
            for (int ks = 0; ks < D / 16; ++ks) {
                s[st] = T::mfma32(as_frag<T>(lds_read128(kb, k_rd[st][ks])), qf[ks], s[st]);
            }
        }
    };

    // ---- dropout (keep mask from the Philox stream) and conversion of P into the 16-bit B
    // operand of P·V
    auto dropout_cvt = [&](f32x16 (&s)[2], int kv0, typename T::frag (&pf)[2][2]) __attribute__((always_inline)) {
        if (DROPOUT) {
            // Keep mask generated in the column-major (backward) layout, transposed through a
            // per-wave LDS image with ds_read_b64_tr_b16.
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                char *img = rng_img + st * (32 * 32 * 2);
                const uint32_t col = (uint32_t)(kv0 + 32 * st + l32);
#pragma unroll
                for (int sg = 0; sg < 2; ++sg) {
                    const uint32_t g = ((uint32_t)(qw >> 5) << 2) | (sg << 1) | hi;
                    u32x4 w = philox7(g, col, bh, rng_ctr3, seed_lo, seed_hi);
                    u32x2 w01 = {w[0], w[1]}, w23 = {w[2], w[3]};
                    lds_write64(img, l32 * 64 + (16 * sg + 4 * hi) * 2, w01);
                    lds_write64(img, l32 * 64 + (16 * sg + 8 + 4 * hi) * 2, w23);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                char *img = rng_img + st * (32 * 32 * 2);
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    u32x2 rv = lds_read_tr(img, (8 * g4 + 4 * hi + qq) * 64 + (16 * grp + 4 * pp) * 2);
                    const uint32_t k01 = keep2(rv[0], keep_thr), k23 = keep2(rv[1], keep_thr);
                    if (!(k01 & 1)) s[st][4 * g4 + 0] = 0.f;
                    if (!(k01 & 2)) s[st][4 * g4 + 1] = 0.f;
                    if (!(k23 & 1)) s[st][4 * g4 + 2] = 0.f;
                    if (!(k23 & 2)) s[st][4 * g4 + 3] = 0.f;
                }
            }
        }
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                u32x4 pk;
#pragma unroll
                for (int e = 0; e < 4; ++e) pk[e] = T::pack2(s[st][8 * s2 + 2 * e], s[st][8 * s2 + 2 * e + 1]);
                pf[st][s2] = as_frag<T>(pk);
            }
    };

    // ---- softmax of one tile in registers: mask, max, deferred rescale, exp, row sum,
    // dropout, and conversion into the 16-bit B operand of P·V.
    auto softmax_tile = [&](f32x16 (&s)[2], int kv0, typename T::frag (&pf)[2][2]) __attribute__((always_inline)) {
        const bool dead = SPARSE && !((lane_cols >> (kv0 >> 8)) & 1);   // row's block is 0 in the layout
        const bool need_mask = (kv0 + C::BN > seqlen_k) || (CAUSAL && kv0 + C::BN - 1 > qw) ||
                               (SPARSE && __builtin_amdgcn_ballot_w64(dead));
        if (need_mask) {
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int kv = kv0 + 32 * st + crow(r, hi);
                    if (dead || kv >= seqlen_k || (CAUSAL && kv > qrow)) s[st][r] = -INFINITY;
                }
        }
        const float mx = pair_max3(max_tree32(s[0], s[1]));
        float mc;
        if (MTHR) {
            // m_thr = m + 2^RESCALE_THR in raw units (-inf before the first key); mc_row = m * c
            const bool grow = mx > m_thr;   // NaN (all -inf) -> false
            if (__builtin_amdgcn_ballot_w64(grow)) {
                // m itself is not kept: alpha and the LSE only need m * c_log2
                const float mcx = mx * c_log2;
                const float alpha = grow ? fast_exp2(m_thr == -INFINITY ? -INFINITY : mc_row - mcx) : 1.f;
                if (grow) {
                    m_thr = mx + thr_raw;
                    mc_row = mcx;
                }
                l_i *= alpha;
#pragma unroll
                for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            }
            mc = mc_row;
        } else {
            const float m_new = fmaxf(m_i, mx);
            const bool grow = (m_new - m_i) * c_log2 > RESCALE_THR;   // NaN (all -inf) -> false
            if (__builtin_amdgcn_ballot_w64(grow)) {
                const float alpha = grow ? fast_exp2((m_i - m_new) * c_log2) : 1.f;
                if (grow) m_i = m_new;
                l_i *= alpha;
#pragma unroll
                for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
            }
            mc = (m_i == -INFINITY ? 0.f : m_i) * c_log2;
        }
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int r = 0; r < 16; ++r) s[st][r] = fast_exp2(fmaf(s[st][r], c_log2, -mc));
        l_i += sum_tree32(s[0], s[1]);

        dropout_cvt(s, kv0, pf);
    };

    // ---- O^T += V^T P^T for one tile
    auto pv = [&](const char *vb, typename T::frag (&pf)[2][2]) __attribute__((always_inline)) {
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    u32x2 lo = lds_read_tr(vb, v_rd[dt][st][s2][0]);
                    u32x2 hv = lds_read_tr(vb, v_rd[dt][st][s2][1]);
                    u32x4 av = {lo[0], lo[1], hv[0], hv[1]};
                    o[dt] = T::mfma32(as_frag<T>(av), pf[st][s2], o[dt]);
                }
    };

    // Dense walk: K[j], V[j] in LDS buffer j & 1.
    // DMA: piece p (1 KiB = RPP rows of the tile image) is written by wave p % NW; lane l lands at
    // byte 16 l of the piece, i.e. row RPP p + l / NC, slot l % NC, which holds chunk slot ^ x(row)
    // KSPLIT: each key group stages its own tiles (its own 4 tile buffers) with its NWR waves
    constexpr int PIECES = C::TILE_BYTES / 1024;
    constexpr int DNW = C::NWR;
    constexpr int PPW = (PIECES + DNW - 1) / DNW;
    constexpr int RPP = 1024 / (2 * D);
    const int dwave = wave - kgrp * C::NWR;
    char *const gsm = smem + kgrp * 4 * C::TILE_BYTES;
    int dma_k_off[PPW], dma_v_off[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int p = dwave + DNW * i;
        const int r = RPP * p + lane / C::NC;
        const int c = (lane % C::NC) ^ S::x(r);
        const bool ok = c * 8 < head_dim;
        dma_k_off[i] = ok ? (r * (int)a.k_row_stride + c * 8) * 2 : OOB;
        dma_v_off[i] = ok ? (r * (int)a.v_row_stride + c * 8) * 2 : OOB;
    }
    // LDS-DMA through inline asm (fa_common.h dma16): through the builtin, hipcc put an
    // s_waitcnt vmcnt(0) for the in-flight DMA in front of the first ds_read_b64_tr_b16 of every tile
    const i32x4 ksrd = make_srd(kbase, n_end * (int)a.k_row_stride * 2);
    const i32x4 vsrd = make_srd(vbase, n_end * (int)a.v_row_stride * 2);
    auto dma_tile = [&](const i32x4 &srd, const int (&off)[PPW], int step_bytes, char *buf, int j)
        __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int p = dwave + DNW * i;
            if (PIECES % DNW == 0 || p < PIECES) dma16(srd, off[i], j * step_bytes, lds_addr(buf + 1024 * p));
        }
    };
    // stage the next K/V tiles: issue the DMA early, wait for it late
    auto stage_issue = [&](char *kb_wr, char *vb_wr, int jk, int jv) __attribute__((always_inline)) {
        dma_tile(ksrd, dma_k_off, k_tile_step, kb_wr, jk);
        dma_tile(vsrd, dma_v_off, v_tile_step, vb_wr, jv);
    };
    auto stage_commit = [&]() __attribute__((always_inline)) { vmcnt0(); };
    // KSPLIT: group g walks tiles [jbeg, jend) = the g-th half of the key range, both groups in
    // the same number of steps (a group past its end only meets the barriers)
    const int jhalf = KSPLIT ? (nt + 1) / 2 : nt;
    const int jbeg = kgrp * jhalf;
    const int jend = KSPLIT ? min(nt, jbeg + jhalf) : nt;
    auto step = [&](auto par_tag, int j) __attribute__((always_inline)) {
        constexpr int P = decltype(par_tag)::value;
        char *kb_rd = gsm + P * C::TILE_BYTES;
        char *vb_rd = gsm + (2 + P) * C::TILE_BYTES;
        char *kb_wr = gsm + (1 - P) * C::TILE_BYTES;
        char *vb_wr = gsm + (3 - P) * C::TILE_BYTES;
        stage_issue(kb_wr, vb_wr, j + 1, j + 1);
        // causal: a wave whose 32 rows all lie above this key tile would add exactly nothing (every
        // P = 0, no rescale): it only stages its share of the next tile and meets the barrier
        if ((!CAUSAL || j * C::BN <= qw + 31) && (!KSPLIT || j < jend)) {
            f32x16 s[2];
            qk(kb_rd, s);
            typename T::frag pf[2][2];
            softmax_tile(s, j * C::BN, pf);
            pv(vb_rd, pf);
        }
        stage_commit();
        __syncthreads();
    };

    if constexpr (SPARSE) {
        // walk the live tiles only: the same double-buffered step with tile indices from
        // next_tile (a dead next tile is never loaded)
        auto sstep = [&](auto par_tag, int j, int jn) __attribute__((always_inline)) {
            constexpr int P = decltype(par_tag)::value;
            char *kb_rd = smem + P * C::TILE_BYTES;
            char *vb_rd = smem + (2 + P) * C::TILE_BYTES;
            gload_k(jn);
            gload_v(jn);
            // a wave whose rows are all dead in this column block skips the math (it still
            // stages its share of the next tile and meets the barrier)
            const bool lane_live = (lane_cols >> (j >> 2)) & 1;
            if (__builtin_amdgcn_ballot_w64(lane_live)) {
                f32x16 s[2];
                qk(kb_rd, s);
                typename T::frag pf[2][2];
                softmax_tile(s, j * C::BN, pf);
                pv(vb_rd, pf);
            }
            lds_store_k(smem + (1 - P) * C::TILE_BYTES);
            lds_store_v(smem + (3 - P) * C::TILE_BYTES);
            __syncthreads();
        };
        int j = next_tile(-1);
        gload_k(j);
        gload_v(j);
        lds_store_k(smem);
        lds_store_v(smem + 2 * C::TILE_BYTES);
        __syncthreads();
        while (j < nt) {
            int jn = next_tile(j);
            sstep(std::integral_constant<int, 0>(), j, jn);
            j = jn;
            if (j >= nt) break;
            jn = next_tile(j);
            sstep(std::integral_constant<int, 1>(), j, jn);
            j = jn;
        }
    } else {
        // prologue: K[jbeg] -> kbuf0, V[jbeg] -> vbuf0 (of the key group)
        stage_issue(gsm, gsm + 2 * C::TILE_BYTES, jbeg, jbeg);
        stage_commit();
        __syncthreads();
        for (int u = 0; u < jhalf; u += 2) {
            step(std::integral_constant<int, 0>(), jbeg + u);
            if (u + 1 < jhalf) step(std::integral_constant<int, 1>(), jbeg + u + 1);
        }
    }

    if constexpr (KSPLIT) {
        // merge the two key groups' partial states through LDS (the tile buffers are free after
        // the last barrier): group 1 writes (O, l, m*c), group 0 rescales both to the larger max
        // and goes on to the epilogue. A group that saw no key (m_thr = -inf) gets weight 0.
        constexpr int NR = 16 * (D / 32);              // O registers per lane
        float *xo = (float *)smem;                     // [row wave][NR / 4][lane][4]
        float *xl = xo + C::NWR * NR * 64;             // [row wave][lane]
        float *xm = xl + C::NWR * 64;
        const float mcx = m_thr == -INFINITY ? -INFINITY : mc_row;
        if (kgrp == 1) {
#pragma unroll
            for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 v = {o[dt][4 * g], o[dt][4 * g + 1], o[dt][4 * g + 2], o[dt][4 * g + 3]};
                    *reinterpret_cast<f32x4 *>(xo + ((dwave * (NR / 4) + 4 * dt + g) * 64 + lane) * 4) = v;
                }
            xl[dwave * 64 + lane] = l_i;
            xm[dwave * 64 + lane] = mcx;
        }
        __syncthreads();
        if (kgrp == 1) return;
        const float mc1 = xm[dwave * 64 + lane];
        const float l1 = xl[dwave * 64 + lane];
        const float mcm = fmaxf(mcx, mc1);
        const float a0 = mcx == -INFINITY ? 0.f : fast_exp2(mcx - mcm);
        const float a1 = mc1 == -INFINITY ? 0.f : fast_exp2(mc1 - mcm);
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const f32x4 v = *reinterpret_cast<const f32x4 *>(xo + ((dwave * (NR / 4) + 4 * dt + g) * 64 + lane) * 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) o[dt][4 * g + e] = o[dt][4 * g + e] * a0 + v[e] * a1;
            }
        l_i = l_i * a0 + l1 * a1;
        if (mcm != -INFINITY) mc_row = mcm;
    }

    // ---- epilogue
    const float l_tot = pair_sum(l_i);
    const bool empty = (l_tot == 0.f) || (l_tot != l_tot);
    float inv = empty ? 1.f : 1.f / l_tot;
    if (DROPOUT) inv *= 1.0f / (1.0f - a.p_dropout);
    if (qrow < seqlen_q) {
        uint16_t *op = (uint16_t *)a.o + (int64_t)(q_start + qrow) * a.o_row_stride + (int64_t)h * a.o_head_stride;
        // 16-byte stores (T21): lanes l and l+32 hold the two 8-byte halves of each 8-column group
        // of the same row; one v_permlane32_swap per word gives lane l group g4 whole and lane
        // l+32 group g4+1 whole, so each lane writes 16 contiguous bytes instead of 2 x 8.
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int g4 = 0; g4 < 4; g4 += 2) {
                const uint32_t a0 = T::pack2(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
                const uint32_t a1 = T::pack2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
                const uint32_t b0 = T::pack2(o[dt][4 * g4 + 4] * inv, o[dt][4 * g4 + 5] * inv);
                const uint32_t b1 = T::pack2(o[dt][4 * g4 + 6] * inv, o[dt][4 * g4 + 7] * inv);
                const auto s0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
                const auto s1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
                const int d = 32 * dt + 8 * (g4 + hi);
                if (d < head_dim) gstore128(op + d, u32x4{s0[0], s1[0], s0[1], s1[1]});
            }
        if (hi == 0) {
            a.softmax_lse[(int64_t)(b * a.nheads + h) * a.lse_stride + qrow] =
                empty ? -INFINITY : (MTHR ? mc_row * LN2 : m_i * a.softmax_scale) + __logf(l_tot);
        }
    }
}

}  // namespace fa
