// fa_bwd_split_kernel.h — FlashAttention backward for large head dims (D = 128) on gfx950.
//
// Same contract and layouts as fa_bwd_kernel.h (see its header for the math). The difference is
// the split of the per-key work between two waves, so that a wave fits in 256 registers and two
// of them share each SIMD:
//   P waves  (0..3): S = Q K^T, P = exp(S - lse) (masked), Pd (dropout), dV^T += dO^T Pd
//   dS waves (4..7): dZ = dO V^T, dS = P (dZ Md / pk - delta), dK^T += Q^T dS, dS image
// A workgroup covers 128 keys (32 per wave pair). P crosses LDS once per query tile in fp32 (the
// dS waves use exactly the P the one-wave kernel keeps in registers), and every wave then takes
// two of the 16 x 16 dQ tiles as in fa_bwd_kernel.h. At D = 128 the one-wave-per-key kernel
// needs ~360 registers (dK^T and dV^T alone are 128), i.e. one wave per SIMD with every LDS
// read and barrier exposed; here each wave keeps one of the two accumulators and one of K / V.
#pragma once

#include "fa_common.h"
#include "fa_bwd_kernel.h"
#include "../../include/fa_hip.h"

namespace fa {

#ifndef FA_BWD_SPLIT_KVL
#define FA_BWD_SPLIT_KVL 1   // 1: split kernels re-read K / V rows from LDS (no 32-register copy)
#endif
#ifndef FA_BWD_SPLIT_KVL_NC
#define FA_BWD_SPLIT_KVL_NC 1   // 1: the non-causal ones too (D=128 non-causal 1.00 -> 0.95 ms)
#endif

template <int D, bool KVL_ = false, bool SKEW_ = false, int SUB_ = 1>
struct BwdSplitCfg {
    // SKEW (dense, no dropout, dQ by the query-major pass): the P waves run one query tile ahead
    // of the dS waves, so Q/dO/lse/delta rotate through 3 buffers and P through 2
    static constexpr bool SKEW = SKEW_;
    // SUB (skewed kernels): 32-row query sub-tiles per step. With 2, each wave runs two
    // independent MFMA chains and twice the matrix work per barrier, and P crosses LDS as the
    // 16-bit words of the dV operand (the fp32 exchange would not fit next to 64-row images)
    static constexpr int SUB = SKEW ? SUB_ : 1;
    static constexpr bool P16 = SUB > 1;
    static constexpr int NQB = SKEW ? 3 : 2;
    static constexpr int NPX = SKEW ? 2 : 1;
    static constexpr int NW = 8;            // waves per workgroup
    static constexpr int NT = 64 * NW;
    static constexpr int KEYW = NW / 2;     // wave pairs, 32 keys each
    static constexpr int BKV = 32 * KEYW;   // keys per workgroup
    static constexpr int BQ = 32 * SUB;
    static constexpr int NC = D / 8;
    // KVL (causal): K and V rows re-read from LDS images per query tile instead of 32 registers
    static constexpr bool KVL = KVL_;
    // the K image: the B operand of dQ (non-skewed kernels) and the KVL reads
    static constexpr bool KIMG = !SKEW || KVL;
    static constexpr int K_IMG = BKV * D * 2;
    static constexpr int Q_IMG = BQ * D * 2;
    static constexpr int DS_IMG = BKV * BQ * 2;
    static constexpr int OFF_K = 0;
    static constexpr int OFF_Q = OFF_K + (KIMG ? K_IMG : 0);   // Q[NQB]
    static constexpr int OFF_DO = OFF_Q + NQB * Q_IMG;   // dO[NQB]
    static constexpr int OFF_DS = OFF_DO + NQB * Q_IMG;
    static constexpr int OFF_LSE = OFF_DS + (SKEW ? 0 : DS_IMG);   // lse[NQB][BQ]
    static constexpr int OFF_DELTA = OFF_LSE + NQB * BQ * 4;
    static constexpr int OFF_QLIVE = OFF_DELTA + NQB * BQ * 4;
    static constexpr int QLIVE_WORDS = 16;
    // P exchange: per wave pair and sub-tile, 4 (fp32) or 2 (16-bit) chunks x 64 lanes x 16 B
    // (chunk-major: conflict-free b128)
    static constexpr int OFF_PX = OFF_QLIVE + QLIVE_WORDS * 8;
    static constexpr int PX_SUB = (P16 ? 2 : 4) * 64 * 16;
    static constexpr int PX_PAIR = SUB * PX_SUB;
    static constexpr int OFF_V = OFF_PX + NPX * KEYW * PX_PAIR;
    static constexpr int LDS_BYTES = OFF_V + (KVL ? K_IMG : 0);
    static constexpr int QCH = (BQ * NC + NT - 1) / NT;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

#ifndef FA_BWD_SPLIT_KVL_SKEW
#define FA_BWD_SPLIT_KVL_SKEW 0   // 0: the skewed kernels keep K / V rows in registers (C4 bwd -3 %, D=128 -4 %)
#endif
#ifndef FA_BWD_SPLIT_PROBE
#define FA_BWD_SPLIT_PROBE 0
#endif
#ifndef FA_BWD_SPLIT_HOIST
#define FA_BWD_SPLIT_HOIST 1  // 1: skewed steps read their row constants and operands ahead, mask unswitched
#endif
#ifndef FA_BWD_SPLIT_SUB
#define FA_BWD_SPLIT_SUB 1    // 32-row query sub-tiles per skewed step (2: C4 even, D=128 -2 %; needs the default scheduler)
#endif
#ifndef FA_BWD_SPLIT_SKEW
#define FA_BWD_SPLIT_SKEW 1   // 1: P waves one query tile ahead of dS waves (dense, no dropout, no dQ)
#endif
constexpr bool bwd_split_skew(bool dq, bool dropout, bool sparse) {
    return FA_BWD_SPLIT_SKEW && !dq && !dropout && !sparse;
}

// the configuration of one instantiation (kernel and launcher)
template <int D, bool CAUSAL, bool DROPOUT, bool SPARSE, bool DQ>
using BwdSplitCfgOf = BwdSplitCfg<D,
                                  bwd_split_skew(DQ, DROPOUT, SPARSE)
                                      ? (bool)FA_BWD_SPLIT_KVL_SKEW
                                      : (CAUSAL || FA_BWD_SPLIT_KVL_NC) && FA_BWD_SPLIT_KVL,
                                  bwd_split_skew(DQ, DROPOUT, SPARSE), FA_BWD_SPLIT_SUB>;

// DQ = false: no dS image and no dQ (fa_bwd_dq_kernel computes dQ query-major, no atomics)
template <int D, typename T, bool CAUSAL, bool DROPOUT, bool SPARSE = false, bool DQ = true>
__global__ __launch_bounds__(512, 2) void fa_bwd_split_kernel(const FaBwdArgs a, const FaBlockMask bm, const int slots) {
    using C = BwdSplitCfgOf<D, CAUSAL, DROPOUT, SPARSE, DQ>;
    using S = Swz<D>;
    constexpr float LOG2E = 1.4426950408889634f;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char *kimg = smem + C::OFF_K;
    char *dsimg = smem + C::OFF_DS;
    char *px_all = smem + C::OFF_PX;
    float *lse_s = (float *)(smem + C::OFF_LSE);
    float *del_s = (float *)(smem + C::OFF_DELTA);

    // block order as in fa_bwd_kernel (FA_BWD_XCD: head-major per XCD, heaviest block first)
    int kb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    if (FA_BWD_XCD) {
        const int nkb = gridDim.x, nbh = gridDim.y * gridDim.z;
        const int L = blockIdx.x + nkb * (blockIdx.y + gridDim.y * blockIdx.z);
        int bh;
        if (CAUSAL && DQ) {
            // dQ by fp32 atomics: a group's key blocks would all add into the same dQ rows at
            // once (C3: 315 vs 271 us), so the global heaviest-first order spreads the heads
            kb = L / nbh;
            bh = L % nbh;
        } else if (CAUSAL) {
            xcd_grouped(L, nkb, nbh, slots, kb, bh);
        } else {
            const int Lp = xcd_contiguous(L, nkb * nbh);
            kb = Lp % nkb;
            bh = Lp / nkb;
        }
        h = bh % gridDim.y;
        b = bh / gridDim.y;
    } else if (CAUSAL) {
        const int nbh = gridDim.y * gridDim.z;
        const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        kb = L / nbh;
        h = (L % nbh) % gridDim.y;
        b = (L % nbh) / gridDim.y;
    }
    const int q_start = a.cu_seqlens_q[b];
    const int seqlen_q = a.cu_seqlens_q[b + 1] - q_start;
    const int k_start = a.cu_seqlens_k[b];
    const int seqlen_k = a.cu_seqlens_k[b + 1] - k_start;
    const int k0 = kb * C::BKV;
    if (k0 >= seqlen_k) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool role_p = wave < C::KEYW;            // wave-uniform
    const int kwave = role_p ? wave : wave - C::KEYW;
    const int l32 = lane & 31;
    const int hi = lane >> 5;
    const int kw = k0 + 32 * kwave;
    const int kvrow = kw + l32;
    const int head_dim = a.head_dim;
    char *px = px_all + kwave * C::PX_PAIR;

    const uint16_t *qp = (const uint16_t *)a.q + (int64_t)q_start * a.q_row_stride + (int64_t)h * a.q_head_stride;
    const uint16_t *dop = (const uint16_t *)a.dout + (int64_t)q_start * a.do_row_stride + (int64_t)h * a.do_head_stride;
    const uint16_t *kp = (const uint16_t *)a.k + (int64_t)k_start * a.k_row_stride + (int64_t)h * a.k_head_stride;
    const uint16_t *vp = (const uint16_t *)a.v + (int64_t)k_start * a.v_row_stride + (int64_t)h * a.v_head_stride;
    const float *lse_g = a.softmax_lse + (int64_t)(b * a.nheads + h) * a.lse_stride;
    const float *del_g = a.softmax_d + (int64_t)(b * a.nheads + h) * a.lse_stride;
    float *dqa = a.dq_accum + ((int64_t)q_start * a.nheads + h) * head_dim;
    const int64_t dqa_row = (int64_t)a.nheads * head_dim;

    // ---- K block image (B operand of dQ = dS K)
    for (int idx = tid; (C::KIMG || C::KVL) && idx < C::BKV * C::NC; idx += C::NT) {
        const int row = idx / C::NC, c = idx % C::NC;
        const int kv = k0 + row;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (kv < seqlen_k && c * 8 < head_dim) v = gload128(kp + (int64_t)kv * a.k_row_stride + c * 8);
        if constexpr (C::KIMG) lds_write128(kimg, S::off(row, c), v);
        if constexpr (C::KVL) {
            u32x4 w = {0u, 0u, 0u, 0u};
            if (kv < seqlen_k && c * 8 < head_dim) w = gload128(vp + (int64_t)kv * a.v_row_stride + c * 8);
            lds_write128(smem + C::OFF_V, S::off(row, c), w);
        }
    }
    // ---- this lane's key row of K (P waves) or V (dS waves) as B operands: B[k=d][col=key]
    const uint16_t *rowp = role_p ? kp + (int64_t)kvrow * a.k_row_stride : vp + (int64_t)kvrow * a.v_row_stride;
    typename T::frag bf[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
        const int c = 2 * ks + hi;
        u32x4 v4 = {0u, 0u, 0u, 0u};
        if (!C::KVL && kvrow < seqlen_k && c * 8 < head_dim) v4 = gload128(rowp + c * 8);
        bf[ks] = as_frag<T>(v4);
    }
    // dV^T (P waves) or dK^T (dS waves): one 32-key x D accumulator per wave
    f32x16 acc[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;

    const float c_log2 = a.softmax_scale * LOG2E;
    const float rp = 1.0f / (1.0f - a.p_dropout);
    const uint32_t keep_thr = (uint32_t)floorf((1.0f - a.p_dropout) * 65535.0f);
    const uint32_t seed_lo = (uint32_t)a.rng_seed, seed_hi = (uint32_t)(a.rng_seed >> 32);
    const uint32_t rng_ctr3 = DROPOUT ? (uint32_t)(rng_offset_of(a) >> 2) : 0u;
    const uint32_t bh = (uint32_t)(b * a.nheads + h);

    const int grp = (lane >> 4) & 1;
    const int qq = (lane & 15) >> 2;
    const int pp = lane & 3;
    const int g4 = lane >> 4;

    const int q_begin = CAUSAL ? k0 : 0;
    const int nqt = seqlen_q > q_begin ? (seqlen_q - q_begin + C::BQ - 1) / C::BQ : 0;

    // ---- query-tile staging (issue early, write late), buffer loads bounded at row seqlen_q
    u32x4 qst[C::QCH], dst[C::QCH];
    float lse_st = 0.f, del_st = 0.f;
    const auto q_rs = make_rsrc_n(qp, seqlen_q * (int)a.q_row_stride * 2);
    const auto do_rs = make_rsrc_n(dop, seqlen_q * (int)a.do_row_stride * 2);
    int qld_off[C::QCH], dold_off[C::QCH];
#pragma unroll
    for (int i = 0; i < C::QCH; ++i) {
        const int idx = tid + C::NT * i;
        const int row = idx / C::NC, c = idx % C::NC;
        const bool okc = idx < C::BQ * C::NC && c * 8 < head_dim;
        qld_off[i] = okc ? (row * (int)a.q_row_stride + c * 8) * 2 : OOB;
        dold_off[i] = okc ? (row * (int)a.do_row_stride + c * 8) * 2 : OOB;
    }
    auto gload_qtile = [&](int q0n) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < C::QCH; ++i) {
            qst[i] = bload128s(q_rs, qld_off[i], q0n * (int)a.q_row_stride * 2);
            dst[i] = bload128s(do_rs, dold_off[i], q0n * (int)a.do_row_stride * 2);
        }
        if (tid < C::BQ) {
            const int qc = min(q0n + tid, seqlen_q - 1);   // rows past seqlen_q are masked (P = 0)
            lse_st = lse_g[qc];
            del_st = del_g[qc];
        }
    };
    auto lds_store_qtile = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < C::QCH; ++i) {
            const int idx = tid + C::NT * i;
            if ((C::BQ * C::NC) % C::NT == 0 || idx < C::BQ * C::NC) {
                const int row = idx / C::NC, c = idx % C::NC;
                lds_write128(smem + C::OFF_Q + buf * C::Q_IMG, S::off(row, c), qst[i]);
                lds_write128(smem + C::OFF_DO + buf * C::Q_IMG, S::off(row, c), dst[i]);
            }
        }
        if (tid < C::BQ) {
            lds_write32(smem + C::OFF_LSE + buf * C::BQ * 4, 4 * tid, lse_st * LOG2E);
            lds_write32(smem + C::OFF_DELTA + buf * C::BQ * 4, 4 * tid, del_st);
        }
    };
    // ---- block sparsity: live 32-row query tiles of this 256-key column block (as fa_bwd_kernel)
    uint64_t *qlive = (uint64_t *)(smem + C::OFF_QLIVE);
    const int cb = k0 >> 8;
    auto row_live = [&](int r) __attribute__((always_inline)) -> bool {
        return r < bm.rows && bm.mask[(int64_t)r * bm.row_stride + cb] != 0;
    };
    if constexpr (SPARSE) {
        for (int chunk = wave; chunk < C::QLIVE_WORDS; chunk += C::NW) {
            const int t = 64 * chunk + lane;
            const int rb = (q_begin >> 4) + 2 * t;
            const bool live = t < nqt && (row_live(rb) || row_live(rb + 1));
            const uint64_t word = __builtin_amdgcn_ballot_w64(live);
            if (lane == 0) qlive[chunk] = word;
        }
        __syncthreads();
    }
    auto next_qt = [&](int t) __attribute__((always_inline)) -> int {
        int n = t + 1;
        if constexpr (!SPARSE) {
            return n;
        } else {
            while (n < nqt) {
                const int w = n >> 6;
                const uint64_t bits = qlive[w] >> (n & 63);
                const uint64_t ub = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(bits >> 32)) << 32) |
                                    __builtin_amdgcn_readfirstlane((uint32_t)bits);
                if (ub) return n + (int)__builtin_ctzll(ub);
                n = 64 * (w + 1);
            }
            return nqt;
        }
    };
    const int t_first = SPARSE ? next_qt(-1) : 0;
    if (t_first < nqt) {
        gload_qtile(q_begin + t_first * C::BQ);
        lds_store_qtile(0);
    }
    __syncthreads();

    auto qstep = [&](auto par_tag, int it, int itn) __attribute__((always_inline)) {
        constexpr int BUF = decltype(par_tag)::value;
        char *qimg = smem + C::OFF_Q + BUF * C::Q_IMG;
        char *doimg = smem + C::OFF_DO + BUF * C::Q_IMG;
        const float *lse_b = lse_s + BUF * C::BQ;
        const float *del_b = del_s + BUF * C::BQ;
        const int q0 = q_begin + it * C::BQ;
        if (itn < nqt) gload_qtile(q_begin + itn * C::BQ);
        const bool dead0 = SPARSE && !row_live(q0 >> 4);
        const bool dead1 = SPARSE && !row_live((q0 >> 4) + 1);
        const bool active = !CAUSAL || (q0 + C::BQ - 1 >= kw);
        f32x16 x;   // P waves: S -> P -> Pd; dS waves: dZ -> dS
        u32x4 rw[2];
        if (active) {
            // ---- S = Q K^T (P waves) or dZ = dO V^T (dS waves): lane = key, registers = query rows
            const char *aimg = role_p ? qimg : doimg;
#pragma unroll
            for (int r = 0; r < 16; ++r) x[r] = 0.f;
#pragma unroll
            for (int ks = 0; ks < D / 16; ++ks) {
                const auto qa = as_frag<T>(lds_read128(aimg, S::off(l32, 2 * ks + hi)));
                if constexpr (C::KVL)
                    x = T::mfma32(qa, as_frag<T>(lds_read128(role_p ? kimg : smem + C::OFF_V,
                                                             S::off(32 * kwave + l32, 2 * ks + hi))), x);
                else
                    x = T::mfma32(qa, bf[ks], x);
            }
            if (DROPOUT) {
#pragma unroll
                for (int sg = 0; sg < 2; ++sg) {
                    const uint32_t g = ((uint32_t)(q0 >> 5) << 2) | (sg << 1) | hi;
                    rw[sg] = philox7(g, (uint32_t)kvrow, bh, rng_ctr3, seed_lo, seed_hi);
                }
            }
            if (role_p) {
                const bool need_mask = (q0 + C::BQ > seqlen_q) || (k0 + C::BKV > seqlen_k) ||
                                       (CAUSAL && q0 < kw + 31) || dead0 || dead1;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 lse4 = *reinterpret_cast<const f32x4 *>(lse_b + 8 * g + 4 * hi);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int r = 4 * g + e;
                        float p = fast_exp2(fmaf(x[r], c_log2, -lse4[e]));
                        if (need_mask) {
                            const int q = q0 + crow(r, hi);
                            if (q >= seqlen_q || kvrow >= seqlen_k || (CAUSAL && kvrow > q) || (r < 8 ? dead0 : dead1))
                                p = 0.f;
                        }
                        x[r] = p;
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    lds_write128(px, j * 1024 + lane * 16,
                                 u32x4{__float_as_uint(x[4 * j]), __float_as_uint(x[4 * j + 1]),
                                       __float_as_uint(x[4 * j + 2]), __float_as_uint(x[4 * j + 3])});
            }
        }
        __syncthreads();   // P is in LDS
        if (active) {
            if (role_p) {
                if (DROPOUT) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int slot = (r & 3) | (((r >> 2) & 1) << 2);
                        const uint32_t word = rw[r >> 3][slot >> 1];
                        const uint32_t rnd = (slot & 1) ? (word >> 16) : (word & 0xFFFFu);
                        x[r] = rnd <= keep_thr ? x[r] * rp : 0.f;
                    }
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const u32x4 pw = lds_read128(px, j * 1024 + lane * 16);
                    const f32x4 del4 = *reinterpret_cast<const f32x4 *>(del_b + 8 * j + 4 * hi);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int r = 4 * j + e;
                        float dpv = x[r];
                        if (DROPOUT) {
                            const int slot = (r & 3) | (((r >> 2) & 1) << 2);
                            const uint32_t word = rw[r >> 3][slot >> 1];
                            const uint32_t rnd = (slot & 1) ? (word >> 16) : (word & 0xFFFFu);
                            dpv = rnd <= keep_thr ? dpv * rp : 0.f;
                        }
                        x[r] = __uint_as_float(pw[e]) * (dpv - del4[e]);
                    }
                }
                // dS^T image: row = key (32*kwave + l32), columns = query rows 8g + 4hi .. +3
                if constexpr (DQ) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        u32x2 w = {T::pack2(x[4 * g + 0], x[4 * g + 1]), T::pack2(x[4 * g + 2], x[4 * g + 3])};
                        lds_write64(dsimg, ds_off(32 * kwave + l32, 8 * g + 4 * hi), w);
                    }
                }
            }
            // ---- dV^T += dO^T Pd (P waves) or dK^T += Q^T dS (dS waves), A operands by transposed reads
            const char *timg = role_p ? doimg : qimg;
#pragma unroll
            for (int sg = 0; sg < 2; ++sg) {
                u32x4 pk;
#pragma unroll
                for (int e = 0; e < 4; ++e) pk[e] = T::pack2(x[8 * sg + 2 * e], x[8 * sg + 2 * e + 1]);
                const int rb = 16 * sg + 4 * hi + qq;
#pragma unroll
                for (int dt = 0; dt < D / 32; ++dt) {
                    const int col = 32 * dt + 16 * grp + 4 * pp;
                    u32x2 a0 = lds_read_tr(timg, S::off8(rb, col));
                    u32x2 a1 = lds_read_tr(timg, S::off8(rb + 8, col));
                    acc[dt] = T::mfma32(as_frag<T>(u32x4{a0[0], a0[1], a1[0], a1[1]}), as_frag<T>(pk), acc[dt]);
                }
            }
        } else if (DQ && !role_p) {
            const u32x2 z = {0u, 0u};
#pragma unroll
            for (int g = 0; g < 4; ++g) lds_write64(dsimg, ds_off(32 * kwave + l32, 8 * g + 4 * hi), z);
        }
        if constexpr (DQ) {
            __syncthreads();   // dS image complete

            // ---- dQ = dS K over the block's keys: 16x16x32 MFMAs, 2 x D/16 tiles dealt to the waves
    #pragma unroll
            for (int t0 = 0; t0 < 2 * (D / 16); t0 += C::NW) {
                const int t = t0 + wave;
                if (t < 2 * (D / 16)) {
                    const int qh = t & 1;
                    const int dbase = 16 * (t >> 1);
                    f32x4 dacc = {0.f, 0.f, 0.f, 0.f};
                    auto dq_operands = [&](int ks, u32x4 &av, u32x4 &bv) __attribute__((always_inline)) {
                        const int r0 = 32 * ks + 8 * g4 + qq;
                        u32x2 a0 = lds_read_tr(dsimg, ds_off(r0, 16 * qh + 4 * pp));
                        u32x2 a1 = lds_read_tr(dsimg, ds_off(r0 + 4, 16 * qh + 4 * pp));
                        av = u32x4{a0[0], a0[1], a1[0], a1[1]};
                        u32x2 b0 = lds_read_tr(kimg, S::off8(r0, dbase + 4 * pp));
                        u32x2 b1 = lds_read_tr(kimg, S::off8(r0 + 4, dbase + 4 * pp));
                        bv = u32x4{b0[0], b0[1], b1[0], b1[1]};
                    };
                    u32x4 av, bv, avn, bvn;
                    dq_operands(0, av, bv);
    #pragma unroll
                    for (int ks = 0; ks < C::BKV / 32; ++ks) {
                        if (ks + 1 < C::BKV / 32) dq_operands(ks + 1, avn, bvn);
                        dacc = T::mfma16(as_frag<T>(av), as_frag<T>(bv), dacc);
                        av = avn;
                        bv = bvn;
                    }
                    const int d = dbase + (lane & 15);
                    if (q0 + C::BQ <= seqlen_q && head_dim == D) {
                        float *base = dqa + (int64_t)(q0 + 16 * qh + 4 * g4) * dqa_row + d;
    #pragma unroll
                        for (int i = 0; i < 4; ++i) atomicAdd(base + i * dqa_row, dacc[i]);
                    } else if (d < head_dim) {
    #pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int q = q0 + 16 * qh + 4 * g4 + i;
                            if (q < seqlen_q) atomicAdd(dqa + (int64_t)q * dqa_row + d, dacc[i]);
                        }
                    }
                }
            }
        }
        if (itn < nqt) lds_store_qtile(1 - BUF);
        __syncthreads();
    };
    // ---- skewed pipeline (C::SKEW): in step u the P waves take query tile u (S, P -> P image u&1,
    // dV) while the dS waves take tile u-1 (dZ, dS from P image (u-1)&1, dK). Neither waits for the
    // other inside a step, so on each SIMD the P wave's exp work runs beside the dS wave's MFMAs and
    // the other way round; one barrier per step. Tile u+1 is prefetched into Q/dO buffer (u+1)%3.
    // FA_BWD_SPLIT_PROBE == 6 (timing probe, wrong dK / dV by design): shader-clock stamps per
    // step phase, summed over the steps and written over the first key row of each wave's output
    uint64_t ph[5] = {0, 0, 0, 0, 0};
    uint64_t tstamp = 0;
    auto stamp = [&](int i) __attribute__((always_inline)) {
        if constexpr (FA_BWD_SPLIT_PROBE == 6) {
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t t = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_sched_barrier(0);
            if (i >= 0) ph[i] += t - tstamp;
            tstamp = t;
        }
    };
    auto sstep = [&](auto qb_tag, int u) __attribute__((always_inline)) {
        constexpr int QB = decltype(qb_tag)::value;           // buffer of tile u
        constexpr int QBD = (QB + 2) % 3;                      // buffer of tile u-1 (dS waves)
        stamp(-1);
        if (u + 1 < nqt && FA_BWD_SPLIT_PROBE != 4) gload_qtile(q_begin + (u + 1) * C::BQ);
        const int tile = role_p ? u : u - 1;
        const int q0 = q_begin + tile * C::BQ;
        const bool has = role_p ? u < nqt : u >= 1;
        const bool active = has && (!CAUSAL || (q0 + C::BQ - 1 >= kw));
        char *pxb = px + ((role_p ? u : u - 1) & 1) * (C::KEYW * C::PX_PAIR);
        if (active) {
            const char *qimg = smem + C::OFF_Q + (role_p ? QB : QBD) * C::Q_IMG;
            const char *doimg = smem + C::OFF_DO + (role_p ? QB : QBD) * C::Q_IMG;
            f32x16 x;
            const char *aimg = role_p ? qimg : doimg;
            // row constants (lse, or delta and the P image of the tile) issued ahead of the product:
            // none of them depends on it, and read behind it they exposed one LDS latency per group
            f32x4 rc4[4];
            u32x4 pw[4];
            if (FA_BWD_SPLIT_HOIST) {
                const float *rcb = role_p ? lse_s + QB * C::BQ : del_s + QBD * C::BQ;
#pragma unroll
                for (int g = 0; g < 4; ++g) rc4[g] = *reinterpret_cast<const f32x4 *>(rcb + 8 * g + 4 * hi);
                if (!role_p) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) pw[j] = lds_read128(pxb, j * 1024 + lane * 16);
                }
            }
            // (dZ's accumulator seeded with -delta, as fa_bwd_kernel does without dropout, measured
            // 3-6 % slower in this kernel: C4 backward 4.01 vs 3.77 ms)
#pragma unroll
            for (int r = 0; r < 16; ++r) x[r] = 0.f;
            if (FA_BWD_SPLIT_HOIST) {
                // operands of all D/16 k-steps read before the chain (the compiler otherwise kept one
                // read in flight per MFMA)
                typename T::frag qa[D / 16], kv[D / 16];
#pragma unroll
                for (int ks = 0; ks < D / 16; ++ks) {
                    qa[ks] = as_frag<T>(lds_read128(aimg, S::off(l32, 2 * ks + hi)));
                    if constexpr (C::KVL)
                        kv[ks] = as_frag<T>(lds_read128(role_p ? kimg : smem + C::OFF_V,
                                                        S::off(32 * kwave + l32, 2 * ks + hi)));
                    else
                        kv[ks] = bf[ks];
                    // keep the reads ahead of the chain and in k-step order (counted waits)
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int ks = 0; ks < D / 16; ++ks) x = T::mfma32(qa[ks], kv[ks], x);
            } else {
#pragma unroll
                for (int ks = 0; ks < D / 16; ++ks) {
                    const auto qa = as_frag<T>(lds_read128(aimg, S::off(l32, 2 * ks + hi)));
                    if constexpr (C::KVL)
                        x = T::mfma32(qa, as_frag<T>(lds_read128(role_p ? kimg : smem + C::OFF_V,
                                                                 S::off(32 * kwave + l32, 2 * ks + hi))), x);
                    else
                        x = T::mfma32(qa, bf[ks], x);
                }
            }
            if (!FA_BWD_SPLIT_HOIST) {
                const float *rcb = role_p ? lse_s + QB * C::BQ : del_s + QBD * C::BQ;
#pragma unroll
                for (int g = 0; g < 4; ++g) rc4[g] = *reinterpret_cast<const f32x4 *>(rcb + 8 * g + 4 * hi);
                if (!role_p) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) pw[j] = lds_read128(pxb, j * 1024 + lane * 16);
                }
            }
            if constexpr (FA_BWD_SPLIT_PROBE == 6) {
                // the chain's result consumed before the stamp
                float z = x[0] + x[15];
                asm volatile("" :: "v"(z));
            }
            stamp(0);
            if (role_p) {
                // P = exp2(S c - lse), the per-element mask in its own copy (taken on the causal
                // diagonal and the ragged edges only)
                auto pexp = [&](auto masked_tag) __attribute__((always_inline)) {
                    constexpr bool MASKED = decltype(masked_tag)::value;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        float p = fast_exp2(fmaf(x[r], c_log2, -rc4[r >> 2][r & 3]));
                        if (MASKED) {
                            const int q = q0 + crow(r, hi);
                            p = mask_min(p, q >= seqlen_q || kvrow >= seqlen_k || (CAUSAL && kvrow > q));
                        }
                        x[r] = p;
                    }
                };
                const bool need_mask = (q0 + C::BQ > seqlen_q) || (k0 + C::BKV > seqlen_k) || (CAUSAL && q0 < kw + 31);
                if (FA_BWD_SPLIT_PROBE == 3)
                    ;
                else if (!FA_BWD_SPLIT_HOIST || __builtin_amdgcn_readfirstlane((int)need_mask))
                    pexp(std::true_type{});
                else
                    pexp(std::false_type{});
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    lds_write128(pxb, j * 1024 + lane * 16,
                                 u32x4{__float_as_uint(x[4 * j]), __float_as_uint(x[4 * j + 1]),
                                       __float_as_uint(x[4 * j + 2]), __float_as_uint(x[4 * j + 3])});
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        x[4 * j + e] = FA_BWD_SPLIT_PROBE == 3 ? x[4 * j + e] + __uint_as_float(pw[j][e])
                                                               : __uint_as_float(pw[j][e]) * (x[4 * j + e] - rc4[j][e]);
                }
            }
            stamp(1);
            // dV^T += dO^T P (P waves) or dK^T += Q^T dS (dS waves), A operands by transposed reads
            const char *timg = role_p ? doimg : qimg;
#pragma unroll
            for (int sg = 0; sg < 2; ++sg) {
                u32x4 pk;
#pragma unroll
                for (int e = 0; e < 4; ++e) pk[e] = T::pack2(x[8 * sg + 2 * e], x[8 * sg + 2 * e + 1]);
                const int rb = 16 * sg + 4 * hi + qq;
#pragma unroll
                for (int dt = 0; dt < D / 32; ++dt) {
                    const int col = 32 * dt + 16 * grp + 4 * pp;
                    u32x2 a0 = lds_read_tr(timg, S::off8(rb, col));
                    u32x2 a1 = lds_read_tr(timg, S::off8(rb + 8, col));
                    acc[dt] = T::mfma32(as_frag<T>(u32x4{a0[0], a0[1], a1[0], a1[1]}), as_frag<T>(pk), acc[dt]);
                }
            }
        }
        if constexpr (FA_BWD_SPLIT_PROBE == 6) {
            float z = acc[0][0] + acc[D / 32 - 1][15];
            asm volatile("" :: "v"(z));
        }
        stamp(2);
        // tile u+1 into buffer (u+1)%3: it held tile u-2, last read by the dS waves in step u-1
        if (u + 1 < nqt && FA_BWD_SPLIT_PROBE != 5) lds_store_qtile((QB + 1) % 3);
        stamp(3);
        // timing probes (wrong results by design): FA_BWD_SPLIT_PROBE 1 = no barrier in odd steps,
        // 2 = no barrier at all, 3 = no exp / dS VALU (P = S), 4 = no query-tile loads, 5 = no query-tile
        // LDS stores
        if (!(FA_BWD_SPLIT_PROBE == 2 || (FA_BWD_SPLIT_PROBE == 1 && (u & 1)))) __syncthreads();
        stamp(4);
    };

    // ---- skewed step over two 32-row sub-tiles (C::SUB == 2): as sstep, with both sub-tiles'
    // chains interleaved (independent accumulators), a four-k-step window of operand reads, and P
    // exchanged as the packed 16-bit words the P waves feed their own dV MFMAs
    auto sstep2 = [&](auto qb_tag, int u) __attribute__((always_inline)) {
        constexpr int QB = decltype(qb_tag)::value;           // buffer of tile u
        // LDS bases past 64 KiB (beyond the 16-bit ds offset) tied to the step (u >> 30 is 0), so
        // per-lane addresses are formed next to their reads, not hoisted as dozens of registers
        const int zu = __builtin_amdgcn_readfirstlane(u >> 30);
        auto step_base = [&](int off) __attribute__((always_inline)) { return off + zu; };
        constexpr int QBD = (QB + 2) % 3;                      // buffer of tile u-1 (dS waves)
        if (u + 1 < nqt) gload_qtile(q_begin + (u + 1) * C::BQ);
        const int tile = role_p ? u : u - 1;
        const int q0 = q_begin + tile * C::BQ;
        const bool has = role_p ? u < nqt : u >= 1;
        const bool active = has && (!CAUSAL || (q0 + C::BQ - 1 >= kw));
        char *pxb = smem + step_base(C::OFF_PX + kwave * C::PX_PAIR + ((role_p ? u : u - 1) & 1) * (C::KEYW * C::PX_PAIR));
        if (active) {
            const int qbuf = role_p ? QB : QBD;
            const char *qimg = smem + step_base(C::OFF_Q + qbuf * C::Q_IMG);
            const char *doimg = smem + step_base(C::OFF_DO + qbuf * C::Q_IMG);
            const char *aimg = role_p ? qimg : doimg;
            constexpr int NKS = D / 16, WIN = 1;
            f32x16 x[2];
#pragma unroll
            for (int r = 0; r < 16; ++r) { x[0][r] = 0.f; x[1][r] = 0.f; }
            u32x4 qa[2][NKS];
            auto rd = [&](int ks) __attribute__((always_inline)) {
#pragma unroll
                for (int sb = 0; sb < 2; ++sb) qa[sb][ks] = lds_read128(aimg, S::off(32 * sb + l32, 2 * ks + hi));
            };
#pragma unroll
            for (int ks = 0; ks < WIN; ++ks) rd(ks);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const auto kf = C::KVL ? as_frag<T>(lds_read128(role_p ? kimg : smem + C::OFF_V,
                                                                S::off(32 * kwave + l32, 2 * ks + hi)))
                                       : bf[ks];
                x[0] = T::mfma32(as_frag<T>(qa[0][ks]), kf, x[0]);
                x[1] = T::mfma32(as_frag<T>(qa[1][ks]), kf, x[1]);
                if (ks + WIN < NKS) rd(ks + WIN);
                __builtin_amdgcn_sched_barrier(0);
            }
            u32x4 pk[2][2];   // [sub-tile][16-row half]: packed 16-bit P (P waves) or dS (dS waves)
            if (role_p) {
                const float *lse_b = (const float *)(smem + step_base(C::OFF_LSE + QB * C::BQ * 4));
#pragma unroll
                for (int sb = 0; sb < 2; ++sb) {
                    const int q0s = q0 + 32 * sb;
                    f32x4 rc4[4];
#pragma unroll
                    for (int g = 0; g < 4; ++g) rc4[g] = *reinterpret_cast<const f32x4 *>(lse_b + 32 * sb + 8 * g + 4 * hi);
                    auto pexp = [&](auto masked_tag) __attribute__((always_inline)) {
                        constexpr bool MASKED = decltype(masked_tag)::value;
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            float p = fast_exp2(fmaf(x[sb][r], c_log2, -rc4[r >> 2][r & 3]));
                            if (MASKED) {
                                const int q = q0s + crow(r, hi);
                                p = mask_min(p, q >= seqlen_q || kvrow >= seqlen_k || (CAUSAL && kvrow > q));
                            }
                            x[sb][r] = p;
                        }
                    };
                    const bool need_mask = (q0s + 32 > seqlen_q) || (k0 + C::BKV > seqlen_k) || (CAUSAL && q0s < kw + 31);
                    if (__builtin_amdgcn_readfirstlane((int)need_mask))
                        pexp(std::true_type{});
                    else
                        pexp(std::false_type{});
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) pk[sb][sg][e] = T::pack2(x[sb][8 * sg + 2 * e], x[sb][8 * sg + 2 * e + 1]);
                        lds_write128(pxb, sb * C::PX_SUB + sg * 1024 + lane * 16, pk[sb][sg]);
                    }
                }
            } else {
                const float *del_b = (const float *)(smem + step_base(C::OFF_DELTA + QBD * C::BQ * 4));
#pragma unroll
                for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
                    for (int sg = 0; sg < 2; ++sg) {
                        const u32x4 pw = lds_read128(pxb, sb * C::PX_SUB + sg * 1024 + lane * 16);
                        const f32x4 dA = *reinterpret_cast<const f32x4 *>(del_b + 32 * sb + 16 * sg + 4 * hi);
                        const f32x4 dB = *reinterpret_cast<const f32x4 *>(del_b + 32 * sb + 16 * sg + 8 + 4 * hi);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            // registers 8 sg + 2e, +1: rows crow(., hi) = 16 sg + (2e < 4 ? 0 : 8) + 4hi + (2e & 3), +1
                            const int r = 8 * sg + 2 * e;
                            const f32x4 &dl = (e < 2) ? dA : dB;
                            const float p0 = T::lo_float(pw[e]), p1 = T::hi_float(pw[e]);
                            const float s0 = p0 * (x[sb][r] - dl[(2 * e) & 3]);
                            const float s1 = p1 * (x[sb][r + 1] - dl[(2 * e + 1) & 3]);
                            pk[sb][sg][e] = T::pack2(s0, s1);
                        }
                    }
                }
            }
            // dV^T += dO^T P (P waves) or dK^T += Q^T dS (dS waves), A operands by transposed reads
            const char *timg = role_p ? doimg : qimg;
#pragma unroll
            for (int sb = 0; sb < 2; ++sb)
#pragma unroll
                for (int sg = 0; sg < 2; ++sg) {
                    const int rb = 32 * sb + 16 * sg + 4 * hi + qq;
#pragma unroll
                    for (int dt = 0; dt < D / 32; ++dt) {
                        const int col = 32 * dt + 16 * grp + 4 * pp;
                        u32x2 a0 = lds_read_tr(timg, S::off8(rb, col));
                        u32x2 a1 = lds_read_tr(timg, S::off8(rb + 8, col));
                        acc[dt] = T::mfma32(as_frag<T>(u32x4{a0[0], a0[1], a1[0], a1[1]}), as_frag<T>(pk[sb][sg]), acc[dt]);
                    }
                }
        }
        // tile u+1 into buffer (u+1)%3: it held tile u-2, last read by the dS waves in step u-1
        if (u + 1 < nqt) lds_store_qtile((QB + 1) % 3);
        __syncthreads();
    };

    if constexpr (C::SKEW) {
        // the prologue stored tile 0 in buffer 0; steps u = 0 .. nqt (the last one: dS waves only)
        int u = 0;
        if constexpr (C::SUB == 2) {
            for (; u + 2 <= nqt; u += 3) {
                sstep2(std::integral_constant<int, 0>(), u);
                sstep2(std::integral_constant<int, 1>(), u + 1);
                sstep2(std::integral_constant<int, 2>(), u + 2);
            }
            if (u <= nqt) sstep2(std::integral_constant<int, 0>(), u++);
            if (u <= nqt) sstep2(std::integral_constant<int, 1>(), u++);
        } else {
            for (; u + 2 <= nqt; u += 3) {
                sstep(std::integral_constant<int, 0>(), u);
                sstep(std::integral_constant<int, 1>(), u + 1);
                sstep(std::integral_constant<int, 2>(), u + 2);
            }
            if (u <= nqt) sstep(std::integral_constant<int, 0>(), u++);
            if (u <= nqt) sstep(std::integral_constant<int, 1>(), u++);
        }
    } else if constexpr (SPARSE) {
        int it = t_first;
        while (it < nqt) {
            int itn = next_qt(it);
            qstep(std::integral_constant<int, 0>(), it, itn);
            it = itn;
            if (it >= nqt) break;
            itn = next_qt(it);
            qstep(std::integral_constant<int, 1>(), it, itn);
            it = itn;
        }
    } else {
        for (int it = 0; it < nqt; it += 2) {
            qstep(std::integral_constant<int, 0>(), it, it + 1);
            if (it + 1 < nqt) qstep(std::integral_constant<int, 1>(), it + 1, it + 2);
        }
    }

    if constexpr (FA_BWD_SPLIT_PROBE == 6) {
        // phases: 0 = operand reads + S / dZ chain, 1 = P / dS VALU (+ P exchange), 2 = update
        // MFMAs (transposed reads, results consumed), 3 = staging LDS stores, 4 = barrier; 5th word:
        // the step count
        if (lane == 0 && kw < seqlen_k) {
            uint64_t *o = (uint64_t *)(role_p ? (uint16_t *)a.dv + (int64_t)(k_start + kw) * a.dv_row_stride + (int64_t)h * a.dv_head_stride
                                              : (uint16_t *)a.dk + (int64_t)(k_start + kw) * a.dk_row_stride + (int64_t)h * a.dk_head_stride);
            for (int i = 0; i < 5; ++i) o[i] = ph[i];
            o[5] = (uint64_t)(nqt + 1);
        }
        return;
    }
    // ---- epilogue: dV (P waves) or scaled dK (dS waves) rows of this lane's key
    if (kvrow < seqlen_k) {
        uint16_t *outp = role_p
            ? (uint16_t *)a.dv + (int64_t)(k_start + kvrow) * a.dv_row_stride + (int64_t)h * a.dv_head_stride
            : (uint16_t *)a.dk + (int64_t)(k_start + kvrow) * a.dk_row_stride + (int64_t)h * a.dk_head_stride;
        const float sc = role_p ? 1.f : a.softmax_scale;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = 32 * dt + 8 * g + 4 * hi;
                if (d < head_dim) {
                    u32x2 w = {T::pack2(acc[dt][4 * g + 0] * sc, acc[dt][4 * g + 1] * sc),
                               T::pack2(acc[dt][4 * g + 2] * sc, acc[dt][4 * g + 3] * sc)};
                    gstore64(outp + d, w);
                }
            }
    }
}

}  // namespace fa
