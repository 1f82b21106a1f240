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
// (q-blocks, H, B); a workgroup = 4 waves = 128 query rows, one wave = 32 rows. Q stays in
// VGPRs for the whole kernel; K/V tiles of 64 keys are register-staged into a double-buffered,
// XOR-swizzled LDS image (issue-early / write-late, one barrier per tile). Scores are computed
// swapped (S^T = K Q^T, v_mfma_f32_32x32x16) so each lane owns one query row: the row max is
// 31 fmax + one v_permlane32_swap, the row sum stays lane-local until the epilogue, and P feeds
// the P·V MFMA straight from registers (accumulator-as-B-operand). V^T operands come from
// ds_read_b64_tr_b16. The N x N score matrix never leaves registers.
#pragma once

#include "fa_common.h"
#include "../../include/fa_hip.h"

namespace fa {

template <int D>
struct FwdCfg {
    static constexpr int NW = 4;                  // waves per workgroup
    static constexpr int BM = 32 * NW;            // query rows per workgroup
    static constexpr int BN = 64;                 // keys per iteration
    static constexpr int NC = D / 8;              // 16-B chunks per row
    static constexpr int TILE_BYTES = BN * D * 2;
    static constexpr int CPT = BN * NC / 256;     // staged chunks per thread per tile
    static constexpr int RNG_BYTES_PER_WAVE = 2 * 32 * 32 * 2;  // two 32x32 u16 images
    static constexpr int lds_bytes(bool dropout) {
        return 4 * TILE_BYTES + (dropout ? NW * RNG_BYTES_PER_WAVE : 0);
    }
};

template <int D, typename T, bool CAUSAL, bool DROPOUT>
__global__ __launch_bounds__(256) void fa_fwd_kernel(const FaFwdArgs a) {
    using C = FwdCfg<D>;
    using S = Swz<D>;
    constexpr float LOG2E = 1.4426950408889634f;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int b = blockIdx.z;
    const int h = blockIdx.y;
    // causal: heaviest query blocks first (LPT order)
    const int qb = CAUSAL ? (int)(gridDim.x - 1 - blockIdx.x) : (int)blockIdx.x;
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
    const int qw = q0 + 32 * wave;       // first query row of this wave
    const int qrow = qw + l32;           // the query row this lane owns
    const int head_dim = a.head_dim;

    const uint16_t *qp = (const uint16_t *)a.q + (int64_t)q_start * a.q_row_stride + (int64_t)h * a.q_head_stride;
    const uint16_t *kp = (const uint16_t *)a.k + (int64_t)k_start * a.k_row_stride + (int64_t)h * a.k_head_stride;
    const uint16_t *vp = (const uint16_t *)a.v + (int64_t)k_start * a.v_row_stride + (int64_t)h * a.v_head_stride;

    char *kbuf0 = smem;
    char *kbuf1 = smem + C::TILE_BYTES;
    char *vbuf0 = smem + 2 * C::TILE_BYTES;
    char *vbuf1 = smem + 3 * C::TILE_BYTES;

    int n_end = seqlen_k;
    if (CAUSAL) n_end = min(n_end, q0 + C::BM);
    const int nt = (n_end + C::BN - 1) / C::BN;

    // ---- Q fragments (B operand of S^T = K Q^T): Q[qrow][16ks + 8hi + j]
    typename T::frag qf[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
        const int c = 2 * ks + hi;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (qrow < seqlen_q && c * 8 < head_dim) v = gload128(qp + (int64_t)qrow * a.q_row_stride + c * 8);
        qf[ks] = as_frag<T>(v);
    }

    // ---- register staging of one K/V tile (issue early, write late: T14)
    u32x4 kst[C::CPT], vst[C::CPT];
    auto gload_tile = [&](int kv0) {
#pragma unroll
        for (int i = 0; i < C::CPT; ++i) {
            const int idx = tid + 256 * i;
            const int row = idx / C::NC, c = idx % C::NC;
            const int kv = kv0 + row;
            const bool ok = kv < seqlen_k && c * 8 < head_dim;
            u32x4 z = {0u, 0u, 0u, 0u};
            kst[i] = ok ? gload128(kp + (int64_t)kv * a.k_row_stride + c * 8) : z;
            vst[i] = ok ? gload128(vp + (int64_t)kv * a.v_row_stride + c * 8) : z;
        }
    };
    auto lds_store_tile = [&](char *kb, char *vb) {
#pragma unroll
        for (int i = 0; i < C::CPT; ++i) {
            const int idx = tid + 256 * i;
            const int row = idx / C::NC, c = idx % C::NC;
            lds_write128(kb, S::off(row, c), kst[i]);
            lds_write128(vb, S::off(row, c), vst[i]);
        }
    };

    f32x16 o[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
    float m_i = -INFINITY;
    float l_i = 0.f;
    const float c_log2 = a.softmax_scale * LOG2E;

    // dropout constants
    const uint32_t keep_thr = (uint32_t)floorf((1.0f - a.p_dropout) * 65535.0f);
    const uint32_t seed_lo = (uint32_t)a.rng_seed, seed_hi = (uint32_t)(a.rng_seed >> 32);
    const uint32_t rng_ctr3 = (uint32_t)(a.rng_offset >> 2);
    const uint32_t bh = (uint32_t)(b * a.nheads + h);
    char *rng_img = smem + 4 * C::TILE_BYTES + wave * C::RNG_BYTES_PER_WAVE;

    // tr-read lane geometry (16-lane group, lane 4qq+pp supplies row qq, columns 4pp..4pp+3)
    const int grp = (lane >> 4) & 1;
    const int qq = (lane & 15) >> 2;
    const int pp = lane & 3;

    if (nt > 0) {
        gload_tile(0);
        lds_store_tile(kbuf0, vbuf0);
    }
    __syncthreads();

    for (int j = 0; j < nt; ++j) {
        const int kv0 = j * C::BN;
        const bool odd = j & 1;
        char *kb = odd ? kbuf1 : kbuf0;
        char *vb = odd ? vbuf1 : vbuf0;
        if (j + 1 < nt) gload_tile(kv0 + C::BN);

        const bool active = (qw < seqlen_q) && (!CAUSAL || kv0 <= qw + 31);
        if (active) {
            // ---- S^T = K Q^T : two 32x32 sub-tiles, lane = query row, registers = keys
            f32x16 s[2];
#pragma unroll
            for (int st = 0; st < 2; ++st) {
#pragma unroll
                for (int r = 0; r < 16; ++r) s[st][r] = 0.f;
#pragma unroll
                for (int ks = 0; ks < D / 16; ++ks) {
                    u32x4 kf = lds_read128(kb, S::off(32 * st + l32, 2 * ks + hi));
                    s[st] = T::mfma32(as_frag<T>(kf), qf[ks], s[st]);
                }
            }
            // ---- mask (only on the ragged last tile and the causal diagonal)
            const bool need_mask = (kv0 + C::BN > seqlen_k) || (CAUSAL && kv0 + C::BN - 1 > qw);
            if (need_mask) {
#pragma unroll
                for (int st = 0; st < 2; ++st)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int kv = kv0 + 32 * st + crow(r, hi);
                        if (kv >= seqlen_k || (CAUSAL && kv > qrow)) s[st][r] = -INFINITY;
                    }
            }
            // ---- online softmax
            float mx = s[0][0];
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[st][r]);
            mx = pair_max(mx);
            const float m_new = fmaxf(m_i, mx);
            const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
            const float mc = m_use * c_log2;
            const float alpha = fast_exp2(m_i * c_log2 - mc);
            float rs = 0.f;
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float p = fast_exp2(fmaf(s[st][r], c_log2, -mc));
                    s[st][r] = p;
                    rs += p;
                }
            l_i = l_i * alpha + rs;
            m_i = m_new;
#pragma unroll
            for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;

            if (DROPOUT) {
                // Generate the keep mask in the column-major (backward) layout, then transpose
                // it through a per-wave LDS image with ds_read_b64_tr_b16.
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

            // ---- P (16-bit) as the B operand: registers 8s2..8s2+7 of sub-tile st
            typename T::frag pf[2][2];
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    u32x4 pk;
#pragma unroll
                    for (int e = 0; e < 4; ++e) pk[e] = T::pack2(s[st][8 * s2 + 2 * e], s[st][8 * s2 + 2 * e + 1]);
                    pf[st][s2] = as_frag<T>(pk);
                }
            // ---- O^T += V^T P^T
#pragma unroll
            for (int dt = 0; dt < D / 32; ++dt) {
                const int col = 32 * dt + 16 * grp + 4 * pp;
#pragma unroll
                for (int st = 0; st < 2; ++st)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const int rb = 32 * st + 16 * s2 + 4 * hi + qq;
                        u32x2 lo = lds_read_tr(vb, S::off8(rb, col));
                        u32x2 hv = lds_read_tr(vb, S::off8(rb + 8, col));
                        u32x4 av = {lo[0], lo[1], hv[0], hv[1]};
                        o[dt] = T::mfma32(as_frag<T>(av), pf[st][s2], o[dt]);
                    }
            }
        }

        if (j + 1 < nt) lds_store_tile(odd ? kbuf0 : kbuf1, odd ? vbuf0 : vbuf1);
        __syncthreads();
    }

    // ---- epilogue
    const float l_tot = pair_sum(l_i);
    const bool empty = (l_tot == 0.f) || (l_tot != l_tot);
    float inv = empty ? 1.f : 1.f / l_tot;
    if (DROPOUT) inv *= 1.0f / (1.0f - a.p_dropout);
    if (qrow < seqlen_q) {
        uint16_t *op = (uint16_t *)a.o + (int64_t)(q_start + qrow) * a.o_row_stride + (int64_t)h * a.o_head_stride;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int d = 32 * dt + 8 * g4 + 4 * hi;
                if (d < head_dim) {
                    u32x2 w = {T::pack2(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv),
                               T::pack2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv)};
                    gstore64(op + d, w);
                }
            }
        if (hi == 0) {
            a.softmax_lse[(int64_t)(b * a.nheads + h) * a.lse_stride + qrow] =
                empty ? -INFINITY : m_i * a.softmax_scale + __logf(l_tot);
        }
    }
}

}  // namespace fa
