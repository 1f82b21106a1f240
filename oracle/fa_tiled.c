/*
 * fa_tiled.c — CPU restatement of the tiled FlashAttention forward. TEST INFRASTRUCTURE ONLY
 * (see oracle/__init__.py): used by tests/ as a checker, by bench.py as the "port" CPU baseline.
 *
 * Follows the reference forward's per-row semantics:
 *   online softmax, exp2 with scale*log2(e) folded     csrc/flash_attn/src/fmha/softmax.h:211-226
 *   sum taken before dropout; O *= 1/sum * 1/p_keep    csrc/flash_attn/src/fmha_fprop_kernel_1xN.h:522-536,637-661
 *   keep <=> rnd16 <= floor(p_keep*65535)              fmha_api.cpp:104, softmax.h:256-296
 *   mask col < seqlen_k, causal col <= row (top-left)  csrc/flash_attn/src/fmha/mask.h:58-72
 *   lse = max*scale + log(sum); empty row -> -inf, out 0  fmha_fprop_kernel_1xN.h:590-623,645
 * with this build's tiling (64-key tiles) and its Philox element map (oracle/philox.py).
 * P is optionally rounded to bf16/fp16 before P·V, as the kernel does.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

void fa_oracle_philox(const uint32_t ctr[4], const uint32_t key[2], int rounds, uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int i = 0; i < rounds; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t fa_oracle_rnd16(uint64_t seed, uint64_t offset, uint32_t bh, int row, int col) {
    uint32_t g = ((uint32_t)(row >> 5) << 2) | (((row >> 4) & 1) << 1) | ((row >> 2) & 1);
    int slot = (row & 3) | (((row >> 3) & 1) << 2);
    uint32_t ctr[4] = {g, (uint32_t)col, bh, (uint32_t)(offset >> 2)};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t o[4];
    fa_oracle_philox(ctr, key, 7, o);
    uint32_t w = o[slot >> 1];
    return (slot & 1) ? (w >> 16) : (w & 0xFFFFu);
}

static float round16(float x, int mode) {
    if (mode == 1) { /* bf16 RNE */
        uint32_t u;
        memcpy(&u, &x, 4);
        if ((u & 0x7F800000u) != 0x7F800000u) u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
        memcpy(&x, &u, 4);
        return x;
    }
    if (mode == 2 && x != 0.f && isfinite(x)) { /* fp16 RNE, subnormals down to 2^-24 */
        int e;
        frexpf(fabsf(x), &e);
        int qe = e - 11;
        if (qe < -24) qe = -24;
        const float quantum = ldexpf(1.0f, qe);
        float r = nearbyintf(fabsf(x) / quantum) * quantum;
        if (r > 65504.f) r = INFINITY;
        return copysignf(r, x);
    }
    return x;
}

/* q: (total_q, H, D), k/v: (total_k, H, D) fp32 contiguous; out (total_q, H, D); lse (B, H, lse_stride). */
void fa_oracle_fwd(const float *q, const float *k, const float *v, const int32_t *cu_q, const int32_t *cu_k,
                   int B, int H, int D, int lse_stride, float scale, float p_drop, uint64_t seed,
                   uint64_t offset, int causal, int round_p, float *out, float *lse) {
    const float LOG2E = 1.4426950408889634f;
    const float c = scale * LOG2E;
    const uint32_t thr = (uint32_t)floorf((1.0f - p_drop) * 65535.0f);
    float acc[128], s[64];
    for (int b = 0; b < B; ++b) {
        const int q0 = cu_q[b], sq = cu_q[b + 1] - cu_q[b];
        const int k0 = cu_k[b], sk = cu_k[b + 1] - cu_k[b];
        for (int h = 0; h < H; ++h) {
            const uint32_t bh = (uint32_t)(b * H + h);
            for (int i = 0; i < sq; ++i) {
                const float *qi = q + ((int64_t)(q0 + i) * H + h) * D;
                float m = -INFINITY, l = 0.f;
                for (int d = 0; d < D; ++d) acc[d] = 0.f;
                int n_end = sk;
                for (int j0 = 0; j0 < n_end; j0 += 64) {
                    const int nj = (n_end - j0) < 64 ? (n_end - j0) : 64;
                    float mx = -INFINITY;
                    for (int jj = 0; jj < nj; ++jj) {
                        const int j = j0 + jj;
                        const float *kj = k + ((int64_t)(k0 + j) * H + h) * D;
                        float dot = 0.f;
                        for (int d = 0; d < D; ++d) dot += qi[d] * kj[d];
                        if (causal && j > i) dot = -INFINITY;
                        s[jj] = dot;
                        if (dot > mx) mx = dot;
                    }
                    const float m_new = m > mx ? m : mx;
                    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
                    const float alpha = exp2f(m * c - m_use * c);
                    float rs = 0.f;
                    for (int jj = 0; jj < nj; ++jj) {
                        s[jj] = exp2f(s[jj] * c - m_use * c);
                        rs += s[jj];
                    }
                    l = l * alpha + rs;
                    m = m_new;
                    for (int d = 0; d < D; ++d) acc[d] *= alpha;
                    for (int jj = 0; jj < nj; ++jj) {
                        float p = s[jj];
                        if (p_drop > 0.f && fa_oracle_rnd16(seed, offset, bh, i, j0 + jj) > thr) p = 0.f;
                        p = round16(p, round_p);
                        const float *vj = v + ((int64_t)(k0 + j0 + jj) * H + h) * D;
                        for (int d = 0; d < D; ++d) acc[d] += p * vj[d];
                    }
                }
                const int empty = (l == 0.f) || (l != l);
                float inv = empty ? 1.f : 1.f / l;
                if (p_drop > 0.f) inv *= 1.0f / (1.0f - p_drop);
                float *oi = out + ((int64_t)(q0 + i) * H + h) * D;
                for (int d = 0; d < D; ++d) oi[d] = acc[d] * inv;
                lse[(int64_t)bh * lse_stride + i] = empty ? -INFINITY : m * scale + logf(l);
            }
        }
    }
}
