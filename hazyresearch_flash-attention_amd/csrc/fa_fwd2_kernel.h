// fa_fwd2_kernel.h — dense forward (no dropout, no block mask) for gfx950: two 32-row query
// blocks per wave, software-pipelined so one block's MFMAs run beside the other block's softmax.
//
// Reference behaviour followed (file:line in /root/reference), identical to fa_fwd_kernel.h:
//   - online softmax with exp2 and scale*log2(e) folded     csrc/flash_attn/src/fmha/softmax.h:211-226
//   - row sum before normalisation, O scaled by 1/sum once  csrc/flash_attn/src/fmha_fprop_kernel_1xN.h:522-536,637-661
//   - mask: col < seqlen_k, causal col <= row (top-left)    csrc/flash_attn/src/fmha/mask.h:58-72
//   - LSE = max*scale + log(sum); empty/NaN row -> -inf, O = 0   fmha_fprop_kernel_1xN.h:590-623,645
//
// Structure (MI355X-first, not the reference's loop):
//   * workgroup = 4 waves = 256 query rows; a wave owns rows [qw, qw+64) as block A (first 32) and
//     block B (last 32). K/V tiles of 64 keys arrive by LDS-DMA into a 3-slot ring (tile j+1 loads
//     while tile j and j-1 are read), one barrier per tile.
//   * per tile j the wave runs four phases, each 8 (D=64) MFMAs with independent VALU work beside them:
//        1: S_A(j)  = K(j) Q_A^T            | softmax of B(j-1), keys 32..63, and its check
//        2: O_B    += V(j-1)^T P_B(j-1)^T  | softmax of A(j),   keys  0..31
//        3: S_B(j)  = K(j) Q_B^T            | softmax of A(j),   keys 32..63, and its check
//        4: O_A    += V(j)^T P_A(j)^T      | softmax of B(j),   keys  0..31
//     so the matrix pipe never waits for a softmax and the K/V fragments read from LDS serve 64 rows.
//   * max-free softmax: after the first tile a row keeps a reference m (its first tile's max) and
//     computes p = exp2(s*c - m*c) with no per-tile max. Each lane checks its tile sum: while it stays
//     <= 2^15 every p does too (fp32/bf16 keep their relative precision at any magnitude, so the
//     result equals the max-normalised one up to rounding). A tile whose sum passes the bound (a new
//     max about 10 log2 units above m, an overflow to inf, NaN) is recomputed from the K tile
//     still in LDS with the exact max-rescale path — rare, wave-uniform, and exact.
#pragma once

#include "fa_common.h"
#include "fa_fwd_kernel.h"
#include "../../include/fa_hip.h"

namespace fa {

#ifndef FA_FWD2_WPE
#define FA_FWD2_WPE 2      // waves per SIMD the register allocation must allow (2 = 256 registers)
#endif
#ifndef FA_FWD2_KREUSE
#define FA_FWD2_KREUSE 0   // 1: K fragments of a tile read once and kept for both blocks' QK^T
#endif
#ifndef FA_FWD2_PF
#define FA_FWD2_PF 2       // LDS-DMA prefetch distance in tiles (1..3); the rings hold PF + 2 tiles
#endif
#ifndef FA_FWD2_PROBE
#define FA_FWD2_PROBE 0    // timing probes for the variant harness only (1/2/3 drop exp / row sum / fma)
#endif
#ifndef FA_FWD2_SCHED
#define FA_FWD2_SCHED 0    // 1: sched_group_barrier interleave of MFMA / VALU / LDS reads per phase
#endif

template <int D>
struct Fwd2Cfg {
    static constexpr int NW = 4;                  // waves per workgroup
    static constexpr int NT = 64 * NW;
    static constexpr int BM = 64 * NW;            // query rows per workgroup
    static constexpr int BN = 64;                 // keys per tile
    static constexpr int TILE_BYTES = BN * D * 2;
    static constexpr int PF = FA_FWD2_PF;         // tiles in flight ahead of the one being read
    static constexpr int SLOTS = PF + 2;          // K ring and V ring: j-1, j, j+1 .. j+PF
    static constexpr int LDS_BYTES = 2 * SLOTS * TILE_BYTES;
    static constexpr int PIECES = TILE_BYTES / 1024;   // 1-KiB LDS-DMA pieces per tile
    static constexpr int PPW = PIECES / NW;
    static constexpr int RPP = 1024 / (2 * D);         // tile rows per piece
    static_assert(PIECES % NW == 0, "pieces per tile must split evenly over the waves");
};

// fast-path bound on a lane's tile sum: every p stays <= 2^15, inside fp16's range
constexpr float FWD2_SUM_THR = 32768.0f;

// Row sums are plain f32 adds: this kernel's translation unit (fa_fwd2.hip) is compiled with
// -fno-slp-vectorize so they stay single v_add_f32 (packed v_pk_add_f32 costs more beside MFMAs).
__device__ __forceinline__ float vadd(float a, float b) { return a + b; }

template <int D, typename T, bool CAUSAL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FA_FWD2_WPE))) void fa_fwd2_kernel(const FaFwdArgs a) {
    using C = Fwd2Cfg<D>;
    using Z = Swz<D>;
    using frag = typename T::frag;
    constexpr int KS = D / 16;    // k-steps of QK^T
    constexpr int DT = D / 32;    // 32-wide output column blocks
    constexpr float LOG2E = 1.4426950408889634f;
    constexpr float LN2 = 0.6931471805599453f;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    // ---- block -> (q-block, head, batch): LPT order for causal, XCD-contiguous runs otherwise
    const int nqb = gridDim.x;
    const int nbh = gridDim.y * gridDim.z;
    const int nwg = nqb * nbh;
    const int L = blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z);
    int qb, bh_lin;
    if (CAUSAL) {
        qb = nqb - 1 - L / nbh;
        bh_lin = L % nbh;
    } else {
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
    const int qw = q0 + 64 * wave;          // first row of block A; block B starts at qw + 32
    const int rowA = qw + l32, rowB = qw + 32 + l32;
    const int head_dim = a.head_dim;

    int n_end = seqlen_k;
    if (CAUSAL) n_end = min(n_end, q0 + C::BM);
    const int nt = (n_end + C::BN - 1) / C::BN;

    // ---- Q fragments (B operand of S^T = K Q^T): Q[row][16ks + 8hi + j]
    const auto qr = make_rsrc((const uint16_t *)a.q + (int64_t)q_start * a.q_row_stride + (int64_t)h * a.q_head_stride);
    frag qa[KS], qbf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int c = 2 * ks + hi;
        const bool okc = c * 8 < head_dim;
        qa[ks] = as_frag<T>(bload128(qr, okc && rowA < seqlen_q ? (rowA * (int)a.q_row_stride + c * 8) * 2 : OOB));
        qbf[ks] = as_frag<T>(bload128(qr, okc && rowB < seqlen_q ? (rowB * (int)a.q_row_stride + c * 8) * 2 : OOB));
    }

    // ---- K/V descriptors end at row n_end: rows past it land in LDS as zeros
    const uint16_t *kbase = (const uint16_t *)a.k + (int64_t)k_start * a.k_row_stride + (int64_t)h * a.k_head_stride;
    const uint16_t *vbase = (const uint16_t *)a.v + (int64_t)k_start * a.v_row_stride + (int64_t)h * a.v_head_stride;
    const auto kr = make_rsrc_n(kbase, n_end * (int)a.k_row_stride * 2);
    const auto vr = make_rsrc_n(vbase, n_end * (int)a.v_row_stride * 2);
    const int k_tile_step = C::BN * (int)a.k_row_stride * 2;
    const int v_tile_step = C::BN * (int)a.v_row_stride * 2;

    // LDS-DMA: piece p (1 KiB = RPP rows) of a tile image is written by wave p % NW; lane l lands at
    // byte 16 l of the piece = row RPP p + l / NC, slot l % NC, which holds chunk slot ^ x(row)
    int dma_k_off[C::PPW], dma_v_off[C::PPW];
#pragma unroll
    for (int i = 0; i < C::PPW; ++i) {
        const int p = wave + C::NW * i;
        const int r = C::RPP * p + lane / (D / 8);
        const int c = (lane % (D / 8)) ^ Z::x(r);
        const bool ok = c * 8 < head_dim;
        dma_k_off[i] = ok ? (r * (int)a.k_row_stride + c * 8) * 2 : OOB;
        dma_v_off[i] = ok ? (r * (int)a.v_row_stride + c * 8) * 2 : OOB;
    }
#if FA_DMA_ASM
    const i32x4 ksrd = make_srd(kbase, n_end * (int)a.k_row_stride * 2);
    const i32x4 vsrd = make_srd(vbase, n_end * (int)a.v_row_stride * 2);
#endif
    auto dma = [&](int j, int slot) __attribute__((always_inline)) {
        char *kb = smem + slot * C::TILE_BYTES;
        char *vb = smem + (C::SLOTS + slot) * C::TILE_BYTES;
#pragma unroll
        for (int i = 0; i < C::PPW; ++i) {
            const int p = wave + C::NW * i;
#if defined(__HIP_DEVICE_COMPILE__)
#if FA_DMA_ASM
            dma16(ksrd, dma_k_off[i], j * k_tile_step, lds_addr(kb + 1024 * p));
            dma16(vsrd, dma_v_off[i], j * v_tile_step, lds_addr(vb + 1024 * p));
#else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(kr, (__attribute__((address_space(3))) void *)(kb + 1024 * p), 16,
                                                     dma_k_off[i], j * k_tile_step, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (__attribute__((address_space(3))) void *)(vb + 1024 * p), 16,
                                                     dma_v_off[i], j * v_tile_step, 0, 0);
#endif
#endif
        }
    };
    // wait until tile j+1 has landed, leaving the younger tiles' DMA (up to PF-1 of them) in flight
    constexpr int OPT = 2 * C::PPW;   // DMA instructions per tile per wave
    auto wait_next = [&](int j) __attribute__((always_inline)) {
        const int younger = min(C::PF - 1, nt - 2 - j);
        if (C::PF >= 3 && younger >= 2) vmcnt_n<OPT * (C::PF >= 3 ? 2 : 0)>();
        else if (C::PF >= 2 && younger >= 1) vmcnt_n<OPT>();
        else vmcnt0();
    };

    // ---- lane-constant LDS offsets (slot bases fold into immediates)
    int k_rd[2][KS];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) k_rd[st][ks] = Z::off(32 * st + l32, 2 * ks + hi);
    const int grp = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
    int v_rd[DT][2][2][2];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int rb = 32 * st + 16 * s2 + 4 * hi + qq;
                const int col = 32 * dt + 16 * grp + 4 * pp;
                v_rd[dt][st][s2][0] = Z::off8(rb, col);
                v_rd[dt][st][s2][1] = Z::off8(rb + 8, col);
            }

    const float c_log2 = a.softmax_scale * LOG2E;

    // ---- building blocks
    auto read_k = [&](const char *kb, frag (&kf)[2][KS]) __attribute__((always_inline)) {
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#if FA_FWD2_PROBE >= 5   // timing probe only: no LDS operand reads
                kf[st][ks] = qa[(ks + st) % KS];
#else
                kf[st][ks] = as_frag<T>(lds_read128(kb, k_rd[st][ks]));
#endif
    };
    auto qk = [&](const frag (&kf)[2][KS], const frag (&q)[KS], f32x16 (&s)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[st][r] = 0.f;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) s[st] = T::mfma32(kf[st][ks], q[ks], s[st]);
        }
    };
    auto qk_lds = [&](const char *kb, const frag (&q)[KS], f32x16 (&s)[2]) __attribute__((always_inline)) {
        frag kf[2][KS];
        read_k(kb, kf);
        qk(kf, q, s);
    };
    auto pv = [&](const char *vb, const frag (&p)[2][2], f32x16 (&o)[DT]) __attribute__((always_inline)) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
#if FA_FWD2_PROBE >= 5
                    o[dt] = T::mfma32(qbf[(dt + st + s2) % KS], p[st][s2], o[dt]);
#else
                    const u32x2 lo = lds_read_tr(vb, v_rd[dt][st][s2][0]);
                    const u32x2 hv = lds_read_tr(vb, v_rd[dt][st][s2][1]);
                    const u32x4 av = {lo[0], lo[1], hv[0], hv[1]};
                    o[dt] = T::mfma32(as_frag<T>(av), p[st][s2], o[dt]);
#endif
                }
    };
    // mask of one block's scores for tile kv0 (only called on tiles that cross seqlen_k or the diagonal)
    auto mask = [&](f32x16 (&s)[2], int kv0, int row) __attribute__((always_inline)) {
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int kv = kv0 + 32 * st + crow(r, hi);
                if (kv >= seqlen_k || (CAUSAL && kv > row)) s[st][r] = -INFINITY;
            }
    };
    // wave-uniform: does tile kv0 need the mask for the block whose first row is row0
    auto needs_mask = [&](int kv0, int row0) __attribute__((always_inline)) {
        return kv0 + C::BN > seqlen_k || (CAUSAL && kv0 + C::BN - 1 > row0);
    };
    // half a tile (32 keys) of the max-free softmax: p = exp2(s c - mc), lane sum, 16-bit B operand
    auto smh = [&](f32x16 &s, float mc, float &ts, frag (&p)[2]) __attribute__((always_inline)) {
#if FA_FWD2_PROBE >= 4   // timing probe only: no softmax arithmetic (skeleton)
#elif FA_FWD2_PROBE == 1    // timing probe only (wrong results): no v_exp
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = fmaf(s[r], c_log2, -mc);
#elif FA_FWD2_PROBE == 3    // timing probe only: no scale/subtract
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = fast_exp2(s[r]);
#else
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = fast_exp2(fmaf(s[r], c_log2, -mc));
#endif
#if FA_FWD2_PROBE == 2 || FA_FWD2_PROBE >= 4   // timing probe only: no row sum
        ts = vadd(ts, s[0]);
#else
        float t0 = vadd(s[0], s[1]), t1 = vadd(s[2], s[3]), t2 = vadd(s[4], s[5]), t3 = vadd(s[6], s[7]);
        t0 = vadd(t0, s[8]); t1 = vadd(t1, s[9]); t2 = vadd(t2, s[10]); t3 = vadd(t3, s[11]);
        t0 = vadd(t0, s[12]); t1 = vadd(t1, s[13]); t2 = vadd(t2, s[14]); t3 = vadd(t3, s[15]);
        ts = vadd(ts, vadd(vadd(t0, t1), vadd(t2, t3)));
#endif
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            u32x4 pk;
#pragma unroll
            for (int e = 0; e < 4; ++e)
#if FA_FWD2_PROBE == 8   // timing probe only: P = raw S bits, no VALU at all
                pk[e] = __float_as_uint(s[8 * s2 + 2 * e]);
#else
                pk[e] = T::pack2(s[8 * s2 + 2 * e], s[8 * s2 + 2 * e + 1]);
#endif
            p[s2] = as_frag<T>(pk);
        }
    };
    // exact path: the tile's row max moves the reference (O and l rescaled), then the whole tile again
    auto exact = [&](f32x16 (&s)[2], float &mc, float &l, f32x16 (&o)[DT], float &ts, frag (&p)[2][2], bool first)
        __attribute__((always_inline)) {
        const float mx = pair_max3(max_tree32(s[0], s[1]));       // -inf: every key masked; NaN-free max
        const float mcx = mx * c_log2;
        if (first) {
            mc = mx == -INFINITY ? 0.f : mcx;
        } else {
            const float mcn = mcx > mc ? mcx : mc;
            const float alpha = fast_exp2(mc - mcn);
            mc = mcn;
            l *= alpha;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        }
        ts = 0.f;
        smh(s[0], mc, ts, p[0]);
        smh(s[1], mc, ts, p[1]);
    };
    // end of a block's tile: fast-path check (wave-uniform), else recompute from the K tile in LDS
    auto finish = [&](f32x16 (&s)[2], const frag (&q)[KS], const char *kb, int kv0, int row, int row0, float &mc,
                      float &l, f32x16 (&o)[DT], float &ts, frag (&p)[2][2]) __attribute__((always_inline)) {
        if (__builtin_amdgcn_ballot_w64(!(ts <= FWD2_SUM_THR))) {
            qk_lds(kb, q, s);
            if (needs_mask(kv0, row0)) mask(s, kv0, row);
            exact(s, mc, l, o, ts, p, false);
        }
        l += ts;
    };
    auto sched_phase = [&](auto nmfma, auto nvalu, auto nds) __attribute__((always_inline)) {
#if FA_FWD2_SCHED
        constexpr int NM = decltype(nmfma)::value, NV = decltype(nvalu)::value, ND = decltype(nds)::value;
#pragma unroll
        for (int i = 0; i < NM; ++i) {
            if (ND) __builtin_amdgcn_sched_group_barrier(0x100, (ND + NM - 1) / NM, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x402, (NV + NM - 1) / NM, 0);
        }
#endif
    };
    using I0 = std::integral_constant<int, 0>;
    constexpr int NM_QK = 2 * KS, NM_PV = 4 * DT;
    using IQK = std::integral_constant<int, NM_QK>;
    using IPV = std::integral_constant<int, NM_PV>;
    using IV = std::integral_constant<int, 56>;
    using IKR = std::integral_constant<int, 2 * KS>;
    using IVR = std::integral_constant<int, 8 * DT>;

    f32x16 oa[DT], ob[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) oa[dt][r] = ob[dt][r] = 0.f;
    float la = 0.f, lb = 0.f, mca = 0.f, mcb = 0.f, tsa = 0.f, tsb = 0.f;
    f32x16 sa[2], sb[2];
    frag pa[2][2], pb[2][2];

    if (nt > 0) {
        // ---- tile 0: exact softmax (sets each row's reference), then the pipeline takes over
        static_for<0, C::PF>([&](auto t) {
            if (t < nt) dma(t, t);
        });
        wait_next(-1);
        __syncthreads();
        if (C::PF < nt) dma(C::PF, C::PF);
        {
            frag kf[2][KS];
            read_k(smem, kf);
            qk(kf, qa, sa);
            qk(kf, qbf, sb);
        }
        if (needs_mask(0, qw)) mask(sa, 0, rowA);
        exact(sa, mca, la, oa, tsa, pa, true);
        la += tsa;
        if (needs_mask(0, qw + 32)) mask(sb, 0, rowB);
        {
            const float mx = pair_max3(max_tree32(sb[0], sb[1]));
            mcb = mx == -INFINITY ? 0.f : mx * c_log2;
        }
        tsb = 0.f;
        smh(sb[0], mcb, tsb, pb[0]);
        pv(smem + C::SLOTS * C::TILE_BYTES, pa, oa);
        wait_next(0);
        __syncthreads();

        // ---- steady state: tile j in slot j % SLOTS (ring unrolled so slot bases are immediates)
        auto step = [&](auto slot_tag, int j) __attribute__((always_inline)) {
            constexpr int CUR = decltype(slot_tag)::value;
            constexpr int PREV = (CUR + C::SLOTS - 1) % C::SLOTS, FILL = (CUR + C::PF) % C::SLOTS;
            const char *kcur = smem + CUR * C::TILE_BYTES;
            const char *vcur = smem + (C::SLOTS + CUR) * C::TILE_BYTES;
            const char *kprev = smem + PREV * C::TILE_BYTES;
            const char *vprev = smem + (C::SLOTS + PREV) * C::TILE_BYTES;
            const int kv0 = j * C::BN;
#if FA_FWD2_PROBE != 7   // probe 7: no steady-state DMA
            if (j + C::PF < nt) dma(j + C::PF, FILL);
#endif
#if FA_FWD2_KREUSE
            frag kf[2][KS];
            read_k(kcur, kf);
#endif
            // phase 1: S_A(j) | softmax B(j-1) keys 32..63
#if FA_FWD2_KREUSE
            qk(kf, qa, sa);
#else
            qk_lds(kcur, qa, sa);
#endif
            smh(sb[1], mcb, tsb, pb[1]);
            sched_phase(IQK(), IV(), IKR());
            __builtin_amdgcn_sched_barrier(0);
            finish(sb, qbf, kprev, kv0 - C::BN, rowB, qw + 32, mcb, lb, ob, tsb, pb);
            if (needs_mask(kv0, qw)) mask(sa, kv0, rowA);
            __builtin_amdgcn_sched_barrier(0);
            // phase 2: O_B += V(j-1) P_B(j-1) | softmax A(j) keys 0..31
            pv(vprev, pb, ob);
            tsa = 0.f;
            smh(sa[0], mca, tsa, pa[0]);
            sched_phase(IPV(), IV(), IVR());
            __builtin_amdgcn_sched_barrier(0);
            // phase 3: S_B(j) | softmax A(j) keys 32..63
#if FA_FWD2_KREUSE
            qk(kf, qbf, sb);
#else
            qk_lds(kcur, qbf, sb);
#endif
            smh(sa[1], mca, tsa, pa[1]);
            sched_phase(IQK(), IV(), std::integral_constant<int, FA_FWD2_KREUSE ? 0 : 2 * KS>());
            __builtin_amdgcn_sched_barrier(0);
            finish(sa, qa, kcur, kv0, rowA, qw, mca, la, oa, tsa, pa);
            if (needs_mask(kv0, qw + 32)) mask(sb, kv0, rowB);
            __builtin_amdgcn_sched_barrier(0);
            // phase 4: O_A += V(j) P_A(j) | softmax B(j) keys 0..31
            pv(vcur, pa, oa);
            tsb = 0.f;
            smh(sb[0], mcb, tsb, pb[0]);
            sched_phase(IPV(), IV(), IVR());
            __builtin_amdgcn_sched_barrier(0);
#if FA_FWD2_PROBE != 6 && FA_FWD2_PROBE != 7   // probes 6/7: no per-tile wait + barrier
            wait_next(j);
            __syncthreads();
#endif
        };
        int j = 1;
        for (; j + C::SLOTS - 1 < nt; j += C::SLOTS)
            static_for<0, C::SLOTS>([&](auto k) { step(std::integral_constant<int, (1 + k) % C::SLOTS>(), j + k); });
        static_for<0, C::SLOTS - 1>([&](auto k) {
            if (j < nt) step(std::integral_constant<int, (1 + k) % C::SLOTS>(), j++);
        });

        // ---- drain: softmax B(nt-1) keys 32..63, its check, O_B += V(nt-1) P_B(nt-1)
        auto tail = [&](auto slot_tag) __attribute__((always_inline)) {
            constexpr int LAST = decltype(slot_tag)::value;
            smh(sb[1], mcb, tsb, pb[1]);
            finish(sb, qbf, smem + LAST * C::TILE_BYTES, (nt - 1) * C::BN, rowB, qw + 32, mcb, lb, ob, tsb, pb);
            pv(smem + (C::SLOTS + LAST) * C::TILE_BYTES, pb, ob);
        };
        const int last = (nt - 1) % C::SLOTS;
        static_for<0, C::SLOTS>([&](auto k) {
            if (last == k) tail(k);
        });
    }

    // ---- epilogue: O / l, 16-byte row stores (T21), LSE
    auto store = [&](const f32x16 (&o)[DT], float l, float mc, int row) __attribute__((always_inline)) {
        const float l_tot = pair_sum(l);
        const bool empty = (l_tot == 0.f) || (l_tot != l_tot);
        const float inv = empty ? 1.f : 1.f / l_tot;
        if (row < seqlen_q) {
            uint16_t *op = (uint16_t *)a.o + (int64_t)(q_start + row) * a.o_row_stride + (int64_t)h * a.o_head_stride;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt)
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
            if (hi == 0)
                a.softmax_lse[(int64_t)(b * a.nheads + h) * a.lse_stride + row] =
                    empty ? -INFINITY : mc * LN2 + __logf(l_tot);
        }
    };
    store(oa, la, mca, rowA);
    store(ob, lb, mcb, rowB);
}

}  // namespace fa
