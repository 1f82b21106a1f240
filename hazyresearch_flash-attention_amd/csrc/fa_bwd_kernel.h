// fa_bwd_kernel.h — FlashAttention backward for gfx950 (CDNA4), hand-written HIP.
//
// The reference branch has no native backward (flash_attn_cuda.bwd is called at
// flash_attn/flash_attn_interface.py:31-33 but never bound, fmha_api.cpp:244-247). Its contract
// is rebuilt from that call signature and from autograd of attention_ref
// (tests/test_flash_attn.py:115-159): with P = softmax(scale*QK^T), M the dropout keep mask,
// pk = 1 - p_drop, Pd = P*M/pk, O = Pd V:
//     dV = Pd^T dO,  dZ = dO V^T,  delta = rowsum(dO*O),  dS = P * (dZ*M/pk - delta),
//     dQ = scale * dS K,  dK = scale * dS^T Q.
//
// Structure (MI355X-first, D <= 64; D = 128 is fa_bwd_split_kernel.h): grid = (key blocks of
// 32 NW, H, B); a workgroup = NW = 8 waves, one wave owns 32 keys and keeps its dK^T, dV^T accumulators in registers
// for the whole kernel; its K, V rows (MFMA B operands) stay in registers too, or, in the causal
// kernels, are re-read per query tile from LDS images. It sweeps 32-row query tiles: Q and dO tiles are staged into swizzled LDS
// images that serve both row reads (S = Q K^T, dZ = dO V^T) and transposed reads
// (dV^T += dO^T Pd, dK^T += Q^T dS). Scores are computed with the key on the MFMA lane, so
// P/dS accumulators are already the B operands of dV^T/dK^T. dS crosses LDS once (a [key][query]
// image, double-buffered) for dQ = dS K, computed one query tile later (so a step needs one
// barrier) with 16x16x32 MFMAs, each wave owning whole dQ tiles summed over all the block's keys,
// then added with fp32 atomics into a workspace; a last kernel scales and converts dQ into the
// (possibly strided) output.
#pragma once

#include "fa_common.h"
#include "../../include/fa_hip.h"

namespace fa {

#ifndef FA_BWD_CAUSAL_NW
#define FA_BWD_CAUSAL_NW 8      // waves (32 keys each) per causal backward workgroup (8: C3 0.405 -> 0.366 ms vs 4)
#endif
#ifndef FA_BWD_NONCAUSAL_NW
#define FA_BWD_NONCAUSAL_NW 8
#endif
#ifndef FA_BWD_KV_LDS
#define FA_BWD_KV_LDS 1         // 1 (D <= 64, causal): K/V B operands re-read from LDS every query tile
#endif
#ifndef FA_BWD_RC_ALL
#define FA_BWD_RC_ALL 0         // 1: every lane of the staging half stages the row constants (no lane branch)
#endif
// timing probes (wrong results by design, A/B builds only): 1 = no barrier per
// query tile, 2 = no dQ phase, 3 = no P / dS VALU
#ifndef FA_BWD_PROBE
#define FA_BWD_PROBE 0
#endif
#ifndef FA_BWD_ROT_WALK
#define FA_BWD_ROT_WALK 1   // non-causal: query-tile walk rotated per key block (see qrow)
#endif
#ifndef FA_BWD_HOIST
#define FA_BWD_HOIST 1   // 1: S / dZ operands read ahead of their MFMA chains (D = 64, dense)
#endif
// per instantiation: C3 (causal, dropout) -2 %, the other D = 64 shapes even, D = 32 even to +2 %
constexpr bool bwd_hoist(int D, bool sparse) { return FA_BWD_HOIST && !sparse && D == 64; }
#ifndef FA_BWD_LANE_BASES
#define FA_BWD_LANE_BASES 1     // 1: LDS reads from loop-invariant lane bases + immediates
#endif

// Waves per workgroup (32 keys each). dQ atomic bytes scale with 1/NW, so both use 8 at D <= 64
// (causal: 4-wave blocks balanced the triangle better but were slower once K/V moved to LDS).
template <bool CAUSAL>
struct BwdWaves { static constexpr int value = CAUSAL ? FA_BWD_CAUSAL_NW : FA_BWD_NONCAUSAL_NW; };

template <int D, int NW_ = 8, bool CAUSAL_ = false>
struct BwdCfg {
    static constexpr int NW = NW_;
    static constexpr int NT = 64 * NW;      // threads per workgroup
    static constexpr int BKV = 32 * NW;     // keys per workgroup
    static constexpr int BQ = 32;           // query rows per iteration
    static constexpr int NC = D / 8;
    static constexpr int K_IMG = BKV * D * 2;
    static constexpr int Q_IMG = BQ * D * 2;
    static constexpr int DS_IMG = BKV * BQ * 2;
    static constexpr int OFF_K = 0;
    static constexpr int OFF_Q = OFF_K + K_IMG;          // Q[2]  (double-buffered query tiles)
    static constexpr int OFF_DO = OFF_Q + 2 * Q_IMG;     // dO[2]
    static constexpr int OFF_DS = OFF_DO + 2 * Q_IMG;
    static constexpr int OFF_LSE = OFF_DS + 2 * DS_IMG;  // dS[2] (dQ runs one tile behind); lse[2][BQ]
    static constexpr int OFF_DELTA = OFF_LSE + 2 * BQ * 4;
    static constexpr int OFF_QLIVE = OFF_DELTA + 2 * BQ * 4;   // block-sparse: live query tiles, 1 bit each
    static constexpr int QLIVE_WORDS = 16;                      // <= 1024 tiles (32768 rows)
    // KV_LDS: a V image beside the K image; K and V fragments are read from LDS per query tile
    // instead of being held in 32 registers for the whole kernel. The causal kernels (mask and
    // LPT bookkeeping on top) spilled inside the loop without it (C3 backward 0.557 -> 0.398 ms
    // on 4-wave blocks); the non-causal ones fit and lose 2-5 % with it.
    static constexpr bool KV_LDS = FA_BWD_KV_LDS && D <= 64 && CAUSAL_;
    static constexpr int OFF_V = OFF_QLIVE + QLIVE_WORDS * 8;
    static constexpr int LDS_BYTES = OFF_V + (KV_LDS ? K_IMG : 0);
};

// byte offset in the dS^T image ([key][query], 64-B rows) of query column q (multiple of 4) of
// key row r. The 8-B slot is XOR-ed with (r>>1)&7 so that both the ds_write_b64 of a 16-lane
// group (16 consecutive rows, one column) and the dQ transposed reads (two 4-row blocks 8 rows
// apart per half-wave) touch every bank once.
__device__ __forceinline__ int ds_off(int r, int q) { return r * 64 + ((q * 2) ^ (((r >> 1) & 7) << 3)); }

// delta = rowsum(dO * O) (softmax_d), and zero the fp32 dQ accumulator (if any). CPR threads per
// row (one 16-B chunk each; CPR = head_dim / 8 rounded up to 4, 8 or 16, so no lane idles at D = 32
// or 64), 256 / CPR rows per 256-thread block, shuffle reduction over the CPR lanes.
template <typename T, int CPR>
__global__ __launch_bounds__(256) void fa_bwd_dot_kernel(const FaBwdArgs a) {
    const int b = blockIdx.z, h = blockIdx.y;
    const int q_start = a.cu_seqlens_q[b];
    const int seqlen_q = a.cu_seqlens_q[b + 1] - q_start;
    const int row = blockIdx.x * (256 / CPR) + (threadIdx.x / CPR);
    const int c = threadIdx.x % CPR;
    const bool ok = row < seqlen_q && c * 8 < a.head_dim;
    float sum = 0.f;
    if (ok) {
        const uint16_t *dop = (const uint16_t *)a.dout + (int64_t)(q_start + row) * a.do_row_stride +
                              (int64_t)h * a.do_head_stride + c * 8;
        const uint16_t *op = (const uint16_t *)a.out + (int64_t)(q_start + row) * a.o_row_stride +
                             (int64_t)h * a.o_head_stride + c * 8;
        const u32x4 x = gload128(dop), y = gload128(op);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sum += T::to_float(x[e] & 0xFFFF) * T::to_float(y[e] & 0xFFFF);
            sum += T::to_float(x[e] >> 16) * T::to_float(y[e] >> 16);
        }
        if (a.dq_accum) {   // NULL when dq is written directly (bwd_dq_direct)
            float *acc = a.dq_accum + ((int64_t)(q_start + row) * a.nheads + h) * a.head_dim + c * 8;
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            *reinterpret_cast<f32x4 *>(acc) = z;
            *reinterpret_cast<f32x4 *>(acc + 4) = z;
        }
    }
#pragma unroll
    for (int w = CPR / 2; w >= 1; w >>= 1) sum += __shfl_xor(sum, w, CPR);
    if (c == 0 && row < seqlen_q) a.softmax_d[(int64_t)(b * a.nheads + h) * a.lse_stride + row] = sum;
}

// dq = scale * dq_accum, converted to 16-bit into the (possibly strided) dq.
template <typename T>
__global__ __launch_bounds__(256) void fa_bwd_dq_convert_kernel(const FaBwdArgs a) {
    const int64_t nchunk_row = a.head_dim / 8;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t total = (int64_t)a.total_q * a.nheads * nchunk_row;
    if (idx >= total) return;
    const int64_t c = idx % nchunk_row;
    const int64_t rh = idx / nchunk_row;
    const int64_t h = rh % a.nheads;
    const int64_t row = rh / a.nheads;
    const float *src = a.dq_accum + (row * a.nheads + h) * a.head_dim + c * 8;
    f32x4 x0 = *reinterpret_cast<const f32x4 *>(src);
    f32x4 x1 = *reinterpret_cast<const f32x4 *>(src + 4);
    const float s = a.softmax_scale;
    u32x4 w = {T::pack2(x0[0] * s, x0[1] * s), T::pack2(x0[2] * s, x0[3] * s),
               T::pack2(x1[0] * s, x1[1] * s), T::pack2(x1[2] * s, x1[3] * s)};
    gstore128((uint16_t *)a.dq + row * a.dq_row_stride + h * a.dq_head_stride + c * 8, w);
}

// two waves per SIMD: one 8-wave workgroup per CU, up to 256 registers per wave
#define FA_BWD_BOUNDS(C) __launch_bounds__((64 * BwdWaves<C>::value), 2)
// DQ = false: no dS image and no dQ (fa_bwd_dq_kernel computes dQ query-major, no atomics)
template <int D, typename T, bool CAUSAL, bool DROPOUT, bool SPARSE = false, bool DQ = true>
__global__ FA_BWD_BOUNDS(CAUSAL) void fa_bwd_kernel(const FaBwdArgs a, const FaBlockMask bm, const int slots) {
    static_assert(D <= 64, "D = 128 takes fa_bwd_split_kernel");
    using C = BwdCfg<D, BwdWaves<CAUSAL>::value, CAUSAL>;
    using S = Swz<D>;
    constexpr float LOG2E = 1.4426950408889634f;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char *kimg = smem + C::OFF_K;
    char *dsimg = smem + C::OFF_DS;
    float *lse_s = (float *)(smem + C::OFF_LSE);
    float *del_s = (float *)(smem + C::OFF_DELTA);

    // causal: key block kb sees queries kb*BKV..end, so block 0 is the heaviest. FA_BWD_XCD:
    // causal in xcd_grouped order (block 0 first within XCD head groups), non-causal head-major
    // per XCD (xcd_contiguous); else all heads' block 0 first, then block 1, ... (global order)
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
    const int l32 = lane & 31;
    const int hi = lane >> 5;
    const int kw = k0 + 32 * wave;
    const int kvrow = kw + l32;
    const int head_dim = a.head_dim;

    const uint16_t *qp = (const uint16_t *)a.q + (int64_t)q_start * a.q_row_stride + (int64_t)h * a.q_head_stride;
    const uint16_t *dop = (const uint16_t *)a.dout + (int64_t)q_start * a.do_row_stride + (int64_t)h * a.do_head_stride;
    const uint16_t *kp = (const uint16_t *)a.k + (int64_t)k_start * a.k_row_stride + (int64_t)h * a.k_head_stride;
    const uint16_t *vp = (const uint16_t *)a.v + (int64_t)k_start * a.v_row_stride + (int64_t)h * a.v_head_stride;
    const float *lse_g = a.softmax_lse + (int64_t)(b * a.nheads + h) * a.lse_stride;
    const float *del_g = a.softmax_d + (int64_t)(b * a.nheads + h) * a.lse_stride;
    float *dqa = a.dq_accum + ((int64_t)q_start * a.nheads + h) * head_dim;
    const int64_t dqa_row = (int64_t)a.nheads * head_dim;

    // ---- stage the K block image (B operand of dQ = dS K, transposed reads)
    for (int idx = tid; idx < C::BKV * C::NC; idx += C::NT) {
        const int row = idx / C::NC, c = idx % C::NC;
        const int kv = k0 + row;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (kv < seqlen_k && c * 8 < head_dim) v = gload128(kp + (int64_t)kv * a.k_row_stride + c * 8);
        lds_write128(kimg, S::off(row, c), v);
        if constexpr (C::KV_LDS) {
            u32x4 w = {0u, 0u, 0u, 0u};
            if (kv < seqlen_k && c * 8 < head_dim) w = gload128(vp + (int64_t)kv * a.v_row_stride + c * 8);
            lds_write128(smem + C::OFF_V, S::off(row, c), w);
        }
    }
    // ---- K, V rows of this lane's key as B operands: B[k=d][col=key]
    typename T::frag kf[D / 16], vf[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
        const int c = 2 * ks + hi;
        u32x4 kv4 = {0u, 0u, 0u, 0u}, vv4 = {0u, 0u, 0u, 0u};
        if (!C::KV_LDS && kvrow < seqlen_k && c * 8 < head_dim) {
            kv4 = gload128(kp + (int64_t)kvrow * a.k_row_stride + c * 8);
            vv4 = gload128(vp + (int64_t)kvrow * a.v_row_stride + c * 8);
        }
        kf[ks] = as_frag<T>(kv4);
        vf[ks] = as_frag<T>(vv4);
    }

    f32x16 dv[D / 32], dk[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) { dv[dt][r] = 0.f; dk[dt][r] = 0.f; }

    const float c_log2 = a.softmax_scale * LOG2E;
    const float rp = 1.0f / (1.0f - a.p_dropout);
    const uint32_t keep_thr = (uint32_t)floorf((1.0f - a.p_dropout) * 65535.0f);
    const uint32_t seed_lo = (uint32_t)a.rng_seed, seed_hi = (uint32_t)(a.rng_seed >> 32);
    const uint32_t rng_ctr3 = DROPOUT ? (uint32_t)(rng_offset_of(a) >> 2) : 0u;
    const uint32_t bh = (uint32_t)(b * a.nheads + h);

    const int grp = (lane >> 4) & 1;   // 16-lane group within the half (32x32 tr reads)
    const int qq = (lane & 15) >> 2;
    const int pp = lane & 3;
    const int g4 = lane >> 4;          // 16-lane group index 0..3 (16x16x32 operands)

    // Loop-invariant LDS lane bases. The D <= 64 swizzles depend on row bits 1..3 (Swz::x, ds_off)
    // only, so a row offset of 16 or 32 is a plain byte offset that folds into the instruction's
    // immediate; written this way the compiler keeps a handful of base registers instead of one
    // computed address per read (which it rematerialized inside the loop under register pressure).
    static_assert(D <= 64, "row offsets of 16 / 32 are additive for the D <= 64 swizzles");
    // (D = 32 keeps the per-read expressions: its translation unit's iterative-ILP scheduler
    // crashes hipcc 7.2 on the lane-base form)
    constexpr bool LB = FA_BWD_LANE_BASES && D == 64;
    // (the dropout kernels, at the 256-register limit with the Philox state, recompute the row-read
    // addresses instead of holding four more registers)
    int qd_base[D / 16];                                   // Q / dO / K / V row reads, k-step ks
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) qd_base[ks] = S::off(l32, 2 * ks + hi);
    auto qd_off = [&](int ks) __attribute__((always_inline)) -> int {
        return (DROPOUT || !LB) ? S::off(l32, 2 * ks + hi) : qd_base[ks];
    };
    int tr_base[2][D / 32];                                // dO^T / Q^T reads: [row +8][d-block]
#pragma unroll
    for (int h8 = 0; h8 < 2; ++h8)
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) tr_base[h8][dt] = S::off8(4 * hi + qq + 8 * h8, 32 * dt + 16 * grp + 4 * pp);

    const int q_begin = CAUSAL ? k0 : 0;   // rows q < k0 see no key of this block
    const int nqt = seqlen_q > q_begin ? (seqlen_q - q_begin + C::BQ - 1) / C::BQ : 0;
    // Non-causal dense kernels walk the query tiles from a per-key-block offset (tile (t + rot) % nqt
    // at step t): the key blocks of one head run at the same time on one XCD, and walking in lockstep
    // from tile 0 they added their dQ partials into the same rows at the same moment (same-address
    // atomics serialise in the L2). Causal blocks start at their own diagonal already.
    constexpr bool ROT = FA_BWD_ROT_WALK && !CAUSAL && !SPARSE && DQ;
    const int rot = ROT && nqt > 0 ? (int)(((int64_t)(k0 / C::BKV) * nqt) / ((seqlen_k + C::BKV - 1) / C::BKV)) % nqt : 0;
    auto qrow = [&](int t) __attribute__((always_inline)) -> int {
        if constexpr (!ROT) {
            return q_begin + t * C::BQ;
        } else {
            int u = t + rot;
            u -= u >= nqt ? nqt : 0;
            return q_begin + u * C::BQ;
        }
    };

    // ---- query-tile staging (T14): a tile is loaded into registers two steps before its use and
    // written to its LDS image one step before. The two halves of the workgroup take turns: half
    // g = tid / (NT/2) stages the tiles of step parity g (thread l of the half: the Q and dO
    // chunk l, and for l < BQ the lse and delta of row l), so each thread holds one tile's
    // registers, and the wait at a tile's LDS write no longer covers the dQ atomics of the step
    // that issued its loads. Loads are buffer loads (lane offset + scalar tile offset; the
    // descriptors end at row seqlen_q, so rows past it read as zeros).
    constexpr int CH = C::BQ * C::NC;
    constexpr int HALF = C::NT / 2;
    static_assert(CH <= HALF && HALF % 64 == 0, "one Q and one dO chunk per thread of a half");
    const int stg_half = tid >= HALF;             // wave-uniform
    const int sl = tid - HALF * stg_half;
    const int crow_ = sl / C::NC, ccol = sl % C::NC;
    const bool chunk_ok = sl < CH && ccol * 8 < head_dim;
    // every lane of a half takes part in the row-constant staging (row sl % BQ: the 8 lanes of a row
    // load and store the same values), so no lane-divergent branch wraps it
    const int crow_c = FA_BWD_RC_ALL ? sl % C::BQ : sl;
    const bool rc_lane = FA_BWD_RC_ALL || sl < C::BQ;   // lanes that stage the row constants
    u32x4 qst = {0u, 0u, 0u, 0u}, dst = {0u, 0u, 0u, 0u};
    float lse_st = 0.f, del_st = 0.f;
    const auto q_rs = make_rsrc_n(qp, seqlen_q * (int)a.q_row_stride * 2);
    const auto do_rs = make_rsrc_n(dop, seqlen_q * (int)a.do_row_stride * 2);
    const int qld_off = chunk_ok ? (crow_ * (int)a.q_row_stride + ccol * 8) * 2 : OOB;
    const int dold_off = chunk_ok ? (crow_ * (int)a.do_row_stride + ccol * 8) * 2 : OOB;
    const int st_off = S::off(crow_, ccol);
    const int cb = k0 >> 8;
    auto row_live = [&](int r) __attribute__((always_inline)) -> bool {
        return r < bm.rows && bm.mask[(int64_t)r * bm.row_stride + cb] != 0;
    };
    auto gload_qtile = [&](int q0n) __attribute__((always_inline)) {
        if (CH == HALF || sl < CH) {
            qst = bload128s(q_rs, qld_off, q0n * (int)a.q_row_stride * 2);
            dst = bload128s(do_rs, dold_off, q0n * (int)a.do_row_stride * 2);
        }
        // row constants of a clamped row (rows past seqlen_q get lse = +inf at the LDS write, so
        // their P = exp2(s c - inf) = 0 with no per-element mask)
        if (rc_lane) {
            const int qc = min(q0n + crow_c, seqlen_q - 1);
            lse_st = lse_g[qc];
            del_st = del_g[qc];
        }
    };
    auto lds_store_qtile = [&](int buf, int q0n) __attribute__((always_inline)) {
        if (CH == HALF || sl < CH) {
            lds_write128(smem + C::OFF_Q + buf * C::Q_IMG, st_off, qst);
            lds_write128(smem + C::OFF_DO + buf * C::Q_IMG, st_off, dst);
        }
        // one lane offset for both rows' constants (the image offsets fold into the instruction).
        // Rows past seqlen_q and (block-sparse) dead 16-row halves get lse = +inf: P = 0 there.
        if (rc_lane) {
            const int qr = q0n + crow_c;
            bool dead = qr >= seqlen_q;
            if constexpr (SPARSE) dead = dead || !row_live(qr >> 4);
            lds_write32(smem + C::OFF_LSE + buf * C::BQ * 4, 4 * crow_c, dead ? INFINITY : lse_st * LOG2E);
            lds_write32(smem + C::OFF_DELTA + buf * C::BQ * 4, 4 * crow_c, -del_st);   // -delta
        }
    };
    // ---- block sparsity (fa_bwd_block): this workgroup's keys lie in one 256-key column block
    // cb; a 32-row query tile is live when either of its 16-row blocks is 1 in column cb. The
    // live tiles are kept as a bit set in LDS and walked in order; dead tiles are never loaded.
    uint64_t *qlive = (uint64_t *)(smem + C::OFF_QLIVE);
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
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    const int t_first = SPARSE ? next_qt(-1) : 0;
    const int t_second = t_first < nqt ? next_qt(t_first) : nqt;
    if (t_first < nqt) {
        if (stg_half == 0) {
            gload_qtile(qrow(t_first));
            lds_store_qtile(0, qrow(t_first));
        } else if (t_second < nqt) {
            gload_qtile(qrow(t_second));
        }
    }
    __syncthreads();

    // ---- dQ[q][d] += dS[q][key] K[key][d] over the BKV keys (16x16x32 MFMAs) of the query tile
    // at row qd, from the dS image dsr; the 2*(D/16) output tiles of 16 query rows x 16 columns
    // are dealt round-robin to the waves, each summing over every key of the block, so one fp32
    // atomic per element per block. store_buf >= 0: the waves holding a dQ tile write the staged
    // query tile into LDS buffer store_buf before their atomics.
    auto dq_phase = [&](const char *dsr, int qd, int store_buf, int store_q0) __attribute__((always_inline)) {
#pragma unroll
        for (int t0 = 0; t0 < 2 * (D / 16); t0 += C::NW) {
            const int t = t0 + wave;
            if (t < 2 * (D / 16)) {
                const int qh = t & 1;
                const int dbase = 16 * (t >> 1);
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                // rows r0 = 32 ks + 8 g4 + qq (+4): key step ks is an immediate offset (32 rows)
                const int ds0 = ds_off(8 * g4 + qq, 16 * qh + 4 * pp), ds1 = ds_off(8 * g4 + qq + 4, 16 * qh + 4 * pp);
                const int kb0 = S::off8(8 * g4 + qq, dbase + 4 * pp), kb1 = S::off8(8 * g4 + qq + 4, dbase + 4 * pp);
                auto dq_operands = [&](int ks, u32x4 &av, u32x4 &bv) __attribute__((always_inline)) {
                    const int r0 = 32 * ks + 8 * g4 + qq;
                    u32x2 a0 = lds_read_tr(dsr, LB ? ds0 + 32 * ks * 64 : ds_off(r0, 16 * qh + 4 * pp));
                    u32x2 a1 = lds_read_tr(dsr, LB ? ds1 + 32 * ks * 64 : ds_off(r0 + 4, 16 * qh + 4 * pp));
                    av = u32x4{a0[0], a0[1], a1[0], a1[1]};
                    u32x2 b0 = lds_read_tr(kimg, LB ? kb0 + 32 * ks * S::ROW_BYTES : S::off8(r0, dbase + 4 * pp));
                    u32x2 b1 = lds_read_tr(kimg, LB ? kb1 + 32 * ks * S::ROW_BYTES : S::off8(r0 + 4, dbase + 4 * pp));
                    bv = u32x4{b0[0], b0[1], b1[0], b1[1]};
                };
                // operands of key step ks+1 are read before the MFMA of step ks
                u32x4 av, bv, avn, bvn;
                dq_operands(0, av, bv);
#pragma unroll
                for (int ks = 0; ks < C::BKV / 32; ++ks) {
                    if (ks + 1 < C::BKV / 32) dq_operands(ks + 1, avn, bvn);
                    acc = T::mfma16(as_frag<T>(av), as_frag<T>(bv), acc);
                    av = avn;
                    bv = bvn;
                }
                const int d = dbase + (lane & 15);
                // the staged query tile goes to LDS first: its vmcnt wait then covers only loads
                // (vmcnt retires in issue order), and these atomics have a whole tile of compute
                // before the next wait
                if (t0 == 0 && store_buf >= 0) lds_store_qtile(store_buf, store_q0);
                if (qd + C::BQ <= seqlen_q && head_dim == D) {
                    // full tile (wave-uniform test): the four atomics without per-lane guards
                    float *base = dqa + (int64_t)(qd + 16 * qh + 4 * g4) * dqa_row + d;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
#ifdef FA_BWD_PROBE_NOATOMIC   // timing probe only (tools/ab_libs.sh builds): no dQ atomics, wrong dQ
                        if (acc[i] == 1.2345e-30f) base[i * dqa_row] = acc[i];
#else
                        atomicAdd(base + i * dqa_row, acc[i]);
#endif
                    }
                } else if (d < head_dim) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int q = qd + 16 * qh + 4 * g4 + i;
                        if (q < seqlen_q) atomicAdd(dqa + (int64_t)q * dqa_row + d, acc[i]);
                    }
                }
            }
        }
    };

    // step of tile `it` (LDS buffer BUF); itn, itnn: the next two live tiles (nqt if none);
    // itp: the previous live tile (-1 if none), whose dQ this step computes
    auto qstep = [&](auto par_tag, int itp, int it, int itn, int itnn) __attribute__((always_inline)) {
        constexpr int BUF = decltype(par_tag)::value;
        // half BUF loads tile itnn now; half 1-BUF writes tile itn (loaded a step ago) to LDS
        const bool my_load = stg_half == BUF, my_store = stg_half != BUF;
        char *qimg = smem + C::OFF_Q + BUF * C::Q_IMG;
        char *doimg = smem + C::OFF_DO + BUF * C::Q_IMG;
        const float *lse_b = lse_s + BUF * C::BQ;
        const float *del_b = del_s + BUF * C::BQ;
        const int q0 = qrow(it);
        char *dsw = dsimg + BUF * C::DS_IMG;
        if (my_load && itnn < nqt) gload_qtile(qrow(itnn));
        // (block sparsity: a dead 16-row half of a live tile has lse = +inf in its row constants)
        const bool active = !CAUSAL || (q0 + C::BQ - 1 >= kw);
        u32x4 pk[2] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}}, sk[2] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
        // ---- dV^T += dO^T Pd ; dK^T += Q^T dS  (A operands by transposed reads). Causal kernels
        // without dropout run it outside the `active` branch (a wave above the diagonal adds
        // zeros): with the accumulator updates inside it, the two paths' dV/dK registers were joined
        // by 64 register moves per step (causal D=64 0.270 -> 0.245 ms); with dropout the branch
        // version measured faster (0.276 vs 0.286 ms).
        constexpr bool DVDK_ALWAYS = CAUSAL && !DROPOUT;
        auto dvdk = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int sg = 0; sg < 2; ++sg) {
                const int ro = 16 * sg * S::ROW_BYTES;    // rows 16 sg + 4 hi + qq (+8)
#pragma unroll
                for (int dt = 0; dt < D / 32; ++dt) {
                    const int rb = 16 * sg + 4 * hi + qq, col = 32 * dt + 16 * grp + 4 * pp;
                    const int o0 = LB ? tr_base[0][dt] + ro : S::off8(rb, col);
                    const int o1 = LB ? tr_base[1][dt] + ro : S::off8(rb + 8, col);
                    u32x2 a0 = lds_read_tr(doimg, o0);
                    u32x2 a1 = lds_read_tr(doimg, o1);
                    u32x4 av = {a0[0], a0[1], a1[0], a1[1]};
                    dv[dt] = T::mfma32(as_frag<T>(av), as_frag<T>(pk[sg]), dv[dt]);
                    u32x2 b0 = lds_read_tr(qimg, o0);
                    u32x2 b1 = lds_read_tr(qimg, o1);
                    u32x4 bv = {b0[0], b0[1], b1[0], b1[1]};
                    dk[dt] = T::mfma32(as_frag<T>(bv), as_frag<T>(sk[sg]), dk[dt]);
                }
            }
        };
        if (active) {
            // ---- S = Q K^T and dZ = dO V^T : lane = key, registers = query rows crow(r,hi)
            // without dropout dZ's accumulator starts at -delta of its row (the image holds -delta) (16-B LDS reads straight
            // into the accumulator registers), so dS = P (dZ - delta) is one multiply per element
            f32x16 sacc, zacc;
#pragma unroll
            for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
            constexpr bool SEED_DZ = !DROPOUT;
            if constexpr (!SEED_DZ) {
#pragma unroll
                for (int r = 0; r < 16; ++r) zacc[r] = 0.f;
            } else {
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 del4 = *reinterpret_cast<const f32x4 *>(del_b + 8 * g + 4 * hi);
#pragma unroll
                    for (int e = 0; e < 4; ++e) zacc[4 * g + e] = del4[e];
                }
            }
            if constexpr (bwd_hoist(D, SPARSE)) {
                // every k-step's operands read before the chains, in k-step order (the compiler
                // otherwise kept one read in flight per MFMA: one exposed LDS latency each)
                u32x4 qa[D / 16], da[D / 16], ka[D / 16], va[D / 16];
#pragma unroll
                for (int ks = 0; ks < D / 16; ++ks) {
                    qa[ks] = lds_read128(qimg, qd_off(ks));
                    da[ks] = lds_read128(doimg, qd_off(ks));
                    if constexpr (C::KV_LDS) {
                        const int ko = qd_off(ks) + 32 * wave * S::ROW_BYTES;
                        ka[ks] = lds_read128(kimg, ko);
                        va[ks] = lds_read128(smem + C::OFF_V, ko);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
                for (int ks = 0; ks < D / 16; ++ks) {
                    if constexpr (C::KV_LDS) {
                        sacc = T::mfma32(as_frag<T>(qa[ks]), as_frag<T>(ka[ks]), sacc);
                        zacc = T::mfma32(as_frag<T>(da[ks]), as_frag<T>(va[ks]), zacc);
                    } else {
                        sacc = T::mfma32(as_frag<T>(qa[ks]), kf[ks], sacc);
                        zacc = T::mfma32(as_frag<T>(da[ks]), vf[ks], zacc);
                    }
                }
            } else {
#pragma unroll
                for (int ks = 0; ks < D / 16; ++ks) {
                    u32x4 qa = lds_read128(qimg, qd_off(ks));
                    u32x4 da = lds_read128(doimg, qd_off(ks));
                    if constexpr (C::KV_LDS) {
                        const int ko = qd_off(ks) + 32 * wave * S::ROW_BYTES;   // row 32 wave + l32
                        sacc = T::mfma32(as_frag<T>(qa), as_frag<T>(lds_read128(kimg, ko)), sacc);
                        zacc = T::mfma32(as_frag<T>(da), as_frag<T>(lds_read128(smem + C::OFF_V, ko)), zacc);
                    } else {
                        sacc = T::mfma32(as_frag<T>(qa), kf[ks], sacc);
                        zacc = T::mfma32(as_frag<T>(da), vf[ks], zacc);
                    }
                }
            }
            // Rows past seqlen_q and dead (block-sparse) rows carry lse = +inf in the staged row
            // constants, so their P is 0 with no test here; only the last key block (keys past
            // seqlen_k) and the causal diagonal tiles take the per-element mask, as a separate copy
            // of the loop behind one wave-uniform branch (no select on every tile).
            const bool need_mask = (k0 + C::BKV > seqlen_k) || (CAUSAL && q0 < kw + 31);
            u32x4 rw[2];
            if (DROPOUT) {
#pragma unroll
                for (int sg = 0; sg < 2; ++sg) {
                    const uint32_t g = ((uint32_t)(q0 >> 5) << 2) | (sg << 1) | hi;
                    rw[sg] = philox7(g, (uint32_t)kvrow, bh, rng_ctr3, seed_lo, seed_hi);
                }
            }
            // P and dS in place: sacc -> Pd (dropped, scaled P), zacc -> dS. Row constants for
            // rows crow(4g+e, hi) = 8g + 4hi + e are one 16-B LDS read per group of 4 registers.
            auto pds = [&](auto masked_tag) __attribute__((always_inline)) {
                constexpr bool MASKED = decltype(masked_tag)::value;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 lse4 = *reinterpret_cast<const f32x4 *>(lse_b + 8 * g + 4 * hi);
                    const f32x4 del4 = *reinterpret_cast<const f32x4 *>(del_b + 8 * g + 4 * hi);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int r = 4 * g + e;
                        float p = fast_exp2(fmaf(sacc[r], c_log2, -lse4[e]));
                        if constexpr (MASKED) p = mask_min(p, kvrow >= seqlen_k || (CAUSAL && kvrow > q0 + crow(r, hi)));
                        float dpv = zacc[r];
                        float pdv = p;
                        if (DROPOUT) {
                            const int slot = (r & 3) | (((r >> 2) & 1) << 2);
                            const uint32_t word = rw[r >> 3][slot >> 1];
                            const uint32_t rnd = (slot & 1) ? (word >> 16) : (word & 0xFFFFu);
                            // one select: the kept scale 1/(1-p) or 0, then two multiplies
                            const float rpk = rnd <= keep_thr ? rp : 0.f;
                            dpv = dpv * rpk;
                            pdv = p * rpk;
                        }
                        sacc[r] = pdv;
                        zacc[r] = SEED_DZ ? p * dpv : p * (dpv + del4[e]);
                    }
                }
            };
            if (FA_BWD_PROBE == 3)
                ;
            else if (__builtin_amdgcn_readfirstlane((int)need_mask))
                pds(std::true_type{});
            else
                pds(std::false_type{});
            // packed 16-bit Pd and dS: the B operands of dV^T / dK^T and the dS image words
#pragma unroll
            for (int sg = 0; sg < 2; ++sg)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    pk[sg][e] = T::pack2(sacc[8 * sg + 2 * e], sacc[8 * sg + 2 * e + 1]);
                    sk[sg][e] = T::pack2(zacc[8 * sg + 2 * e], zacc[8 * sg + 2 * e + 1]);
                }
            if constexpr (!DVDK_ALWAYS) dvdk();
        }
        if constexpr (DVDK_ALWAYS) dvdk();
        // ---- dS^T image: row = key (32*wave + l32), columns = query rows 8g + 4hi .. +3
        if constexpr (DQ) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                u32x2 w = {sk[g >> 1][2 * (g & 1)], sk[g >> 1][2 * (g & 1) + 1]};
                lds_write64(dsw, ds_off(32 * wave + l32, 8 * g + 4 * hi), w);
            }
        }
        const int store_buf = my_store && itn < nqt ? 1 - BUF : -1;
        bool stored = false;
        if constexpr (DQ) {
            // dQ runs one tile behind: the previous tile's dS image is complete since the barrier
            // that closed the previous step, so each step needs a single barrier (the dS image of
            // this tile is read in the next step, the other buffer)
            if (itp >= 0 && FA_BWD_PROBE != 2) {
                dq_phase(dsimg + (1 - BUF) * C::DS_IMG, qrow(itp), store_buf, qrow(itn));
                stored = true;
            }
        }
        // waves without a dQ tile (or steps without a dQ phase) store the staged tile here
        if (store_buf >= 0 && !(stored && wave < 2 * (D / 16))) lds_store_qtile(store_buf, qrow(itn));
        if (FA_BWD_PROBE != 1) __syncthreads();
    };
    int ilast = -1, blast = 0;   // last tile and its buffer (its dQ runs after the walk)
    if constexpr (SPARSE) {
        int itp = -1, it = t_first, itn = t_second;
        while (it < nqt) {
            int itnn = itn < nqt ? next_qt(itn) : nqt;
            qstep(I0(), itp, it, itn, itnn);
            ilast = it; blast = 0;
            itp = it;
            it = itn;
            itn = itnn;
            if (it >= nqt) break;
            itnn = itn < nqt ? next_qt(itn) : nqt;
            qstep(I1(), itp, it, itn, itnn);
            ilast = it; blast = 1;
            itp = it;
            it = itn;
            itn = itnn;
        }
    } else {
        for (int it = 0; it < nqt; it += 2) {
            qstep(I0(), it - 1, it, it + 1, it + 2);
            if (it + 1 < nqt) qstep(I1(), it, it + 1, it + 2, it + 3);
        }
        ilast = nqt - 1;
        blast = (nqt - 1) & 1;
    }
    if constexpr (DQ) {
        // dQ of the last tile (its dS image is complete since the last step's closing barrier)
        if (ilast >= 0) {
            if (blast)
                dq_phase(dsimg + C::DS_IMG, qrow(ilast), -1, 0);
            else
                dq_phase(dsimg, qrow(ilast), -1, 0);
        }
    }

    // ---- epilogue: dV, dK (scaled) rows of this lane's key
    if (kvrow < seqlen_k) {
        uint16_t *dvp = (uint16_t *)a.dv + (int64_t)(k_start + kvrow) * a.dv_row_stride + (int64_t)h * a.dv_head_stride;
        uint16_t *dkp = (uint16_t *)a.dk + (int64_t)(k_start + kvrow) * a.dk_row_stride + (int64_t)h * a.dk_head_stride;
        const float sc = a.softmax_scale;
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = 32 * dt + 8 * g + 4 * hi;
                if (d < head_dim) {
                    u32x2 wv = {T::pack2(dv[dt][4 * g + 0], dv[dt][4 * g + 1]),
                                T::pack2(dv[dt][4 * g + 2], dv[dt][4 * g + 3])};
                    u32x2 wk = {T::pack2(dk[dt][4 * g + 0] * sc, dk[dt][4 * g + 1] * sc),
                                T::pack2(dk[dt][4 * g + 2] * sc, dk[dt][4 * g + 3] * sc)};
                    gstore64(dvp + d, wv);
                    gstore64(dkp + d, wk);
                }
            }
    }
}

// Attention probabilities for return_attn_probs (test-only path, reference S_dmask
// semantics of csrc/flash_attn/src/fmha/softmax.h:256-296 with this build's own layout):
// s[b][h][row][col] = softmax(scale*QK^T)[row][col], negated where dropout dropped it,
// 0 where masked or padded. Row-major (B, H, s_rows, s_cols).
template <typename T, bool CAUSAL, bool DROPOUT>
__global__ __launch_bounds__(256) void fa_probs_kernel(const FaFwdArgs a, const FaBlockMask bm) {
    // block = 32 query rows x 64 keys; thread = one key column x 8 rows (one Philox call)
    constexpr float LOG2E = 1.4426950408889634f;
    __shared__ float qs[32][129];
    __shared__ float ks[64][129];
    const int b = blockIdx.z, h = blockIdx.y;
    const int q0 = blockIdx.x * 32;
    const int q_start = a.cu_seqlens_q[b];
    const int seqlen_q = a.cu_seqlens_q[b + 1] - q_start;
    const int k_start = a.cu_seqlens_k[b];
    const int seqlen_k = a.cu_seqlens_k[b + 1] - k_start;
    const int tid = threadIdx.x;
    const int D = a.head_dim;
    const uint16_t *qp = (const uint16_t *)a.q + (int64_t)q_start * a.q_row_stride + (int64_t)h * a.q_head_stride;
    const uint16_t *kp = (const uint16_t *)a.k + (int64_t)k_start * a.k_row_stride + (int64_t)h * a.k_head_stride;
    const float *lse_g = a.softmax_lse + (int64_t)(b * a.nheads + h) * a.lse_stride;
    uint16_t *sp = (uint16_t *)a.s_dmask + (int64_t)(b * a.nheads + h) * a.s_rows * a.s_cols;
    const float c_log2 = a.softmax_scale * LOG2E;
    const uint32_t keep_thr = (uint32_t)floorf((1.0f - a.p_dropout) * 65535.0f);
    const uint32_t bh = (uint32_t)(b * a.nheads + h);

    for (int idx = tid; idx < 32 * D; idx += 256) {
        const int r = idx / D, d = idx % D;
        const int q = q0 + r;
        qs[r][d] = q < seqlen_q ? T::to_float(qp[(int64_t)q * a.q_row_stride + d]) : 0.f;
    }
    const int col_l = tid & 63;
    const int sg = (tid >> 6) & 1;
    const int hh = tid >> 7;
    for (int kv0 = 0; kv0 < a.s_cols; kv0 += 64) {
        __syncthreads();
        for (int idx = tid; idx < 64 * D; idx += 256) {
            const int r = idx / D, d = idx % D;
            const int kv = kv0 + r;
            ks[r][d] = kv < seqlen_k ? T::to_float(kp[(int64_t)kv * a.k_row_stride + d]) : 0.f;
        }
        __syncthreads();
        const int col = kv0 + col_l;
        if (col >= a.s_cols) continue;
        u32x4 w = {0u, 0u, 0u, 0u};
        if (DROPOUT) {
            const uint32_t g = ((uint32_t)(q0 >> 5) << 2) | (sg << 1) | hh;
            w = philox7(g, (uint32_t)col, bh, (uint32_t)(rng_offset_of(a) >> 2), (uint32_t)a.rng_seed,
                        (uint32_t)(a.rng_seed >> 32));
        }
        for (int slot = 0; slot < 8; ++slot) {
            const int r = 16 * sg + 4 * hh + (slot & 3) + 8 * (slot >> 2);
            const int q = q0 + r;
            if (q >= a.s_rows) continue;
            float val = 0.f;
            bool valid = q < seqlen_q && col < seqlen_k && !(CAUSAL && col > q);
            if (valid && bm.mask) valid = (q >> 4) < bm.rows && bm.mask[(int64_t)(q >> 4) * bm.row_stride + (col >> 8)] != 0;
            if (valid) {
                float acc = 0.f;
                for (int d = 0; d < D; ++d) acc = fmaf(qs[r][d], ks[col_l][d], acc);
                val = fast_exp2(acc * c_log2 - lse_g[q] * LOG2E);
                if (DROPOUT) {
                    const uint32_t word = w[slot >> 1];
                    const uint32_t rnd = (slot & 1) ? (word >> 16) : (word & 0xFFFFu);
                    if (rnd > keep_thr) val = -val;
                }
            }
            sp[(int64_t)q * a.s_cols + col] = T::from_float(val);
        }
    }
}

}  // namespace fa
