// fa_common.h — shared device helpers for the gfx950 FlashAttention kernels.
//
// Fragment maps used everywhere (cdna_hip_programming.md §3, v_mfma_f32_32x32x16_{bf16,f16}):
//   lane l, r = l & 31, h = l >> 5
//   A operand element j (0..7):  A[row r][k = 8h + j]
//   B operand element j (0..7):  B[k = 8h + j][col r]
//   C/D register i (0..15):      C[row crow(i, h)][col r],  crow(i,h) = (i&3) + 8(i>>2) + 4h
// An accumulator X used as the B operand of k-step s takes registers 8s..8s+7 (converted to
// 16-bit) and represents X rows 16s + 8(j>>2) + 4h + (j&3) — the other operand must supply
// the same k order (what ds_read_b64_tr_b16 delivers below).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace fa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) void lds_void;

// The backward's masking relies on IEEE infinities: rows past seqlen_q and dead block-sparse rows
// carry lse = +inf so that exp2 gives P = 0, and mask_min() is fminf(p, inf) on live elements. A
// finite-math build (-ffast-math, -ffinite-math-only) may fold both and unmask those rows.
#if defined(__FINITE_MATH_ONLY__) && __FINITE_MATH_ONLY__
#error "fa kernels need IEEE inf semantics (lse = +inf row masking, mask_min): build without -ffinite-math-only"
#endif

// Timing probes of the backward kernels (FA_BWD_PROBE, FA_BWD_PROBE_NOATOMIC, FA_BWD_SPLIT_PROBE)
// compute wrong gradients by design. They compile only in an explicit A/B probe build
// (-DFA_AB_PROBE_BUILD, tools only; build.py refuses to write the product library with one set).
#if !defined(FA_AB_PROBE_BUILD)
#if (defined(FA_BWD_PROBE) && FA_BWD_PROBE != 0) || defined(FA_BWD_PROBE_NOATOMIC) || \
    (defined(FA_BWD_SPLIT_PROBE) && FA_BWD_SPLIT_PROBE != 0)
#error "backward timing probe set without -DFA_AB_PROBE_BUILD: such a library computes wrong gradients"
#endif
#endif

// 16-bit element traits: storage is raw 16-bit, MFMA operand type differs by dtype.
struct Bf16 {
    typedef bf16x8 frag;
    static __device__ __forceinline__ uint16_t from_float(float x) {
        __bf16 b = (__bf16)x;  // v_cvt_pk_bf16_f32, RNE, NaN-preserving
        return __builtin_bit_cast(uint16_t, b);
    }
    static __device__ __forceinline__ float to_float(uint16_t x) {
        return __uint_as_float(((uint32_t)x) << 16);
    }
    static __device__ __forceinline__ uint32_t pack2(float a, float b) {
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        bf16x2 v = {(__bf16)a, (__bf16)b};
        return __builtin_bit_cast(uint32_t, v);
    }
    // the two halves of a pack2 word back to fp32 (exact)
    static __device__ __forceinline__ float lo_float(uint32_t w) { return __uint_as_float(w << 16); }
    static __device__ __forceinline__ float hi_float(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
    static __device__ __forceinline__ f32x16 mfma32(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ f32x4 mfma16(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};

struct Fp16 {
    typedef f16x8 frag;
    static __device__ __forceinline__ uint16_t from_float(float x) {
        _Float16 h = (_Float16)x;  // RNE
        return __builtin_bit_cast(uint16_t, h);
    }
    static __device__ __forceinline__ float to_float(uint16_t x) {
        return (float)__builtin_bit_cast(_Float16, x);
    }
    static __device__ __forceinline__ uint32_t pack2(float a, float b) {
        typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
        f16x2 v = {(_Float16)a, (_Float16)b};
        return __builtin_bit_cast(uint32_t, v);
    }
    static __device__ __forceinline__ float lo_float(uint32_t w) { return to_float((uint16_t)(w & 0xFFFFu)); }
    static __device__ __forceinline__ float hi_float(uint32_t w) { return to_float((uint16_t)(w >> 16)); }
    static __device__ __forceinline__ f32x16 mfma32(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ f32x4 mfma16(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
};

template <typename T>
__device__ __forceinline__ typename T::frag as_frag(u32x4 v) {
    return __builtin_bit_cast(typename T::frag, v);
}

__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// p (an exp2 result, >= 0) forced to 0 where `masked`: min(p, masked ? 0 : inf). Written as a
// select of `p` itself, the compiler sank the exp into the unmasked arm and gave every element
// its own divergent branch; the min keeps the exp on both arms, so the mask stays two VALU ops.
// (IEEE inf required: see the finite-math guard at the top of this file)
__device__ __forceinline__ float mask_min(float p, bool masked) { return fminf(p, masked ? 0.f : INFINITY); }

// XCD-aware work order. The dispatcher hands workgroup L (linear id) to XCD L & 7, and each XCD
// takes its share in order of L >> 3; this maps L to a position Lp such that every XCD covers a
// contiguous run of [0, nwg) (bijective for any nwg). Grids ordered head-major in Lp keep the
// blocks of one head on one XCD at about the same time, so the rows they all stream (the
// forward's and the dQ pass's K/V, the key-major backward's Q/dO/lse/delta) come from that XCD's
// L2 instead of eight.
__device__ __forceinline__ int xcd_contiguous(int L, int nwg) {
    const int xcd = L & 7, q8 = nwg >> 3, r8 = nwg & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
}

// Causal grids (blocks of unequal work, rank 0 the heaviest): per XCD, its nbh / 8 heads in groups
// of G, G * nblk ~ the workgroups one XCD runs at once (`slots`), heaviest-first across the group's
// heads, groups one after the other. One group's rows fit one L2 (a head-major order alone left
// C3's few blocks per head unbalanced; a global heaviest-first order spread ~24 heads per XCD at
// C4: 5.5 GB fetched for 0.8 GB of Q/K/V/dO). nbh not a multiple of 8: the global order.
__device__ __forceinline__ void xcd_grouped(int L, int nblk, int nbh, int slots, int &rank, int &bh) {
    if ((nbh & 7) == 0) {
        const int nh = nbh >> 3, x = L & 7, i = L >> 3;
        int G = (slots + nblk - 1) / nblk;
        G = G < 1 ? 1 : (G > nh ? nh : G);
        const int per = G * nblk;
        const int grp = i / per, w = i - grp * per;
        const int gh = nh - grp * G < G ? nh - grp * G : G;
        rank = w / gh;
        bh = x * nh + grp * G + (w - rank * gh);
    } else {
        rank = L / nbh;
        bh = L % nbh;
    }
}

#ifndef FA_BWD_XCD
#define FA_BWD_XCD 1   // 1: backward grids in xcd_contiguous head-major order (0: the round-2 orders)
#endif

// ---------------------------------------------------------------------------------------
// LDS tile image: [rows][D] 16-bit, 16-byte chunks XOR-swizzled so that
//   (a) ds_read_b128 row reads (lane -> row r = l&31, fixed chunk) and
//   (b) ds_read_b64_tr_b16 transposed reads (4 consecutive rows x 32 columns per half-wave)
// are both bank-conflict free (derivation in DESIGN.md §4).
// ---------------------------------------------------------------------------------------
template <int D>
struct Swz {
    static constexpr int NC = D / 8;          // 16-B chunks per row
    static constexpr int ROW_BYTES = D * 2;
    static __device__ __forceinline__ int x(int r) {
        if constexpr (D == 32) {
            return (r >> 2) & 3;
        } else if constexpr (D == 64) {
            int u = (r >> 1) & 7;
            return ((u & 1) << 2) | (u >> 1);
        } else {  // 128
            return ((r & 3) << 2) | ((r >> 2) & 3);
        }
    }
    // byte offset of chunk c of row r
    static __device__ __forceinline__ int off(int r, int c) { return r * ROW_BYTES + ((c ^ x(r)) << 4); }
    // byte offset of the 8-byte half holding columns col..col+3 (col % 4 == 0) of row r
    static __device__ __forceinline__ int off8(int r, int col) {
        return off(r, col >> 3) + ((col >> 2) & 1) * 8;
    }
};

__device__ __forceinline__ u32x4 lds_read128(const char *lds, int byte_off) {
    return *reinterpret_cast<const __attribute__((address_space(3))) u32x4 *>(
        (const __attribute__((address_space(3))) char *)lds + byte_off);
}
__device__ __forceinline__ void lds_write128(char *lds, int byte_off, u32x4 v) {
    *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(
        (__attribute__((address_space(3))) char *)lds + byte_off) = v;
}
__device__ __forceinline__ void lds_write32(char *lds, int byte_off, float v) {
    *reinterpret_cast<__attribute__((address_space(3))) float *>(
        (__attribute__((address_space(3))) char *)lds + byte_off) = v;
}
__device__ __forceinline__ void lds_write64(char *lds, int byte_off, u32x2 v) {
    *reinterpret_cast<__attribute__((address_space(3))) u32x2 *>(
        (__attribute__((address_space(3))) char *)lds + byte_off) = v;
}
// Transposed read: within each 16-lane group, lane 4q+p supplies the address of row q,
// columns 4p..4p+3 of a 4x16 block; lane i of the group receives column i of the 4 rows.
__device__ __forceinline__ u32x2 lds_read_tr(const char *lds, int byte_off) {
    i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) i16x4 *)((__attribute__((address_space(3))) char *)lds + byte_off));
    return __builtin_bit_cast(u32x2, v);
}

// Global 16-byte load / 8-byte store helpers.
__device__ __forceinline__ u32x4 gload128(const void *p) { return *reinterpret_cast<const u32x4 *>(p); }
__device__ __forceinline__ void gstore64(void *p, u32x2 v) { *reinterpret_cast<u32x2 *>(p) = v; }
__device__ __forceinline__ void gstore128(void *p, u32x4 v) { *reinterpret_cast<u32x4 *>(p) = v; }

// Buffer descriptors (T8/T20): 32-bit per-lane offsets against a wave-uniform base, hardware
// bounds check; an offset of OOB reads zeros / drops the store or atomic, so edge handling needs
// no branches (and the compiler can count outstanding memory operations exactly).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_n(const void *base, int num_bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, num_bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 bload128(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
// lane offset + wave-uniform (SGPR) offset: the per-tile advance costs no vector instruction
__device__ __forceinline__ u32x4 bload128s(__amdgpu_buffer_rsrc_t r, int byte_off, int soff) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, soff, 0));
}
constexpr int OOB = (int)0x80000000;  // any offset past num_records reads as zero

// ---- LDS-DMA issued as inline asm (buffer_load_dwordx4 ... lds). Through the builtin, hipcc
// orders every later ds_read_b64_tr_b16 behind an s_waitcnt vmcnt(0) for the in-flight DMA, so a
// tile prefetched at the top of a step is waited for at that step's first V^T read; issued here the
// DMA is invisible to the compiler's counters and the caller waits itself (vmcnt + barrier).
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
// wave-uniform buffer descriptor words (base, stride 0, num_records, raw-buffer flags) in SGPRs
__device__ __forceinline__ i32x4 make_srd(const void *base, int num_bytes) {
    const uint64_t p = (uint64_t)base;
    i32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));
    r[2] = __builtin_amdgcn_readfirstlane(num_bytes);
    r[3] = 0x00020000;
    return r;
}
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)p;
}
// s_waitcnt vmcnt(0) that the compiler's counters see (it then knows its own loads are done too)
__device__ __forceinline__ void vmcnt0() {
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) expcnt(7) lgkmcnt(15)
    asm volatile("" ::: "memory");
}
// s_waitcnt vmcnt(N): all but the N youngest vector-memory operations done (N compile-time)
template <int N>
__device__ __forceinline__ void vmcnt_n() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
    asm volatile("" ::: "memory");
}
// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>());
        static_for<B + 1, E>(f);
    }
}
// one 1-KiB piece: lane l's 16 bytes from srd[voff + soff] land at LDS byte lds + 16 l
__device__ __forceinline__ void dma16(i32x4 srd, int voff, int soff, uint32_t lds) {
#if defined(__HIP_DEVICE_COMPILE__)   // (the host pass never runs it)
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(srd), "s"(soff), "s"(__builtin_amdgcn_readfirstlane(lds))
                 : "memory");
#endif
}
__device__ __forceinline__ float bload32f(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}
__device__ __forceinline__ void batomic_add(__amdgpu_buffer_rsrc_t r, int byte_off, float v) {
    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v, r, byte_off, 0, 0);
}

// Max over the lane pair (l, l^32) with v_permlane32_swap (T12).
__device__ __forceinline__ float pair_max(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ---------------------------------------------------------------------------------------
// Rotary embedding of 8 consecutive features (4 interleaved pairs) of one row, rounded like torch's
// eager evaluation of flash_attn/rotary.py:31-41 (every product and the sum rounded to T):
//   forward  y0 = rnd(rnd(x0 c0) + rnd(-x1 s0)),  y1 = rnd(rnd(x1 c1) + rnd(x0 s1))
//   inverse  y0 = rnd(rnd(x0 c0) + rnd(x1 s1)),   y1 = rnd(rnd(x1 c1) + rnd(-(x0 s0)))   (autograd)
// Shared by fa_rotary (separate pass) and the Q load of fa_fwd_kernel so both give the same bits.
// ---------------------------------------------------------------------------------------
template <typename T, bool INVERSE>
__device__ __forceinline__ u32x4 rotary8(u32x4 xv, u32x4 cv, u32x4 sv) {
    // no contraction: a fused multiply-add would round once less than torch's mul, mul, add
#pragma clang fp contract(off)
    u32x4 out;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const float x0 = T::to_float((uint16_t)(xv[w] & 0xFFFF)), x1 = T::to_float((uint16_t)(xv[w] >> 16));
        const float c0 = T::to_float((uint16_t)(cv[w] & 0xFFFF)), c1 = T::to_float((uint16_t)(cv[w] >> 16));
        const float s0 = T::to_float((uint16_t)(sv[w] & 0xFFFF)), s1 = T::to_float((uint16_t)(sv[w] >> 16));
        auto rnd = [](float v) { return T::to_float(T::from_float(v)); };
        float y0, y1;
        if (!INVERSE) {
            y0 = rnd(x0 * c0) + rnd(-x1 * s0);
            y1 = rnd(x1 * c1) + rnd(x0 * s1);
        } else {
            y0 = rnd(x0 * c0) + rnd(x1 * s1);
            y1 = rnd(x1 * c1) + rnd(-(x0 * s0));
        }
        out[w] = T::pack2(y0, y1);
    }
    return out;
}

// ---------------------------------------------------------------------------------------
// Dropout RNG: Philox-4x32 with 7 rounds (6 keyed rounds + final), the generator of the
// reference (csrc/flash_attn/src/philox.cuh:30-59, 121-136), used as a pure counter-based
// function of (seed, offset, bh, row, col) so forward and backward agree under any tiling:
//
//   g    = (row >> 5) << 2 | ((row >> 4) & 1) << 1 | ((row >> 2) & 1)
//   slot = (row & 3) | ((row >> 3) & 1) << 2
//   out  = Philox7(key = {seed_lo, seed_hi}, ctr = {g, col, bh, offset >> 2})
//   rnd16(row, col) = 16-bit word `slot` of out (word slot>>1, low half first)
//   keep(row, col)  = rnd16 <= floor((1 - p) * 65535)   (fmha_api.cpp:104, softmax.h:256-296)
//
// One Philox call serves the 8 rows {16s+4h+0..3, 16s+8+4h+0..3} of one column: exactly the
// registers 8s..8s+7 of a 32x32 accumulator whose lane is the column (the backward's layout).
// ---------------------------------------------------------------------------------------
// a ^ b ^ k with k wave-uniform (a Philox key word): one v_bitop3_b32 (truth table 0x96 = XOR3)
// instead of two v_xor_b32; hipcc does not form it from the C expression.
__device__ __forceinline__ uint32_t xor3_key(uint32_t a, uint32_t b, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(__builtin_amdgcn_readfirstlane(k)));
    return r;
#else
    return a ^ b ^ k;
#endif
}

__device__ __forceinline__ u32x4 philox7(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = xor3_key((uint32_t)(p1 >> 32), c1, k0);
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = xor3_key((uint32_t)(p0 >> 32), c3, k1);
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    u32x4 r = {c0, c1, c2, c3};
    return r;
}

// Philox stream offset of a launch: the host-reserved rng_offset plus, when given, a device word
// that a captured graph advances on every replay (FaFwdArgs::rng_offset_dev).
template <typename A>
__device__ __forceinline__ uint64_t rng_offset_of(const A &a) {
    return a.rng_offset + (a.rng_offset_dev ? *a.rng_offset_dev : 0ull);
}

__device__ __forceinline__ uint32_t rng_group(int row) {
    return ((uint32_t)(row >> 5) << 2) | (((row >> 4) & 1) << 1) | ((row >> 2) & 1);
}

// Compare both 16-bit halves of w against thr; returns keep bits (bit0 = low half).
__device__ __forceinline__ uint32_t keep2(uint32_t w, uint32_t thr) {
    return ((w & 0xFFFFu) <= thr ? 1u : 0u) | ((w >> 16) <= thr ? 2u : 0u);
}

}  // namespace fa
