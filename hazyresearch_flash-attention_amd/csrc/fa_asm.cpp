// fa_asm.cpp — launcher of the hand-scheduled gfx950 assembly forward (csrc/asm/gen_fwd.py).
//
// The kernel is generated as AMDGPU assembly, assembled into a code object at build time
// (build.py) and embedded in libfa_hip.so as a byte array (build/fa_asm_blobs.cpp). It is
// loaded per device on first use with hipModuleLoadData and launched with hipModuleLaunchKernel
// on the caller's stream (so it is captured into hipGraphs like the HIP kernels).
//
// It serves head_dim <= 32 (the D=32 tile, round 6), (32, 64] (the D=64 tile), 80 and 96 (the D=96 tile: the D=128 layout computing
// 96 columns) and 128 (the D=128 tile), fp16/bf16, causal or not, no dropout, dense (no block mask), no
// fused rotary. Everything else keeps the HIP kernels of fa_fwd_kernel.h. Semantics are the same: var-len sequences through cu_seqlens,
// rows past a sequence neither read nor written, LSE = m*scale + ln(sum) (-inf for no keys).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>

#include "fa_launch.h"

extern "C" {
extern const unsigned char fa_asm_fwd_d64_bf16[];
extern const unsigned long fa_asm_fwd_d64_bf16_size;
extern const unsigned char fa_asm_fwd_d64_f16[];
extern const unsigned long fa_asm_fwd_d64_f16_size;
extern const unsigned char fa_asm_fwd_d128_bf16[];
extern const unsigned long fa_asm_fwd_d128_bf16_size;
extern const unsigned char fa_asm_fwd_d128_f16[];
extern const unsigned long fa_asm_fwd_d128_f16_size;
extern const unsigned char fa_asm_fwd_d64p_bf16[];
extern const unsigned long fa_asm_fwd_d64p_bf16_size;
extern const unsigned char fa_asm_fwd_d64p_f16[];
extern const unsigned long fa_asm_fwd_d64p_f16_size;
extern const unsigned char fa_asm_fwd_d128p_bf16[];
extern const unsigned long fa_asm_fwd_d128p_bf16_size;
extern const unsigned char fa_asm_fwd_d128p_f16[];
extern const unsigned long fa_asm_fwd_d128p_f16_size;
extern const unsigned char fa_asm_fwd_d96_bf16[];
extern const unsigned long fa_asm_fwd_d96_bf16_size;
extern const unsigned char fa_asm_fwd_d96_f16[];
extern const unsigned long fa_asm_fwd_d96_f16_size;
extern const unsigned char fa_asm_fwd_d96p_bf16[];
extern const unsigned long fa_asm_fwd_d96p_bf16_size;
extern const unsigned char fa_asm_fwd_d96p_f16[];
extern const unsigned long fa_asm_fwd_d96p_f16_size;
extern const unsigned char fa_asm_fwd_d32_bf16[];
extern const unsigned long fa_asm_fwd_d32_bf16_size;
extern const unsigned char fa_asm_fwd_d32_f16[];
extern const unsigned long fa_asm_fwd_d32_f16_size;
extern const unsigned char fa_asm_fwd_d32p_bf16[];
extern const unsigned long fa_asm_fwd_d32p_bf16_size;
extern const unsigned char fa_asm_fwd_d32p_f16[];
extern const unsigned long fa_asm_fwd_d32p_f16_size;
}

namespace fa {

// Kernel argument block; the byte offsets are the ones gen_fwd.py's prologue loads.
struct FaAsmFwdArgs {
    const void *q, *k, *v;
    void *o;
    float *lse;
    const int32_t *cu_q, *cu_k;
    uint64_t q_hs, k_hs, v_hs, o_hs;       // head strides, bytes
    uint32_t q_rs, k_rs, v_rs, o_rs;       // row strides, bytes
    uint32_t nheads;
    uint32_t lse_row_bytes;                // lse_stride * 4
    float c;                               // softmax_scale * log2(e)
    float thr;                             // rescale threshold 2^8 in raw score units (8 / c)
    uint32_t nqb;                          // 256-row query blocks per head (grid x)
    uint32_t nwg;                          // workgroups in the grid
    uint32_t magic_nqb;                    // ceil(2^32 / (2 nqb)): Lp / nqb = mulhi(2 Lp, magic)
    uint32_t magic_h;                      // ceil(2^32 / (2 H))
    uint32_t head_dim;
    uint32_t nbh;                          // batch * heads
    uint32_t causal;                       // top-left causal mask (col <= row), heaviest q-blocks first
    uint32_t magic_nbh;                    // ceil(2^32 / (2 nbh))
    // causal XCD groups (fa_common.h xcd_grouped): each XCD runs its nbh / 8 heads in groups of G,
    // heaviest q-block first across a group; per = G nqb (0: the global heaviest-first order)
    uint32_t per, magic_per, group, magic_group;
    // persistent form only (gen_fwd.py --persist, KARG_BYTES 176): workgroups in the 1-D grid; each
    // walks logical blocks L = blockIdx.x + r * persist_grid
    uint32_t persist_grid, pad;
};
static_assert(sizeof(FaAsmFwdArgs) == 176, "FaAsmFwdArgs layout (gen_fwd.py KARG_BYTES)");
static_assert(offsetof(FaAsmFwdArgs, q_rs) == 88 && offsetof(FaAsmFwdArgs, c) == 112 &&
              offsetof(FaAsmFwdArgs, magic_nqb) == 128 && offsetof(FaAsmFwdArgs, head_dim) == 136 &&
                  offsetof(FaAsmFwdArgs, causal) == 144,
              "FaAsmFwdArgs offsets (gen_fwd.py prologue)");

namespace {

constexpr int kRows = 256;            // query rows per workgroup
#ifndef FA_ASM_GROUP_WGS
#define FA_ASM_GROUP_WGS 64          // causal D > 64: workgroups per XCD head group (2x the 32 a XCD runs)
#endif
constexpr int kMaxDev = 64;
constexpr float kRescaleThr = 8.0f;   // fa_fwd_kernel.h RESCALE_THR

// kernels: [form (0: D=64, 1: D=128, 2: D=64 persistent, 3: D=128 persistent, 4: D=96, 5: D=96
// persistent, 6: D=32, 7: D=32 persistent) * 2 + dtype (0: bf16, 1: f16)]. The two-waves-per-SIMD
// form (gen_fwd.py --waves 8, FA_IMPL_ASM8) measured even or slower in every A/B
// and left the library in round 6; the generator keeps it for A/B builds. The D=32 tile (head_dim
// <= 32, zero-padded) joined in round 6, when it measured faster than the HIP D=32 forward.
constexpr int kNumFns = 16;
struct DevFns {
    hipModule_t mod[kNumFns] = {};
    hipFunction_t fn[kNumFns] = {};
};
std::mutex g_mu;
DevFns g_fns[kMaxDev];
// assembly-forward launches enqueued (or captured) by this process: fa_query(FA_QUERY_ASM_LAUNCHES)
std::atomic<int64_t> g_asm_launches{0};

// Every form of the device is loaded at its first asm call, under the mutex, so that after any one
// eager call no later call (whatever form its grid picks) loads a module: a call inside a hipGraph
// capture then only launches. If the very first asm call of a device happens inside a capture, the
// loads run with this thread's capture mode exchanged to relaxed (module loading is not a stream
// operation; in global mode the runtime may refuse it), and if they still fail the caller falls back
// to the HIP kernels (fa_api.cpp) instead of failing the capture.
// Each module loads on its own (one that fails does not stop the others); the call reports the status
// of the requested form `want` only.
hipError_t load_all(DevFns &d, int want) {
    static const void *const imgs[kNumFns] = {fa_asm_fwd_d64_bf16,   fa_asm_fwd_d64_f16,
                                              fa_asm_fwd_d128_bf16,  fa_asm_fwd_d128_f16,
                                              fa_asm_fwd_d64p_bf16,  fa_asm_fwd_d64p_f16,
                                              fa_asm_fwd_d128p_bf16, fa_asm_fwd_d128p_f16,
                                              fa_asm_fwd_d96_bf16,   fa_asm_fwd_d96_f16,
                                              fa_asm_fwd_d96p_bf16,  fa_asm_fwd_d96p_f16,
                                              fa_asm_fwd_d32_bf16,   fa_asm_fwd_d32_f16,
                                              fa_asm_fwd_d32p_bf16,  fa_asm_fwd_d32p_f16};
    static const char *const names[kNumFns] = {"fa_fwd_d64_bf16_asm",   "fa_fwd_d64_f16_asm",
                                               "fa_fwd_d128_bf16_asm",  "fa_fwd_d128_f16_asm",
                                               "fa_fwd_d64p_bf16_asm",  "fa_fwd_d64p_f16_asm",
                                               "fa_fwd_d128p_bf16_asm", "fa_fwd_d128p_f16_asm",
                                               "fa_fwd_d96_bf16_asm",   "fa_fwd_d96_f16_asm",
                                               "fa_fwd_d96p_bf16_asm",  "fa_fwd_d96p_f16_asm",
                                               "fa_fwd_d32_bf16_asm",   "fa_fwd_d32_f16_asm",
                                               "fa_fwd_d32p_bf16_asm",  "fa_fwd_d32p_f16_asm"};
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    const bool exchanged = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
    hipError_t want_e = hipErrorNotFound;
    for (int k = 0; k < kNumFns; ++k) {
        if (d.fn[k]) {
            if (k == want) want_e = hipSuccess;
            continue;
        }
        hipModule_t m = nullptr;
        hipError_t e = hipModuleLoadData(&m, imgs[k]);
        if (e == hipSuccess) {
            e = hipModuleGetFunction(&d.fn[k], m, names[k]);
            if (e == hipSuccess) {
                d.mod[k] = m;
            } else {
                d.fn[k] = nullptr;
                (void)hipModuleUnload(m);
            }
        }
        if (k == want) want_e = e;
    }
    if (exchanged) hipThreadExchangeStreamCaptureMode(&mode);
    return want_e;
}

hipError_t get_function(int dtype, int form, hipFunction_t *out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    const int k = 2 * form + (dtype == FA_DTYPE_BF16 ? 0 : 1);
    std::lock_guard<std::mutex> lk(g_mu);
    DevFns &d = g_fns[dev];
    if (!d.fn[k]) {
        e = load_all(d, k);
        if (e != hipSuccess || !d.fn[k]) return e != hipSuccess ? e : hipErrorNotFound;
    }
    *out = d.fn[k];
    return hipSuccess;
}

uint32_t magic_half(uint32_t d) {   // ceil(2^32 / (2 d)) for d >= 1
    const uint64_t dd = 2ull * d;
    return (uint32_t)(((1ull << 32) + dd - 1) / dd);
}

}  // namespace

bool fwd_asm_eligible(const FaFwdArgs &a, const FaBlockMask &bm) {
    if (a.impl == FA_IMPL_HIP) return false;
    if (bm.mask || a.p_dropout > 0.f || a.rot_cos) return false;
    // D = 32 tile: head_dim <= 32, D = 64 tile: head_dim in (32, 64] (both zero-padded); D = 128 tile:
    // head_dim == 128 only (its Q loads and O stores address whole rows from one base); D = 96 tile (the
    // D = 128 layout computing 96 columns): head_dim 96, or 80 (k-step 5 of Q loaded as zeros, O
    // columns 80..95 not stored)
    if (!(a.head_dim <= 64 || a.head_dim == 80 || a.head_dim == 96 || a.head_dim == 128)) return false;
    if (a.max_seqlen_q <= 0) return false;
    // byte strides must fit the kernel's 32-bit row strides; the magic divisions are exact for
    // n * d <= 2^30 (n < workgroups, d = q-blocks per head or heads)
    const int64_t rs_max = (int64_t)1 << 31;
    if (a.q_row_stride * 2 >= rs_max || a.k_row_stride * 2 >= rs_max || a.v_row_stride * 2 >= rs_max ||
        a.o_row_stride * 2 >= rs_max || (int64_t)a.lse_stride * 4 >= rs_max)
        return false;
    const int64_t nqb = (a.max_seqlen_q + kRows - 1) / kRows;
    const int64_t nwg = nqb * a.nheads * a.batch;
    const int64_t nbh = (int64_t)a.nheads * a.batch;
    int64_t dmax = nqb > a.nheads ? nqb : a.nheads;
    if (nbh > dmax) dmax = nbh;
    if (nwg >= ((int64_t)1 << 30) / dmax) return false;
    if (nqb > 65535 || a.nheads > 65535 || a.batch > 65535) return false;
    return true;
}


// CUs of the current device rounded down to whole XCD rounds (8): the persistent grid, so that
// workgroup P walks L = P, P + G, ... in the XCD-aware block order of the one-block launch.
static int persist_grid() {
    static std::atomic<int> cache[kMaxDev] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 0;
    int g = cache[dev].load(std::memory_order_relaxed);
    if (!g) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
        g = n / 8 * 8;
        cache[dev].store(g, std::memory_order_relaxed);
    }
    return g;
}

// The persistent form (D=64, D=96 and D=128 tiles, non-causal): by default when the grid has more
// blocks than CUs (measured -1.8 % at the north star's 3 rounds, -3.4 % at 6; D=128 -1.6 % at 3
// rounds, even at 12); FA_IMPL_ASM4P forces it. Causal grids keep the dispatcher's dynamic balance.
// Every form computes fp32-exact scores (round 5: the pre-scaled Q of round 4, gen_fwd.py PRESCALE,
// is out of the product), so the choice is by grid shape only, never by key count.
static int persistent_grid_for(const FaFwdArgs &a, uint32_t nwg) {
    if (a.is_causal || a.impl == FA_IMPL_ASM4) return 0;
    const int g = persist_grid();
    if (g < 8) return 0;
    if (a.impl == FA_IMPL_ASM4P) return (int)(nwg < (uint32_t)g ? nwg : (uint32_t)g);
    return nwg > (uint32_t)g ? g : 0;
}

// The code object launch_fwd_asm runs for these arguments (form index of kNumFns / 2) and the
// persistent grid (0: one workgroup per block).
static int asm_form(const FaFwdArgs &a, int *pgrid) {
    const uint32_t nqb0 = (uint32_t)((a.max_seqlen_q + kRows - 1) / kRows);
    *pgrid = persistent_grid_for(a, nqb0 * (uint32_t)a.nheads * (uint32_t)a.batch);
    const bool d128 = a.head_dim > 96, d96 = a.head_dim > 64 && !d128, d32 = a.head_dim <= 32;
    return *pgrid ? (d128 ? 3 : d96 ? 5 : d32 ? 7 : 2) : (d128 ? 1 : d96 ? 4 : d32 ? 6 : 0);
}

const char *asm_kernel_name(const FaFwdArgs &a) {
    static const char *const names[kNumFns] = {"fa_fwd_d64_bf16_asm",   "fa_fwd_d64_f16_asm",
                                               "fa_fwd_d128_bf16_asm",  "fa_fwd_d128_f16_asm",
                                               "fa_fwd_d64p_bf16_asm",  "fa_fwd_d64p_f16_asm",
                                               "fa_fwd_d128p_bf16_asm", "fa_fwd_d128p_f16_asm",
                                               "fa_fwd_d96_bf16_asm",   "fa_fwd_d96_f16_asm",
                                               "fa_fwd_d96p_bf16_asm",  "fa_fwd_d96p_f16_asm",
                                               "fa_fwd_d32_bf16_asm",   "fa_fwd_d32_f16_asm",
                                               "fa_fwd_d32p_bf16_asm",  "fa_fwd_d32p_f16_asm"};
    int pgrid = 0;
    return names[2 * asm_form(a, &pgrid) + (a.dtype == FA_DTYPE_BF16 ? 0 : 1)];
}

hipError_t launch_fwd_asm(const FaFwdArgs &a, hipStream_t stream, bool *unavailable) {
    hipFunction_t fn = nullptr;
    *unavailable = false;
    int pgrid = 0;
    const int form = asm_form(a, &pgrid);
    hipError_t e = get_function(a.dtype, form, &fn);
    if (e != hipSuccess) {
        (void)hipGetLastError();   // the load error is not the caller's launch error
        *unavailable = true;
        return hipSuccess;
    }
    FaAsmFwdArgs k;
    std::memset(&k, 0, sizeof(k));
    k.q = a.q;
    k.k = a.k;
    k.v = a.v;
    k.o = a.o;
    k.lse = a.softmax_lse;
    k.cu_q = a.cu_seqlens_q;
    k.cu_k = a.cu_seqlens_k;
    k.q_hs = (uint64_t)a.q_head_stride * 2;
    k.k_hs = (uint64_t)a.k_head_stride * 2;
    k.v_hs = (uint64_t)a.v_head_stride * 2;
    k.o_hs = (uint64_t)a.o_head_stride * 2;
    k.q_rs = (uint32_t)(a.q_row_stride * 2);
    k.k_rs = (uint32_t)(a.k_row_stride * 2);
    k.v_rs = (uint32_t)(a.v_row_stride * 2);
    k.o_rs = (uint32_t)(a.o_row_stride * 2);
    k.nheads = (uint32_t)a.nheads;
    k.lse_row_bytes = (uint32_t)a.lse_stride * 4;
    k.c = a.softmax_scale * 1.4426950408889634f;
    k.thr = kRescaleThr / k.c;
    const uint32_t nqb = (uint32_t)((a.max_seqlen_q + kRows - 1) / kRows);
    k.nqb = nqb;
    k.nwg = nqb * (uint32_t)a.nheads * (uint32_t)a.batch;
    k.magic_nqb = magic_half(nqb);
    k.magic_h = magic_half((uint32_t)a.nheads);
    k.head_dim = (uint32_t)a.head_dim;
    k.nbh = (uint32_t)a.nheads * (uint32_t)a.batch;
    k.causal = a.is_causal ? 1u : 0u;
    k.magic_nbh = magic_half(k.nbh);
    // causal XCD groups only for the D=128 tile (its 2 MB of K/V per head at S=4096 want one L2): at
    // D=64 the global heaviest-first order measured faster (tools/asm_group_ab.py, B8 H12 S2048: 69.3
    // vs 75.4-90.3 us for G = 1..4; C4 D=128: G = 4 764.8 vs 836.4 us global)
    if (a.is_causal && k.nbh % 8 == 0 && a.head_dim > 64) {
        // G nqb ~ 2x the workgroups one XCD runs at once (one per CU: 32), G dividing the XCD's
        // nbh / 8 heads so that every group is full (the HIP kernels' measured choice, x2 slots)
        const uint32_t nh = k.nbh / 8, want = (FA_ASM_GROUP_WGS + nqb - 1) / nqb;
        uint32_t g = 1;
        for (uint32_t c = 1; c <= nh && c <= want; ++c)
            if (nh % c == 0) g = c;
        k.per = g * nqb;
        k.magic_per = magic_half(k.per);
        k.group = g;
        k.magic_group = magic_half(g);
    }
    k.persist_grid = (uint32_t)pgrid;
    // the one-block forms take the 168-byte block (their kernarg segment size)
    size_t size = pgrid ? sizeof(k) : offsetof(FaAsmFwdArgs, persist_grid);
    void *config[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &k, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size, HIP_LAUNCH_PARAM_END};
    if (pgrid)
        e = hipModuleLaunchKernel(fn, (unsigned)pgrid, 1, 1, kRows, 1, 1, 0, stream, nullptr, config);
    else
        e = hipModuleLaunchKernel(fn, nqb, (unsigned)a.nheads, (unsigned)a.batch, kRows, 1, 1, 0, stream, nullptr,
                                  config);
    if (e != hipSuccess) return e;
    e = hipGetLastError();
    if (e == hipSuccess) g_asm_launches.fetch_add(1, std::memory_order_relaxed);
    return e;
}

int64_t asm_launch_count() { return g_asm_launches.load(std::memory_order_relaxed); }

}  // namespace fa
