// valu_rate.hip — issue cost of single VALU instructions on gfx950 (the Philox rounds of the
// dropout mask are integer multiplies: which form is cheapest?). Each wave runs CH independent
// chains of one instruction (inline asm, so exactly that opcode), timed with s_memtime (shader
// cycles); prints cycles per instruction per wave at 1 and 2 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/valu_rate.hip -o tools/micro/valu_rate && tools/micro/valu_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int CH = 8, UNROLL = 8;

template <int OP>
__device__ __forceinline__ void op(uint32_t &x, uint32_t y) {
    if constexpr (OP == 0) {
        uint64_t r;
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(x), "v"(y) : "vcc");
        x = (uint32_t)r;
    } else if constexpr (OP == 1) {
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 2) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 3) {
        asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 4) {
        asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 5) {
        asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 6) {
        asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 7) {
        asm volatile("v_exp_f32 %0, %0" : "+v"(x));
    } else if constexpr (OP == 8) {
        asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 9) {
        asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 10) {
        asm volatile("v_cmp_le_u32_sdwa vcc, %0, %1 src0_sel:WORD_1 src1_sel:DWORD" : : "v"(x), "v"(y) : "vcc");
    } else if constexpr (OP == 11) {
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 12) {
        asm volatile("v_exp_f16 %0, %0" : "+v"(x));
    } else if constexpr (OP == 13) {
        asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(x));
    } else if constexpr (OP == 14) {
        asm volatile("v_fma_mixlo_f16 %0, %1, %1, -%0" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 15) {
        asm volatile("v_fma_mixhi_f16 %0, %1, %1, -%0" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 16) {
        asm volatile("v_cvt_pk_bf16_f32 %0, %0, %1" : "+v"(x) : "v"(y));
    } else if constexpr (OP == 17) {
        asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
    }
}

template <int OP>
__global__ __launch_bounds__(512) void valu_loop(uint64_t *cyc, uint32_t *sink, int iters) {
    uint32_t x[CH];
    const uint32_t y = 0x3F800001u + threadIdx.x;
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 7 + c;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) op<OP>(x[c], y);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s ^= x[c];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char *name, uint64_t *cyc, uint32_t *sink) {
    const int iters = 2000;
    printf("%-22s", name);
    for (int wps = 1; wps <= 2; ++wps) {
        const int blocks = 256, threads = 256 * wps;   // one block per CU: wps waves per SIMD
        hipLaunchKernelGGL(valu_loop<OP>, dim3(blocks), dim3(threads), 0, 0, cyc, sink, iters);
        hipLaunchKernelGGL(valu_loop<OP>, dim3(blocks), dim3(threads), 0, 0, cyc, sink, iters);
        hipDeviceSynchronize();
        std::vector<uint64_t> h(blocks * threads / 64);
        hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
        double avg = 0;
        for (auto v : h) avg += (double)v;
        avg /= h.size();
        // cycles per instruction of one wave; per SIMD = that / wps
        const double per = avg / ((double)iters * UNROLL * CH);
        printf("  %d wave/SIMD: %6.2f cyc/instr/wave (%5.2f per SIMD)", wps, per, per / wps);
    }
    printf("\n");
}

int main() {
    uint64_t *cyc;
    uint32_t *sink;
    hipMalloc(&cyc, 256 * 8 * 8);
    hipMalloc(&sink, 256 * 512 * 4);
    run<0>("v_mad_u64_u32", cyc, sink);
    run<1>("v_mul_hi_u32", cyc, sink);
    run<2>("v_mul_lo_u32", cyc, sink);
    run<3>("v_bitop3_b32", cyc, sink);
    run<4>("v_fma_f32", cyc, sink);
    run<5>("v_mul_u32_u24", cyc, sink);
    run<6>("v_mul_hi_u32_u24", cyc, sink);
    run<7>("v_exp_f32", cyc, sink);
    run<8>("v_xor_b32", cyc, sink);
    run<9>("v_mad_u32_u24", cyc, sink);
    run<10>("v_cmp_le_u32_sdwa", cyc, sink);
    run<11>("v_mul_f32", cyc, sink);
    run<12>("v_exp_f16", cyc, sink);
    run<13>("v_exp_f16_sdwa(hi)", cyc, sink);
    run<14>("v_fma_mixlo_f16", cyc, sink);
    run<15>("v_fma_mixhi_f16", cyc, sink);
    run<16>("v_cvt_pk_bf16_f32", cyc, sink);
    run<17>("v_or3_b32", cyc, sink);
    return 0;
}
