// mfma_rate.hip — what a bare v_mfma_f32_32x32x16_bf16 stream sustains on this MI355X:
// CHAINS independent accumulators per wave (each MFMA depends on the one CHAINS back), WPS waves
// per SIMD, random or zero operands. Prints TFLOP/s per configuration (kernel time by hipEvent).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/mfma_rate.hip -o /tmp/mfma_rate && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CHAINS>
__global__ __launch_bounds__(512) void mfma_loop(const bf16x8 *in, float *out, int iters) {
    const int lane = threadIdx.x & 63;
    bf16x8 a = in[(blockIdx.x * 512 + threadIdx.x) % 4096];
    bf16x8 b = in[(blockIdx.x * 512 + threadIdx.x + 1234) % 4096];
    f32x16 acc[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 16; ++s) acc[s % CHAINS] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[s % CHAINS], 0, 0, 0);
    }
    float t = 0.f;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += acc[c][r];
    if (t == 12345.f) out[lane] = t;   // keep the chain alive
}

template <int CHAINS>
float run(const bf16x8 *in, float *out, int blocks, int threads, int iters) {
    hipEvent_t s, e;
    hipEventCreate(&s);
    hipEventCreate(&e);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(mfma_loop<CHAINS>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
    hipEventRecord(s);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(mfma_loop<CHAINS>, dim3(blocks), dim3(threads), 0, 0, in, out, iters);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms;
    hipEventElapsedTime(&ms, s, e);
    const double flops = (double)blocks * (threads / 64) * iters * 16 * 32.0 * 32 * 16 * 2 * reps;
    return (float)(flops / (ms * 1e-3) / 1e12);
}

int main() {
    std::vector<__bf16> h(4096 * 8);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (__bf16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
    bf16x8 *rnd, *zero;
    float *out;
    hipMalloc(&rnd, h.size() * 2);
    hipMalloc(&zero, h.size() * 2);
    hipMalloc(&out, 4096);
    hipMemcpy(rnd, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMemset(zero, 0, h.size() * 2);
    const int iters = 2000;
    for (int data = 0; data < 2; ++data) {
        const bf16x8 *in = data ? zero : rnd;
        for (int wps : {1, 2, 4}) {   // waves per SIMD: 256 CUs x (4 * wps) waves; 512-thread blocks
            const int blocks = 256 * wps / 2 > 0 ? 256 * wps / 2 : 1;
            const int threads = wps == 1 ? 256 : 512;
            const int nb = wps == 1 ? 256 : blocks;
            printf("%s wps=%d  chains1 %7.1f  chains2 %7.1f  chains4 %7.1f  chains8 %7.1f TF/s\n",
                   data ? "zero  " : "random", wps, run<1>(in, out, nb, threads, iters), run<2>(in, out, nb, threads, iters),
                   run<4>(in, out, nb, threads, iters), run<8>(in, out, nb, threads, iters));
        }
    }
    return 0;
}
