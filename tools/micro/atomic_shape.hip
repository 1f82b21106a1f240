// Rate of no-return fp32 atomic adds by the shape of one wave-instruction's addresses, at the
// backward's dQ footprint (B8 H12 S2048 D64: 50 MB of fp32 rows of 256 B, 8 adds per element):
//   mode 0  16x16 accumulator tile as fa_bwd_kernel issues it: lane l -> row 4 (l >> 4) + i,
//           column l & 15 (four 64-B segments in four rows per instruction)
//   mode 1  32x32-style: lane l -> row 2 i + (l >> 5), column l & 31 (two 128-B segments)
//   mode 2  256 contiguous bytes: lane l -> column l of one row
// Each wave adds a 16-row x 16..64-column tile per step; tiles walk the buffer so every element
// gets 8 adds. Prints one JSON line per mode: event time and added bytes per second.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(512) atomic_kernel(float *buf, int rows, int steps, float v) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwg = blockDim.x >> 6;
    const int gw = blockIdx.x * nwg + wave, nw = gridDim.x * nwg;
    // a "tile" = 256 floats = one wave-instruction set of 4 instructions x 64 lanes
    const int64_t ntiles = (int64_t)rows * 64 / 256;
    for (int s = 0; s < steps; ++s) {
        const int64_t t = ((int64_t)s * nw + gw) % ntiles;
        // tile t covers 16 rows x 16 columns (MODE 0), 8 rows x 32 columns (MODE 1) or 4 rows x 64 (MODE 2)
        float *p;
        int stride;
        if (MODE == 0) {
            const int64_t r0 = (t / 4) * 16, c0 = (t % 4) * 16;
            p = buf + (r0 + 4 * (lane >> 4)) * 64 + c0 + (lane & 15);
            stride = 64;
        } else if (MODE == 1) {
            const int64_t r0 = (t / 2) * 8, c0 = (t % 2) * 32;
            p = buf + (r0 + (lane >> 5)) * 64 + c0 + (lane & 31);
            stride = 2 * 64;
        } else {
            const int64_t r0 = t * 4;
            p = buf + r0 * 64 + lane;
            stride = 64;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(p + i * stride, v);
    }
}

template <int MODE>
static void run(float *buf, int rows, int grid, int nwaves, int steps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(atomic_kernel<MODE>, dim3(grid), dim3(64 * nwaves), 0, 0, buf, rows, steps, 1.f);
    hipEventRecord(e0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(atomic_kernel<MODE>, dim3(grid), dim3(64 * nwaves), 0, 0, buf, rows, steps, 1.f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double bytes = (double)grid * nwaves * steps * 4 * 64 * 4;   // waves x steps x 4 instr x 64 lanes x 4 B
    printf("{\"mode\": %d, \"grid\": %d, \"waves\": %d, \"us_per_launch\": %.1f, \"added_TBps\": %.3f}\n", MODE, grid, nwaves,
           ms * 1e3 / reps, bytes * reps / (ms * 1e-3) / 1e12);
}

int main() {
    const int rows = 8 * 12 * 2048;      // dQ rows of B8 H12 S2048, 64 fp32 each
    float *buf;
    if (hipMalloc(&buf, (size_t)rows * 64 * 4) != hipSuccess) return 1;
    hipMemset(buf, 0, (size_t)rows * 64 * 4);
    // 4 workgroups of 4 waves per CU, or one of 8 (the backward's shape)
    const int shapes[2][2] = {{1024, 4}, {256, 8}};
    for (int rep = 0; rep < 2; ++rep) {
        for (auto &sh : shapes) {
            const int steps = (int)((int64_t)rows * 64 / 256 * 8 / (sh[0] * sh[1]));   // 8 adds per element
            run<0>(buf, rows, sh[0], sh[1], steps);
            run<1>(buf, rows, sh[0], sh[1], steps);
            run<2>(buf, rows, sh[0], sh[1], steps);
        }
    }
    hipFree(buf);
    return 0;
}
