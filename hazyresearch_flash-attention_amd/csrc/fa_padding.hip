// fa_padding.hip — first-axis gather / scatter for the var-len layout.
//
// Replaces the tensor indexing inside the reference's flash_attn/bert_padding.py:
//   index_first_axis       (IndexFirstAxis, :11-38)          dst[i] = src[idx[i]]
//   index_put_first_axis   (IndexPutFirstAxis, :41-64)       dst = 0; dst[idx[i]] = src[i]
//   index_first_axis_residual backward (:82-94)              dst[idx[i]] += src[i]
// unpad_input (:99-119) and pad_input (:122-134) are these plus a few tiny torch index ops.
//
// All three are HBM-bound row copies: one thread moves one 16-byte chunk (4- or 2-byte words
// when the row size or strides do not allow 16), so a wave covers 1 KiB of consecutive row
// bytes and every access is coalesced. The zero-filling scatter writes each output row exactly
// once through an inverse index map (inv[r] = i or -1), so the padded output costs one write
// of the output plus one read of the packed rows: the algorithmic minimum.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fa_launch.h"

namespace fa {

template <int W> struct Word;
template <> struct Word<16> { typedef uint4 type; };
template <> struct Word<4> { typedef uint32_t type; };
template <> struct Word<2> { typedef uint16_t type; };

// Each thread moves UNR words spaced one block apart (all loads issued before the stores, so a
// wave keeps UNR KiB in flight).
constexpr int UNR = 4;

// Both row copies run on a row-block grid: workgroup g moves rows [g RPB, (g + 1) RPB) (RPB chosen
// so a workgroup moves about 256 UNR words), its threads over the block's words in 32-bit arithmetic,
// UNR words per thread with every load issued before the first store. (A flat grid over all words
// with 64-bit divisions per word ran the gather at 4.1 TB/s.)
__device__ __forceinline__ void row_word(int t, int wpr, int &row, int &c) {
    row = t / wpr;
    c = t - row * wpr;
}

// dst[i][c] = src[idx[i]][c]; rows outside [0, src_rows) read as zeros
template <int W>
__global__ __launch_bounds__(256) void gather_rows_kernel(const char *__restrict__ src, int64_t src_rows,
                                                          int64_t src_stride, const int64_t *__restrict__ idx,
                                                          int64_t n, char *__restrict__ dst, int64_t dst_stride,
                                                          int wpr, int rpb) {
    typedef typename Word<W>::type T;
    const int64_t i0 = (int64_t)blockIdx.x * rpb;
    const int nr = n - i0 < rpb ? (int)(n - i0) : rpb;
    const int words = nr * wpr;
    for (int t0 = threadIdx.x; t0 < words; t0 += blockDim.x * UNR) {
        T v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int t = t0 + u * blockDim.x;
            v[u] = T{};
            if (t < words) {
                int li, c;
                row_word(t, wpr, li, c);
                const int64_t r = idx[i0 + li];
                if (r >= 0 && r < src_rows) v[u] = *reinterpret_cast<const T *>(src + r * src_stride + (int64_t)c * W);
            }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int t = t0 + u * blockDim.x;
            if (t < words) {
                int li, c;
                row_word(t, wpr, li, c);
                *reinterpret_cast<T *>(dst + (i0 + li) * dst_stride + (int64_t)c * W) = v[u];
            }
        }
    }
}

__global__ __launch_bounds__(256) void inverse_index_kernel(const int64_t *__restrict__ idx, int64_t n,
                                                            int32_t *__restrict__ inv, int64_t dst_rows) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = idx[i];
    if (r >= 0 && r < dst_rows) inv[r] = (int32_t)i;
}

// dst[r][c] = inv[r] >= 0 ? src[inv[r]][c] : 0 over every output row
template <int W>
__global__ __launch_bounds__(256) void pad_rows_kernel(const char *__restrict__ src, int64_t src_stride,
                                                       const int32_t *__restrict__ inv, int64_t dst_rows,
                                                       char *__restrict__ dst, int64_t dst_stride,
                                                       int wpr, int rpb) {
    typedef typename Word<W>::type T;
    const int64_t r0 = (int64_t)blockIdx.x * rpb;
    const int nr = dst_rows - r0 < rpb ? (int)(dst_rows - r0) : rpb;
    const int words = nr * wpr;
    for (int t0 = threadIdx.x; t0 < words; t0 += blockDim.x * UNR) {
        T v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int t = t0 + u * blockDim.x;
            v[u] = T{};
            if (t < words) {
                int lr, c;
                row_word(t, wpr, lr, c);
                const int32_t i = inv[r0 + lr];
                if (i >= 0) v[u] = *reinterpret_cast<const T *>(src + (int64_t)i * src_stride + (int64_t)c * W);
            }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int t = t0 + u * blockDim.x;
            if (t < words) {
                int lr, c;
                row_word(t, wpr, lr, c);
                *reinterpret_cast<T *>(dst + (r0 + lr) * dst_stride + (int64_t)c * W) = v[u];
            }
        }
    }
}

// dst[idx[i]][e] += src[i][e] (indices unique, as unpad_input produces them)
template <int DT>   // FA_DTYPE_FP16, FA_DTYPE_BF16 or FA_DTYPE_FP32
__global__ __launch_bounds__(256) void scatter_add_rows_kernel(const char *__restrict__ src, int64_t src_stride,
                                                               const int64_t *__restrict__ idx, int64_t n,
                                                               char *__restrict__ dst, int64_t dst_rows,
                                                               int64_t dst_stride, int64_t elems_per_row) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * elems_per_row) return;
    const int64_t i = t / elems_per_row, e = t - i * elems_per_row;
    const int64_t r = idx[i];
    if (r < 0 || r >= dst_rows) return;
    if constexpr (DT == FA_DTYPE_FP32) {
        const float a = *reinterpret_cast<const float *>(src + i * src_stride + e * 4);
        float *d = reinterpret_cast<float *>(dst + r * dst_stride + e * 4);
        *d = *d + a;
    } else if constexpr (DT == FA_DTYPE_BF16) {
        const __bf16 a = *reinterpret_cast<const __bf16 *>(src + i * src_stride + e * 2);
        __bf16 *d = reinterpret_cast<__bf16 *>(dst + r * dst_stride + e * 2);
        *d = (__bf16)((float)*d + (float)a);
    } else {
        const _Float16 a = *reinterpret_cast<const _Float16 *>(src + i * src_stride + e * 2);
        _Float16 *d = reinterpret_cast<_Float16 *>(dst + r * dst_stride + e * 2);
        *d = (_Float16)((float)*d + (float)a);
    }
}

static int word_size(const void *a, const void *b, int64_t s0, int64_t s1, int64_t row_bytes) {
    const uint64_t m = (uint64_t)(uintptr_t)a | (uint64_t)(uintptr_t)b | (uint64_t)s0 | (uint64_t)s1 |
                       (uint64_t)row_bytes;
    if ((m & 15) == 0) return 16;
    if ((m & 3) == 0) return 4;
    return 2;
}

static unsigned blocks_for(int64_t threads) { return (unsigned)((threads + 255) / 256); }

// rows per workgroup of the row copies: about 256 UNR words (at least one row)
static int rows_per_block(int wpr) {
    const int r = 256 * UNR / (wpr > 0 ? wpr : 1);
    return r < 1 ? 1 : r;
}

hipError_t launch_gather_rows(const void *src, int64_t src_rows, int64_t src_stride, const int64_t *idx, int64_t n,
                              void *dst, int64_t dst_stride, int64_t row_bytes, hipStream_t s) {
    const int w = word_size(src, dst, src_stride, dst_stride, row_bytes);
    const int wpr = (int)(row_bytes / w);
    if (n * wpr == 0) return hipSuccess;
    const int rpb = rows_per_block(wpr);
    const dim3 grid((unsigned)((n + rpb - 1) / rpb));
    const char *sp = (const char *)src;
    char *dp = (char *)dst;
    if (w == 16)
        hipLaunchKernelGGL(gather_rows_kernel<16>, grid, dim3(256), 0, s, sp, src_rows, src_stride, idx, n, dp, dst_stride, wpr, rpb);
    else if (w == 4)
        hipLaunchKernelGGL(gather_rows_kernel<4>, grid, dim3(256), 0, s, sp, src_rows, src_stride, idx, n, dp, dst_stride, wpr, rpb);
    else
        hipLaunchKernelGGL(gather_rows_kernel<2>, grid, dim3(256), 0, s, sp, src_rows, src_stride, idx, n, dp, dst_stride, wpr, rpb);
    return hipGetLastError();
}

hipError_t launch_pad_rows(const void *src, int64_t src_stride, const int64_t *idx, int64_t n, void *dst,
                           int64_t dst_rows, int64_t dst_stride, int64_t row_bytes, int32_t *inv, hipStream_t s) {
    if (dst_rows == 0 || row_bytes == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(inv, 0xFF, (size_t)dst_rows * sizeof(int32_t), s);   // -1
    if (e != hipSuccess) return e;
    if (n > 0) hipLaunchKernelGGL(inverse_index_kernel, dim3(blocks_for(n)), dim3(256), 0, s, idx, n, inv, dst_rows);
    const int w = word_size(src, dst, src_stride, dst_stride, row_bytes);
    const int wpr = (int)(row_bytes / w);
    const int rpb = rows_per_block(wpr);
    const dim3 grid((unsigned)((dst_rows + rpb - 1) / rpb));
    const char *sp = (const char *)src;
    char *dp = (char *)dst;
    if (w == 16)
        hipLaunchKernelGGL(pad_rows_kernel<16>, grid, dim3(256), 0, s, sp, src_stride, inv, dst_rows, dp, dst_stride, wpr, rpb);
    else if (w == 4)
        hipLaunchKernelGGL(pad_rows_kernel<4>, grid, dim3(256), 0, s, sp, src_stride, inv, dst_rows, dp, dst_stride, wpr, rpb);
    else
        hipLaunchKernelGGL(pad_rows_kernel<2>, grid, dim3(256), 0, s, sp, src_stride, inv, dst_rows, dp, dst_stride, wpr, rpb);
    return hipGetLastError();
}

hipError_t launch_scatter_add_rows(const void *src, int64_t src_stride, const int64_t *idx, int64_t n, void *dst,
                                   int64_t dst_rows, int64_t dst_stride, int64_t elems_per_row, int dtype,
                                   hipStream_t s) {
    if (n * elems_per_row == 0) return hipSuccess;
    const dim3 grid(blocks_for(n * elems_per_row));
    const char *sp = (const char *)src;
    char *dp = (char *)dst;
    if (dtype == FA_DTYPE_FP32)
        hipLaunchKernelGGL(scatter_add_rows_kernel<FA_DTYPE_FP32>, grid, dim3(256), 0, s, sp, src_stride, idx, n, dp, dst_rows, dst_stride, elems_per_row);
    else if (dtype == FA_DTYPE_BF16)
        hipLaunchKernelGGL(scatter_add_rows_kernel<FA_DTYPE_BF16>, grid, dim3(256), 0, s, sp, src_stride, idx, n, dp, dst_rows, dst_stride, elems_per_row);
    else
        hipLaunchKernelGGL(scatter_add_rows_kernel<FA_DTYPE_FP16>, grid, dim3(256), 0, s, sp, src_stride, idx, n, dp, dst_rows, dst_stride, elems_per_row);
    return hipGetLastError();
}

}  // namespace fa
