// fa_rotary.hip — rotary position embedding applied to q/k in HBM.
//
// Replaces the torch element-wise chain of the reference's flash_attn/rotary.py:
//   apply_rotary_pos_emb (:31-41): y = x*cos + rotate_half(x)*sin, rotate_half pairs (2i, 2i+1)
//   -> (-x[2i+1], x[2i]) (:22-28), cos/sin repeated per pair (:76-77), every op in x's dtype.
// Rounding follows torch's eager evaluation exactly, so results are bit-identical to the
// reference path: p = rnd(x*cos), r = rnd(rotate_half(x)*sin), y = rnd(p + r), each product and
// the sum formed in fp32 (exact products of two 16-bit values) and rounded to the 16-bit type.
// The backward (inverse = 1) is autograd's transpose of the same chain:
//   dx[2i] = rnd(rnd(g[2i]*cos) + rnd(g[2i+1]*sin)),  dx[2i+1] = rnd(rnd(g[2i+1]*cos) + rnd(-g[2i]*sin)).
//
// Layout: x and y are (B, S, NSLOT, H, D) with element strides (y may alias x: in place); slots
// [0, nrot) are rotated and the others copied when y != x — so one launch rotates q and k of a
// packed qkv in place, or rotates them into a fresh buffer together with v. One thread handles
// 8 consecutive features (16 B) of one row; the cos/sin rows (shared by every batch, slot and
// head) stay in L2. HBM-bound: algorithmic bytes = read x + write y of the touched slots.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fa_common.h"
#include "fa_launch.h"

namespace fa {

template <typename T, bool INVERSE>
__global__ __launch_bounds__(256) void rotary_kernel(const FaRotaryArgs a) {
    const int chunks = a.head_dim / 8;
    const int64_t rows = (int64_t)a.batch * a.seqlen * a.nslot * a.nheads;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= rows * chunks) return;
    const int c = (int)(t % chunks);
    int64_t r = t / chunks;
    const int h = (int)(r % a.nheads);
    r /= a.nheads;
    const int slot = (int)(r % a.nslot);
    r /= a.nslot;
    const int s = (int)(r % a.seqlen);
    const int b = (int)(r / a.seqlen);
    const uint16_t *xp = (const uint16_t *)a.x + b * a.x_strides[0] + s * a.x_strides[1] + slot * a.x_strides[2] +
                         h * a.x_strides[3] + 8 * c;
    uint16_t *yp = (uint16_t *)a.y + b * a.y_strides[0] + s * a.y_strides[1] + slot * a.y_strides[2] +
                   h * a.y_strides[3] + 8 * c;
    const u32x4 xv = *reinterpret_cast<const u32x4 *>(xp);
    if (slot >= a.nrot) {
        if (a.y != a.x) *reinterpret_cast<u32x4 *>(yp) = xv;
        return;
    }
    const u32x4 cv = *reinterpret_cast<const u32x4 *>((const uint16_t *)a.cos + s * a.table_stride + 8 * c);
    const u32x4 sv = *reinterpret_cast<const u32x4 *>((const uint16_t *)a.sin + s * a.table_stride + 8 * c);
    const u32x4 out = rotary8<T, INVERSE>(xv, cv, sv);
    *reinterpret_cast<u32x4 *>(yp) = out;
}

hipError_t launch_rotary(const FaRotaryArgs &a, hipStream_t s) {
    const int64_t threads = (int64_t)a.batch * a.seqlen * a.nslot * a.nheads * (a.head_dim / 8);
    if (threads == 0) return hipSuccess;
    const dim3 grid((unsigned)((threads + 255) / 256));
    if (a.dtype == FA_DTYPE_BF16) {
        if (a.inverse) hipLaunchKernelGGL((rotary_kernel<Bf16, true>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((rotary_kernel<Bf16, false>), grid, dim3(256), 0, s, a);
    } else {
        if (a.inverse) hipLaunchKernelGGL((rotary_kernel<Fp16, true>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((rotary_kernel<Fp16, false>), grid, dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace fa
