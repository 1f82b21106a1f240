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

// Grid: blockIdx.y = batch, blockIdx.x = a run of RPOS positions; the threads go over the
// (position, slot, head, 16-byte chunk) cells of the run in 32-bit arithmetic, RUNR cells per
// thread with every load issued before the first store (cells are distinct, so in place is safe);
// in place (y == x) only the rotated slots are visited. (A flat grid over every chunk of the tensor
// with 64-bit index arithmetic and idle threads for the unrotated v slot ran at 0.42 of HBM.)
#ifndef FA_ROT_RPOS
#define FA_ROT_RPOS 4
#endif
#ifndef FA_ROT_UNR
#define FA_ROT_UNR 4
#endif
constexpr int RPOS = FA_ROT_RPOS, RUNR = FA_ROT_UNR;
template <typename T, bool INVERSE>
__global__ __launch_bounds__(256) void rotary_kernel(const FaRotaryArgs a) {
    const int b = blockIdx.y;
    const int s0 = blockIdx.x * RPOS;
    const int npos = a.seqlen - s0 < RPOS ? a.seqlen - s0 : RPOS;
    const int chunks = a.head_dim >> 3;
    const int nact = a.y == a.x ? a.nrot : a.nslot;        // slots this launch touches
    const int per_slot = a.nheads * chunks;
    const int per_pos = nact * per_slot;
    const int cells = npos * per_pos;
    const uint16_t *xb = (const uint16_t *)a.x + b * a.x_strides[0];
    uint16_t *yb = (uint16_t *)a.y + b * a.y_strides[0];
    for (int t0 = threadIdx.x; t0 < cells; t0 += blockDim.x * RUNR) {
        u32x4 xv[RUNR];
        int64_t yo[RUNR];
        int sc[RUNR], cc[RUNR];
#pragma unroll
        for (int u = 0; u < RUNR; ++u) {
            const int t = t0 + u * blockDim.x;
            sc[u] = -1;
            if (t < cells) {
                const int pos = t / per_pos;
                int rem = t - pos * per_pos;
                const int slot = rem / per_slot;
                rem -= slot * per_slot;
                const int h = rem / chunks;
                const int c = rem - h * chunks;
                const int s = s0 + pos;
                xv[u] = *reinterpret_cast<const u32x4 *>(xb + s * a.x_strides[1] + slot * a.x_strides[2] +
                                                         h * a.x_strides[3] + 8 * c);
                yo[u] = s * a.y_strides[1] + slot * a.y_strides[2] + h * a.y_strides[3] + 8 * c;
                sc[u] = slot < a.nrot ? s : -2 - s;      // rotated: position; copied: -2 - position
                cc[u] = c;
            }
        }
#pragma unroll
        for (int u = 0; u < RUNR; ++u) {
            if (sc[u] == -1) continue;
            u32x4 out = xv[u];
            if (sc[u] >= 0) {
                const int64_t to = sc[u] * a.table_stride + 8 * cc[u];
                const u32x4 cv = *reinterpret_cast<const u32x4 *>((const uint16_t *)a.cos + to);
                const u32x4 sv = *reinterpret_cast<const u32x4 *>((const uint16_t *)a.sin + to);
                out = rotary8<T, INVERSE>(xv[u], cv, sv);
            }
            *reinterpret_cast<u32x4 *>(yb + yo[u]) = out;
        }
    }
}

hipError_t launch_rotary(const FaRotaryArgs &args, hipStream_t s) {
    const int64_t cells = (int64_t)(args.y == args.x ? args.nrot : args.nslot) * args.nheads * (args.head_dim / 8);
    if (cells == 0 || args.batch == 0 || args.seqlen == 0) return hipSuccess;
    const unsigned nt = cells * RPOS >= 256 ? 256u : (unsigned)((cells * RPOS + 63) / 64 * 64);
    // grid (seqlen, batch): batches beyond the 65535 grid-y limit go in further launches
    for (int b0 = 0; b0 < args.batch; b0 += 65535) {
        FaRotaryArgs a = args;
        a.batch = args.batch - b0 < 65535 ? args.batch - b0 : 65535;
        a.x = (const uint16_t *)args.x + (int64_t)b0 * args.x_strides[0];
        a.y = (uint16_t *)args.y + (int64_t)b0 * args.y_strides[0];
        const dim3 grid((unsigned)((a.seqlen + RPOS - 1) / RPOS), (unsigned)a.batch);
        if (a.dtype == FA_DTYPE_BF16) {
            if (a.inverse) hipLaunchKernelGGL((rotary_kernel<Bf16, true>), grid, dim3(nt), 0, s, a);
            else hipLaunchKernelGGL((rotary_kernel<Bf16, false>), grid, dim3(nt), 0, s, a);
        } else {
            if (a.inverse) hipLaunchKernelGGL((rotary_kernel<Fp16, true>), grid, dim3(nt), 0, s, a);
            else hipLaunchKernelGGL((rotary_kernel<Fp16, false>), grid, dim3(nt), 0, s, a);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace fa
