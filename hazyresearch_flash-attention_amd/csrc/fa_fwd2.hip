// fa_fwd2.hip — instantiations of the pipelined dense forward (fa_fwd2_kernel.h). Its own
// translation unit because it is compiled with -fno-slp-vectorize (build.py): the softmax row
// sums must stay single v_add_f32 beside the MFMAs.
#include <cstdlib>

#include "fa_launch.h"
#include "fa_fwd2_kernel.h"

namespace fa {

template <int D, typename T, bool CAUSAL>
static hipError_t launch_fwd2_t(const FaFwdArgs &a, hipStream_t stream) {
    using C = Fwd2Cfg<D>;
    auto kern = fa_fwd2_kernel<D, T, CAUSAL>;
    FA_ENSURE_LDS(kern, C::LDS_BYTES);
    dim3 grid((a.max_seqlen_q + C::BM - 1) / C::BM, a.nheads, a.batch);
    hipLaunchKernelGGL(kern, grid, dim3(C::NT), C::LDS_BYTES, stream, a);
    return hipGetLastError();
}

template <int D>
hipError_t launch_fwd2(const FaFwdArgs &a, hipStream_t s) {
    if (a.dtype == FA_DTYPE_BF16)
        return a.is_causal ? launch_fwd2_t<D, Bf16, true>(a, s) : launch_fwd2_t<D, Bf16, false>(a, s);
    return a.is_causal ? launch_fwd2_t<D, Fp16, true>(a, s) : launch_fwd2_t<D, Fp16, false>(a, s);
}

template hipError_t launch_fwd2<32>(const FaFwdArgs &, hipStream_t);
template hipError_t launch_fwd2<64>(const FaFwdArgs &, hipStream_t);
template hipError_t launch_fwd2<128>(const FaFwdArgs &, hipStream_t);

}  // namespace fa
