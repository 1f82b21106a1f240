// Backward kernels for head-dim tile 32.
#include "fa_kernels_impl.h"
FA_INSTANTIATE_BWD(32)
