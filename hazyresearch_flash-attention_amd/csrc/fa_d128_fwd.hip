// Forward kernels for head-dim tile 128.
#include "fa_kernels_impl.h"
FA_INSTANTIATE_FWD(128)
