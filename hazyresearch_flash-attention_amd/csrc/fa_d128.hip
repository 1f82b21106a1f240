// Kernels for head-dim tile 128.
#include "fa_kernels_impl.h"
FA_INSTANTIATE(128)
