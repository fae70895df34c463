// GEMM instantiations: activation mode A_CONV3, halo tiles (conv_halo_kernel, gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3, SET_HALO, halo)
