// GEMM instantiations: activation mode A_DENSE, small tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_DENSE, SET_SMALL, small)
