// GEMM instantiations: activation mode A_CONV3_UP, small tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3_UP, SET_SMALL, small)
