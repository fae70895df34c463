// GEMM instantiations: activation mode A_DENSE, 2-stage 64-row tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_DENSE, SET_SHALLOW, shallow)
