// GEMM instantiations: activation mode A_DENSE, deep-ring 64-row tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_DENSE, SET_DEEP, deep)
