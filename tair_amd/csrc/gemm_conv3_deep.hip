// GEMM instantiations: activation mode A_CONV3, deep-ring 64-row tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3, SET_DEEP, deep)
