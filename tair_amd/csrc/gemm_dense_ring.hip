// GEMM instantiations: activation mode A_DENSE, BK=32 deep-ring tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_DENSE, SET_RING, ring)
