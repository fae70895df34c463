// GEMM instantiations: activation mode A_CONV3_UP, BK=32 deep-ring tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3_UP, SET_RING, ring)
