// GEMM instantiations: activation mode A_CONV3, BK=32 deep-ring tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3, SET_RING, ring)
