// GEMM instantiations: activation mode A_CONV3_S2, big tile set (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3_S2, SET_BIG, big)
