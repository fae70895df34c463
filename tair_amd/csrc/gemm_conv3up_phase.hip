// GEMM instantiations: activation mode A_CONV3_UP, 4-phase 256-row kernel (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3_UP, SET_PHASE, phase)
