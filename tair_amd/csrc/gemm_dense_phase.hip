// GEMM instantiations: activation mode A_DENSE, 4-phase 256-row kernel (gemm_kern.h).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_DENSE, SET_PHASE, phase)
