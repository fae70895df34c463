// GEMM instantiations: activation mode A_CONV3 with e4m3 operands (fp8 ResBlock convs, gemm_kern.h act_src_f8).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3, SET_F8, f8)
