// GEMM instantiations: A_CONV3_SMALLC (first convs, 4 / 8 input channels; register-staged kernel).
#include "gemm_kern.h"

TAIR_GEMM_SET_TU(A_CONV3_SMALLC, SET_REG, reg)
