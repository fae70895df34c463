// GEMM instantiations for A_CONV3_SMALLC: first convs, 4 / 8 input channels (unet.py:491, controlnet.py:168).
#include "gemm_kern.h"

TAIR_GEMM_MODE_TU(A_CONV3_SMALLC, reg)
