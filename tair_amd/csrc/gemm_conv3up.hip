// GEMM instantiations for A_CONV3_UP: Upsample: nearest x2 + 3x3 conv (unet.py:51-79).
#include "gemm_kern.h"

TAIR_GEMM_MODE_TU(A_CONV3_UP, dma)
