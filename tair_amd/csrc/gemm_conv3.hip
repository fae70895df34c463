// GEMM instantiations for A_CONV3: 3x3 conv, stride 1 (unet.py:111-223).
#include "gemm_kern.h"

TAIR_GEMM_MODE_TU(A_CONV3, dma)
