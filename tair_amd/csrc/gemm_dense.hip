// GEMM instantiations for A_DENSE: Linear / 1x1 conv (attention.py:19-353, controlnet.py:318).
#include "gemm_kern.h"

TAIR_GEMM_MODE_TU(A_DENSE, dma)
