// GEMM instantiations for A_CONV3_S2: Downsample conv, stride 2 (unet.py:82-108).
#include "gemm_kern.h"

TAIR_GEMM_MODE_TU(A_CONV3_S2, dma)
