// Timing-only ablation switch of attn_kernel (attention.hip), for variant builds only
// (python -m tair_amd.build --variant NAME -D ATTN_ABL=...; tools/attn_ablate.py): the results of an
// ablated build are invalid.  Bits: 1 no K/V loads, 2 no QK^T MFMA, 4 no exp, 8 no PV MFMA.  The product
// library is always built with ATTN_ABL = 0.
#pragma once
#ifndef ATTN_ABL
#define ATTN_ABL 0
#endif
