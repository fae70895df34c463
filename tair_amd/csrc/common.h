// Shared device/host definitions for the tair_amd gfx950 kernels.
// Activations live in HBM as NHWC bf16 ("token-major": [B*H*W, C] row-major); statistics and
// accumulators are fp32.  Everything here is CDNA4-only (64-wide waves, MFMA 16x16x32 bf16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // native vector: SROA-friendly

#define TAIR_DEV __device__ __forceinline__

// Kernel-argument snapshots (gemm_kern.h epi_args / main_args, norm.hip gn_args, attention.hip): an empty asm
// over the loaded fields keeps them in registers as one batch of loads.  TAIR_PIN=0 (A/B builds only) drops it.
#ifndef TAIR_PIN
#define TAIR_PIN 1
#endif
#if TAIR_PIN
#define TAIR_PIN_ASM(...) asm volatile(__VA_ARGS__)
#else
#define TAIR_PIN_ASM(...) ((void)0)
#endif

TAIR_DEV float bf2f(bf16 x) { return (float)x; }
TAIR_DEV bf16 f2bf(float x) { return (bf16)x; }

TAIR_DEV float silu_f(float x) { return x / (1.0f + __expf(-x)); }
// SiLU of the GroupNorm applies (gn_apply_kernel and the GEMMs' GroupNorm-on-load): the hardware
// reciprocal (1 ulp) instead of an IEEE division, ~10 fewer VALU instructions per value
TAIR_DEV float silu_gn(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// erf for the GEGLU epilogue: Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 output's
// 2^-9 step) with the hardware reciprocal and exp: ~12 VALU instructions and no branches, against the
// library erff's piecewise polynomial (TAIR_FAST_ERF=0 keeps erff: A/B builds)
#ifndef TAIR_FAST_ERF
#define TAIR_FAST_ERF 1
#endif
TAIR_DEV float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, ax, 1.0f));
  const float y =
      ((((1.061405429f * t - 1.453152027f) * t + 1.421413741f) * t - 0.284496736f) * t + 0.254829592f) * t;
  return copysignf(1.0f - y * __expf(-ax * ax), x);
}
TAIR_DEV float gelu_erf(float x) {
  const float u = x * 0.70710678118654752f;
  return 0.5f * x * (1.0f + (TAIR_FAST_ERF ? erf_fast(u) : erff(u)));
}

TAIR_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
TAIR_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------------------------
// Host-side launch helpers
// ---------------------------------------------------------------------------------------------
namespace tair {

// Error bookkeeping for the C ABI: every launcher returns hipError_t; the runtime turns a
// failure into a status code + thread-local message (tair_last_error()).
void set_error(const char* fmt, ...);

#define TAIR_HIP_CHECK(expr)                                                     \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) {                                                      \
      ::tair::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),   \
                        __FILE__, __LINE__);                                     \
      return _e;                                                                 \
    }                                                                            \
  } while (0)

inline int cdiv(int a, int b) { return (a + b - 1) / b; }

}  // namespace tair
