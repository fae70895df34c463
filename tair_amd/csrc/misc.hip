// Small bandwidth-bound kernels on the ControlLDM path: GEGLU, timestep embedding, layout
// conversion at the drop-in boundary (NCHW fp32 <-> NHWC bf16) and the fused v-parameterised
// ancestral sampler step.
#include <algorithm>

#include "kernels.h"

namespace tair {
namespace {

// attention.py:19-26: [T, 2D] -> x * gelu_erf(gate), x = cols [0, D), gate = cols [D, 2D)
__global__ __launch_bounds__(256) void geglu_kernel(const bf16* __restrict__ xg, int T, int D,
                                                    bf16* __restrict__ y) {
  const int dv = D / 8;
  const long total = (long)T * dv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long t = i / dv;
    const int c = (int)(i - t * dv) * 8;
    union { uint4 u; bf16 h[8]; } a, g, out;
    a.u = *(const uint4*)(xg + (size_t)t * 2 * D + c);
    g.u = *(const uint4*)(xg + (size_t)t * 2 * D + D + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) out.h[e] = f2bf(bf2f(a.h[e]) * gelu_erf(bf2f(g.h[e])));
    *(uint4*)(y + (size_t)t * D + c) = out.u;
  }
}

// util.py:128-148 (repeat_only=False): [n, dim] = cat[cos(t*f), sin(t*f)], f_i = 10000^(-i/half)
__global__ void sinusoid_kernel(const int64_t* __restrict__ t, int n, int dim, float* __restrict__ out) {
  const int half = dim / 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * half) return;
  const int r = i / half, c = i - r * half;
  // same float32 formula as the reference: exp(-ln(10000) * c / half)
  const float freq = expf(-9.210340371976184f * (float)c / (float)half);
  const float arg = (float)t[r] * freq;
  out[(size_t)r * dim + c] = cosf(arg);
  out[(size_t)r * dim + half + c] = sinf(arg);
}

__global__ void silu_f32_kernel(const float* __restrict__ x, int n, float* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = silu_f(x[i]);
}

// zero a buffer of n 16-byte words (the per-step GroupNorm statistics slots; a kernel node instead
// of a memset node keeps the captured step graph all-kernel)
__global__ void zero16_kernel(uint4* __restrict__ p, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = make_uint4(0, 0, 0, 0);
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, int n, bf16* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f2bf(x[i]);
}

// NCHW fp32 -> NHWC bf16 (one thread per (b, pixel, channel); C is tiny at the boundary)
__global__ void nchw2nhwc_kernel(const float* __restrict__ x, int B, int C, int HW, bf16* __restrict__ y,
                                 int ldy, int c_off) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long total = (long)B * C * HW;
  if (i >= total) return;
  const long b = i / ((long)C * HW);
  const long rem = i - b * C * HW;
  const int p = (int)(rem % HW), c = (int)(rem / HW);
  y[(size_t)(b * HW + p) * ldy + c_off + c] = f2bf(x[i]);
}

__global__ void nhwc2nchw_kernel(const bf16* __restrict__ x, int ldx, int B, int C, int HW,
                                 float* __restrict__ y) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long total = (long)B * C * HW;
  if (i >= total) return;
  const long b = i / ((long)C * HW);
  const long rem = i - b * C * HW;
  const int p = (int)(rem % HW), c = (int)(rem / HW);
  y[i] = bf2f(x[(size_t)(b * HW + p) * ldx + c]);
}

__global__ void nhwcf2nchw_kernel(const float* __restrict__ x, int B, int C, int HW, float* __restrict__ y) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long total = (long)B * C * HW;
  if (i >= total) return;
  const long b = i / ((long)C * HW);
  const long rem = i - b * C * HW;
  const int p = (int)(rem % HW), c = (int)(rem / HW);
  y[i] = x[(size_t)(b * HW + p) * C + c];
}

// spaced_sampler.py:141-189, parameterization 'v':
//   x0 = sqrt(abar_t) x - sqrt(1-abar_t) v ; mean = c1_t x0 + c2_t x ; x' = mean + [t!=0] sqrt(var_t) eps
// tabs = [4][n_steps] fp32 rows: sqrt_abar, sqrt_1m_abar, coef1, coef2, posterior_variance (5 rows)
__global__ void sampler_step_kernel(const float* __restrict__ x, const float* __restrict__ v,
                                    const float* __restrict__ noise, const float* __restrict__ tabs,
                                    const int* __restrict__ step_idx, int n, float* __restrict__ xo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int t = step_idx[0];
  const int ns = step_idx[1];
  const float sa = tabs[0 * ns + t], s1a = tabs[1 * ns + t];
  const float c1 = tabs[2 * ns + t], c2 = tabs[3 * ns + t], var = tabs[4 * ns + t];
  const float xv = x[i];
  const float x0 = sa * xv - s1a * v[i];
  const float mean = c1 * x0 + c2 * xv;
  xo[i] = (t != 0) ? mean + sqrtf(var) * noise[i] : mean;
}

}  // namespace

static inline int blocks_for(long n, int bs) { return (int)((n + bs - 1) / bs); }

hipError_t geglu(const bf16* xg, int T, int D, bf16* y, hipStream_t s) {
  const long total = (long)T * (D / 8);
  int blocks = blocks_for(total, 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(geglu_kernel, dim3(blocks), dim3(256), 0, s, xg, T, D, y);
  return hipGetLastError();
}

hipError_t timestep_sinusoid(const int64_t* t, int n, int dim, float* out, hipStream_t s) {
  hipLaunchKernelGGL(sinusoid_kernel, dim3(blocks_for((long)n * (dim / 2), 256)), dim3(256), 0, s, t, n, dim, out);
  return hipGetLastError();
}

hipError_t silu_f32(const float* x, int n, float* y, hipStream_t s) {
  hipLaunchKernelGGL(silu_f32_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, x, n, y);
  return hipGetLastError();
}

hipError_t zero_bytes(void* p, size_t bytes, hipStream_t s) {
  const long n = (long)(bytes / 16);
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<long>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(zero16_kernel, dim3(blocks), dim3(256), 0, s, (uint4*)p, n);
  return hipGetLastError();
}

hipError_t f32_to_bf16(const float* x, int n, bf16* y, hipStream_t s) {
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, x, n, y);
  return hipGetLastError();
}

hipError_t nchw_f32_to_nhwc_bf16(const float* x, int B, int C, int HW, bf16* y, int ldy, int c_off,
                                 hipStream_t s) {
  const long total = (long)B * C * HW;
  hipLaunchKernelGGL(nchw2nhwc_kernel, dim3(blocks_for(total, 256)), dim3(256), 0, s, x, B, C, HW, y, ldy, c_off);
  return hipGetLastError();
}

hipError_t nhwc_bf16_to_nchw_f32(const bf16* x, int ldx, int B, int C, int HW, float* y, hipStream_t s) {
  const long total = (long)B * C * HW;
  hipLaunchKernelGGL(nhwc2nchw_kernel, dim3(blocks_for(total, 256)), dim3(256), 0, s, x, ldx, B, C, HW, y);
  return hipGetLastError();
}

hipError_t nhwc_f32_to_nchw_f32(const float* x, int B, int C, int HW, float* y, hipStream_t s) {
  const long total = (long)B * C * HW;
  hipLaunchKernelGGL(nhwcf2nchw_kernel, dim3(blocks_for(total, 256)), dim3(256), 0, s, x, B, C, HW, y);
  return hipGetLastError();
}

hipError_t sampler_step_v(const float* x, const float* v, const float* noise, const float* tabs,
                          const int* step_idx, int n, float* x_out, hipStream_t s) {
  hipLaunchKernelGGL(sampler_step_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, x, v, noise, tabs,
                     step_idx, n, x_out);
  return hipGetLastError();
}

}  // namespace tair
