// GroupNorm / LayerNorm for NHWC bf16 activations (fp32 statistics).
//
// GroupNorm32 (util.py:176-193, eps 1e-5) and the transformer's nn.GroupNorm (attention.py:48-51,
// eps 1e-6) are split into
//   (1) a partial-statistics pass over (b, group, pixel-chunk) blocks with pivot-shifted sums
//       (x - x_pivot), so E[x^2]-E[x]^2 does not cancel when |mean| >> std,
//   (2) a finalize pass producing per-(b, channel) scale/shift (gamma*rstd, beta-mean*gamma*rstd),
//   (3) an apply pass y = act(x*scale + shift) with 16-byte vector loads/stores.
// LayerNorm (attention.py:255-257, eps 1e-5): one wave per token, exact two-pass in registers.
#include "kernels.h"

namespace tair {
namespace {

constexpr int GN_MAX_SPLIT = 64;

__global__ __launch_bounds__(256) void gn_partial_kernel(const bf16* __restrict__ x, int ldx, int HW,
                                                         int C, int G, int splits,
                                                         float* __restrict__ part) {
  const int bg = blockIdx.x, s = blockIdx.y;
  const int G_ = G;
  const int b = bg / G_, g = bg - b * G_;
  const int cg = C / G_;
  const long n_el = (long)HW * cg;
  const long per = (n_el + splits - 1) / splits;
  const long e0 = s * per, e1 = min(n_el, e0 + per);
  const bf16* xb = x + (size_t)b * HW * ldx + g * cg;
  const float pivot = bf2f(xb[0]);
  float sum = 0.f, sq = 0.f;
  for (long e = e0 + threadIdx.x; e < e1; e += 256) {
    const int p = (int)(e / cg), c = (int)(e - (long)p * cg);
    const float v = bf2f(xb[(size_t)p * ldx + c]) - pivot;
    sum += v;
    sq += v * v;
  }
  __shared__ float red[2][4];
  sum = wave_sum(sum);
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = sum; red[1][threadIdx.x >> 6] = sq; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float* o = part + ((size_t)bg * GN_MAX_SPLIT + s) * 2;
    o[0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    o[1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ __launch_bounds__(64) void gn_finalize_kernel(const bf16* __restrict__ x, int ldx, int HW,
                                                         int C, int G, int splits, float eps,
                                                         const float* __restrict__ part,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         float* __restrict__ ss) {
  const int bg = blockIdx.x;
  const int b = bg / G, g = bg - b * G;
  const int cg = C / G;
  float sum = 0.f, sq = 0.f;
  for (int s = threadIdx.x; s < splits; s += 64) {
    sum += part[((size_t)bg * GN_MAX_SPLIT + s) * 2];
    sq += part[((size_t)bg * GN_MAX_SPLIT + s) * 2 + 1];
  }
  sum = wave_sum(sum);
  sq = wave_sum(sq);
  const float n = (float)HW * (float)cg;
  const float pivot = bf2f(x[(size_t)b * HW * ldx + g * cg]);
  const float dm = sum / n;
  const float var = fmaxf(sq / n - dm * dm, 0.f);
  const float mean = pivot + dm;
  const float rstd = rsqrtf(var + eps);
  for (int c = threadIdx.x; c < cg; c += 64) {
    const int ch = g * cg + c;
    const float sc = (gamma ? gamma[ch] : 1.f) * rstd;
    const float sh = (beta ? beta[ch] : 0.f) - mean * sc;
    ss[((size_t)b * C + ch) * 2] = sc;
    ss[((size_t)b * C + ch) * 2 + 1] = sh;
  }
}

__global__ __launch_bounds__(256) void gn_apply_kernel(const bf16* __restrict__ x, int ldx, int B, int HW,
                                                       int C, const float* __restrict__ ss, int silu,
                                                       bf16* __restrict__ y, int ldy) {
  const int cv = C / 8;
  const long total = (long)B * HW * cv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long row = i / cv;
    const int c0 = (int)(i - row * cv) * 8;
    const int b = (int)(row / HW);
    union { uint4 u; bf16 h[8]; } in, out;
    in.u = *(const uint4*)(x + (size_t)row * ldx + c0);
    const float4* sp = (const float4*)(ss + ((size_t)b * C + c0) * 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 t = sp[q];
      float a0 = bf2f(in.h[2 * q]) * t.x + t.y;
      float a1 = bf2f(in.h[2 * q + 1]) * t.z + t.w;
      if (silu) { a0 = silu_f(a0); a1 = silu_f(a1); }
      out.h[2 * q] = f2bf(a0);
      out.h[2 * q + 1] = f2bf(a1);
    }
    *(uint4*)(y + (size_t)row * ldy + c0) = out.u;
  }
}

template <int VPL>  // 8-wide vectors per lane
__global__ __launch_bounds__(256) void layernorm_kernel(const bf16* __restrict__ x, int T, int C,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps,
                                                        bf16* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int cv = C / 8;
  const bf16* xr = x + (size_t)t * C;
  float v[VPL][8];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int vi = lane + 64 * j;
    if (vi < cv) {
      union { uint4 u; bf16 h[8]; } in;
      in.u = *(const uint4*)(xr + vi * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) { v[j][e] = bf2f(in.h[e]); sum += v[j][e]; }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][e] = 0.f;
    }
  }
  const float mean = wave_sum(sum) / C;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    if (lane + 64 * j < cv) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[j][e] - mean; sq += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / C + eps);
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int vi = lane + 64 * j;
    if (vi < cv) {
      union { uint4 u; bf16 h[8]; } out;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = vi * 8 + e;
        out.h[e] = f2bf((v[j][e] - mean) * rstd * gamma[c] + beta[c]);
      }
      *(uint4*)(y + (size_t)t * C + vi * 8) = out.u;
    }
  }
}

}  // namespace

hipError_t groupnorm_scale_shift(const bf16* x, int ldx, int B, int HW, int C, int G, float eps,
                                 const float* gamma, const float* beta, float* ss, float* ws,
                                 hipStream_t s) {
  if (C % G) { set_error("groupnorm: C=%d not divisible by G=%d", C, G); return hipErrorInvalidValue; }
  const long n_el = (long)HW * (C / G);
  int splits = (int)((n_el + 2047) / 2048);
  if (splits > GN_MAX_SPLIT) splits = GN_MAX_SPLIT;
  if (splits < 1) splits = 1;
  hipLaunchKernelGGL(gn_partial_kernel, dim3(B * G, splits), dim3(256), 0, s, x, ldx, HW, C, G, splits, ws);
  TAIR_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(B * G), dim3(64), 0, s, x, ldx, HW, C, G, splits, eps, ws,
                     gamma, beta, ss);
  return hipGetLastError();
}

hipError_t groupnorm_apply(const bf16* x, int ldx, int B, int HW, int C, const float* ss, int silu,
                           bf16* y, int ldy, hipStream_t s) {
  if (C % 8) { set_error("groupnorm_apply: C=%d not a multiple of 8", C); return hipErrorInvalidValue; }
  const long total = (long)B * HW * (C / 8);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(gn_apply_kernel, dim3(blocks), dim3(256), 0, s, x, ldx, B, HW, C, ss, silu, y, ldy);
  return hipGetLastError();
}

hipError_t layernorm(const bf16* x, int T, int C, const float* gamma, const float* beta, float eps,
                     bf16* y, hipStream_t s) {
  const int cv = C / 8;
  dim3 grid(cdiv(T, 4));
  if (C % 8) { set_error("layernorm: C=%d", C); return hipErrorInvalidValue; }
  if (cv <= 64) hipLaunchKernelGGL(layernorm_kernel<1>, grid, dim3(256), 0, s, x, T, C, gamma, beta, eps, y);
  else if (cv <= 128) hipLaunchKernelGGL(layernorm_kernel<2>, grid, dim3(256), 0, s, x, T, C, gamma, beta, eps, y);
  else if (cv <= 192) hipLaunchKernelGGL(layernorm_kernel<3>, grid, dim3(256), 0, s, x, T, C, gamma, beta, eps, y);
  else if (cv <= 320) hipLaunchKernelGGL(layernorm_kernel<5>, grid, dim3(256), 0, s, x, T, C, gamma, beta, eps, y);
  else { set_error("layernorm: C=%d too wide", C); return hipErrorInvalidValue; }
  return hipGetLastError();
}

}  // namespace tair
