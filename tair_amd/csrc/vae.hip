// Kernels of the split-precision VAE decoder (reference: terediff/model/vae.py:120-282 AttnBlock,
// 429-559 Decoder) that are not GEMMs or GroupNorms: the attention softmax and the V transpose.
// Values are carried as three bf16 planes (hi, lo, hi) / (hi, hi, lo) so that bf16 MFMA GEMMs over
// 3K reproduce fp32 products to ~2^-16 (kernels.h GemmArgs::out_split).
#include "kernels.h"

namespace tair {
namespace {

// One block per row: P = softmax(S[row, :L]) written as hi / lo / hi planes [3L].
__global__ __launch_bounds__(256) void softmax_split_kernel(const float* __restrict__ S, int lds, int L,
                                                            bf16* __restrict__ P) {
  const float* s = S + (size_t)blockIdx.x * lds;
  bf16* p = P + (size_t)blockIdx.x * 3 * L;
  __shared__ float red[4];
  float m = -INFINITY;
  for (int i = threadIdx.x; i < L; i += 256) m = fmaxf(m, s[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int i = threadIdx.x; i < L; i += 256) sum += expf(s[i] - m);
  sum = wave_sum(sum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  const float inv = 1.f / ((red[0] + red[1]) + (red[2] + red[3]));
  for (int i = threadIdx.x; i < L; i += 256) {
    const float v = expf(s[i] - m) * inv;
    const bf16 hi = f2bf(v);
    p[i] = hi;
    p[L + i] = f2bf(v - bf2f(hi));
    p[2 * L + i] = hi;
  }
}

// x [B][L][3C] (hi, lo, hi) -> y [B][C][3L] (hi, hi, lo), through 64 x 64 LDS tiles.
__global__ __launch_bounds__(256) void transpose_split_kernel(const bf16* __restrict__ x, int L, int C,
                                                              bf16* __restrict__ y) {
  __shared__ bf16 th[64][65], tl[64][65];
  const int b = blockIdx.z;
  const int l0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const bf16* xb = x + (size_t)b * L * 3 * C;
  bf16* yb = y + (size_t)b * C * 3 * L;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e / 64, c = e % 64;  // r: l within tile, c: channel within tile (coalesced on c)
    const int l = l0 + r, ch = c0 + c;
    if (l < L && ch < C) {
      th[r][c] = xb[(size_t)l * 3 * C + ch];
      tl[r][c] = xb[(size_t)l * 3 * C + C + ch];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e / 64, c = e % 64;  // r: channel within tile, c: l within tile (coalesced on l)
    const int ch = c0 + r, l = l0 + c;
    if (l < L && ch < C) {
      bf16* o = yb + (size_t)ch * 3 * L + l;
      o[0] = th[c][r];
      o[L] = th[c][r];
      o[2 * L] = tl[c][r];
    }
  }
}

}  // namespace

hipError_t softmax_split(const float* S, int lds, int rows, int L, bf16* P, hipStream_t s) {
  hipLaunchKernelGGL(softmax_split_kernel, dim3(rows), dim3(256), 0, s, S, lds, L, P);
  return hipGetLastError();
}

hipError_t transpose_split(const bf16* x, int B, int L, int C, bf16* y, hipStream_t s) {
  hipLaunchKernelGGL(transpose_split_kernel, dim3(cdiv(L, 64), cdiv(C, 64), B), dim3(256), 0, s, x, L, C, y);
  return hipGetLastError();
}

}  // namespace tair
