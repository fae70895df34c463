// Multi-scale deformable attention sampling of the stage-3 TESTR spotter.
//
// out[n][q][m*D + c] = sum_l sum_p attn[n][q][m][l][p] * bilinear(value_l[n][:, m, c], loc[n][q][m][l][p])
// with grid_sample semantics (align_corners = False, zero padding): pixel coordinates
// (x, y) = (loc_x * W_l - 0.5, loc_y * H_l - 0.5), the four neighbours outside the level read 0 and a
// point outside (-1, W) x (-1, H) contributes nothing.  The same arithmetic and summation order (levels,
// then points; corners w1..w4) as the reference's ms_deformable_im2col_gpu_kernel
// (testr/adet/layers/csrc/DeformAttn/ms_deform_im2col_cuda.cuh:33-83,238-299), which the reference calls
// from MSDeformAttn.forward (testr/adet/layers/ms_deform_attn.py:116-153).
//
// Layout: value (N, S, M, D) fp32 (S = sum of H_l * W_l, level-major rows), loc (N, Q, M, L, P, 2) as
// (x, y) in [0, 1], attn (N, Q, M, L, P), out (N, Q, M * D).  A wave covers 64 / D (query, head) pairs,
// lane = channel: each neighbour read is one D-float line per pair, the locations / weights are
// wave-uniform per pair (broadcast loads).  Level shapes travel in the kernel argument block (no device
// copies: the call is capturable).
#include "kernels.h"

namespace tair {
namespace {

__global__ __launch_bounds__(256) void msda_kernel(const MsdaArgs A, const float* __restrict__ value,
                                                   const float* __restrict__ loc, const float* __restrict__ attn,
                                                   float* __restrict__ out) {
  const long total = (long)A.N * A.Q * A.M * A.D;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = (int)(idx % A.D);
  long t = idx / A.D;
  const int m = (int)(t % A.M);
  t /= A.M;
  const int q = (int)(t % A.Q);
  const int n = (int)(t / A.Q);
  const int LP = A.L * A.P;
  const long pair = ((long)n * A.Q + q) * A.M + m;
  const float* w = attn + pair * LP;
  const float2* xy = (const float2*)(loc + pair * LP * 2);
  const int rstride = A.M * A.D;  // one value row (pixel) = M heads x D channels
  const float* vb = value + (long)n * A.S * rstride + m * A.D + c;
  float col = 0.f;
  for (int l = 0; l < A.L; ++l) {
    const int H = A.h[l], W = A.w[l];
    const float* vl = vb + (long)A.start[l] * rstride;
    for (int p = 0; p < A.P; ++p) {
      const float2 g = xy[l * A.P + p];
      const float aw = w[l * A.P + p];
      const float hi = g.y * H - 0.5f, wi = g.x * W - 0.5f;
      if (hi > -1.f && wi > -1.f && hi < H && wi < W) {
        const int h0 = (int)floorf(hi), w0 = (int)floorf(wi);
        const int h1 = h0 + 1, w1 = w0 + 1;
        const float lh = hi - h0, lw = wi - w0, hh = 1.f - lh, hw = 1.f - lw;
        const float v1 = (h0 >= 0 && w0 >= 0) ? vl[((long)h0 * W + w0) * rstride] : 0.f;
        const float v2 = (h0 >= 0 && w1 <= W - 1) ? vl[((long)h0 * W + w1) * rstride] : 0.f;
        const float v3 = (h1 <= H - 1 && w0 >= 0) ? vl[((long)h1 * W + w0) * rstride] : 0.f;
        const float v4 = (h1 <= H - 1 && w1 <= W - 1) ? vl[((long)h1 * W + w1) * rstride] : 0.f;
        col += (hh * hw * v1 + hh * lw * v2 + lh * hw * v3 + lh * lw * v4) * aw;
      }
    }
  }
  out[idx] = col;
}

}  // namespace

hipError_t ms_deform_attn(const MsdaArgs& a, const float* value, const float* loc, const float* attn, float* out,
                          hipStream_t s) {
  if (a.N < 1 || a.Q < 1 || a.M < 1 || a.D < 1 || a.L < 1 || a.L > MSDA_MAX_LEVELS || a.P < 1 || !value || !loc ||
      !attn || !out) {
    set_error("ms_deform_attn: N %d Q %d M %d D %d L %d P %d", a.N, a.Q, a.M, a.D, a.L, a.P);
    return hipErrorInvalidValue;
  }
  long s_sum = 0;
  for (int l = 0; l < a.L; ++l) {
    if (a.h[l] < 1 || a.w[l] < 1 || a.start[l] != s_sum) {
      set_error("ms_deform_attn: level %d shape %dx%d start %d (expected %ld)", l, a.h[l], a.w[l], a.start[l], s_sum);
      return hipErrorInvalidValue;
    }
    s_sum += (long)a.h[l] * a.w[l];
  }
  if (s_sum != a.S) {
    set_error("ms_deform_attn: levels cover %ld rows, value has %d", s_sum, a.S);
    return hipErrorInvalidValue;
  }
  const long total = (long)a.N * a.Q * a.M * a.D;
  hipLaunchKernelGGL(msda_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a, value, loc, attn, out);
  return hipGetLastError();
}

}  // namespace tair
