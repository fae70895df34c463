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

// scale/shift of the cg channels of group (b, g) from its pivot-shifted sums
TAIR_DEV void gn_scale_shift(float sum, float sq, float pivot, float n, float eps, int b, int g, int C, int cg,
                             const float* __restrict__ gamma, const float* __restrict__ beta,
                             float* __restrict__ ss, int lane) {
  const float dm = sum / n;
  const float var = fmaxf(sq / n - dm * dm, 0.f);
  const float mean = pivot + dm;
  const float rstd = rsqrtf(var + eps);
  for (int c = lane; c < cg; c += 64) {
    const int ch = g * cg + c;
    const float sc = (gamma ? gamma[ch] : 1.f) * rstd;
    const float sh = (beta ? beta[ch] : 0.f) - mean * sc;
    ss[((size_t)b * C + ch) * 2] = sc;
    ss[((size_t)b * C + ch) * 2 + 1] = sh;
  }
}

// Partial sums of (b, group, pixel-chunk) blocks.  With a ticket array the last chunk of each group
// to arrive also finalizes it (scale/shift), so stats + finalize are one launch: the partials are
// stored write-through (sc1) and drained before an agent-scope ticket, and the finalizing wave
// reads them back with sc1 loads (gfx950 per-XCD L2s are not coherent; no fences needed).
__global__ __launch_bounds__(256) void gn_partial_kernel(const GnGroup P, int HW, int C, int G, int splits,
                                                         float eps) {
  const GnArgs& A = P.g[blockIdx.z];
  const bf16* __restrict__ x = A.x;
  const int ldx = A.ldx;
  float* __restrict__ part = A.ws;
  int* __restrict__ tickets = A.tickets;
  const float* __restrict__ gamma = A.gamma;
  const float* __restrict__ beta = A.beta;
  float* __restrict__ ss = A.ss;
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
    const size_t o = (size_t)p * ldx + c;
    const float v = bf2f(xb[o]) + (A.x_lo ? bf2f(xb[o + A.x_lo]) : 0.f) - pivot;
    sum += v;
    sq += v * v;
  }
  __shared__ float red[2][4];
  sum = wave_sum(sum);
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = sum; red[1][threadIdx.x >> 6] = sq; }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  float* o = part + ((size_t)bg * GN_MAX_SPLIT + s) * 2;
  const float tsum = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const float tsq = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  if (!tickets) {
    if (threadIdx.x == 0) { o[0] = tsum; o[1] = tsq; }
    return;
  }
  int last = 0;
  if (threadIdx.x == 0) {
    __hip_atomic_store(o, tsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(o + 1, tsq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(tickets + bg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == splits - 1;
  }
  last = __shfl(last, 0, 64);
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float psum = 0.f, psq = 0.f;  // splits <= 64: one partial per lane, summed in a fixed tree order
  if ((int)threadIdx.x < splits) {
    const float* q = part + ((size_t)bg * GN_MAX_SPLIT + threadIdx.x) * 2;
    psum = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    psq = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  psum = wave_sum(psum);
  psq = wave_sum(psq);
  gn_scale_shift(psum, psq, pivot, (float)HW * (float)cg, eps, b, g, C, cg, gamma, beta, ss, threadIdx.x);
  if (threadIdx.x == 0) __hip_atomic_store(tickets + bg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(64) void gn_finalize_kernel(const GnGroup P, int HW, int C, int G, int splits,
                                                         float eps) {
  const GnArgs& A = P.g[blockIdx.y];
  const bf16* __restrict__ x = A.x;
  const int ldx = A.ldx;
  const float* __restrict__ part = A.ws;
  const float* __restrict__ gamma = A.gamma;
  const float* __restrict__ beta = A.beta;
  float* __restrict__ ss = A.ss;
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
  const float pivot = bf2f(x[(size_t)b * HW * ldx + g * cg]);
  gn_scale_shift(sum, sq, pivot, (float)HW * (float)cg, eps, b, g, C, cg, gamma, beta, ss, threadIdx.x);
}

// x (|x| <= 448) rounded to the e4m3 grid, nearest even, exactly in fp32.  gfx950's
// v_cvt_pk_fp8_f32 does not round an fp32 value correctly on its own: it drops the low mantissa bits
// before rounding, so 272.00003 (just above the 256/288 midpoint) became 256 (measured,
// tools/fp8_quant_diag.py).  Handing it a value already on the grid makes the conversion exact.
__device__ __forceinline__ float e4m3_grid_rne(float x) {
  int e = (int)((__float_as_uint(x) >> 23) & 0xff) - 127;  // floor(log2 |x|) for normal x
  e = e < -6 ? -6 : e;                                       // e4m3 subnormal spacing 2^-9
  const float up = __uint_as_float((uint32_t)(3 - e + 127) << 23);   // 1 / ulp = 2^(3 - e)
  const float ulp = __uint_as_float((uint32_t)(e - 3 + 127) << 23);  // 2^(e - 3)
  return rintf(x * up) * ulp;                                // power-of-two scalings: exact
}

// 8 scaled values (|q| <= 448 up to the last ulp) -> 8 OCP e4m3 bytes, round to nearest even
__device__ __forceinline__ uint2 pack_e4m3x8_scaled(float (&q)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) q[e] = e4m3_grid_rne(fminf(fmaxf(q[e], -448.f), 448.f));
  uint32_t lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], lo, true);
  uint32_t hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[4], q[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(q[6], q[7], hi, true);
  return uint2{lo, hi};
}
// 8 values x * inv -> 8 OCP e4m3 bytes (|x * inv| <= 448 by construction, the clamp only catches the
// last-ulp excess of amax * (448 / amax))
__device__ __forceinline__ uint2 pack_e4m3x8(const float (&x)[8], float inv) {
  float q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) q[e] = x[e] * inv;
  return pack_e4m3x8_scaled(q);
}

// y = act(x*scale + shift).  A block owns RB rows (pixels) of one batch element; each thread keeps
// ONE 8-channel vector (its scale/shift formed once) and at most two rows (RB <= 2 * rows per pass),
// so the stats are read once per thread instead of once per element vector.
//
// With producer statistics (A.st: the fp64 (sum, sum^2) replicas a GEMM epilogue accumulated, see
// StatTgt) the block first finalises mean / rstd of every group of its batch element in LDS, and
// each thread forms its scale/shift from them: no separate statistics pass.  The thread's rows and
// gamma / beta are loaded BEFORE that finalisation, so the block pays one memory latency, not three.
// GnArgs fields in registers, loaded as one batch: read through the kernel-argument reference, the compiler
// rematerialised them at every use (an s_load + lgkmcnt(0) round trip each, ~47 per thread on the apply
// path: the bulk of a B = 1 apply's ~5 us); one empty asm over all of them makes them opaque (gemm_kern.h pin)
// (pointers pinned as global address-space pointers: a generic pointer out of an asm statement would turn
// every access into a flat_* operation)
#define TAIR_G(T) __attribute__((address_space(1))) T*
TAIR_DEV GnArgs gn_args(const GnArgs& a) {
  GnArgs g = a;
  TAIR_G(const bf16) x = (TAIR_G(const bf16))a.x;
  TAIR_G(const float) gamma = (TAIR_G(const float))a.gamma;
  TAIR_G(const float) beta = (TAIR_G(const float))a.beta;
  TAIR_G(float) ss = (TAIR_G(float))a.ss;
  TAIR_G(bf16) y = (TAIR_G(bf16))a.y;
  TAIR_G(const double) st = (TAIR_G(const double))a.st;
  TAIR_G(uint8_t) y8 = (TAIR_G(uint8_t))a.y8;
  TAIR_G(const float) inv8 = (TAIR_G(const float))a.inv8;
  TAIR_PIN_ASM(""
               : "+s"(x), "+s"(g.ldx), "+s"(gamma), "+s"(beta), "+s"(ss), "+s"(y), "+s"(g.ldy), "+s"(st),
                 "+s"(g.st_rs), "+s"(g.eps), "+s"(g.x_lo), "+s"(g.y_split), "+s"(y8), "+s"(g.ld8), "+s"(inv8));
  g.x = (const bf16*)x; g.gamma = (const float*)gamma; g.beta = (const float*)beta; g.ss = (float*)ss;
  g.y = (bf16*)y; g.st = (const double*)st; g.y8 = (uint8_t*)y8; g.inv8 = (const float*)inv8;
  return g;
}

#ifndef TAIR_GN_PREFETCH
#define TAIR_GN_PREFETCH 1
#endif
__global__ __launch_bounds__(256) void gn_apply_kernel(const GnGroup P, int B, int HW, int C, int silu, int RB,
                                                       int G) {
  const GnArgs A = gn_args(P.g[blockIdx.y]);
  const bf16* __restrict__ x = A.x;
  const int ldx = A.ldx;
  const float* __restrict__ ss = A.ss;
  bf16* __restrict__ y = A.y;
  const int ldy = A.ldy;
  const int cv = C / 8;
  const int row0 = blockIdx.x * RB;
  const int b = row0 / HW;
  const int t = threadIdx.x;
  typedef union { uint4 u; bf16 h[8]; } V8;
  auto apply = [&](int row, int c0, const V8& in, const V8& in2, const float (&sc)[8], const float (&sh)[8]) {
    V8 out, out2;
    float a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xv = A.x_lo ? bf2f(in.h[e]) + bf2f(in2.h[e]) : bf2f(in.h[e]);
      a[e] = xv * sc[e] + sh[e];
      if (silu) a[e] = silu_gn(a[e]);
      out.h[e] = f2bf(a[e]);
    }
    if (A.y8) {  // e4m3 operand of an fp8 consumer: y / a_c with the static per-channel power-of-two scale
      float q[8];
      const float4 i0 = *(const float4*)(A.inv8 + c0), i1 = *(const float4*)(A.inv8 + c0 + 4);
      const float iv[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = bf2f(out.h[e]) * iv[e];  // the bf16 path's rounding first
      uint8_t* yr8 = A.y8 + (size_t)row * A.ld8;
      *(uint2*)(yr8 + c0) = pack_e4m3x8_scaled(q);
      if (c0 + 8 == C)  // the dense consumer's 128-value K-tile padding
        for (int c = C; c < A.ld8; c += 8) *(uint2*)(yr8 + c) = uint2{0u, 0u};
      return;
    }
    bf16* yr = y + (size_t)row * ldy + c0;
    *(uint4*)yr = out.u;
    if (A.y_split) {
#pragma unroll
      for (int e = 0; e < 8; ++e) out2.h[e] = f2bf(a[e] - bf2f(out.h[e]));
      *(uint4*)(yr + C) = out2.u;
      *(uint4*)(yr + 2 * C) = out.u;
    }
  };
  auto load_row = [&](int row, int c0, V8& in, V8& in2) {
    in.u = *(const uint4*)(x + (size_t)row * ldx + c0);
    if (A.x_lo) in2.u = *(const uint4*)(x + (size_t)row * ldx + A.x_lo + c0);
  };
  __shared__ float mr[2 * 64];  // mean, rstd per group (producer-statistics path)
  const int cg = C / G;
  auto finalize_stats = [&]() {
    if (t < G) {
      double s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int r = 0; r < STAT_REPL; ++r) {
        const double* q = A.st + (size_t)r * A.st_rs + ((size_t)b * G + t) * 2;
        s1 += q[0];
        s2 += q[1];
      }
      const double cnt = (double)HW * cg;
      const double mean = s1 / cnt;
      const double var = fmax(s2 / cnt - mean * mean, 0.0);
      mr[2 * t] = (float)mean;
      mr[2 * t + 1] = (float)(1.0 / sqrt(var + (double)A.eps));
    }
    __syncthreads();
  };
  auto form_ss = [&](int c0, const float4 (&gb)[4], float (&sc)[8], float (&sh)[8]) {
    if (A.st) {
      const float gg[8] = {gb[0].x, gb[0].y, gb[0].z, gb[0].w, gb[1].x, gb[1].y, gb[1].z, gb[1].w};
      const float bb[8] = {gb[2].x, gb[2].y, gb[2].z, gb[2].w, gb[3].x, gb[3].y, gb[3].z, gb[3].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int g = (c0 + e) / cg;
        sc[e] = gg[e] * mr[2 * g + 1];
        sh[e] = bb[e] - mr[2 * g] * sc[e];
      }
      return;
    }
    const float4* sp = (const float4*)(ss + ((size_t)b * C + c0) * 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = sp[q];
      sc[2 * q] = v.x; sh[2 * q] = v.y; sc[2 * q + 1] = v.z; sh[2 * q + 1] = v.w;
    }
  };
  auto load_gb = [&](int c0, float4 (&gb)[4]) {
    if (A.st) {
      gb[0] = *(const float4*)(A.gamma + c0);
      gb[1] = *(const float4*)(A.gamma + c0 + 4);
      gb[2] = *(const float4*)(A.beta + c0);
      gb[3] = *(const float4*)(A.beta + c0 + 4);
    }
  };
  float sc[8], sh[8];
  float4 gb[4];
  if (cv <= 256) {
    const int rpp = 256 / cv;
    const bool active = t < rpp * cv;
    const int c0 = (t % cv) * 8;
    const int ra = t / cv, rb = ra + rpp;  // the host keeps RB <= 2 * rpp
    V8 xa, xa2, xb, xb2;
    if (active) {  // independent of the statistics: in flight while they are finalised
      if (ra < RB) load_row(row0 + ra, c0, xa, xa2);
      if (rb < RB) load_row(row0 + rb, c0, xb, xb2);
      load_gb(c0, gb);
    }
    if (A.st) finalize_stats();
    if (!active) return;
    form_ss(c0, gb, sc, sh);
#if TAIR_GN_PREFETCH
    // large grids: more rows per block (the statistics finalised once per block); the next two rows are
    // loaded before the current two are applied, so four rows per thread are in flight
    for (int r = ra; r < RB; r += 2 * rpp) {
      V8 na, na2, nb, nb2;
      const int rn = r + 2 * rpp;
      if (rn < RB) load_row(row0 + rn, c0, na, na2);
      if (rn + rpp < RB) load_row(row0 + rn + rpp, c0, nb, nb2);
      apply(row0 + r, c0, xa, xa2, sc, sh);
      if (r + rpp < RB) apply(row0 + r + rpp, c0, xb, xb2, sc, sh);
      xa = na; xa2 = na2; xb = nb; xb2 = nb2;
    }
#else
    if (ra < RB) apply(row0 + ra, c0, xa, xa2, sc, sh);
    if (rb < RB) apply(row0 + rb, c0, xb, xb2, sc, sh);
    // large grids: more rows per block (the statistics finalised once per block), two rows in flight
    for (int r = ra + 2 * rpp; r < RB; r += 2 * rpp) {
      load_row(row0 + r, c0, xa, xa2);
      if (r + rpp < RB) load_row(row0 + r + rpp, c0, xb, xb2);
      apply(row0 + r, c0, xa, xa2, sc, sh);
      if (r + rpp < RB) apply(row0 + r + rpp, c0, xb, xb2, sc, sh);
    }
#endif
  } else {
    if (A.st) finalize_stats();
    for (int v = t; v < cv; v += 256) {
      load_gb(v * 8, gb);
      form_ss(v * 8, gb, sc, sh);
#pragma unroll 4
      for (int r = 0; r < RB; ++r) {
        V8 in, in2;
        load_row(row0 + r, v * 8, in, in2);
        apply(row0 + r, v * 8, in, in2, sc, sh);
      }
    }
  }
}

// one wave per weight row: absmax -> scale, e4m3 bytes (quant_rows_fp8)
__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(const bf16* __restrict__ w, int rows, int K, int ldw,
                                                             uint8_t* __restrict__ q, int ldq, float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const bf16* wr = w + (size_t)r * ldw;
  float amax = 0.f;
  for (int k = lane; k < K; k += 64) amax = fmaxf(amax, fabsf(bf2f(wr[k])));
  amax = wave_max(amax);
  // q = e4m3(w / s) with the stored scale s itself (a correctly rounded division per element, once
  // at load): dequantisation q * s pairs with exactly this s
  const float sc = amax > 0.f ? amax / 448.f : 1.f;
  if (lane == 0) scale[r] = sc;
  uint8_t* qr = q + (size_t)r * ldq;
  for (int k8 = lane; k8 < ldq / 8; k8 += 64) {
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = k8 * 8 + e < K ? bf2f(wr[k8 * 8 + e]) / sc : 0.f;
    *(uint2*)(qr + k8 * 8) = pack_e4m3x8_scaled(x);
  }
}

// fp8 weights of the GroupNorm-fed convs / linears (static activation scales): one wave per row r,
// x[k] = w[r][k] * a[k] (a = the consumer's per-input-channel activation scale, folded here), s[r] =
// the power of two >= max_k |x[k]| / 448 (1 for a zero row), q[r][k] = e4m3(x[k] / s) for k < K, zeros
// to k8, then the bf16 K-extension (skip conv) columns w[r][K + j] / s as bf16 (exact: s is a power
// of two) at byte k8 + 2j.  q rows are ldq bytes.
__global__ __launch_bounds__(256) void quant_rows_fp8_ex_kernel(const bf16* __restrict__ w, int rows, int K, int Kx,
                                                                int ldw, const float* __restrict__ a,
                                                                uint8_t* __restrict__ q, int ldq, int k8,
                                                                float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const bf16* wr = w + (size_t)r * ldw;
  float amax = 0.f;
  for (int k = lane; k < K; k += 64) amax = fmaxf(amax, fabsf(bf2f(wr[k]) * (a ? a[k] : 1.f)));
  amax = wave_max(amax);
  float sc = 1.f;
  if (amax > 0.f) {
    int ex;
    const float m = frexpf(amax / 448.f, &ex);  // amax / 448 = m * 2^ex, m in [0.5, 1)
    sc = ldexpf(1.f, m == 0.5f ? ex - 1 : ex);
  }
  const float inv = 1.f / sc;
  if (lane == 0) scale[r] = sc;
  uint8_t* qr = q + (size_t)r * ldq;
  for (int k0 = lane * 8; k0 < k8; k0 += 64 * 8) {
    float x[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = k0 + e < K ? bf2f(wr[k0 + e]) * (a ? a[k0 + e] : 1.f) * inv : 0.f;
    *(uint2*)(qr + k0) = pack_e4m3x8_scaled(x);
  }
  bf16* tail = (bf16*)(qr + k8);
  for (int j = lane; j < Kx; j += 64) tail[j] = f2bf(bf2f(wr[K + j]) * inv);
}

template <int VPL>  // 8-wide vectors per lane
__global__ __launch_bounds__(256) void layernorm_kernel(const LnGroup P, int T, int C, float eps) {
  const LnArgs& A = P.g[blockIdx.y];
  const bf16* __restrict__ x = A.x;
  const float* __restrict__ gamma = A.gamma;
  const float* __restrict__ beta = A.beta;
  bf16* __restrict__ y = A.y;
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
  if (A.y8) {  // e4m3 output with a per-token scale
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int vi = lane + 64 * j;
      if (vi < cv) {
        const float4 g0 = *(const float4*)(gamma + vi * 8), g1 = *(const float4*)(gamma + vi * 8 + 4);
        const float4 b0 = *(const float4*)(beta + vi * 8), b1 = *(const float4*)(beta + vi * 8 + 4);
        const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // the bf16 path's rounding first: the fp8 operand quantises the same activation
          v[j][e] = bf2f(f2bf((v[j][e] - mean) * rstd * gg[e] + bb[e]));
          amax = fmaxf(amax, fabsf(v[j][e]));
        }
      }
    }
    amax = wave_max(amax);
    const float inv = amax > 0.f ? 448.f / amax : 1.f;
    if (lane == 0) A.s8[t] = amax > 0.f ? amax / 448.f : 1.f;
    uint8_t* yr = A.y8 + (size_t)t * A.ld8;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int vi = lane + 64 * j;
      if (vi < cv) *(uint2*)(yr + vi * 8) = pack_e4m3x8(v[j], inv);
    }
    for (int vi = cv + lane; vi < A.ld8 / 8; vi += 64) *(uint2*)(yr + vi * 8) = uint2{0u, 0u};
    return;
  }
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int vi = lane + 64 * j;
    if (vi < cv) {
      union { uint4 u; bf16 h[8]; } out;
      const float4 g0 = *(const float4*)(gamma + vi * 8), g1 = *(const float4*)(gamma + vi * 8 + 4);
      const float4 b0 = *(const float4*)(beta + vi * 8), b1 = *(const float4*)(beta + vi * 8 + 4);
      const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) out.h[e] = f2bf((v[j][e] - mean) * rstd * gg[e] + bb[e]);
      *(uint4*)(y + (size_t)t * C + vi * 8) = out.u;
    }
  }
}

}  // namespace

hipError_t groupnorm_stats_grouped(const GnArgs* a, int n, int B, int HW, int C, int G, float eps,
                                   hipStream_t s) {
  if (C % G) { set_error("groupnorm: C=%d not divisible by G=%d", C, G); return hipErrorInvalidValue; }
  if (n < 1 || n > MAX_GROUP) { set_error("groupnorm: group of %d", n); return hipErrorInvalidValue; }
  const long n_el = (long)HW * (C / G);
  int splits = (int)((n_el + 2047) / 2048);
  if (splits > GN_MAX_SPLIT) splits = GN_MAX_SPLIT;
  if (splits < 1) splits = 1;
  GnGroup P;
  bool fused = true;
  for (int i = 0; i < MAX_GROUP; ++i) {
    P.g[i] = a[i < n ? i : 0];
    fused = fused && P.g[i].tickets;
  }
  if (!fused)
    for (int i = 0; i < MAX_GROUP; ++i) P.g[i].tickets = nullptr;
  hipLaunchKernelGGL(gn_partial_kernel, dim3(B * G, splits, n), dim3(256), 0, s, P, HW, C, G, splits, eps);
  TAIR_HIP_CHECK(hipGetLastError());
  if (fused) return hipSuccess;
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(B * G, n), dim3(64), 0, s, P, HW, C, G, splits, eps);
  return hipGetLastError();
}

hipError_t groupnorm_apply_grouped(const GnArgs* a, int n, int B, int HW, int C, int silu, hipStream_t s, int G) {
  if (C % 8) { set_error("groupnorm_apply: C=%d not a multiple of 8", C); return hipErrorInvalidValue; }
  if (a[0].st && (G < 1 || G > 64 || C % G)) {
    set_error("groupnorm_apply: %d groups over %d channels", G, C);
    return hipErrorInvalidValue;
  }
  if (n < 1 || n > MAX_GROUP) { set_error("groupnorm: group of %d", n); return hipErrorInvalidValue; }
  for (int i = 0; i < n; ++i)
    if (a[i].y8 && (!a[i].inv8 || a[i].ld8 < C || a[i].ld8 % 8 || a[i].y_split)) {
      set_error("groupnorm_apply: e4m3 output needs per-channel scales and ld8 >= C, %% 8 (ld8 %d)", a[i].ld8);
      return hipErrorInvalidValue;
    }
  GnGroup P;
  for (int i = 0; i < MAX_GROUP; ++i) P.g[i] = a[i < n ? i : 0];
  // rows per block: a power of two dividing HW, ~1024 / (C/8) so each thread handles ~4 vectors
  const int cv = C / 8;
  // (and at most two rows per thread when a thread owns one channel vector)
  const int rmax = cv <= 256 ? 2 * (256 / cv) : 32;
  int RB = 1;
  while (RB < 32 && RB * 2 * cv <= 1024 && RB * 2 <= rmax && HW % (RB * 2) == 0) RB *= 2;
  if (cv <= 256 && RB > rmax) {  // the kernel keeps at most two rows per thread in flight
    set_error("groupnorm_apply: %d rows per block for C=%d", RB, C);
    return hipErrorInvalidValue;
  }
  // batched grids: grow the block's rows (looped two at a time) while >= 4096 blocks remain -- each block
  // finalises the statistics once, and at B = 64 that per-block latency, not HBM, bounded the pass
  // (profiles/r04_gn_apply_bw.log: one- and two-plane inputs took the same time)
  if (cv <= 256)
    while (RB < 64 && (long)B * HW / (RB * 2) >= 4096 && HW % (RB * 2) == 0) RB *= 2;
  hipLaunchKernelGGL(gn_apply_kernel, dim3(B * HW / RB, n), dim3(256), 0, s, P, B, HW, C, silu, RB, G);
  return hipGetLastError();
}

hipError_t groupnorm_scale_shift(const bf16* x, int ldx, int B, int HW, int C, int G, float eps,
                                 const float* gamma, const float* beta, float* ss, float* ws,
                                 hipStream_t s, int* tickets) {
  GnArgs a{x, ldx, gamma, beta, ss, ws, tickets, nullptr, 0};
  return groupnorm_stats_grouped(&a, 1, B, HW, C, G, eps, s);
}

hipError_t groupnorm_apply(const bf16* x, int ldx, int B, int HW, int C, const float* ss, int silu,
                           bf16* y, int ldy, hipStream_t s) {
  GnArgs a{x, ldx, nullptr, nullptr, const_cast<float*>(ss), nullptr, nullptr, y, ldy};
  return groupnorm_apply_grouped(&a, 1, B, HW, C, silu, s);
}

hipError_t layernorm_grouped(const LnArgs* a, int n, int T, int C, float eps, hipStream_t s) {
  if (C % 8) { set_error("layernorm: C=%d", C); return hipErrorInvalidValue; }
  if (n < 1 || n > MAX_GROUP) { set_error("layernorm: group of %d", n); return hipErrorInvalidValue; }
  for (int i = 0; i < n; ++i)
    if (a[i].y8 && (!a[i].s8 || a[i].ld8 < C || a[i].ld8 % 8)) {
      set_error("layernorm: fp8 output needs a scale vector and ld8 >= C, %% 8 (ld8 %d)", a[i].ld8);
      return hipErrorInvalidValue;
    }
  LnGroup P;
  for (int i = 0; i < MAX_GROUP; ++i) P.g[i] = a[i < n ? i : 0];
  const int cv = C / 8;
  const dim3 grid(cdiv(T, 4), n);
  if (cv <= 64) hipLaunchKernelGGL(layernorm_kernel<1>, grid, dim3(256), 0, s, P, T, C, eps);
  else if (cv <= 128) hipLaunchKernelGGL(layernorm_kernel<2>, grid, dim3(256), 0, s, P, T, C, eps);
  else if (cv <= 192) hipLaunchKernelGGL(layernorm_kernel<3>, grid, dim3(256), 0, s, P, T, C, eps);
  else if (cv <= 320) hipLaunchKernelGGL(layernorm_kernel<5>, grid, dim3(256), 0, s, P, T, C, eps);
  else { set_error("layernorm: C=%d too wide", C); return hipErrorInvalidValue; }
  return hipGetLastError();
}

hipError_t quant_rows_fp8(const bf16* w, int rows, int K, int ldw, uint8_t* q, int ldq, float* scale,
                          hipStream_t s) {
  if (rows < 1 || K < 1 || ldq < K || ldq % 8 || K > ldw) {
    set_error("quant_rows_fp8: rows %d K %d ldw %d ldq %d", rows, K, ldw, ldq);
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(quant_rows_fp8_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, w, rows, K, ldw, q, ldq, scale);
  return hipGetLastError();
}

hipError_t quant_rows_fp8_ex(const bf16* w, int rows, int K, int Kx, int ldw, const float* a, uint8_t* q, int ldq,
                             int k8, float* scale, hipStream_t s) {
  if (rows < 1 || K < 1 || k8 < K || k8 % 8 || K + Kx > ldw || ldq < k8 + 2 * Kx || ldq % 16) {
    set_error("quant_rows_fp8_ex: rows %d K %d Kx %d ldw %d k8 %d ldq %d", rows, K, Kx, ldw, k8, ldq);
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(quant_rows_fp8_ex_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, s, w, rows, K, Kx, ldw, a, q, ldq,
                     k8, scale);
  return hipGetLastError();
}

hipError_t layernorm(const bf16* x, int T, int C, const float* gamma, const float* beta, float eps,
                     bf16* y, hipStream_t s) {
  LnArgs a{x, gamma, beta, y};
  return layernorm_grouped(&a, 1, T, C, eps, s);
}

}  // namespace tair
