// bf16 MFMA GEMM / implicit-GEMM convolution for gfx950.
//
// One kernel serves every matmul-shaped op on the ControlLDM path:
//   * Linear layers and 1x1 convs (A_DENSE)                       attention.py:19-353, controlnet.py:318
//   * 3x3 convs as implicit GEMM, stride 1 / stride 2 / fused
//     nearest-x2 upsample (A_CONV3*), k = tap*C + c (NHWC)         unet.py:51-223
//   * ResBlock 1x1 skip conv fused as a K-extension of conv2      unet.py:182-189, 223
// Roles: the MFMA A operand is the weight tile (rows = output channels n), the B operand is the
// activation tile (cols = pixels/tokens m), so each lane ends with 4 consecutive channels of one
// pixel and the NHWC epilogue store is an 8-byte vector.
// Tiles: BM x BN x 64, 256 threads = 2x2 waves, v_mfma_f32_16x16x32_bf16, register-staged
// double-buffered LDS with an XOR swizzle (chunk ^ (row & 7)) that makes both the ds_write_b128
// staging and the ds_read_b128 fragment reads bank-conflict free (checked against the gfx950
// lane groups of MI355X_MICROARCH.md §LDS).  One barrier per K-tile.
#include "kernels.h"

namespace tair {
namespace {

constexpr int BK = 64;

TAIR_DEV uint4 zero4() { return make_uint4(0, 0, 0, 0); }

template <int AMODE>
struct ARow {
  int m;       // global row (pixel) index, or -1
  int pix;     // pixel base of the batch element in the input (b*H*W)
  int yo, xo;  // output coordinates
};

template <int AMODE>
TAIR_DEV ARow<AMODE> make_row(const GemmArgs& p, int m) {
  ARow<AMODE> r;
  r.m = (m < p.M) ? m : -1;
  r.pix = 0; r.yo = 0; r.xo = 0;
  if constexpr (AMODE != A_DENSE) {
    if (r.m >= 0) {
      const int hw = p.Ho * p.Wo;
      const int b = m / hw, rem = m - b * hw;
      r.yo = rem / p.Wo;
      r.xo = rem - r.yo * p.Wo;
      r.pix = b * p.H * p.W;
    }
  }
  return r;
}

// Load 8 consecutive k of activation row r for the K-tile starting at k0 (16 bytes).
template <int AMODE>
TAIR_DEV uint4 load_act(const GemmArgs& p, const ARow<AMODE>& r, int k0, int chunk) {
  if (r.m < 0) return zero4();
  const int k = k0 + chunk * 8;
  if (k0 >= p.K) {  // fused skip-conv K-extension: centre pixel of X, plain
    if (k - p.K >= p.Kx) return zero4();
    return *(const uint4*)(p.X + (size_t)r.m * p.ldx + (k - p.K));
  }
  if constexpr (AMODE == A_DENSE) {
    return *(const uint4*)(p.A + (size_t)r.m * p.lda + k);
  } else if constexpr (AMODE == A_CONV3_SMALLC) {
    // generic gather: every element its own tap (C not a multiple of 8)
    union { uint4 u; bf16 h[8]; } v;
    const int kreal = 9 * p.C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = k + e;
      bf16 val = (bf16)0.0f;
      if (kk < kreal) {
        const int tap = kk / p.C, c = kk - tap * p.C;
        const int ky = tap / 3, kx = tap - ky * 3;
        const int yi = r.yo + ky - 1, xi = r.xo + kx - 1;
        if (yi >= 0 && yi < p.H && xi >= 0 && xi < p.W)
          val = p.A[(size_t)(r.pix + yi * p.W + xi) * p.lda + c];
      }
      v.h[e] = val;
    }
    return v.u;
  } else {
    const int tap = k0 / p.C;           // a 64-wide K-tile never straddles taps (C % 64 == 0)
    const int c = k - tap * p.C;
    const int ky = tap / 3, kx = tap - ky * 3;
    int yi, xi;
    if constexpr (AMODE == A_CONV3) {
      yi = r.yo + ky - 1; xi = r.xo + kx - 1;
    } else if constexpr (AMODE == A_CONV3_S2) {
      yi = 2 * r.yo + ky - 1; xi = 2 * r.xo + kx - 1;
    } else {  // A_CONV3_UP: conv over the 2x nearest-upsampled grid
      const int yu = r.yo + ky - 1, xu = r.xo + kx - 1;
      if (yu < 0 || yu >= 2 * p.H || xu < 0 || xu >= 2 * p.W) return zero4();
      yi = yu >> 1; xi = xu >> 1;
    }
    if (yi < 0 || yi >= p.H || xi < 0 || xi >= p.W) return zero4();
    return *(const uint4*)(p.A + (size_t)(r.pix + yi * p.W + xi) * p.lda + c);
  }
}

TAIR_DEV int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

// Epilogue for 4 consecutive channels n..n+3 of pixel m.
TAIR_DEV void epilogue4(const GemmArgs& p, int m, int n, f32x4 acc) {
  float v[4] = {acc[0] * p.alpha, acc[1] * p.alpha, acc[2] * p.alpha, acc[3] * p.alpha};
  const bool full = (n + 3 < p.N);
  const float bscale = p.scale_bias ? p.alpha : 1.f;
  const float* embrow = nullptr;
  if (p.emb) {
    const int b = m / p.rows_per_b;
    embrow = p.emb + (size_t)p.emb_row[b] * p.ld_emb;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int nn = n + r;
    if (!full && nn >= p.N) break;
    if (p.bias) v[r] += bscale * p.bias[nn];
    if (embrow) v[r] += embrow[nn];
    if (p.res) v[r] += bf2f(p.res[(size_t)m * p.ld_res + nn]);
    if (p.act == 1) v[r] = silu_f(v[r]);
  }
  if (p.out_f32) {
    float* o = (float*)p.out + (size_t)m * p.ldo + n;
    if (full && ((((size_t)m * p.ldo + n) & 3) == 0)) {
      *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int r = 0; r < 4 && n + r < p.N; ++r) o[r] = v[r];
    }
  } else {
    bf16* o = (bf16*)p.out + (size_t)m * p.ldo + n;
    if (full && ((((size_t)m * p.ldo + n) & 3) == 0)) {
      bf16x4 w = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
      *(bf16x4*)o = w;
    } else {
      for (int r = 0; r < 4 && n + r < p.N; ++r) o[r] = f2bf(v[r]);
    }
  }
}

template <int BM, int BN, int AMODE>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmArgs p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int LA = BM / 32, LB = BN / 32;  // 16-byte loads per thread per K-tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sA = (bf16*)smem;                // [2][BM][BK] activations
  bf16* sB = sA + 2 * BM * BK;           // [2][BN][BK] weights

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wm = wid & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  const int ktot = (p.K + p.Kx) / BK;
  const int per = (ktot + p.splits - 1) / p.splits;
  const int kt0 = blockIdx.z * per;
  const int kt1 = min(ktot, kt0 + per);

  const int lrow = tid >> 3, chunk = tid & 7;
  ARow<AMODE> rows[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) rows[i] = make_row<AMODE>(p, m0 + lrow + 32 * i);
  const bf16* wrow[LB];
  bool wval[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int n = n0 + lrow + 32 * i;
    wval[i] = n < p.N;
    wrow[i] = p.Wt + (size_t)(wval[i] ? n : 0) * p.ldw + chunk * 8;
  }

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[LA], rb[LB];
  auto gload = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < LA; ++i) ra[i] = load_act<AMODE>(p, rows[i], k0, chunk);
#pragma unroll
    for (int i = 0; i < LB; ++i) rb[i] = wval[i] ? *(const uint4*)(wrow[i] + k0) : zero4();
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LA; ++i)
      *(uint4*)(sA + buf * BM * BK + swz(lrow + 32 * i, chunk)) = ra[i];
#pragma unroll
    for (int i = 0; i < LB; ++i)
      *(uint4*)(sB + buf * BN * BK + swz(lrow + 32 * i, chunk)) = rb[i];
  };

  if (kt0 < kt1) {
    gload(kt0);
    sstore(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) gload(kt + 1);
      const bf16* a_s = sA + buf * BM * BK;
      const bf16* b_s = sB + buf * BN * BK;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = 4 * s + (lane >> 4);
        bf16x8 wf[FN], xf[FM];
#pragma unroll
        for (int j = 0; j < FN; ++j)
          wf[j] = *(const bf16x8*)(b_s + swz(wn * WN + j * 16 + (lane & 15), ch));
#pragma unroll
        for (int i = 0; i < FM; ++i)
          xf[i] = *(const bf16x8*)(a_s + swz(wm * WM + i * 16 + (lane & 15), ch));
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
      }
      if (more) sstore(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // acc[j][i][r] = out[m = m0 + wm*WM + i*16 + (lane&15)][n = n0 + wn*WN + j*16 + (lane>>4)*4 + r]
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * WM + i * 16 + (lane & 15);
      if (m >= p.M || n >= p.N) continue;
      if (p.splits > 1) {
        float* dst = p.partial + ((size_t)blockIdx.z * p.M + m) * p.N + n;
        if (n + 3 < p.N && (p.N & 3) == 0) {
          *(float4*)dst = make_float4(acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]);
        } else {
          for (int r = 0; r < 4 && n + r < p.N; ++r) dst[r] = acc[j][i][r];
        }
      } else {
        epilogue4(p, m, n, acc[j][i]);
      }
    }
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmArgs p) {
  const int n4 = (p.N + 3) / 4;
  const long total = (long)p.M * n4;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int m = (int)(idx / n4), n = (int)(idx - (long)m * n4) * 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < p.splits; ++z) {
      const float* src = p.partial + ((size_t)z * p.M + m) * p.N + n;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < p.N) acc[r] += src[r];
    }
    epilogue4(p, m, n, acc);
  }
}

template <int BM, int BN, int AMODE>
hipError_t set_attr() {
  const size_t lds = (size_t)2 * (BM + BN) * BK * sizeof(bf16);
  TAIR_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, AMODE>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  return hipSuccess;
}

template <int AMODE>
hipError_t set_attrs_mode() {
  TAIR_HIP_CHECK((set_attr<128, 128, AMODE>()));
  TAIR_HIP_CHECK((set_attr<64, 128, AMODE>()));
  TAIR_HIP_CHECK((set_attr<64, 64, AMODE>()));
  return hipSuccess;
}

template <int BM, int BN, int AMODE>
hipError_t launch_tile(const GemmArgs& a, int splits, hipStream_t s) {
  const size_t lds = (size_t)2 * (BM + BN) * BK * sizeof(bf16);
  dim3 grid(cdiv(a.M, BM), cdiv(a.N, BN), splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, AMODE>), grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

template <int AMODE>
hipError_t launch_mode(const GemmArgs& a, int bm, int bn, int splits, hipStream_t s) {
  if (bm == 128 && bn == 128) return launch_tile<128, 128, AMODE>(a, splits, s);
  if (bm == 64 && bn == 128) return launch_tile<64, 128, AMODE>(a, splits, s);
  return launch_tile<64, 64, AMODE>(a, splits, s);
}

}  // namespace

// Kernel attributes are set once, outside any stream capture (hipFuncSetAttribute is not a
// capturable operation).
hipError_t gemm_init() {
  static bool done = false;
  if (done) return hipSuccess;
  TAIR_HIP_CHECK(set_attrs_mode<A_DENSE>());
  TAIR_HIP_CHECK(set_attrs_mode<A_CONV3>());
  TAIR_HIP_CHECK(set_attrs_mode<A_CONV3_S2>());
  TAIR_HIP_CHECK(set_attrs_mode<A_CONV3_UP>());
  TAIR_HIP_CHECK(set_attrs_mode<A_CONV3_SMALLC>());
  done = true;
  return hipSuccess;
}

void gemm_plan(const GemmArgs& a, int* bm, int* bn, int* splits) {
  const int ktiles = (a.K + a.Kx) / BK;
  const int t128 = cdiv(a.M, 128) * cdiv(a.N, 128);
  const int t64x128 = cdiv(a.M, 64) * cdiv(a.N, 128);
  const int t64 = cdiv(a.M, 64) * cdiv(a.N, 64);
  int s = 1;
  if (t128 >= 240 && a.N >= 256) {
    *bm = 128; *bn = 128;
  } else if (t64x128 >= 240 && a.N >= 128) {
    *bm = 64; *bn = 128;
  } else {
    *bm = 64; *bn = 64;
    if (t64 < 200) {
      s = cdiv(256, t64);
      s = s > ktiles / 2 ? ktiles / 2 : s;  // keep >= 2 K-tiles per split
      if (s > 32) s = 32;
      if (s < 1) s = 1;
    }
  }
  *splits = s;
}

size_t gemm_partial_elems(const GemmArgs& a) {
  int bm, bn, s;
  gemm_plan(a, &bm, &bn, &s);
  return s > 1 ? (size_t)s * a.M * a.N : 0;
}

hipError_t gemm(const GemmArgs& a0, hipStream_t s) {
  TAIR_HIP_CHECK(gemm_init());
  GemmArgs a = a0;
  if (a.amode != A_CONV3_SMALLC && (a.K % BK) != 0) {
    set_error("gemm: K=%d not a multiple of %d", a.K, BK);
    return hipErrorInvalidValue;
  }
  if (a.Kx % BK) {
    set_error("gemm: Kx=%d not a multiple of %d", a.Kx, BK);
    return hipErrorInvalidValue;
  }
  if (a.amode != A_DENSE && a.amode != A_CONV3_SMALLC && (a.C % BK) != 0) {
    set_error("gemm: conv input channels %d not a multiple of %d", a.C, BK);
    return hipErrorInvalidValue;
  }
  int bm, bn, splits;
  gemm_plan(a, &bm, &bn, &splits);
  if (a.force_bm) bm = a.force_bm;
  if (a.force_bn) bn = a.force_bn;
  if (a.force_splits) splits = a.force_splits;
  while (splits > 1 && (a.partial == nullptr || (size_t)splits * a.M * a.N > a.partial_cap)) --splits;
  a.splits = splits;
  hipError_t e;
  switch (a.amode) {
    case A_DENSE: e = launch_mode<A_DENSE>(a, bm, bn, splits, s); break;
    case A_CONV3: e = launch_mode<A_CONV3>(a, bm, bn, splits, s); break;
    case A_CONV3_S2: e = launch_mode<A_CONV3_S2>(a, bm, bn, splits, s); break;
    case A_CONV3_UP: e = launch_mode<A_CONV3_UP>(a, bm, bn, splits, s); break;
    case A_CONV3_SMALLC: e = launch_mode<A_CONV3_SMALLC>(a, bm, bn, splits, s); break;
    default: set_error("gemm: bad amode %d", a.amode); return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  if (splits > 1) {
    const long total = (long)a.M * ((a.N + 3) / 4);
    int blocks = (int)((total + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, a);
    e = hipGetLastError();
  }
  return e;
}

}  // namespace tair
