// Flash-style attention, head dim 64, bf16 in / fp32 softmax / bf16 out, gfx950 MFMA 16x16x32.
//
// Semantics = attention.py:168-216 (SDPCrossAttention / xformers memory_efficient_attention):
// O = softmax(Q K^T * d^-1/2) V per (batch, head), no mask, no bias.  Used for the 16+7 self-
// attention layers (S = 4096/1024/256/64 tokens) and the cross-attention layers (77 context keys,
// padded to 64-key tiles and masked).
//
// Structure (one workgroup = 4 waves = 64*QSETS queries of one (b, h)):
//  * S^T = K * Q^T ("swapped" product): each lane ends with 4 consecutive keys x 1 query per
//    16-key block, so the row max / row sum of softmax are lane-local plus two xor-shuffles.
//  * The probabilities feed P*V as the MFMA B operand straight from registers; the key order inside
//    each 32-key step is permuted (keys 4h..4h+3 and 16+4h..16+4h+3 for lane half h) and V^T is read
//    from LDS with the same permutation, so no P round trip through LDS is needed.
//  * K tile [64 keys][64 d] bf16 with the GEMM XOR swizzle (ds_read_b128, conflict free);
//    V staged transposed [64 d][72] (row pad 8 -> the ds_read_b64 of both lane halves conflict free).
//  * K/V tiles double buffered in LDS, next tile prefetched to registers during compute.
#include "kernels.h"

namespace tair {
namespace {

constexpr int KT = 64;      // keys per tile
constexpr int VT_LD = 72;   // padded row of the transposed V tile

TAIR_DEV int kswz(int row, int chunk) { return row * 64 + ((chunk ^ (row & 7)) << 3); }

template <int QSETS>
__global__ __launch_bounds__(256) void attn_kernel(const bf16* __restrict__ q, int ldq,
                                                   const bf16* __restrict__ k, int ldk,
                                                   const bf16* __restrict__ v, int ldv,
                                                   bf16* __restrict__ o, int ldo, int H, int Sq,
                                                   int Skv, int kv_bstride, float scale_log2) {
  __shared__ __attribute__((aligned(16))) bf16 sK[2][KT * 64];
  __shared__ __attribute__((aligned(16))) bf16 sVt[2][64 * VT_LD];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hi = lane >> 4, lo = lane & 15;
  const int bh = blockIdx.y;
  const int b = bh / H, h = bh - b * H;
  const int q0 = blockIdx.x * (64 * QSETS) + wid * (16 * QSETS);

  // Q^T fragments (MFMA B operand): lane holds Q[q = lo][d = 32s + 8hi .. +7]
  bf16x8 qf[QSETS][2];
#pragma unroll
  for (int qs = 0; qs < QSETS; ++qs) {
    const int qi = q0 + qs * 16 + lo;
    const bf16* qr = q + ((size_t)b * Sq + (qi < Sq ? qi : 0)) * ldq + h * 64;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (qi < Sq) qf[qs][s] = *(const bf16x8*)(qr + 32 * s + 8 * hi);
      else qf[qs][s] = bf16x8{};
    }
  }

  const bf16* kb = k + (size_t)b * kv_bstride * ldk + h * 64;
  const bf16* vb = v + (size_t)b * kv_bstride * ldv + h * 64;

  // staging: 64 keys x 8 chunks = 512 chunks per operand, 2 per thread
  const int srow = tid >> 3, schunk = tid & 7;
  uint4 rk[2], rv[2];
  auto gload = [&](int t0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = t0 + srow + 32 * i;
      if (key < Skv) {
        rk[i] = *(const uint4*)(kb + (size_t)key * ldk + schunk * 8);
        rv[i] = *(const uint4*)(vb + (size_t)key * ldv + schunk * 8);
      } else {
        rk[i] = make_uint4(0, 0, 0, 0);
        rv[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = srow + 32 * i;
      *(uint4*)(&sK[buf][kswz(key, schunk)]) = rk[i];
      union { uint4 u; bf16 e[8]; } t;
      t.u = rv[i];
#pragma unroll
      for (int e = 0; e < 8; ++e) sVt[buf][(schunk * 8 + e) * VT_LD + key] = t.e[e];
    }
  };

  float m_run[QSETS], l_run[QSETS];
  f32x4 oacc[QSETS][4];  // O^T[d = 16db + 4hi + r][q = lo]
#pragma unroll
  for (int qs = 0; qs < QSETS; ++qs) {
    m_run[qs] = -INFINITY;
    l_run[qs] = 0.f;
#pragma unroll
    for (int db = 0; db < 4; ++db) oacc[qs][db] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int ntiles = (Skv + KT - 1) / KT;
  gload(0);
  sstore(0);
  __syncthreads();
  int buf = 0;
  for (int t = 0; t < ntiles; ++t) {
    const bool more = t + 1 < ntiles;
    if (more) gload((t + 1) * KT);
    const bf16* Ks = sK[buf];
    const bf16* Vs = sVt[buf];

    // S^T blocks: sacc[qs][kb][r] = S[q = lo][key = 16kb + 4hi + r]
    f32x4 sacc[QSETS][4];
#pragma unroll
    for (int qs = 0; qs < QSETS; ++qs)
#pragma unroll
      for (int kb4 = 0; kb4 < 4; ++kb4) sacc[qs][kb4] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int kb4 = 0; kb4 < 4; ++kb4) {
        const bf16x8 kf = *(const bf16x8*)(Ks + kswz(kb4 * 16 + lo, 4 * s + hi));
#pragma unroll
        for (int qs = 0; qs < QSETS; ++qs)
          sacc[qs][kb4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qs][s], sacc[qs][kb4], 0, 0, 0);
      }
    }

    // online softmax per query (lane-local + xor 16/32 across the four lane quarters)
    bf16x8 pf[QSETS][2];
    const int key0 = t * KT;
#pragma unroll
    for (int qs = 0; qs < QSETS; ++qs) {
      float mx = -INFINITY;
#pragma unroll
      for (int kb4 = 0; kb4 < 4; ++kb4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = key0 + kb4 * 16 + hi * 4 + r;
          float sv = sacc[qs][kb4][r] * scale_log2;
          if (key >= Skv) sv = -INFINITY;
          sacc[qs][kb4][r] = sv;
          mx = fmaxf(mx, sv);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m_run[qs], mx);
      const float alpha = exp2f(m_run[qs] - mnew);
      m_run[qs] = mnew;
      float ls = 0.f;
      float pv[4][4];
#pragma unroll
      for (int kb4 = 0; kb4 < 4; ++kb4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pe = exp2f(sacc[qs][kb4][r] - mnew);
          pv[kb4][r] = pe;
          ls += pe;
        }
      l_run[qs] = l_run[qs] * alpha + ls;
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int r = 0; r < 4; ++r) oacc[qs][db][r] *= alpha;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pf[qs][s][r] = f2bf(pv[2 * s][r]);
          pf[qs][s][4 + r] = f2bf(pv[2 * s + 1][r]);
        }
      }
    }

    // O^T += V^T P^T with the matching key permutation
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const bf16* vrow = Vs + (db * 16 + lo) * VT_LD + 32 * s + 4 * hi;
        const bf16x4 v0 = *(const bf16x4*)(vrow);
        const bf16x4 v1 = *(const bf16x4*)(vrow + 16);
        const bf16x8 vf = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int qs = 0; qs < QSETS; ++qs)
          oacc[qs][db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qs][s], oacc[qs][db], 0, 0, 0);
      }
    }

    if (more) sstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

#pragma unroll
  for (int qs = 0; qs < QSETS; ++qs) {
    float lt = l_run[qs];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const float inv = 1.f / lt;
    const int qi = q0 + qs * 16 + lo;
    if (qi < Sq) {
      bf16* orow = o + ((size_t)b * Sq + qi) * ldo + h * 64;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        bf16x4 w = {f2bf(oacc[qs][db][0] * inv), f2bf(oacc[qs][db][1] * inv),
                    f2bf(oacc[qs][db][2] * inv), f2bf(oacc[qs][db][3] * inv)};
        *(bf16x4*)(orow + db * 16 + hi * 4) = w;
      }
    }
  }
}

}  // namespace

hipError_t attention(const bf16* q, int ldq, const bf16* k, int ldk, const bf16* v, int ldv, bf16* o,
                     int ldo, int B, int H, int Sq, int Skv, int kv_bstride, float scale, hipStream_t s) {
  const float sl2 = scale * 1.4426950408889634f;
  const int blocks64 = cdiv(Sq, 64) * B * H;
  if (blocks64 >= 512 && Sq >= 128) {
    dim3 grid(cdiv(Sq, 128), B * H);
    hipLaunchKernelGGL(attn_kernel<2>, grid, dim3(256), 0, s, q, ldq, k, ldk, v, ldv, o, ldo, H, Sq, Skv,
                       kv_bstride, sl2);
  } else {
    dim3 grid(cdiv(Sq, 64), B * H);
    hipLaunchKernelGGL(attn_kernel<1>, grid, dim3(256), 0, s, q, ldq, k, ldk, v, ldv, o, ldo, H, Sq, Skv,
                       kv_bstride, sl2);
  }
  return hipGetLastError();
}

}  // namespace tair
