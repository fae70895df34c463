// Flash-style attention, head dim 64, bf16 in / fp32 softmax / bf16 out, gfx950 MFMA 16x16x32.
//
// Semantics = attention.py:168-216 (SDPCrossAttention / xformers memory_efficient_attention):
// O = softmax(Q K^T * d^-1/2) V per (batch, head), no mask, no bias.  Used for the 16+7 self-
// attention layers (S = 4096/1024/256/64 tokens) and the cross-attention layers (77 context keys,
// the partial last 64-key tile masked).
//
// Structure (one workgroup = 4 waves = 64*QSETS queries of one (b, h), one KV split):
//  * S^T = K * Q^T ("swapped" product): each lane ends with 4 consecutive keys x 1 query per
//    16-key block, so the row max / row sum of softmax are lane-local plus two permlane swaps.
//  * The probabilities feed P*V as the MFMA B operand straight from registers; the key order inside
//    each 32-key step is permuted (keys 4h..4h+3 and 16+4h..16+4h+3 for lane quarter h), and the
//    V^T operand is read with the same permutation by ds_read_b64_tr_b16 from a ROW-MAJOR V tile
//    (hardware transpose; no transposed staging writes).
//  * K tile [64 keys][64 d] bf16 with the GEMM XOR swizzle chunk ^ (row & 7) (ds_read_b128
//    conflict free); V tile [64 keys][64 d] with chunk ^ (2*((row >> 1) & 3)) (the transposed
//    reads of each 32-lane half cover 8 rows x 2 chunks = all 64 banks once).
//  * K/V tiles double buffered in LDS, the next tile prefetched to registers during compute
//    (issue early / write late), one barrier per tile.
//  * KV split (flash-decoding): at B = 1 a layer has only 80..320 (b, h, 128-query) blocks for 256
//    CUs, so the keys are split over blockIdx.z; each split writes its normalised partial O (bf16)
//    and (m, l) (fp32), and attn_combine_kernel merges them. One split writes O directly.
#include "kernels.h"

namespace tair {
namespace {

constexpr int KT = 64;  // keys per tile
#include "attn_ablate.h"  // ATTN_ABL: 0 in the product (timing-only ablation builds: tools/attn_ablate.py)

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

TAIR_DEV int kswz(int row, int chunk) { return row * 64 + ((chunk ^ (row & 7)) << 3); }
TAIR_DEV int vswz(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 1) & 3) << 1)) << 3); }

// softmax exponent: the bare v_exp_f32 (TAIR_ATTN_RAWEXP=1). exp2f adds a denormal-range guard around it
// (compare, two selects, add, ldexp: 6 VALU per value, half the main loop's VALU); its only effect is on
// probabilities below 2^-126, which vanish against the row sum (>= 1) and the bf16 P operand
#ifndef TAIR_ATTN_RAWEXP
#define TAIR_ATTN_RAWEXP 1
#endif
#ifndef TAIR_ATTN_SPLIT_MIN
#define TAIR_ATTN_SPLIT_MIN 32  // key tiles below which attention_plan does not split the keys
#endif
#ifndef TAIR_ATTN_WPE
#define TAIR_ATTN_WPE 2  // __launch_bounds__ minimum waves per SIMD
#endif
TAIR_DEV float sm_exp2(float x) {
#if TAIR_ATTN_RAWEXP
  return __builtin_amdgcn_exp2f(x);
#else
  return exp2f(x);
#endif
}

TAIR_DEV float xmax16(float x) {  // max(x[l], x[l ^ 16])
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
TAIR_DEV float xmax32(float x) {  // max(x[l], x[l ^ 32])
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
TAIR_DEV float xsum16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
TAIR_DEV float xsum32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

TAIR_DEV s16x4 tr_read(const bf16* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p); }

template <int QSETS, bool MASK>
__global__ __launch_bounds__(256, TAIR_ATTN_WPE) void attn_kernel(const AttnGroup P, int H, int Sq, int Skv, float c,
                                                      int kv_split, int nsplit, int ink) {
  // XCD-aware block order: the hardware deals workgroups round-robin over the 8 XCDs, so consecutive
  // (query-block, head, split) indices are remapped to one XCD: the query blocks of a (batch, head) then
  // read its K / V through one L2 instead of eight (gemm_kern.h xcd_remap, m-fastest form)
  int bxq, bhy, bzs;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const int nwg = gx * gy * gridDim.z;
    const int orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int qq = nwg >> 3, rr = nwg & 7, xcd = orig & 7;
    const int id = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
    bxq = id % gx;
    const int rest = id / gx;
    bhy = rest % gy;
    bzs = rest / gy;
  }
  const int grp = bzs / nsplit;  // grouped launch: which independent attention
  AttnArgs A = P.g[grp];
  // every field in registers, loaded as one batch (an empty asm over all of them: the compiler otherwise
  // rematerialises kernel-argument loads at their uses, one s_load + lgkmcnt(0) round trip each); pointers
  // pinned as global address-space pointers (a generic one out of an asm would make every access flat_*)
  typedef __attribute__((address_space(1))) const bf16* gcb;
  typedef __attribute__((address_space(1))) bf16* gb;
  typedef __attribute__((address_space(1))) char* gc;
  gcb aq = (gcb)A.q, ak = (gcb)A.k, av = (gcb)A.v;
  gb ao = (gb)A.o;
  gc aws = (gc)A.ws;
  typedef __attribute__((address_space(1))) int* gi;
  gi atk = (gi)A.tickets;
  TAIR_PIN_ASM("" : "+s"(aq), "+s"(A.ldq), "+s"(ak), "+s"(A.ldk), "+s"(av), "+s"(A.ldv), "+s"(ao), "+s"(A.ldo),
               "+s"(A.kv_bstride), "+s"(aws), "+s"(atk));
  A.q = (const bf16*)aq; A.k = (const bf16*)ak; A.v = (const bf16*)av; A.o = (bf16*)ao; A.ws = (void*)aws;
  A.tickets = (int*)atk;
  const bf16* __restrict__ q = A.q;
  const bf16* __restrict__ k = A.k;
  const bf16* __restrict__ v = A.v;
  bf16* __restrict__ o = A.o;
  const int ldq = A.ldq, ldk = A.ldk, ldv = A.ldv, ldo = A.ldo, kv_bstride = A.kv_bstride;
  bf16* __restrict__ opart = nsplit > 1 ? (bf16*)A.ws : nullptr;
  float* __restrict__ mlpart =
      nsplit > 1 ? (float*)((char*)A.ws + (size_t)nsplit * (gridDim.y / H) * Sq * H * 64 * 2) : nullptr;
  __shared__ __attribute__((aligned(16))) bf16 sK[2][KT * 64];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][KT * 64];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hi = lane >> 4, lo = lane & 15;
  const int bh = bhy;
  const int b = bh / H, h = bh - b * H;
  const int split = bzs - grp * nsplit;
  const int kbeg = split * kv_split;
  const int kend = min(Skv, kbeg + kv_split);
  const int q0 = bxq * (64 * QSETS) + wid * (16 * QSETS);

  // Q^T fragments (MFMA B operand): lane holds Q[q = lo][d = 32s + 8hi .. +7]
  bf16x8 qf[QSETS][2];
#pragma unroll
  for (int qs = 0; qs < QSETS; ++qs) {
    const int qi = min(q0 + qs * 16 + lo, Sq - 1);
    const bf16* qr = q + ((size_t)b * Sq + qi) * ldq + h * 64;
#pragma unroll
    for (int s = 0; s < 2; ++s) qf[qs][s] = *(const bf16x8*)(qr + 32 * s + 8 * hi);
  }

  const bf16* kb = k + (size_t)b * kv_bstride * ldk + h * 64;
  const bf16* vb = v + (size_t)b * kv_bstride * ldv + h * 64;

  // staging: 64 keys x 8 chunks = 512 chunks per operand, 2 per thread; rows past kend re-read
  // the last valid key (finite data, masked to p = 0)
  const int srow = tid >> 3, schunk = tid & 7;
  u32x4 rk[2], rv[2];
  auto gload_k = [&](int t0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) rk[i] = *(const u32x4*)(kb + (size_t)min(t0 + srow + 32 * i, kend - 1) * ldk + schunk * 8);
  };
  auto gload_v = [&](int t0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) rv[i] = *(const u32x4*)(vb + (size_t)min(t0 + srow + 32 * i, kend - 1) * ldv + schunk * 8);
  };
  auto sstore_k = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *(u32x4*)(&sK[buf][kswz(srow + 32 * i, schunk)]) = rk[i];
  };
  auto sstore_v = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *(u32x4*)(&sV[buf][vswz(srow + 32 * i, schunk)]) = rv[i];
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

  // per-lane transposed-read offsets (elements) of V rows 4hi + (lo >> 2) (+16), d = 16db + 4(lo & 3)
  int voff[2][4];
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int row = 16 * e + 4 * hi + (lo >> 2);
      const int chunk = 2 * db + ((lo & 3) >> 1);
      voff[e][db] = vswz(row, chunk) + 4 * (lo & 1);  // + 32 rows per s step: same swizzle (row & 7)
    }

  typedef f32x4 Sblk[QSETS][4];
  // S^T blocks: sacc[qs][kb][r] = S[q = lo][key = 16kb + 4hi + r]
  auto qk = [&](const bf16* Ks, Sblk& sacc) __attribute__((always_inline)) {
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
          if constexpr (!(ATTN_ABL & 2))
            sacc[qs][kb4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qs][s], sacc[qs][kb4], 0, 0, 0);
          else
            sacc[qs][kb4] += f32x4{1.f, 1.f, 1.f, 1.f};
      }
    }
  };

  // online softmax per query in base 2: p = 2^(s*c - m), m tracked in scaled units; rescales O and l
  auto softmax = [&](Sblk& sacc, int key0, bf16x8 (&pf)[QSETS][2]) __attribute__((always_inline)) {
    const bool partial_tile = MASK && (key0 + KT > kend);
#pragma unroll
    for (int qs = 0; qs < QSETS; ++qs) {
      if (partial_tile) {
#pragma unroll
        for (int kb4 = 0; kb4 < 4; ++kb4)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (key0 + kb4 * 16 + hi * 4 + r >= kend) sacc[qs][kb4][r] = -INFINITY;
      }
      float mx = fmaxf(fmaxf(sacc[qs][0][0], sacc[qs][0][1]), fmaxf(sacc[qs][0][2], sacc[qs][0][3]));
#pragma unroll
      for (int kb4 = 1; kb4 < 4; ++kb4)
        mx = fmaxf(mx, fmaxf(fmaxf(sacc[qs][kb4][0], sacc[qs][kb4][1]), fmaxf(sacc[qs][kb4][2], sacc[qs][kb4][3])));
      mx = xmax32(xmax16(mx));
      const float mold = m_run[qs];
      const float mnew = fmaxf(mold, mx * c);
      m_run[qs] = mnew;
      float ls = 0.f;
      float pv[4][4];
#pragma unroll
      for (int kb4 = 0; kb4 < 4; ++kb4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = __builtin_fmaf(sacc[qs][kb4][r], c, -mnew);
          const float pe = (ATTN_ABL & 4) ? x : sm_exp2(x);
          pv[kb4][r] = pe;
          ls += pe;
        }
      {
        const float alpha = sm_exp2(mold - mnew);
        l_run[qs] = l_run[qs] * alpha + ls;
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
          for (int r = 0; r < 4; ++r) oacc[qs][db][r] *= alpha;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pf[qs][s][r] = f2bf(pv[2 * s][r]);
          pf[qs][s][4 + r] = f2bf(pv[2 * s + 1][r]);
        }
      }
    }
  };

  // O^T += V^T P^T: A operand = V^T[d = 16db + lo][keys 32s + 4hi + j | 32s + 16 + 4hi + j]
  auto pv_mma = [&](const bf16* Vs, const bf16x8 (&pf)[QSETS][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const s16x4 v0 = tr_read(Vs + 32 * s * 64 + voff[0][db]);
        const s16x4 v1 = tr_read(Vs + 32 * s * 64 + voff[1][db]);
        const s16x4 vv[2] = {v0, v1};
        bf16x8 vf;
        __builtin_memcpy(&vf, vv, 16);
#pragma unroll
        for (int qs = 0; qs < QSETS; ++qs)
          if constexpr (!(ATTN_ABL & 8))
            oacc[qs][db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qs][s], oacc[qs][db], 0, 0, 0);
          else
            oacc[qs][db][0] += (float)vf[0] + (float)pf[qs][s][0];
      }
    }
  };

  const int ntiles = (kend - kbeg + KT - 1) / KT;
  gload_k(kbeg);
  gload_v(kbeg);
  sstore_k(0);
  sstore_v(0);
  // the Q fragments' loads complete here, before the loop: otherwise the wait for them that the compiler
  // places at their first use inside the loop (static, so executed every iteration) also waits for that
  // iteration's K / V prefetch, and the prefetch hides nothing (s_waitcnt vmcnt(1) / vmcnt(0) between the
  // QK^T MFMAs of every tile)
#pragma unroll
  for (int qs = 0; qs < QSETS; ++qs)
#pragma unroll
    for (int s = 0; s < 2; ++s) asm volatile("" ::"v"(qf[qs][s]));
  __syncthreads();
  int buf = 0;
  for (int t = 0; t < ntiles; ++t) {
    const bool more = t + 1 < ntiles && !(ATTN_ABL & 1);
    const int key0 = kbeg + t * KT;
    if (more) {
      gload_k(key0 + KT);
      gload_v(key0 + KT);
    }
    Sblk sacc;
    qk(sK[buf], sacc);
    bf16x8 pf[QSETS][2];
    softmax(sacc, key0, pf);
    pv_mma(sV[buf], pf);
    if (more) {
      sstore_k(buf ^ 1);
      sstore_v(buf ^ 1);
    }
    __syncthreads();
    buf ^= 1;
  }

#pragma unroll
  for (int qs = 0; qs < QSETS; ++qs) {
    const float lt = xsum32(xsum16(l_run[qs]));
    const float inv = 1.f / lt;
    const int qi = q0 + qs * 16 + lo;
    if (qi < Sq) {
      const size_t row = (size_t)b * Sq + qi;
      bf16* orow;
      if (opart) {
        const size_t prow = (size_t)split * (gridDim.y / H) * Sq + row;  // [split][B*Sq] rows
        orow = opart + prow * (H * 64) + h * 64;
        if (hi == 0) {
          float2* ml = (float2*)mlpart + prow * H + h;
          const float2 mv = make_float2(m_run[qs], lt);
          if (ink)  // write-through: the merging split may run on another XCD
            __hip_atomic_store((unsigned long long*)ml, __builtin_bit_cast(unsigned long long, mv), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          else
            *ml = mv;
        }
      } else {
        orow = o + row * ldo + h * 64;
      }
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        bf16x4 w = {f2bf(oacc[qs][db][0] * inv), f2bf(oacc[qs][db][1] * inv),
                    f2bf(oacc[qs][db][2] * inv), f2bf(oacc[qs][db][3] * inv)};
        if (opart && ink)
          __hip_atomic_store((unsigned long long*)(orow + db * 16 + hi * 4), __builtin_bit_cast(unsigned long long, w),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          *(bf16x4*)(orow + db * 16 + hi * 4) = w;
      }
    }
  }
  if (!(opart && ink)) return;
  // in-kernel merge of the key splits (attn_combine_kernel's arithmetic and order: the same bits): every split
  // stores its partial rows write-through, drains them and takes the (query block, head) ticket; the last to
  // arrive resets it and merges all splits' rows, each lane the 16 d values of its rows it wrote itself
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    int* tk = A.tickets + 32 * ((grp * gridDim.y + bh) * gridDim.x + bxq);  // one 128-byte line each
    const int tkt = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = tkt == nsplit - 1;
    if (s_last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  const size_t rows_all = (size_t)(gridDim.y / H) * Sq;
  // sc1 buffer loads (Guideline 16 R1: no acquire fence needed for write-through data), every split's (m, l)
  // and then four splits' partial rows at a time in flight (relaxed atomic loads were issued one round trip
  // at a time: the merge then cost more than the merge launch it replaces)
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const __amdgpu_buffer_rsrc_t rml = __builtin_amdgcn_make_buffer_rsrc((void*)mlpart, 0,
                                                                       (int)(nsplit * rows_all * H * 8), 0x00020000);
  const __amdgpu_buffer_rsrc_t rop = __builtin_amdgcn_make_buffer_rsrc((void*)opart, 0,
                                                                       (int)(nsplit * rows_all * H * 128), 0x00020000);
  constexpr int SMAX = 16;  // attention_plan keeps splits <= 16
#pragma unroll
  for (int qs = 0; qs < QSETS; ++qs) {
    const int qi = q0 + qs * 16 + lo;
    if (qi >= Sq) continue;
    const size_t row = (size_t)b * Sq + qi;
    float2 ml[SMAX];
    static_for<0, SMAX>([&](auto P_) {
      constexpr int pp = decltype(P_)::value;
      if (pp < nsplit)
        ml[pp] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(
                                                rml, (int)((((size_t)pp * rows_all + row) * H + h) * 8), 0, 16 /* sc1 */));
    });
    float M = -INFINITY;
    static_for<0, SMAX>([&](auto P_) {
      if (decltype(P_)::value < nsplit) M = fmaxf(M, ml[decltype(P_)::value].x);
    });
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
    float W = 0.f;
    static_for<0, SMAX / 4>([&](auto G_) {
      constexpr int g0 = 4 * decltype(G_)::value;
      if (g0 >= nsplit) return;
      bf16x4 x[4][4];
      static_for<0, 4>([&](auto Q_) {
        constexpr int pp = g0 + decltype(Q_)::value;
        if (pp < nsplit) {
          const int base = (int)((((size_t)pp * rows_all + row) * H + h) * 128 + hi * 8);
#pragma unroll
          for (int db = 0; db < 4; ++db)
            x[decltype(Q_)::value][db] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(
                                                                        rop, base + db * 32, 0, 16 /* sc1 */));
        }
      });
      static_for<0, 4>([&](auto Q_) {
        constexpr int pp = g0 + decltype(Q_)::value;
        if (pp < nsplit) {
          const float w = exp2f(ml[pp].x - M) * ml[pp].y;
          W += w;
#pragma unroll
          for (int db = 0; db < 4; ++db)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[db * 4 + r] += w * bf2f(x[decltype(Q_)::value][db][r]);
        }
      });
    });
    const float inv = 1.f / W;
    bf16* orow = o + row * ldo + h * 64;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      bf16x4 y = {f2bf(acc[db * 4] * inv), f2bf(acc[db * 4 + 1] * inv), f2bf(acc[db * 4 + 2] * inv),
                  f2bf(acc[db * 4 + 3] * inv)};
      *(bf16x4*)(orow + db * 16 + hi * 4) = y;
    }
  }
}

// O = sum_p w_p O_p / sum_p w_p, w_p = 2^(m_p - M) l_p; one thread per (row, head, 8 d values)
__global__ __launch_bounds__(256) void attn_combine_kernel(const AttnGroup G, int P, int rows, int H) {
  const AttnArgs& A = G.g[blockIdx.y];
  const bf16* __restrict__ opart = (const bf16*)A.ws;
  const float* __restrict__ mlpart = (const float*)((const char*)A.ws + (size_t)P * rows * H * 64 * 2);
  bf16* __restrict__ o = A.o;
  const int ldo = A.ldo;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int total = rows * H * 8;
  if (idx >= total) return;
  const int ch = idx & 7;
  const int rh = idx >> 3;
  const int h = rh % H, row = rh / H;
  const float2* ml = (const float2*)mlpart;
  float M = -INFINITY;
  for (int p = 0; p < P; ++p) M = fmaxf(M, ml[((size_t)p * rows + row) * H + h].x);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float W = 0.f;
  for (int p = 0; p < P; ++p) {
    const float2 e = ml[((size_t)p * rows + row) * H + h];
    const float w = exp2f(e.x - M) * e.y;
    W += w;
    const bf16x8 x = *(const bf16x8*)(opart + ((size_t)p * rows + row) * (H * 64) + h * 64 + ch * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += w * bf2f(x[j]);
  }
  const float inv = 1.f / W;
  bf16x8 y;
#pragma unroll
  for (int j = 0; j < 8; ++j) y[j] = f2bf(acc[j] * inv);
  *(bf16x8*)(o + (size_t)row * ldo + h * 64 + ch * 8) = y;
}

template <int QSETS, bool MASK>
void launch_attn(dim3 grid, hipStream_t s, const AttnGroup& P, int H, int Sq, int Skv, float c, int kv_split,
                 int nsplit, int ink) {
  hipLaunchKernelGGL((attn_kernel<QSETS, MASK>), grid, dim3(256), 0, s, P, H, Sq, Skv, c, kv_split, nsplit, ink);
}

}  // namespace

AttnPlan attention_plan(int B, int H, int Sq, int Skv, size_t ws_bytes, int force_qsets, int force_splits) {
  AttnPlan p;
  // from the MI355X sweep (tools/attn_bench.py, B = 1): 32 queries per wave once the grid has
  // >= 256 64-query blocks, then split the keys until ~1280 workgroups, keeping >= 4 tiles a split
  const int base64 = cdiv(Sq, 64) * B * H;
  // cross-attention (<= 2 key tiles): 16 queries per wave at every batch (profiles/r05_attn_q4_sweep_b64.log:
  // B = 64 4096 x 77 130 vs 145 us, 1024 x 77 61-64 vs 71, 256 x 77 35-36 vs 40)
  p.qsets = force_qsets ? force_qsets : (base64 >= 256 && Skv > 2 * KT ? 2 : 1);
  const int blocks = cdiv(Sq, 64 * p.qsets) * B * H;
  const int ktiles = cdiv(Skv, KT);
  int splits = force_splits ? force_splits : (1280 + blocks / 2) / blocks;
  // below 32 key tiles the merge launch costs more than the split saves (profiles/r05_attn_b1_sweep*.log,
  // B = 1 1024 tokens: unsplit 15.3 / 15.9 us, 4 splits + merge 17.4 / 18.0; 4096 tokens: 8 splits 45.8 vs 65)
  splits = std::max(1, std::min(splits, force_splits ? ktiles : (ktiles >= TAIR_ATTN_SPLIT_MIN ? ktiles / 4 : 1)));
  // workspace: per split, rows x H x (64 bf16 + 2 fp32)
  const size_t per_split = (size_t)B * Sq * H * (64 * 2 + 8);
  if (splits > 1 && per_split * splits > ws_bytes) splits = (int)std::max<size_t>(1, ws_bytes / per_split);
  const int tiles_per_split = cdiv(ktiles, splits);
  p.kv_split = tiles_per_split * KT;
  p.splits = cdiv(ktiles, tiles_per_split);
  return p;
}

hipError_t attention_grouped(const AttnArgs* a, int n, int B, int H, int Sq, int Skv, float scale, hipStream_t s,
                             int force_qsets, int force_splits) {
  if (Sq <= 0 || Skv <= 0) return hipSuccess;
  if (n < 1 || n > MAX_GROUP) { set_error("attention: group of %d", n); return hipErrorInvalidValue; }
  const float c = scale * 1.4426950408889634f;
  size_t ws_bytes = (size_t)-1;
  for (int i = 0; i < n; ++i) ws_bytes = std::min(ws_bytes, a[i].ws ? a[i].ws_bytes : (size_t)0);
  const AttnPlan p = attention_plan(B, H, Sq, Skv, ws_bytes, force_qsets, force_splits);
  if (p.qsets != 1 && p.qsets != 2) return hipErrorInvalidValue;
  AttnGroup P;
  for (int i = 0; i < MAX_GROUP; ++i) P.g[i] = a[i < n ? i : 0];
  const dim3 grid(cdiv(Sq, 64 * p.qsets), B * H, p.splits * n);
  const bool mask = (Skv % KT) != 0;
  // key splits merged in-kernel by the last split of each (query block, head) when every lane has tickets
  // for all its blocks (one 128-byte line each), else by attn_combine_kernel
  // (the in-kernel merge addresses the partials through 32-bit buffer-resource ranges: nsplit * rows * H * 128
  // bytes must fit, else the merge kernel, whose offsets are size_t, takes them)
  bool ink = p.splits > 1 && p.splits <= 16 && (long long)p.splits * B * Sq * H * 128 < (1LL << 31);
  for (int i = 0; i < n && ink; ++i)
    ink = a[i].tickets && (long)grid.x * grid.y * n * 32 <= a[i].tickets_cap;
#define TAIR_ATTN(QS, MK) launch_attn<QS, MK>(grid, s, P, H, Sq, Skv, c, p.kv_split, p.splits, ink ? 1 : 0)
  if (p.qsets == 2) {
    if (mask) TAIR_ATTN(2, true); else TAIR_ATTN(2, false);
  } else {
    if (mask) TAIR_ATTN(1, true); else TAIR_ATTN(1, false);
  }
#undef TAIR_ATTN
  if (p.splits > 1 && !ink) {
    const int rows = B * Sq;
    const int total = rows * H * 8;
    hipLaunchKernelGGL(attn_combine_kernel, dim3(cdiv(total, 256), n), dim3(256), 0, s, P, p.splits, rows, H);
  }
  return hipGetLastError();
}

hipError_t attention(const bf16* q, int ldq, const bf16* k, int ldk, const bf16* v, int ldv, bf16* o,
                     int ldo, int B, int H, int Sq, int Skv, int kv_bstride, float scale, hipStream_t s,
                     void* ws, size_t ws_bytes, int force_qsets, int force_splits) {
  AttnArgs a{q, ldq, k, ldk, v, ldv, o, ldo, kv_bstride, ws, ws ? ws_bytes : 0};
  return attention_grouped(&a, 1, B, H, Sq, Skv, scale, s, force_qsets, force_splits);
}

}  // namespace tair
