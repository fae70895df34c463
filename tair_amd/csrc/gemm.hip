// Host side of the bf16 MFMA GEMM: tile / split-K planner, grouped launcher, split-K reduce.
#include <algorithm>

#include "gemm_kern.h"
#ifndef TAIR_BATCH_XCD
#define TAIR_BATCH_XCD 1  // round-6 batched-grid tile order + split recompute (0: round-5 rules, A/B builds only)
#endif

namespace tair {
namespace {

// Sum of the split-K slabs + epilogue (+ GroupNorm statistics of the result).  Block = RB rows x
// CB4 column quads; every thread keeps ONE column quad (fixed groups) and walks rows, so its
// statistics accumulate in registers.  S (the split count) is a template parameter: the 2 x S slab
// loads of a row pair are unrolled and all in flight before the first add (a runtime split loop
// waited one memory latency per split: 7.4 us average per launch at B = 1).
template <int S>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmGroup P, int RB, int CB4) {
  const EpiArgs p = epi_args(P.g[blockIdx.z]);  // one batch of kernel-argument loads, kept in registers
  __shared__ double red[4 * STAT_NG];
  const int n4 = (p.N + 3) / 4;
  const size_t slab = (size_t)p.M * p.N;
  const bool vec = (p.N & 3) == 0;
  const bool stats = p.st[0].acc != nullptr;
  const int rpp = 256 / CB4;
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * RB;
  const int c4_0 = blockIdx.y * CB4;
  if (stats) {
    for (int i = t; i < 4 * STAT_NG; i += 256) red[i] = 0.0;
    __syncthreads();
  }
  const int c4 = c4_0 + t % CB4;
  const int n = c4 * 4;
  const bool active = t < rpp * CB4 && c4 < n4;
  Stat4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
  if (active) {
    // two rows per iteration: both rows' slab loads are in flight before the first add
    for (int r = t / CB4; r < RB; r += 2 * rpp) {
      const int mA = r0 + r, mB = r0 + r + rpp;
      if (mA >= p.M) break;
      const bool okB = (r + rpp < RB) && mB < p.M;
      f32x4 accA = {0.f, 0.f, 0.f, 0.f}, accB = {0.f, 0.f, 0.f, 0.f};
      const float* srcA = p.partial + (size_t)mA * p.N + n;
      const float* srcB = p.partial + (size_t)(okB ? mB : mA) * p.N + n;
      if (vec) {
        f32x4 xa[S], xb[S];
#pragma unroll
        for (int z = 0; z < S; ++z) {
          xa[z] = *(const f32x4*)(srcA + z * slab);
          xb[z] = *(const f32x4*)(srcB + z * slab);
        }
#pragma unroll
        for (int z = 0; z < S; ++z) {
          accA += xa[z];
          accB += xb[z];
        }
      } else {
        for (int z = 0; z < S; ++z)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < p.N) {
              accA[e] += srcA[z * slab + e];
              accB[e] += srcB[z * slab + e];
            }
      }
      float v[4];
      epilogue4(p, mA, n, accA, v);
      if (stats) {
        stat_add(p.st[0], n, v, a0);
        if (p.st[1].acc) stat_add(p.st[1], n, v, a1);
      }
      if (okB) {
        epilogue4(p, mB, n, accB, v);
        if (stats) {
          stat_add(p.st[0], n, v, a0);
          if (p.st[1].acc) stat_add(p.st[1], n, v, a1);
        }
      }
    }
  }
  if (!stats) return;
  if (active) {
    lds_stat_add(red, p.st[0], n, (p.st[0].c_off + 4 * c4_0) / p.st[0].cg, a0);
    if (p.st[1].acc) lds_stat_add(red + 2 * STAT_NG, p.st[1], n, (p.st[1].c_off + 4 * c4_0) / p.st[1].cg, a1);
  }
  __syncthreads();
  stat_flush(p, red, r0 / p.st[0].hw, 4 * c4_0, min(p.N, 4 * (c4_0 + CB4)), (blockIdx.x + blockIdx.y) & (STAT_REPL - 1));
}

}  // namespace

// Device fault counter of the GEMM kernels (GemmGroup.fault), one per device, allocated by gemm_init.
static int* g_fault[16] = {};
static int* fault_word() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  return g_fault[dev];
}

hipError_t gemm_fault_count(int* count, bool reset) {
  *count = 0;
  int* f = fault_word();
  if (!f) return hipSuccess;
  TAIR_HIP_CHECK(hipMemcpy(count, f, sizeof(int), hipMemcpyDeviceToHost));
  if (reset && *count) TAIR_HIP_CHECK(hipMemset(f, 0, sizeof(int)));
  return hipSuccess;
}

// Kernel attributes are set once, outside any stream capture (hipFuncSetAttribute is not a
// capturable operation).
hipError_t gemm_init() {
  {
    int dev = 0;
    TAIR_HIP_CHECK(hipGetDevice(&dev));
    if (dev >= 0 && dev < 16 && !g_fault[dev]) {
      TAIR_HIP_CHECK(hipMalloc(&g_fault[dev], sizeof(int)));
      TAIR_HIP_CHECK(hipMemset(g_fault[dev], 0, sizeof(int)));
    }
  }
  static bool done = false;
  if (done) return hipSuccess;
  TAIR_HIP_CHECK((gemm_set_attrs<A_DENSE, SET_SMALL>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_DENSE, SET_BIG>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3, SET_SMALL>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3, SET_BIG>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_S2, SET_SMALL>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_S2, SET_BIG>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_UP, SET_SMALL>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_UP, SET_BIG>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_SMALLC, SET_REG>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_DENSE, SET_RING>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3, SET_RING>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_S2, SET_RING>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_UP, SET_RING>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_DENSE, SET_PHASE>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_DENSE, SET_SHALLOW>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3, SET_PHASE>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_S2, SET_PHASE>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3_UP, SET_PHASE>()));
  TAIR_HIP_CHECK(set_attrs_f8<A_DENSE>());
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3, SET_F8>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3, SET_HALO>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_DENSE, SET_DEEP>()));
  TAIR_HIP_CHECK((gemm_set_attrs<A_CONV3, SET_DEEP>()));
  done = true;
  return hipSuccess;
}

namespace {
hipError_t launch_set(int amode, GemmGroup& P, int n, int bm, int bn, int splits, int kern, hipStream_t s) {
  if (kern == GEMM_KERN_SHALLOW) return gemm_set_launch<A_DENSE, SET_SHALLOW>(P, n, bm, bn, splits, s);
  if (kern == GEMM_KERN_HALO) return gemm_set_launch<A_CONV3, SET_HALO>(P, n, bm, bn, splits, s);
  if (kern == GEMM_KERN_DEEP)
    return amode == A_DENSE ? gemm_set_launch<A_DENSE, SET_DEEP>(P, n, bm, bn, splits, s)
                            : gemm_set_launch<A_CONV3, SET_DEEP>(P, n, bm, bn, splits, s);
  if (kern == GEMM_KERN_PHASE) {
    switch (amode) {
      case A_DENSE: return gemm_set_launch<A_DENSE, SET_PHASE>(P, n, bm, bn, splits, s);
      case A_CONV3: return gemm_set_launch<A_CONV3, SET_PHASE>(P, n, bm, bn, splits, s);
      case A_CONV3_S2: return gemm_set_launch<A_CONV3_S2, SET_PHASE>(P, n, bm, bn, splits, s);
      default: return gemm_set_launch<A_CONV3_UP, SET_PHASE>(P, n, bm, bn, splits, s);
    }
  }
  if (bm < 0) {  // BK = 32 deep-ring tile
    switch (amode) {
      case A_DENSE: return gemm_set_launch<A_DENSE, SET_RING>(P, n, -bm, bn, splits, s);
      case A_CONV3: return gemm_set_launch<A_CONV3, SET_RING>(P, n, -bm, bn, splits, s);
      case A_CONV3_S2: return gemm_set_launch<A_CONV3_S2, SET_RING>(P, n, -bm, bn, splits, s);
      default: return gemm_set_launch<A_CONV3_UP, SET_RING>(P, n, -bm, bn, splits, s);
    }
  }
  const bool big = gemm_tile_is_big(bm, bn);
  switch (amode) {
    case A_DENSE:
      return big ? gemm_set_launch<A_DENSE, SET_BIG>(P, n, bm, bn, splits, s)
                 : gemm_set_launch<A_DENSE, SET_SMALL>(P, n, bm, bn, splits, s);
    case A_CONV3:
      return big ? gemm_set_launch<A_CONV3, SET_BIG>(P, n, bm, bn, splits, s)
                 : gemm_set_launch<A_CONV3, SET_SMALL>(P, n, bm, bn, splits, s);
    case A_CONV3_S2:
      return big ? gemm_set_launch<A_CONV3_S2, SET_BIG>(P, n, bm, bn, splits, s)
                 : gemm_set_launch<A_CONV3_S2, SET_SMALL>(P, n, bm, bn, splits, s);
    case A_CONV3_UP:
      return big ? gemm_set_launch<A_CONV3_UP, SET_BIG>(P, n, bm, bn, splits, s)
                 : gemm_set_launch<A_CONV3_UP, SET_SMALL>(P, n, bm, bn, splits, s);
    default:
      return gemm_set_launch<A_CONV3_SMALLC, SET_REG>(P, n, bm, bn, splits, s);
  }
}
}  // namespace

// Tile / split-K choice (tools/gemm_probe.py on MI355X at B = 16, profiles/r02_gemm_probe_*.log).
// * Short-K linears (K <= 640, proj / q / qkv / GEGLU-in at 64^2 and 32^2): 64x64 tiles at every
//   size; several workgroups per CU overlap one another's prologue and epilogue, which a one-per-CU
//   large tile cannot (ff1 at B = 16: 64x64 414 us vs 128x256 446, 128x320 479, 256x256 482); from
//   M >= 16384 the 2-stage variant (4-5 workgroups per CU: ff1 389 -> 318 us).
// * Large grids otherwise: 128x320 tiles when 320 | N (every UNet channel count), 128x256 else; the
//   4-phase 256x320 kernel for the widest projections (N >= 5120: ff1 at 16^2, 612 vs 536 TF/s).
//   K is not split once the grid fills a round of CUs (a 4-way in-kernel split of conv64 at B = 16:
//   238 us vs 177 unsplit); below that, split to ~256 workgroups.
// * Small grids (the B = 1 network) keep 4-wave 64-row tiles and split K: convs until ~400
//   workgroups (>= 3 K-tiles per split), linears until ~240 (>= 5 K-tiles per split).
// fp8 (a.f8): the e4m3 tiles 64x64 / 64x128 / 128x128 / 128x256 / 128x320.  A K-tile holds 128 values, so
// the fp8 linears are all short-K (qkv/q2: 3 K-tiles at C = 320, ff1: 3-10): batched grids take the
// widest tile that still gives >= 256 workgroups; small (B = 1) grids split K like the bf16 linears.
// halo tiles (conv_halo_kernel): bf16 stride-1 3x3 convs without a K-extension over whole image rows of
// width 16 / 32 / 64 (256-pixel tiles never straddle two images)
bool conv_halo_ok(const GemmArgs& a) {
  static const bool on = [] { const char* e = getenv("TAIR_HALO"); return !e || atoi(e) != 0; }();
  return on && !a.f8 && a.amode == A_CONV3 && a.Kx == 0 && a.C % 64 == 0 && a.K == 9 * a.C && a.H == a.Ho &&
         a.W == a.Wo && (a.W == 64 || a.W == 32 || a.W == 16) && (a.H * a.W) % 256 == 0 && a.M % 256 == 0 &&
         a.lda % 8 == 0;
}

bool halo_tile_built(int W, int bm, int bn) {
  if (bm != 256) return false;
  if (W == 64) return bn == 64 || bn == 128 || bn == 160;
  return (W == 32 || W == 16) && (bn == 128 || bn == 160 || bn == 192);
}

void gemm_plan(const GemmArgs& a, int* bm, int* bn, int* splits, int* kern) {
  const int ktiles = (a.K + a.Kx) / BK;
  const bool conv = a.amode != A_DENSE;
  *splits = 1;
  if (kern) *kern = GEMM_KERN_TILE;
  // halo tiles (one 256-pixel tile per CU), measured per shape against the tile kernels
  // (profiles/r04_halo_probe_pipe.log): 256x160 at M >= 4096 rows on 16/32-wide and M >= 16384 on 64-wide
  // images (5-14% faster at B = 16 / 64), split over 64-channel chunks only below 256 tiles (in the network
  // the fp32 slabs of a split 64x64-level conv cost more than the halo saves: profiles/r04_b64_launch_*);
  // the B <= 3 levels and narrow outputs (conv_out, N = 4) stay on the tile kernels: 256x64 halo tiles with
  // split-K at the B = 1 64x64 level were faster in isolation but need the reduce launch that the 64-row
  // tile plans fold in-kernel (B = 1 step +0.15 ms, profiles/r04_step_summary_b1.txt)
  if (conv_halo_ok(a) && a.N >= 64 && (a.W == 64 ? a.M >= 16384 : a.M >= 4096)) {
    *bm = 256;
    *bn = 160;
    const long tiles = (long)cdiv(a.M, 256) * cdiv(a.N, *bn);
    *splits = std::max(1, std::min((int)((256 + tiles - 1) / tiles), std::min(a.C / 64, 16)));
    if (kern) *kern = GEMM_KERN_HALO;
    return;
  }
  if (a.f8) {
    // batched short-K linears (K <= 640 values, a.K counts byte pairs): the bf16 rule, 2-stage 64x64 tiles
    if (!conv && 2 * (a.K + a.Kx) <= 640 && a.M >= 16384) {
      *bm = 64;
      *bn = 64;
      if (kern) *kern = GEMM_KERN_SHALLOW;
      return;
    }
    if (a.M >= 4096) {
      // the widest 128-row tile whose column waste is least (320 | N for the UNet's convs and linears), as
      // long as the grid keeps >= 256 workgroups
      *bm = 128;
      int best = 128;
      long waste = (long)cdiv(a.N, 128) * 128 - a.N;
      for (int w : {256, 320}) {
        const long ws = (long)cdiv(a.N, w) * w - a.N;
        if (ws <= waste && (long)cdiv(a.M, 128) * cdiv(a.N, w) >= 256) {
          best = w;
          waste = ws;
        }
      }
      *bn = best;
      if ((long)cdiv(a.M, 128) * cdiv(a.N, *bn) >= 256) return;
    }
    *bm = 64;
    *bn = a.N >= 1024 ? 128 : 64;
    const long tiles = (long)cdiv(a.M, 64) * cdiv(a.N, *bn);
    int s = (int)((240 + tiles / 2) / tiles);
    if (s > ktiles / 2) s = ktiles / 2;
    if (s > 16) s = 16;
    *splits = s < 1 ? 1 : s;
    return;
  }
  const bool short_k = !conv && a.K + a.Kx <= 640;
  // wide batched linears (GEGLU-in at every level, q|k|v at 32x32): 256x128 tiles (8 waves, pipelined
  // loop) -- 3-23% faster than the 2-stage 64x64 tiles / the 4-phase kernel on these shapes
  // (profiles/r04_shortk_probe.log: GEGLU-in at B = 64 64x64 / 32x32 / 16x16 1405 / 1154 / 797 ->
  // 1374 / 884 / 652 us); plans that produce LayerNorm row statistics keep <= 128-row tiles.  Round 6: where
  // 256 | N (GEGLU-in at every level) the 256x256 tiles (8 waves, 2-stage ring) take over: 1383 / 856 / 653 ->
  // 1097 / 718 / 536 us at B = 64 (profiles/r06_sweep_b64_ff1.log; the 256x128 plans' rows are re-read from
  // beyond L2 once the 20-40 n-tiles of an m-tile outlast their L2 lines)
  if (!conv && !a.rst && a.N >= 1920 && a.N % 128 == 0 &&
      ((short_k && a.M >= 16384) || (!short_k && a.N >= 5120 && a.M >= 4096))) {
    *bm = 256;
    *bn = TAIR_BATCH_XCD && a.N % 256 == 0 ? 256 : 128;
    return;
  }
  if (a.amode != A_CONV3_SMALLC && !short_k && a.M >= 2048) {
    const bool phase = !conv && a.N >= 5120 && a.N % 320 == 0 && a.M >= 4096;
    const int wide = phase || a.N % 320 == 0 ? 320 : (a.N >= 256 ? 256 : 0);
    if (wide) {
      const int BMc = phase ? 256 : 128;
      const long tiles = (long)cdiv(a.M, BMc) * cdiv(a.N, wide);
      if (tiles >= 48) {
        int s = 1;
        if (tiles < 200 && !phase && a.act != 2) {
          s = (int)(256 / tiles);
          if (s > 6) s = 6;
          if (s > ktiles / 6) s = ktiles / 6;
          if (s < 1) s = 1;
        }
        *bm = BMc;
        *bn = wide;
        *splits = s;
        if (kern && phase) *kern = GEMM_KERN_PHASE;
        return;
      }
    }
  }
  // wide tiles for the B >= 64 short-K linears (round 5 sweep, profiles/r05_sk_plans_b64.log: q|k|v 64^2 596 -> 413 us
  // on 128x256, proj 64^2 197 -> 157 on 256x160, proj 32^2 108 -> 88 on 256x128; at B = 16 the 64x64 tiles stay
  // ahead, r04_shortk_probe.log); plain epilogues only, LayerNorm-statistics producers keep <= 128-row tiles.
  // Round 5 kept them off for a parity drift that was not in these kernels (they are bitwise the 64x64 plan,
  // tests/test_lnfold_gpu.py) but in the fold decision (gemm_rowstats_ok); configs[2] 2.857 -> 2.883 Mpix/s
  // paired (profiles/r06_cfg2_skw_*.log)
  // round 6: the B >= 64 short-K linears whose epilogue the register-staged path takes (bias, folded LayerNorm, a
  // bf16 residual in place, LayerNorm row statistics; gemm_kern.h epilogue_regstage) on 128x320 tiles where 320 | N:
  // proj_in 64^2 / 32^2 216 / 129 -> 160 / 90 us, the out-projections 230 / 135 -> 207 / 107, q 158 / 91 -> 144 / 85
  // at B = 64 in isolation (profiles/r06_sk320_probe.log); TAIR_SK320=0 keeps the round-5/6 plans (A/B)
  static const bool sk320_env = [] { const char* e = getenv("TAIR_SK320"); return !e || atoi(e) != 0; }();
  const bool regstage_epi = !a.emb && !a.res_lo && !a.out_lo && !a.st[0].acc && !a.out_split && !a.out_f32 &&
                            a.act == 0 && !a.f8 && a.bias;
  if (sk320_env && short_k && regstage_epi && a.M >= 65536 && a.N % 320 == 0) {
    *bm = 128;
    *bn = 320;
    return;
  }
  const bool plain_epi = !a.res && !a.res_lo && !a.out_lo && !a.st[0].acc && !a.out_split && !a.out_f32;
  if (short_k && !a.rst && plain_epi && (a.M >= 262144 || (a.M >= 65536 && a.K + a.Kx >= 640))) {
    // 256x128 where 128 | N, 256x160 for N = 160 / 320, 128x256 else
    const int pick = a.N % 128 == 0 ? 1 : (a.N <= 320 && a.N % 160 == 0) ? 2 : 4;
    *bm = pick == 4 ? 128 : 256;
    *bn = pick == 1 ? 128 : pick == 2 ? 160 : 256;
    return;
  }
  if (short_k && a.M >= 16384) {  // batched short-K linears: 2-stage 64x64 tiles, no split
    *bm = 64;
    *bn = 64;
    if (kern) *kern = GEMM_KERN_SHALLOW;
    return;
  }
  // (round 5, with the cooperative split-K combine: profiles/r05_sweep_b1_coop.log) the stride-2 convs up to
  // 640 channels take 64-column tiles in <= 6 slices (down32 / down16: 13.4 / 14.9 vs 15.4 / 16.1 us); the linears split toward ~200
  // workgroups (lin32proj unsplit 8.1 vs 10.3 us at 2 slices) with at least 2.5 K-tiles per slice
  // (lin8proj 8 slices: 7.7 vs 8.2 us), and a long-K linear keeps >= 2 slices below a round of CUs
  // (lin32ff2: 17.0 vs 19.0 us unsplit)
  // (round 6: 128-row tiles for the 64x64-level linears and ~400-workgroup splits for FF-out were faster in
  // isolation -- GEGLU-in 35.0 -> 24.8 us, q|k|v 15.6 -> 12.2, profiles/r06_sweep_b1_lin.log -- but the B = 1 step
  // did not move (4.70 / 4.73 vs 4.69 / 4.71 ms, paired): not taken)
  const bool s2_narrow = a.amode == A_CONV3_S2 && a.N <= 640;
  const int BNc = (a.N >= 256 && (conv || a.M >= 16384) && !s2_narrow) ? 128 : 64;
  const int BMc = 64;
  const long tiles = (long)cdiv(a.M, BMc) * cdiv(a.N, BNc);
  const long target = s2_narrow ? 480 : conv ? 400 : 200;
  int s = (int)((target + tiles / 2) / tiles);
  int smax = conv ? ktiles / 3 : (2 * ktiles) / 5;
  if (s2_narrow && smax > 6) smax = 6;
  if (!conv && s < 2 && ktiles >= 32 && tiles < 256) s = 2;
  if (s > smax) s = smax;
  if (s > 16) s = 16;
  if (s < 1) s = 1;
  *bm = BMc;
  *bn = BNc;
  *splits = s;
}

bool gemm_rowstats_ok(const GemmArgs& a) {
  // planned as the row-statistics producer it would become (gemm_plan keeps producers off the > 128-row
  // plans; planning the bare linear could pick a wide plan and turn the fold off: round 5's wide-plan drift)
  static double probe_rst[2];
  GemmArgs b = a;
  if (!b.rst) b.rst = probe_rst;
  int bm, bn, s, kern;
  gemm_plan(b, &bm, &bn, &s, &kern);
  if (a.force_bm) bm = a.force_bm;
  return kern != GEMM_KERN_PHASE && (bm < 0 ? -bm : bm) <= 128 && !a.out_f32 && !a.out_split && a.act != 2 &&
         !a.st[0].acc;
}

size_t gemm_partial_elems(const GemmArgs& a) {
  int bm, bn, s;
  gemm_plan(a, &bm, &bn, &s);
  return s > 1 ? (size_t)s * a.M * a.N : 0;
}

static bool g_skip_reduce = false;  // TAIR_ABLATE bit 8 (timing experiments only)
void gemm_set_skip_reduce(bool on) { g_skip_reduce = on; }

// Largest split count combined in-kernel (splitk_combine); larger splits use splitk_reduce_kernel.
// TAIR_INK_SMAX overrides (A/B experiments; 0 or 1 = never in-kernel).
static int ink_smax() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("TAIR_INK_SMAX");
    v = e ? atoi(e) : 3;
    if (v > INK_SMAX_BUILT) v = INK_SMAX_BUILT;
  }
  return v;
}

namespace {
thread_local bool g_gemm_dry = false;  // gemm_gn_ok / gemm_plan_query: validate and plan only
thread_local int g_dry_plan[4];         // the plan the dry run would have launched (bm, bn, splits, kernel)
thread_local bool g_gn_halo_only = false;  // gemm_gn_ok: the product plans GroupNorm on load into halo tiles only
// dynamic LDS of a plan's staging memory (the GroupNorm-on-load table goes behind it)
size_t plan_lds(int kern, int bm, int bn, int W, bool halo_s2) {
  if (kern == GEMM_KERN_HALO) {
    const int hrp = W == 64 ? (bn == 64 ? 448 : 400) : W == 32 ? (bn == 128 ? 384 : 344) : (bn == 128 ? 384 : 328);
    const int st = bn == 64 ? 4 : halo_s2 ? 2 : 3;
    return (size_t)2 * hrp * 128 + (size_t)st * bn * 128;
  }
  const int st = kern == GEMM_KERN_SHALLOW ? 2 : (bm == 128 && bn == 320) || (bm == 256 && bn >= 256) ? 2 : 3;
  return (size_t)st * (bm + bn) * 128;
}
bool deep_built(int bm, int bn, int st) {
  return bm == 64 && ((bn == 64 && (st == 4 || st == 5 || st == 6 || st == 8)) || (bn == 128 && st >= 4 && st <= 6));
}
}  // namespace

bool gemm_gn_ok(const GemmArgs& a) {
  g_gemm_dry = g_gn_halo_only = true;
  const hipError_t e = gemm_grouped(&a, 1, nullptr);
  g_gemm_dry = g_gn_halo_only = false;
  return e == hipSuccess;
}

hipError_t gemm_plan_query(const GemmArgs& a, int* bm, int* bn, int* splits, int* kern) {
  g_gemm_dry = true;
  const hipError_t e = gemm_grouped(&a, 1, nullptr);
  g_gemm_dry = false;
  *bm = g_dry_plan[0];
  *bn = g_dry_plan[1];
  *splits = g_dry_plan[2];
  *kern = g_dry_plan[3];
  return e;
}

hipError_t gemm_grouped(const GemmArgs* args, int n, hipStream_t s) {
  if (!g_gemm_dry) TAIR_HIP_CHECK(gemm_init());  // (a dry planning run touches no device: CPU-testable)
  if (n < 1 || n > MAX_GROUP) {
    set_error("gemm: group of %d GEMMs (max %d)", n, MAX_GROUP);
    return hipErrorInvalidValue;
  }
  const GemmArgs& a = args[0];
  for (int i = 1; i < n; ++i) {
    const GemmArgs& b = args[i];
    if (b.M != a.M || b.N != a.N || b.K != a.K || b.Kx != a.Kx || b.amode != a.amode || b.C != a.C ||
        b.H != a.H || b.W != a.W || b.Ho != a.Ho || b.Wo != a.Wo || b.act != a.act || b.out_f32 != a.out_f32) {
      set_error("gemm: grouped GEMMs must share shape, mode and epilogue kind");
      return hipErrorInvalidValue;
    }
  }
  const int kq = (a.force_bm < 0) ? 32 : BK;  // BK = 32 ring tiles take K, Kx in multiples of 32
  if (a.amode != A_CONV3_SMALLC && (a.K % kq) != 0) {
    set_error("gemm: K=%d not a multiple of %d", a.K, kq);
    return hipErrorInvalidValue;
  }
  if (a.out_split && (a.act == 2 || a.out_f32 || a.ldo < 3 * a.N)) {
    set_error("gemm: split output needs a plain epilogue and ldo >= 3N (N=%d, ldo=%d)", a.N, a.ldo);
    return hipErrorInvalidValue;
  }
  if (a.act == 2 && (a.N % 4 || a.out_f32)) {
    set_error("gemm: GEGLU epilogue needs N %% 4 == 0 and bf16 output (N=%d)", a.N);
    return hipErrorInvalidValue;
  }
  if (a.out_lo && (a.out_f32 || a.out_split || a.act == 2)) {
    set_error("gemm: two-plane (out_lo) output needs a plain bf16 epilogue");
    return hipErrorInvalidValue;
  }
  if (a.x_wrap && (a.Kx != 2 * a.x_wrap || a.x_wrap % kq)) {
    set_error("gemm: x_wrap %d needs Kx = 2 * x_wrap (Kx %d)", a.x_wrap, a.Kx);
    return hipErrorInvalidValue;
  }
  if (a.Kx % kq) {
    set_error("gemm: Kx=%d not a multiple of %d", a.Kx, kq);
    return hipErrorInvalidValue;
  }
  if (a.amode != A_DENSE && a.amode != A_CONV3_SMALLC && (a.C % BK) != 0) {
    set_error("gemm: conv input channels %d not a multiple of %d", a.C, BK);
    return hipErrorInvalidValue;
  }
  // fp8: dense (LayerNorm / GroupNorm-fed linears; row scales optional) or the stride-1 3x3 conv with
  // e4m3 activations (static per-channel scales folded into the weights) and an optional bf16 K-extension
  if (a.f8 && ((a.amode != A_DENSE && a.amode != A_CONV3) || (a.Kx && a.amode != A_CONV3) || !a.col_scale ||
                a.out_split || a.force_stages || a.force_bm < 0 || (a.amode == A_CONV3 && a.C % 64))) {
    set_error("gemm: fp8 operands take a dense GEMM or a stride-1 3x3 conv (C %% 64 == 0) with column scales");
    return hipErrorInvalidValue;
  }
  for (int i = 1; i < n; ++i)
    if (args[i].f8 != a.f8 || (a.f8 && (!args[i].col_scale || !args[i].row_scale != !a.row_scale))) {
      set_error("gemm: grouped GEMMs must share the operand type");
      return hipErrorInvalidValue;
    }
  if (a.rst && (a.out_f32 || a.out_split || a.act == 2 || a.st[0].acc || (a.probe & ~128))) {
    set_error("gemm: LayerNorm row statistics need a plain bf16 epilogue without GroupNorm targets");
    return hipErrorInvalidValue;
  }
  if (a.lnst && (!a.lncs || a.amode != A_DENSE || a.Kx || a.f8 || !(a.ln_c > 0.f) || a.rst || a.st[0].acc ||
                 (a.N & 7))) {
    set_error("gemm: a folded LayerNorm takes a dense bf16 GEMM with column sums and 1/C");
    return hipErrorInvalidValue;
  }
  for (int i = 1; i < n; ++i)
    if ((args[i].rst != nullptr) != (a.rst != nullptr) || (args[i].lnst != nullptr) != (a.lnst != nullptr)) {
      set_error("gemm: grouped GEMMs must share the LayerNorm roles");
      return hipErrorInvalidValue;
    }
  int bm, bn, splits, kern;
  gemm_plan(a, &bm, &bn, &splits, &kern);
  if (a.force_bm) bm = a.force_bm;
  if (a.force_bn) bn = a.force_bn;
  if (a.force_splits) splits = a.force_splits;
  if (splits < 1 || splits > 16) {
    set_error("gemm: %d K splits (1..16)", splits);
    return hipErrorInvalidValue;
  }
  int tile_stages = 0;
  if (a.force_bm || a.force_stages)
    kern = a.force_stages >= 100 ? GEMM_KERN_DEEP
           : a.force_stages == 9 ? GEMM_KERN_HALO
           : a.force_stages >= 4 ? GEMM_KERN_PHASE : a.force_stages == 2 ? GEMM_KERN_SHALLOW : GEMM_KERN_TILE;
  if (kern == GEMM_KERN_DEEP) {
    tile_stages = a.force_stages - 100;
    if (a.f8 || (a.amode != A_DENSE && a.amode != A_CONV3) || !deep_built(bm, bn, tile_stages) || a.gn_st) {
      set_error("gemm: deep-ring tile %dx%d with %d stages not built (bf16 dense / stride-1 conv only)", bm, bn,
                tile_stages);
      return hipErrorInvalidValue;
    }
  }
  if (kern == GEMM_KERN_HALO && (!conv_halo_ok(a) || !halo_tile_built(a.W, bm, bn))) {
    set_error("gemm: halo tiles take bf16 stride-1 3x3 convs over 16/32/64-wide images, tile %dx%d not built "
              "for width %d", bm, bn, a.W);
    return hipErrorInvalidValue;
  }
  if (kern == GEMM_KERN_SHALLOW && (a.amode != A_DENSE || bm != 64 || (bn != 64 && bn != 128) || splits > 1)) {
    set_error("gemm: the 2-stage tiles are dense 64x64 / 64x128 without split-K (got %dx%d, mode %d, %d splits)", bm,
              bn, a.amode, splits);
    return hipErrorInvalidValue;
  }
  if (kern == GEMM_KERN_PHASE) splits = 1;  // built without the split-K epilogue (register budget)
  if (kern == GEMM_KERN_PHASE && (a.amode == A_CONV3_SMALLC || bm != 256 || (bn != 256 && bn != 320))) {
    set_error("gemm: the 4-phase kernel takes 256x256 / 256x320 tiles (got %dx%d, mode %d)", bm, bn, a.amode);
    return hipErrorInvalidValue;
  }
  int st_hw = 0;  // GroupNorm statistics in the epilogue: validate, and keep tiles batch-uniform
  for (int i = 0; i < n; ++i) {
    const GemmArgs& b = args[i];
    for (int k = 0; k < 2; ++k) {
      const StatTgt& t = b.st[k];
      if (!t.acc) continue;
      // (8 aligned channels of the epilogue touch at most two groups: cg >= 8, or 4-aligned groups of 4)
      const bool groups_ok = t.cg >= 8 || (t.cg % 4 == 0 && t.c_off % 4 == 0);
      if ((k == 1 && !b.st[0].acc) || (b.out_f32 && !b.out_split) || b.act == 2 || !groups_ok || t.G < 1 ||
          t.hw < 1 || (b.M % t.hw) != 0 || (st_hw && t.hw != st_hw)) {
        set_error("gemm: unsupported GroupNorm statistics target (cg %d, hw %d, M %d)", t.cg, t.hw, b.M);
        return hipErrorInvalidValue;
      }
      st_hw = t.hw;
    }
  }
  if (st_hw && kern == GEMM_KERN_PHASE && st_hw % 256) {  // a tile must not straddle two batch elements
    kern = GEMM_KERN_TILE;
    bn = 128;
  }
  if (st_hw) {
    const int sg = bm < 0 ? -1 : 1;
    int abm = bm * sg;
    while (abm > 64 && st_hw % abm) {  // a tile must not straddle two batch elements
      abm >>= 1;
      if (sg > 0 ? !gemm_tile_built(a.amode, abm, bn) : !gemm_ring_built(abm, bn)) bn = 128;
    }
    bm = abm * sg;
    // the split was planned for the wider tile: a grid that the smaller tile now fills no longer needs it (B = 64
    // 8x8-level convs: 128x320/s2 -> 64x128, whose 640 tiles ran with fp32 slabs and a combine for nothing)
    if (TAIR_BATCH_XCD && splits > 1 && kern == GEMM_KERN_TILE && (long)cdiv(a.M, abm) * cdiv(a.N, bn) >= 512) splits = 1;
    if (st_hw % abm) {
      set_error("gemm: GroupNorm statistics need hw %% 64 == 0 (hw %d)", st_hw);
      return hipErrorInvalidValue;
    }
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < 2; ++k)
        if (args[i].st[k].acc && bn / args[i].st[k].cg + 2 > STAT_NG) {
          set_error("gemm: %d-channel groups too narrow for a %d-wide tile", args[i].st[k].cg, bn);
          return hipErrorInvalidValue;
        }
  }
  // GroupNorm on load: the software-pipelined tile kernels (<= 128-row tiles, or 256 x 128) and the halo
  // tiles, a tile inside one batch element, bf16 conv (stride 1) or dense operands
  for (int i = 1; i < n; ++i)
    if ((args[i].gn_st != nullptr) != (a.gn_st != nullptr)) {
      set_error("gemm: grouped GEMMs must share the GroupNorm-on-load role");
      return hipErrorInvalidValue;
    }
  if (a.gn_st) {
    const int cin = a.amode == A_DENSE ? a.K : a.C;
    if ((a.amode != A_CONV3 && a.amode != A_DENSE) || a.f8 || !a.gn_gamma || !a.gn_beta || a.gn_G < 1 || a.gn_G > 64 ||
        cin % a.gn_G || cin / a.gn_G < 8 || cin % 64 || a.rows_per_b < 1 || (a.amode == A_CONV3 && a.H * a.W != a.rows_per_b) ||
        a.M % a.rows_per_b) {
      set_error("gemm: GroupNorm on load takes a bf16 stride-1 conv or dense GEMM with >= 8-channel groups");
      return hipErrorInvalidValue;
    }
    if (kern == GEMM_KERN_PHASE) {
      kern = GEMM_KERN_TILE;
      bm = 128;
      bn = a.amode == A_DENSE ? 256 : 320;
    }
    if (kern == GEMM_KERN_TILE && bm == 256 && bn != 128) bm = 128;
    if (kern == GEMM_KERN_TILE && bm == 128 && bn == 160) bn = 128;
    if (kern != GEMM_KERN_HALO)
      while (bm > 64 && a.rows_per_b % bm) bm >>= 1;
    // the tile kernels' pipelined loop: 8-wave tiles (128x256 / 128x320 / 256x128) or the shallow ones
    const bool pipe_tile = kern == GEMM_KERN_SHALLOW || (bm == 128 && (bn == 256 || bn == 320)) ||
                           (bm == 256 && bn == 128);
    if (bm < 0 || (kern != GEMM_KERN_TILE && kern != GEMM_KERN_SHALLOW && kern != GEMM_KERN_HALO) ||
        (kern != GEMM_KERN_HALO && (a.rows_per_b % bm || !gemm_tile_built(a.amode, bm, bn) || !pipe_tile))) {
      set_error("gemm: no GroupNorm-on-load plan (tile %dx%d, kernel %d)", bm, bn, kern);
      return hipErrorInvalidValue;
    }
  }
  for (int i = 0; i < n; ++i) {
    const GemmArgs& b = args[i];
    while (splits > 1 && (b.partial == nullptr || (size_t)splits * b.M * b.N > b.partial_cap)) --splits;
  }
  {
    // no empty K slice: a slice takes cdiv(units, splits) K-tiles (halo tiles: 64-channel chunks), so a split
    // count that does not divide the units can leave trailing slices without work that still launch, write a
    // zero slab and join the combine (e.g. 5 chunks in 4 splits of 2)
    const int units = kern == GEMM_KERN_HALO ? a.C / 64 : (a.K + a.Kx) / (bm < 0 ? 32 : BK);
    while (splits > 1 && (long)(splits - 1) * cdiv(units, splits) >= units) --splits;
  }
  // B = 1 grids (TAIR_B1_DEEP, A/B experiment): the 64-row tiles take the deepest ring that keeps the grid's
  // number of rounds over the 256 CUs (workgroups per CU limited by the LDS), at most one stage beyond the
  // slice's K-tiles
  static const int b1_deep = [] { const char* e = getenv("TAIR_B1_DEEP"); return e ? atoi(e) : 0; }();
  if (b1_deep && kern == GEMM_KERN_TILE && !a.force_bm && !a.force_stages && !a.f8 && !a.gn_st && bm == 64 &&
      (bn == 64 || bn == 128) && (a.amode == A_DENSE || a.amode == A_CONV3)) {
    const long wgs = (long)cdiv(a.M, bm) * cdiv(a.N, bn) * splits * n;
    const int per = cdiv((a.K + a.Kx) / BK, splits);
    const long sb = (long)(bm + bn) * BK * 2;
    auto rounds = [&](int st) { const long slots = 256L * std::max(1L, (160L * 1024) / (st * sb)); return (wgs + slots - 1) / slots; };
    const long r0 = rounds(3);
    for (int st : {8, 6, 5, 4})
      if (st <= per + 1 && deep_built(bm, bn, st) && rounds(st) <= r0) {
        kern = GEMM_KERN_DEEP;
        tile_stages = st;
        break;
      }
  }
  // cooperative split-K (gemm_kern.h splitk_coop): 64-row tile kernels with tickets, on grids the chip holds
  // at once (2 workgroups per CU at most: a tile's slices then wait only for resident or next-dispatched
  // workgroups); TAIR_COOP=0 turns it off (A/B experiments: the last-arriver combine / reduce kernel)
  static const bool coop_env = [] { const char* e = getenv("TAIR_COOP"); return !e || atoi(e) != 0; }();
  const bool coop_kind = coop_env && !g_skip_reduce && kern == GEMM_KERN_TILE && bm == 64 &&
                         a.amode != A_CONV3_SMALLC && !(a.probe & 4);
  // LayerNorm row statistics come from the one epilogue that sees final values: K slices must combine
  // in-kernel (64-row tile kernels: cooperatively, or at most ink_smax() slices), else K is not split
  if (a.rst && splits > 1)
    splits = ((kern == GEMM_KERN_TILE || kern == GEMM_KERN_DEEP) && bm == 64 && a.tile_sem)
                 ? (coop_kind ? splits : std::min(splits, std::max(1, ink_smax()))) : 1;
  if (a.amode < A_DENSE || a.amode > A_CONV3_SMALLC) {
    set_error("gemm: bad amode %d", a.amode);
    return hipErrorInvalidValue;
  }
  const bool f8_tile = (bm == 64 && (bn == 64 || bn == 128)) || (bm == 128 && (bn == 128 || bn == 256 || bn == 320));
  if (a.f8 && !f8_tile) {
    set_error("gemm: fp8 tile %dx%d not built", bm, bn);
    return hipErrorInvalidValue;
  }
  if (!a.f8 && kern != GEMM_KERN_PHASE && kern != GEMM_KERN_HALO &&
      (bm < 0 ? (a.amode == A_CONV3_SMALLC || !gemm_ring_built(-bm, bn) || (a.K % 32) || (a.Kx % 32))
              : !gemm_tile_built(a.amode, bm, bn))) {
    set_error("gemm: tile %dx%d not built for mode %d", bm, bn, a.amode);
    return hipErrorInvalidValue;
  }
  // in-kernel split-K combine: small split counts, tile kernels with tickets and room for
  // [tiles][splits][BM * BN] slabs (the register-staged and phase kernels always use the reduce kernel)
  const int abm = bm < 0 ? -bm : bm;
  const long tiles_all = (long)cdiv(a.M, abm) * cdiv(a.N, bn);
  const long grid_wgs = tiles_all * splits * n;
  // (the launcher re-checks the grid against the device's CU count x the chosen kernel's occupancy and falls back
  // to the last-arriver combine when the grid is not resident at once; 512 = the 256-CU part at 2 per CU bounds
  // the plans that ask)
  bool coop = splits > 1 && coop_kind && grid_wgs <= 2L * 256;
  for (int i = 0; i < n && coop; ++i)
    coop = args[i].tile_sem && tiles_all <= args[i].sem_cap &&
           (size_t)tiles_all * splits * abm * bn <= args[i].partial_cap;
  bool ink = splits > 1 && (coop || splits <= ink_smax() || (a.probe & 4)) && !g_skip_reduce &&
             a.amode != A_CONV3_SMALLC && (kern == GEMM_KERN_TILE || kern == GEMM_KERN_DEEP) &&
             bm == 64;  // 4-wave 64-row tiles: <= 8 fragments per wave
  for (int i = 0; i < n && ink; ++i)
    ink = args[i].tile_sem && tiles_all <= args[i].sem_cap &&
          (size_t)tiles_all * splits * abm * bn <= args[i].partial_cap;
  if (a.rst && splits > 1 && !ink) splits = 1;  // row statistics need the final values: no K split then
  if (a.rst && (kern == GEMM_KERN_PHASE || (bm < 0 ? -bm : bm) > 128 || (splits > 1 && !ink))) {
    set_error("gemm: LayerNorm row statistics need a <= 128-row tile plan (got %dx%d, %d splits)", bm, bn, splits);
    return hipErrorInvalidValue;
  }
  GemmGroup P;
  P.fault = g_gemm_dry ? nullptr : fault_word();
  // tile order: n fastest once the activation operand outgrows an XCD's 4 MiB L2 several times over
  P.xcd = ((size_t)a.M * (a.K + a.Kx) * 2 > ((size_t)16 << 20) && a.N > (bn < 0 ? -bn : bn)) ? 2 : 1;
  {
    // small grids (B = 1): when the activation operand outweighs the weights, n-fastest order keeps an
    // m-range's activation rows on one XCD (each weight slice is then fetched by several XCDs instead)
    // (measured B = 1 step: m-fastest 5.53, this rule 5.47, always n-fastest 5.45 ms; B = 16 unchanged,
    // profiles/r03_bench_xcd_*.log).  TAIR_XCD = 1 / 2 forces m- / n-fastest (A/B experiments).
    static const int xo = [] { const char* e = getenv("TAIR_XCD"); return e ? atoi(e) : 3; }();
    if (xo == 1 || xo == 2) P.xcd = xo;
    if (xo == 3 && a.N > (bn < 0 ? -bn : bn)) {
      const double ab = (double)a.M * (a.amode == A_DENSE ? a.K : a.C) * 2.0 + (double)a.M * a.Kx;
      const double wb = (double)a.N * (a.K + a.Kx) * 2.0;
      const long gx = cdiv(a.M, bm < 0 ? -bm : bm), gy = cdiv(a.N, bn);
      if (TAIR_BATCH_XCD && gx * gy * splits * n > 512) {
        // batched grids (round 6): the order with fewer bytes fetched across the 8 XCDs -- n fastest reads the
        // activation once and every weight slice on every XCD that holds one of its m-tiles, m fastest the
        // reverse (B = 64 8x8-level convs: 29.5 MB of weights per launch fetched by all 8 XCDs, 12.5x the
        // algorithmic bytes, profiles/r05_pmc_summary_b64.txt)
        const double nf = ab + wb * (double)std::min(8L, gx), mf = ab * (double)std::min(8L, gy) + wb;
        P.xcd = nf <= mf ? 2 : 1;
      } else if (ab > wb) {
        P.xcd = 2;
      }
    }
  }
  // halo tiles: the 2-stage weight ring where a fused GroupNorm table needs the LDS (TAIR_HALO_S2=1
  // forces it for 256x160 tiles: A/B measurements)
  static const bool halo_s2_env = [] { const char* e = getenv("TAIR_HALO_S2"); return e && atoi(e) != 0; }();
  // TAIR_EPI_REG=0 (A/B measurements): the wide tiles keep the LDS-staged epilogue (GemmArgs.probe bit 7)
  static const bool epi_reg_env = [] { const char* e = getenv("TAIR_EPI_REG"); return !e || atoi(e) != 0; }();
  for (int i = 0; i < n; ++i) {
    P.g[i] = args[i];
    if (!epi_reg_env) P.g[i].probe |= 128;
    P.g[i].halo_s2 = kern == GEMM_KERN_HALO && bn == 160 && (halo_s2_env || args[i].gn_st);
    P.g[i].tile_stages = tile_stages;
    P.g[i].splits = splits;
    P.g[i].coop = coop;
    // tickets one 128-byte line apart where they fit: the arrivals (and the cooperative polls) of
    // different tiles then do not queue on one line
    P.g[i].sem_stride = (long)tiles_all * 32 <= args[i].sem_cap ? 32 : 1;
    if (!ink) P.g[i].tile_sem = nullptr;  // summed by splitk_reduce_kernel below
  }
  if (coop) P.xcd = P.xcd == 2 ? 4 : 3;  // a tile's K slices on consecutive workgroups
  // blocked order (xcd_remap mode 5) for wide one-slice dense grids whose weight slices outgrow an XCD's L2 per m-row
  // (B = 64 GEGLU-in at 32^2 / 16^2: n fastest re-streamed the 6.5 / 26 MB of weights once per m-row, 25x the
  // algorithmic bytes at 16^2, profiles/r06_pmc_xcd_geglu.txt); TAIR_XCD_BLOCK=0 keeps the round-6 rules (A/B)
  static const bool xcd_block_env = [] { const char* e = getenv("TAIR_XCD_BLOCK"); return !e || atoi(e) != 0; }();
  static const bool xcd_forced = getenv("TAIR_XCD") != nullptr;
  if (xcd_block_env && !xcd_forced && !coop && splits == 1 && a.amode == A_DENSE && bm > 0 && kern == GEMM_KERN_TILE &&
      (P.xcd == 1 || P.xcd == 2)) {
    const long gx = cdiv(a.M, bm) * n, gy = cdiv(a.N, bn);
    const double wslice = (double)bn * (a.K + a.Kx) * 2.0, wb = wslice * gy;
    const double ab = (double)a.M * (a.K + a.Kx) * 2.0 * n;
    if (gx * gy > 512 && wb > (2 << 20)) {
      // bytes fetched beyond L2: n fastest streams W per m-tile, m fastest A per n-tile, blocked A per BNC n-tiles
      // and W per BMR m-tiles
      double best = std::min(ab + wb * (double)gx, ab * (double)gy + wb);
      int pick = 0;
      for (int bnc = 1; bnc <= 16; ++bnc)
        for (int bmr = 1; bmr <= 16; ++bmr) {
          if (gy % bnc || gx % bmr || bmr * bnc < 16 || bmr * bnc > 64) continue;
          if (((gx / bmr) * (gy / bnc)) % 8) continue;
          const double c = ab * (double)(gy / bnc) + wb * (double)(gx / bmr);
          if (c < 0.7 * best) {
            best = c;
            pick = 5 | (bmr << 8) | (bnc << 16);
          }
        }
      if (pick) P.xcd = pick;
    }
  }
  for (int i = n; i < MAX_GROUP; ++i) P.g[i] = P.g[0];

  if (a.gn_st && plan_lds(kern, bm, bn, a.W, P.g[0].halo_s2) + gn_extra_lds(P.g[0], splits) > 160 * 1024) {
    set_error("gemm: GroupNorm-on-load table does not fit the LDS (tile %dx%d, %d splits)", bm, bn, splits);
    return hipErrorInvalidValue;
  }
  // the product plans GroupNorm on load only into halo tiles (the tile kernels re-normalise every
  // K-tile's rows in the latency-bound loop: B = 1 0.90 -> 0.82 Mpix/s, profiles/r04_gn_b1_*.log)
  if (g_gemm_dry) {
    g_dry_plan[0] = bm;
    g_dry_plan[1] = bn;
    g_dry_plan[2] = splits;
    g_dry_plan[3] = kern;
    if (g_gn_halo_only && a.gn_st && kern != GEMM_KERN_HALO) return hipErrorNotSupported;
    return hipSuccess;
  }
  hipError_t e = !a.f8 ? launch_set(a.amode, P, n, bm, bn, splits, kern, s)
                 : a.amode == A_DENSE ? launch_f8<A_DENSE>(P, n, bm, bn, splits, s, kern == GEMM_KERN_SHALLOW)
                                      : gemm_set_launch<A_CONV3, SET_F8>(P, n, bm, bn, splits, s);
  if (e != hipSuccess) return e;
  if (splits > 1 && !g_skip_reduce && !ink) {
    // block = RB rows x CB4 column quads; RB a power of two dividing M (and the statistics' hw),
    // grown until the grid would drop below ~256 blocks
    const int n4 = (a.N + 3) / 4;
    const int CB4 = n4 < 64 ? n4 : 64;  // 4+ rows per pass: more blocks for the short-M (B = 1) plans
    const int cblocks = cdiv(n4, CB4);
    const int hw = st_hw ? st_hw : a.M;
    // (at most ~4 rows per thread: a thread's rows are serial memory latencies, two at a time)
    const int rpp = 256 / CB4;
    int RB = 1;
    while ((a.M % (RB * 2)) == 0 && (hw % (RB * 2)) == 0 && RB * 2 <= 4 * rpp &&
           (long)(a.M / (RB * 2)) * cblocks * n >= 256)
      RB *= 2;
    using RedFn = void (*)(const GemmGroup, int, int);
    static const RedFn red_fn[17] = {nullptr, nullptr,
                                     splitk_reduce_kernel<2>, splitk_reduce_kernel<3>, splitk_reduce_kernel<4>,
                                     splitk_reduce_kernel<5>, splitk_reduce_kernel<6>, splitk_reduce_kernel<7>,
                                     splitk_reduce_kernel<8>, splitk_reduce_kernel<9>, splitk_reduce_kernel<10>,
                                     splitk_reduce_kernel<11>, splitk_reduce_kernel<12>, splitk_reduce_kernel<13>,
                                     splitk_reduce_kernel<14>, splitk_reduce_kernel<15>, splitk_reduce_kernel<16>};
    hipLaunchKernelGGL(red_fn[splits], dim3(a.M / RB + (a.M % RB != 0), cblocks, n), dim3(256), 0, s, P, RB, CB4);
    e = hipGetLastError();
  }
  return e;
}

hipError_t gemm(const GemmArgs& a, hipStream_t s) { return gemm_grouped(&a, 1, s); }

}  // namespace tair