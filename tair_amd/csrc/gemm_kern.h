// Kernel templates of the bf16 MFMA GEMM / implicit-GEMM convolution (gfx950).
//
// One kernel serves every matmul-shaped op on the ControlLDM path:
//   * Linear layers and 1x1 convs (A_DENSE)                       attention.py:19-353, controlnet.py:318
//   * 3x3 convs as implicit GEMM, stride 1 / stride 2 / fused
//     nearest-x2 upsample (A_CONV3*), k = tap*C + c (NHWC)         unet.py:51-223
//   * ResBlock 1x1 skip conv fused as a K-extension of conv2      unet.py:182-189, 223
//
// Roles: the MFMA A operand is the weight tile (rows = output channels n), the B operand is the
// activation tile (cols = pixels/tokens m), so each lane ends with 4 consecutive channels of one
// pixel and the NHWC epilogue store is an 8-byte vector.
//
// Main kernel: gemm_tile_kernel (LDS-DMA ring, see its comment), v_mfma_f32_16x16x32_bf16, BK = 64.
// Every global load is unconditional: out-of-range rows, conv padding taps and padded weight rows
// read a 1 KiB device zero page through a pointer select, so hipcc emits no branch and no vmcnt(0)
// per element (the "register or load" trap of cdna_hip_programming.md §5 item 4(c)).  LDS rows are
// 128 B with the XOR swizzle chunk ^ (row & 7): the ds_read_b128 fragment reads are bank-conflict
// free.
#pragma once
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"

namespace tair {

// Instantiations live in gemm_<mode>_<set>.hip (one translation unit per activation mode and tile
// set, compiled in parallel); gemm.hip holds the planner, the grouped launcher and the split-K
// reduce kernel.
namespace {

__device__ __attribute__((aligned(1024))) uint4 g_zero_page[64];  // 1 KiB of zeros (static init)

constexpr int BK = 64;

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).  Used wherever an index
// selects an accumulator fragment: `#pragma unroll` is only a request, and a nest it gives up on
// (a long epilogue body) leaves acc[][] in scratch memory.
// The kernel's argument block read in place from the kernarg segment.  Indexing the by-value
// parameter (P.g[grp], grp from blockIdx) makes clang copy the whole ~600-byte GemmGroup into
// scratch and reload fields from there inside the main loop, each reload an s_waitcnt vmcnt(0)
// that drains every LDS-DMA in flight.  Valid for a kernel whose FIRST parameter is the struct.
template <class T>
TAIR_DEV const T& kernarg0() {
#if __HIP_DEVICE_COMPILE__
  return *(const T*)(const void*)__builtin_amdgcn_kernarg_segment_ptr();
#else
  return *(const T*)nullptr;  // host pass of a __global__ body: never executed
#endif
}

// Phase stamps of a measurement build (-DTAIR_STAMPS=1, tools/b1_stamps.py): lane 0 of wave 0 writes
// s_memrealtime (100 MHz) into p.stamps[linear block][slot] with a vector store; compiled out otherwise.
#ifndef TAIR_STAMPS
#define TAIR_STAMPS 0
#endif
template <class PA>
TAIR_DEV void stamp(const PA& p, int slot) {
  if constexpr (TAIR_STAMPS) {
    if (p.stamps && threadIdx.x == 0) {
      const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
      __hip_atomic_store(p.stamps + (size_t)b * 8 + slot, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// TAIR_STAMPS >= 2: also per-iteration stamps of the main loop for linear blocks 0..3 (iterations < 64):
// stamps[65536 * 8 + ((block * 64 + it) * 4 + k)], k = 0 iteration start, 1 after the wait + barrier,
// 2 after the DMA issue, 3 after the MFMAs
TAIR_DEV void stamp_it(unsigned long long* st, int it, int k) {
  if constexpr (TAIR_STAMPS >= 2) {
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (st && threadIdx.x == 0 && b < 4 && it < 64)
      __hip_atomic_store(st + 65536 * 8 + ((size_t)(b * 64 + it) * 4 + k),
                         (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int B, int E, class F>
TAIR_DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

TAIR_DEV int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

// XCD-aware block order (cdna_hip_programming.md T1): hardware deals blocks round-robin over the 8
// XCDs, so consecutive LOGICAL tiles are given to blocks that share an XCD.  enable = 1: m fastest
// (then n, then the K slice): the m-tiles that stream the same weight tile hit one L2 (small grids,
// weight-bound); 2: n fastest, for activations far larger than an L2 (batched tiles): the N-tiles of
// an M-tile read its rows once.  Bijective for any count (mode 5, blocked: for the grids the host checks).
TAIR_DEV void xcd_remap(int& bx, int& by, int& bz, int enable) {
  const int gx = gridDim.x, gy = gridDim.y;
  if (!enable) {
    bx = blockIdx.x;
    by = blockIdx.y;
    bz = blockIdx.z;
    return;
  }
  const int nwg = gx * gy * gridDim.z;
  const int orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if ((enable & 0xff) == 5) {
    // blocked (round 6): the grid is cut into super-blocks of BMR m-tiles x BNC n-tiles, super-block s belongs to
    // XCD s % 8, and an XCD walks its super-blocks in order, n fastest inside one: the ~32 tiles an XCD runs at
    // once share a few activation row panels AND a few weight slices in its L2 (n fastest alone re-streams every
    // weight slice per m-row once gy slices outgrow the L2; m fastest re-streams the activations per n-tile).
    // The host picks it only for one-slice grids whose super-block count is a multiple of 8 (gemm.hip), so the
    // workgroups of each XCD are exactly its super-blocks' tiles.
    const int bmr = (enable >> 8) & 0xff, bnc = (enable >> 16) & 0xff, per = bmr * bnc;
    const int k = orig >> 3, j = k / per, w = k - j * per;
    const int sb = (orig & 7) + 8 * j, snb = gy / bnc;
    const int sm = sb / snb, sn = sb - sm * snb;
    bx = sm * bmr + w / bnc;
    by = sn * bnc + (w - (w / bnc) * bnc);
    bz = 0;
    return;
  }
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  if (enable >= 3) {  // K slices fastest (cooperative split-K), then m (3) or n (4)
    bz = id % gridDim.z;
    const int rest = id / gridDim.z;
    if (enable == 3) {
      bx = rest % gx;
      by = rest / gx;
    } else {
      by = rest % gy;
      bx = rest / gy;
    }
    return;
  }
  if (enable == 2) {  // n fastest: the N-tiles of one M-tile share an XCD (activation rows read once)
    by = id % gy;
    const int rest = id / gy;
    bx = rest % gx;
    bz = rest / gx;
    return;
  }
  bx = id % gx;
  const int rest = id / gx;
  by = rest % gy;
  bz = rest / gy;
}

// Per-lane source row of the activation operand, packed into 3 registers (it is live across the
// whole main loop, once per DMA row of the lane): element offsets from A / X (32-bit: every operand
// of the network is < 2^32 elements) and the output pixel's (yo, xo) as one word; INVALID marks a
// row past M (every tap and the K-extension then read the zero page).
constexpr int ROW_INVALID = (int)0x80000000;
template <int AMODE>
struct RowInfo {
  uint32_t off;   // dense: m*lda + 8*chunk ; conv: (b*H*W)*lda + 8*chunk
  uint32_t xoff;  // K-extension: m*ldx + 8*chunk
  int yx;         // conv: (yo << 16) | (xo & 0xffff); dense: 0; ROW_INVALID past M
};

template <int AMODE, class PA>
TAIR_DEV RowInfo<AMODE> row_info(const PA& p, int m, int chunk) {
  RowInfo<AMODE> r;
  const bool valid = m < p.M;
  const int mm = valid ? m : 0;
  r.yx = 0;
  if constexpr (AMODE == A_DENSE) {
    r.off = (uint32_t)mm * (uint32_t)p.lda + chunk * 8;
  } else {
    const int hw = p.Ho * p.Wo;
    const int b = mm / hw, rem = mm - b * hw;
    const int yo = rem / p.Wo, xo = rem - yo * p.Wo;
    r.yx = (yo << 16) | (xo & 0xffff);
    r.off = (uint32_t)b * (uint32_t)(p.H * p.W) * (uint32_t)p.lda + chunk * 8;
  }
  r.xoff = (uint32_t)mm * (uint32_t)p.ldx + chunk * 8;
  if (!valid) r.yx = ROW_INVALID;
  return r;
}
template <int AMODE>
TAIR_DEV int row_yo(const RowInfo<AMODE>& r) { return r.yx >> 16; }
template <int AMODE>
TAIR_DEV int row_xo(const RowInfo<AMODE>& r) { return (int)(short)(r.yx & 0xffff); }

// The GemmArgs fields the activation source needs, copied into registers once per workgroup: read through
// the kernel-argument reference inside the main loop, the compiler re-loaded them (s_load + lgkmcnt(0),
// which also drains the LDS fragment reads in flight) behind a branch at every DMA issue.
struct ActArgs {
  const bf16* A;
  const bf16* X;
  int K, x_wrap, H, W, lda, s2_shift, C;
};
TAIR_DEV ActArgs act_args(const GemmArgs& p) { return {p.A, p.X, p.K, p.x_wrap, p.H, p.W, p.lda, p.s2_shift, p.C}; }

// A kernel argument held in a register: the compiler treats loads from the kernarg segment as invariant and
// REMATERIALISES them at every use instead of keeping them live, each an s_load + s_waitcnt lgkmcnt(0) round
// trip (~0.12 us from L2) on the critical path -- at B = 1 the epilogue's item loop re-read ~8 fields per item
// behind their branches and the prologue chained 8 such round trips before its first DMA (phase stamps,
// tools/b1_stamps.py: items 2.5 us, prologue 1.0 us of a 9 us launch).  An empty asm with the value as an
// in/out operand makes it opaque (not rematerialisable), so a field snapshot is loaded once, as one batch.
template <class T>
TAIR_DEV T pin(T v) {
  TAIR_PIN_ASM("" : "+s"(v));
  return v;
}
TAIR_DEV StatTgt pin_st(const StatTgt& t) {
  return StatTgt{pin(t.acc), pin(t.rs), pin(t.cg), pin(t.G), pin(t.c_off), pin(t.hw)};
}

// The GemmArgs fields of the epilogues (epilogue_tile / epilogue_direct / splitk_reduce_kernel), snapshotted
// into registers once (pin): same field names, so the epilogue code reads either struct.
struct EpiArgs {
  int M, N;
  float alpha;
  int scale_bias, act, probe, splits, rows_per_b, ld_emb, ld_res, res_lo, ldo, out_f32, out_split, out_lo, coop,
      sem_stride;
  float ln_c, ln_eps;
  const float* bias;
  const float* emb;
  const int* emb_row;
  const bf16* res;
  void* out;
  float* partial;
  int* tile_sem;
  const float* row_scale;
  const float* col_scale;
  const double* lnst;
  const float* lncs;
  double* rst;
  StatTgt st[2];
  unsigned long long* stamps;
};
#define TAIR_GPTR(T) __attribute__((address_space(1))) T*
// pointer fields are pinned as global (address space 1) pointers and cast back: a generic pointer that
// comes out of an asm statement would lose its provenance and turn every access into a flat_* operation
// (ordered on both vmcnt and lgkmcnt, so each one waits for everything in flight)
TAIR_DEV EpiArgs epi_args(const GemmArgs& p) {
  EpiArgs e;
  e.M = p.M; e.N = p.N; e.alpha = p.alpha;
  e.scale_bias = p.scale_bias; e.act = p.act; e.probe = p.probe; e.splits = p.splits;
  e.rows_per_b = p.rows_per_b; e.ld_emb = p.ld_emb; e.ld_res = p.ld_res; e.res_lo = p.res_lo;
  e.ldo = p.ldo; e.out_f32 = p.out_f32; e.out_split = p.out_split; e.out_lo = p.out_lo; e.coop = p.coop;
  e.sem_stride = p.sem_stride;
  e.ln_c = p.ln_c; e.ln_eps = p.ln_eps;
  e.st[0] = p.st[0];
  e.st[1] = p.st[1];
  TAIR_GPTR(const float) bias = (TAIR_GPTR(const float))p.bias;
  TAIR_GPTR(const float) emb = (TAIR_GPTR(const float))p.emb;
  TAIR_GPTR(const int) emb_row = (TAIR_GPTR(const int))p.emb_row;
  TAIR_GPTR(const bf16) res = (TAIR_GPTR(const bf16))p.res;
  TAIR_GPTR(char) out = (TAIR_GPTR(char))p.out;
  TAIR_GPTR(float) partial = (TAIR_GPTR(float))p.partial;
  TAIR_GPTR(int) tile_sem = (TAIR_GPTR(int))p.tile_sem;
  TAIR_GPTR(const float) row_scale = (TAIR_GPTR(const float))p.row_scale;
  TAIR_GPTR(const float) col_scale = (TAIR_GPTR(const float))p.col_scale;
  TAIR_GPTR(const double) lnst = (TAIR_GPTR(const double))p.lnst;
  TAIR_GPTR(const float) lncs = (TAIR_GPTR(const float))p.lncs;
  TAIR_GPTR(double) rst = (TAIR_GPTR(double))p.rst;
  TAIR_GPTR(double) st0 = (TAIR_GPTR(double))p.st[0].acc;
  TAIR_GPTR(double) st1 = (TAIR_GPTR(double))p.st[1].acc;
  TAIR_GPTR(unsigned long long) stamps = (TAIR_GPTR(unsigned long long))(TAIR_STAMPS ? p.stamps : nullptr);
  // ONE asm for every field: each asm volatile is a scheduling boundary, so per-field pins would serialise
  // the loads (one round trip each); behind a single one they issue as a batch (s_load_dwordx16s, one wait)
  TAIR_PIN_ASM(""
               : "+s"(e.M), "+s"(e.N), "+s"(e.alpha), "+s"(e.scale_bias), "+s"(e.act), "+s"(e.probe), "+s"(e.splits),
                 "+s"(e.rows_per_b), "+s"(e.ld_emb), "+s"(e.ld_res), "+s"(e.res_lo), "+s"(e.ldo), "+s"(e.out_f32),
                 "+s"(e.out_split), "+s"(e.out_lo), "+s"(e.coop), "+s"(e.sem_stride), "+s"(e.ln_c), "+s"(e.ln_eps), "+s"(bias), "+s"(emb),
                 "+s"(emb_row), "+s"(res), "+s"(out), "+s"(partial), "+s"(tile_sem), "+s"(row_scale),
                 "+s"(col_scale), "+s"(lnst), "+s"(lncs), "+s"(rst), "+s"(st0), "+s"(e.st[0].rs),
                 "+s"(e.st[0].cg), "+s"(e.st[0].G), "+s"(e.st[0].c_off), "+s"(e.st[0].hw), "+s"(st1),
                 "+s"(e.st[1].rs), "+s"(e.st[1].cg), "+s"(e.st[1].G), "+s"(e.st[1].c_off), "+s"(e.st[1].hw),
                 "+s"(stamps));
  e.bias = (const float*)bias; e.emb = (const float*)emb; e.emb_row = (const int*)emb_row; e.res = (const bf16*)res;
  e.out = (void*)out; e.partial = (float*)partial; e.tile_sem = (int*)tile_sem; e.row_scale = (const float*)row_scale;
  e.col_scale = (const float*)col_scale; e.lnst = (const double*)lnst; e.lncs = (const float*)lncs;
  e.rst = (double*)rst; e.st[0].acc = (double*)st0; e.st[1].acc = (double*)st1;
  e.stamps = (unsigned long long*)stamps;
  return e;
}

// The GemmArgs fields of the prologue / main loop of the tile and halo kernels, one batch (see pin).
struct MainArgs {
  int M, N, K, Kx, splits, lda, ldx, ldw, Ho, Wo, H, W, x_wrap, s2_shift, C;
  const bf16* A;
  const bf16* X;
  const bf16* Wt;
  const double* gn_st;
  unsigned long long* stamps;
};
TAIR_DEV MainArgs main_args(const GemmArgs& p) {
  MainArgs a;
  a.M = p.M; a.N = p.N; a.K = p.K; a.Kx = p.Kx; a.splits = p.splits; a.lda = p.lda; a.ldx = p.ldx; a.ldw = p.ldw;
  a.Ho = p.Ho; a.Wo = p.Wo; a.H = p.H; a.W = p.W; a.x_wrap = p.x_wrap; a.s2_shift = p.s2_shift; a.C = p.C;
  TAIR_GPTR(const bf16) A = (TAIR_GPTR(const bf16))p.A;
  TAIR_GPTR(const bf16) X = (TAIR_GPTR(const bf16))p.X;
  TAIR_GPTR(const bf16) Wt = (TAIR_GPTR(const bf16))p.Wt;
  TAIR_GPTR(const double) gn_st = (TAIR_GPTR(const double))p.gn_st;
  TAIR_GPTR(unsigned long long) stamps = (TAIR_GPTR(unsigned long long))(TAIR_STAMPS >= 2 ? p.stamps : nullptr);
  TAIR_PIN_ASM(""
               : "+s"(a.M), "+s"(a.N), "+s"(a.K), "+s"(a.Kx), "+s"(a.splits), "+s"(a.lda), "+s"(a.ldx), "+s"(a.ldw),
                 "+s"(a.Ho), "+s"(a.Wo), "+s"(a.H), "+s"(a.W), "+s"(a.x_wrap), "+s"(a.s2_shift), "+s"(a.C), "+s"(A),
                 "+s"(X), "+s"(Wt), "+s"(gn_st), "+s"(stamps));
  a.A = (const bf16*)A; a.X = (const bf16*)X; a.Wt = (const bf16*)Wt; a.gn_st = (const double*)gn_st;
  a.stamps = (unsigned long long*)stamps;
  return a;
}
TAIR_DEV ActArgs act_args(const MainArgs& p) { return {p.A, p.X, p.K, p.x_wrap, p.H, p.W, p.lda, p.s2_shift, p.C}; }

// Source of the 16-byte activation chunk of row r for K-tile k0 (branch-free pointer select; conv
// padding taps and rows past M read the zero page).  Not for A_CONV3_SMALLC.  PA: GemmArgs or ActArgs.
template <int AMODE, class PA>
TAIR_DEV const bf16* act_src(const PA& p, const RowInfo<AMODE>& r, int k0) {
  const bf16* zp = (const bf16*)g_zero_page;
  const bool valid = r.yx != ROW_INVALID;
  if (k0 >= p.K) {  // fused skip-conv K-extension (x_wrap: the same activation twice, [W_hi | W_lo])
    int kx = k0 - p.K;
    if (p.x_wrap && kx >= p.x_wrap) kx -= p.x_wrap;
    return valid ? p.X + r.xoff + kx : zp;
  }
  if constexpr (AMODE == A_DENSE) {
    return valid ? p.A + r.off + k0 : zp;
  } else {
    // channel-chunk-major K (kernels.h A_CONV3): k = (c64 * 9 + tap) * 64 + (c % 64); a K-tile (64 or
    // 32 wide) never straddles a tap
    const int q = k0 >> 6, chunk = q / 9, tap = q - 9 * chunk;
    const int c = chunk * 64 + (k0 & 63);
    const int ky = tap / 3, kx = tap - ky * 3;
    const int yo = row_yo(r), xo = row_xo(r);  // yo = -32768 for an invalid row: every tap fails
    int yi, xi;
    bool ok;
    if constexpr (AMODE == A_CONV3_S2) {
      yi = 2 * yo + ky - 1 + p.s2_shift;
      xi = 2 * xo + kx - 1 + p.s2_shift;
      ok = yi >= 0 && yi < p.H && xi >= 0 && xi < p.W;
    } else if constexpr (AMODE == A_CONV3_UP) {  // conv over the 2x nearest-upsampled grid
      const int yu = yo + ky - 1, xu = xo + kx - 1;
      ok = yu >= 0 && yu < 2 * p.H && xu >= 0 && xu < 2 * p.W;
      yi = yu >> 1;
      xi = xu >> 1;
    } else {
      yi = yo + ky - 1;
      xi = xo + kx - 1;
      ok = yi >= 0 && yi < p.H && xi >= 0 && xi < p.W;
    }
    return ok ? p.A + r.off + (uint32_t)((yi * p.W + xi) * p.lda + c) : zp;
  }
}

// fp8 (e4m3) 3x3 convs: the activation is e4m3 bytes [pixel][C] addressed in byte PAIRS (lda = row
// bytes / 2, r.off in pairs with the lane's chunk * 8 pairs folded in).  The K order is the bf16
// path's channel-chunk-major one, k = slot * 64 + c % 64 with slot = (c / 64) * 9 + tap, at one byte
// per value: a 128-value K-tile t holds slots 2t (chunks 0-3 of the LDS row) and 2t + 1 (chunks 4-7),
// so the lane's source depends on its half (dchunk >> 2); an odd slot count leaves the last half on
// the zero page (its weights are zero too: quant_rows_fp8 pads K to the 128-value tile).
template <int AMODE, class PA>
TAIR_DEV const bf16* act_src_f8(const PA& p, const RowInfo<AMODE>& r, int k0, int dchunk) {
  const bf16* zp = (const bf16*)g_zero_page;
  const bool valid = r.yx != ROW_INVALID;
  if (k0 >= p.K) {  // bf16 K-extension (skip conv), as act_src
    int kx = k0 - p.K;
    if (p.x_wrap && kx >= p.x_wrap) kx -= p.x_wrap;
    return valid ? p.X + r.xoff + kx : zp;
  }
  const int s = 2 * (k0 >> 6) + (dchunk >> 2);
  const int chunk = s / 9, tap = s - 9 * chunk;
  const int ky = tap / 3, kx = tap - ky * 3;
  const int yo = row_yo(r), xo = row_xo(r);
  int yi, xi;
  bool ok;
  if constexpr (AMODE == A_CONV3_S2) {
    yi = 2 * yo + ky - 1 + p.s2_shift;
    xi = 2 * xo + kx - 1 + p.s2_shift;
    ok = yi >= 0 && yi < p.H && xi >= 0 && xi < p.W;
  } else if constexpr (AMODE == A_CONV3_UP) {
    const int yu = yo + ky - 1, xu = xo + kx - 1;
    ok = yu >= 0 && yu < 2 * p.H && xu >= 0 && xu < 2 * p.W;
    yi = yu >> 1;
    xi = xu >> 1;
  } else {
    yi = yo + ky - 1;
    xi = xo + kx - 1;
    ok = yi >= 0 && yi < p.H && xi >= 0 && xi < p.W;
  }
  ok = ok && chunk * 64 < p.C;  // the zero half of an odd slot count
  // r.off holds chunk (dchunk) * 8 pairs; this lane's 16 bytes are pairs chunk*32 + (dchunk & 3) * 8
  const uint32_t o = r.off + (uint32_t)((yi * p.W + xi) * p.lda) + (uint32_t)(chunk * 32 + (dchunk & 3) * 8) -
                     (uint32_t)(dchunk * 8);
  return ok ? p.A + o : zp;
}

// 16-byte activation chunk of row r for K-tile k0, branch-free.
template <int AMODE>
TAIR_DEV u32x4 load_act(const GemmArgs& p, const RowInfo<AMODE>& r, int k0, int chunk) {
  if constexpr (AMODE == A_CONV3_SMALLC) {
    const bf16* zp = (const bf16*)g_zero_page;
    const bool valid = r.yx != ROW_INVALID;
    if (k0 >= p.K) {
      int kx = k0 - p.K;
      if (p.x_wrap && kx >= p.x_wrap) kx -= p.x_wrap;
      return *(const u32x4*)(valid ? p.X + r.xoff + kx : zp);
    }
    // C not a multiple of 8 (first convs): element gather, tiny layers only
    union { u32x4 u; bf16 h[8]; } v;
    const int kreal = 9 * p.C;
    const bf16* a = p.A + r.off - chunk * 8;
    const int yo = row_yo(r), xo = row_xo(r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = k0 + chunk * 8 + e;
      const int tap = kk / p.C, c = kk - tap * p.C;
      const int ky = tap / 3, kx = tap - ky * 3;
      const int yi = yo + ky - 1, xi = xo + kx - 1;
      const bool ok = kk < kreal && yi >= 0 && yi < p.H && xi >= 0 && xi < p.W;
      const bf16* ptr = ok ? a + (size_t)(yi * p.W + xi) * p.lda + c : zp;
      v.h[e] = *ptr;
    }
    return v.u;
  } else {
    return *(const u32x4*)act_src<AMODE>(p, r, k0);
  }
}

// The epilogues' shared arithmetic with the fused multiply-adds spelled out and no other contraction, so every
// epilogue (epilogue4 / epilogue8 / epilogue_regstage) gives the same bits whichever operations the compiler
// would otherwise have fused (the register-staged epilogue differed from the LDS-staged one in 0.005% of the
// folded-LayerNorm outputs by one bf16 rounding before: test_lnfold_plans_bitwise_identical)
TAIR_DEV float epi_alpha(float x, float al) {
#pragma clang fp contract(off)
  return x * al;
}
TAIR_DEV float epi_lnfold(float a, float mu, float rstd, float cs) {  // rstd (a - mean colsum)
#pragma clang fp contract(off)
  return rstd * __builtin_fmaf(-mu, cs, a);
}
TAIR_DEV float epi_bias(float v, float bscale, float b) { return __builtin_fmaf(bscale, b, v); }

// mean / rstd of row m from the fp64 LayerNorm statistics a producer accumulated (GemmArgs.lnst)
template <class PA>
TAIR_DEV void ln_row(const PA& p, int m, float& mu, float& rstd) {
  const double s = p.lnst[2 * (size_t)m], q = p.lnst[2 * (size_t)m + 1];
  const double mean = s / (double)p.ln_c;
  const double var = fmax(q / (double)p.ln_c - mean * mean, 0.0);
  mu = (float)mean;
  rstd = (float)(1.0 / sqrt(var + (double)p.ln_eps));
}

// Epilogue for 4 consecutive channels n..n+3 of pixel m (n % 4 == 0).  The full-vector path loads
// bias / emb as float4 and the residual as one 8-byte bf16x4 (all channel counts and offsets of the
// network are multiples of 4); the tail path is scalar.
template <class PA>
TAIR_DEV void epilogue4(const PA& p, int m, int n, f32x4 acc, float (&stored)[4]) {
  float v[4] = {epi_alpha(acc[0], p.alpha), epi_alpha(acc[1], p.alpha), epi_alpha(acc[2], p.alpha),
               epi_alpha(acc[3], p.alpha)};
  const bool full = (n + 3 < p.N);
  if (p.row_scale || p.col_scale) {  // fp8 dequantisation
    const float rs = p.row_scale ? p.row_scale[m] : 1.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= rs * (n + r < p.N ? p.col_scale[n + r] : 0.f);
  }
  if (p.lnst) {  // folded LayerNorm: v = rstd (acc - mean * colsum)
    float mu, rstd;
    ln_row(p, m, mu, rstd);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = n + r < p.N ? epi_lnfold(v[r], mu, rstd, p.lncs[n + r]) : 0.f;
  }
  const float bscale = p.scale_bias ? p.alpha : 1.f;
  const float* embrow = nullptr;
  if (p.emb) {
    const int b = m / p.rows_per_b;
    embrow = p.emb + (size_t)p.emb_row[b] * p.ld_emb;
  }
  if (full) {
    if (p.bias) {
      const float* bp = p.bias + n;
      const float4 b4 = ((uintptr_t)bp & 15) == 0 ? *(const float4*)bp : make_float4(bp[0], bp[1], bp[2], bp[3]);
      v[0] = epi_bias(v[0], bscale, b4.x); v[1] = epi_bias(v[1], bscale, b4.y);
      v[2] = epi_bias(v[2], bscale, b4.z); v[3] = epi_bias(v[3], bscale, b4.w);
    }
    if (embrow) {
      const float* ep = embrow + n;
      const float4 e4 = ((uintptr_t)ep & 15) == 0 ? *(const float4*)ep : make_float4(ep[0], ep[1], ep[2], ep[3]);
      v[0] += e4.x; v[1] += e4.y; v[2] += e4.z; v[3] += e4.w;
    }
    if (p.res && p.res_lo) {  // split residual: hi + lo is exact in fp32
      const bf16* rp = p.res + (size_t)m * p.ld_res + n;
      const bf16x4 h4 = *(const bf16x4*)rp, l4 = *(const bf16x4*)(rp + p.res_lo);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += bf2f(h4[r]) + bf2f(l4[r]);
    } else if (p.res) {
      const bf16* rp = p.res + (size_t)m * p.ld_res + n;
      if (((uintptr_t)rp & 7) == 0) {
        const bf16x4 r4 = *(const bf16x4*)rp;
        v[0] += bf2f(r4[0]); v[1] += bf2f(r4[1]); v[2] += bf2f(r4[2]); v[3] += bf2f(r4[3]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bf2f(rp[r]);
      }
    }
    if (p.act == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = silu_f(v[r]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int nn = n + r;
      if (nn >= p.N) break;
      if (p.bias) v[r] = epi_bias(v[r], bscale, p.bias[nn]);
      if (embrow) v[r] += embrow[nn];
      if (p.res) {
        const bf16* rp = p.res + (size_t)m * p.ld_res + nn;
        v[r] += p.res_lo ? bf2f(rp[0]) + bf2f(rp[p.res_lo]) : bf2f(rp[0]);
      }
      if (p.act == 1) v[r] = silu_f(v[r]);
    }
  }
  if (p.act == 2) {  // GEGLU pair (x_2q, x_2q+1, gate_2q, gate_2q+1) -> out columns 2q, 2q+1 (N % 4 == 0)
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 y = {f2bf(v[0] * gelu_erf(v[2])), f2bf(v[1] * gelu_erf(v[3]))};
    if (p.probe & 1) {
      asm volatile("" ::"v"(y));
      return;
    }
    *(bf16x2*)((bf16*)p.out + (size_t)m * p.ldo + (n >> 1)) = y;
    return;
  }
  if (p.out_split) {  // 3-plane split output (the statistics see the fp32 value)
    bf16x4 hi, lo;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      hi[r] = f2bf(v[r]);
      lo[r] = f2bf(v[r] - bf2f(hi[r]));
      stored[r] = (n + r < p.N) ? v[r] : 0.f;
    }
    bf16* o = (bf16*)p.out + (size_t)m * p.ldo + n;
    bf16* o1 = o + p.N;
    bf16* o2 = o + 2 * p.N;
    const bf16x4 second = p.out_split == 1 ? lo : hi, third = p.out_split == 1 ? hi : lo;
    if (full && ((((size_t)m * p.ldo + n) & 3) == 0) && (p.N & 3) == 0) {
      *(bf16x4*)o = hi;
      *(bf16x4*)o1 = second;
      *(bf16x4*)o2 = third;
    } else {
      for (int r = 0; r < 4 && n + r < p.N; ++r) {
        o[r] = hi[r];
        o1[r] = second[r];
        o2[r] = third[r];
      }
    }
    return;
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
    const bf16x4 w = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
    if (p.probe & 1) {  // measurement probe: the values are formed but not stored
      asm volatile("" ::"v"(w));
      return;
    }
    if (p.out_lo) {  // two-plane storage: hi + lo carries v to ~2^-16; consumers (and the statistics) see v
      const bf16x4 lo = {f2bf(v[0] - bf2f(w[0])), f2bf(v[1] - bf2f(w[1])), f2bf(v[2] - bf2f(w[2])),
                         f2bf(v[3] - bf2f(w[3]))};
#pragma unroll
      for (int r = 0; r < 4; ++r) stored[r] = (n + r < p.N) ? v[r] : 0.f;
      if (full && ((((size_t)m * p.ldo + n) & 3) == 0)) {
        *(bf16x4*)o = w;
        *(bf16x4*)(o + p.out_lo) = lo;
      } else {
        for (int r = 0; r < 4 && n + r < p.N; ++r) {
          o[r] = w[r];
          o[p.out_lo + r] = lo[r];
        }
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) stored[r] = (n + r < p.N) ? bf2f(w[r]) : 0.f;
    if (full && ((((size_t)m * p.ldo + n) & 3) == 0)) {
      *(bf16x4*)o = w;
    } else {
      for (int r = 0; r < 4 && n + r < p.N; ++r) o[r] = w[r];
    }
  }
}

// ---- GroupNorm statistics of the stored output (StatTgt, kernels.h) -------------------------
// A lane's 4 consecutive channels n..n+3 touch at most two groups (cg >= 4): gA = group of n and
// gA + 1 for the channels at or past the boundary.  Sums are kept in fp64 from the first add (a
// GroupNorm input can have |mean| >> std, so sum x^2 - (sum x)^2 / n must not cancel in fp32),
// reduced over the lanes that share the channels, added into LDS per group of the block, and
// flushed once per block with fp64 atomics into replica (block % STAT_REPL).
constexpr int STAT_NG = 64;  // groups per block per target (host guarantees BN / cg + 2 <= STAT_NG)
struct Stat4 {
  double sa, qa, sb, qb;
};
TAIR_DEV void stat_add(const StatTgt& t, int n, const float (&v)[4], Stat4& a) {
  const int c = t.c_off + n;
  const int bnd = (c / t.cg + 1) * t.cg - c;  // channels r < bnd belong to group gA
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const double d = v[r];
    if (r < bnd) { a.sa += d; a.qa += d * d; }
    else { a.sb += d; a.qb += d * d; }
  }
}
TAIR_DEV void stat_shfl16(Stat4& a) {  // sum over the 16 lanes (lane & 15) of each lane group
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    a.sa += __shfl_xor(a.sa, o, 64);
    a.qa += __shfl_xor(a.qa, o, 64);
    a.sb += __shfl_xor(a.sb, o, 64);
    a.qb += __shfl_xor(a.qb, o, 64);
  }
}
TAIR_DEV void lds_stat_add(double* red, const StatTgt& t, int n, int gbase, const Stat4& a) {
  const int gA = (t.c_off + n) / t.cg - gbase;
  atomicAdd(red + 2 * gA, a.sa);
  atomicAdd(red + 2 * gA + 1, a.qa);
  if (a.sb != 0.0 || a.qb != 0.0) {
    atomicAdd(red + 2 * gA + 2, a.sb);
    atomicAdd(red + 2 * gA + 3, a.qb);
  }
}
// red: [2][STAT_NG][2] doubles of LDS, zeroed and filled by the block; flush by threads < 2*STAT_NG
template <class PA>
TAIR_DEV void stat_flush(const PA& p, const double* red, int b, int n_lo, int n_hi, int rep) {
  const int t = threadIdx.x;
  if (t >= 2 * STAT_NG) return;
  const int k = t / STAT_NG, gl = t - k * STAT_NG;
  // field-wise selects: a dynamic index into p.st would make the compiler copy the whole argument
  // struct to scratch memory (and reload its fields with vmcnt(0) waits inside the main loop)
  double* const acc = k ? p.st[1].acc : p.st[0].acc;
  if (!acc) return;
  const int c_off = k ? p.st[1].c_off : p.st[0].c_off, cg = k ? p.st[1].cg : p.st[0].cg;
  const int G = k ? p.st[1].G : p.st[0].G, rs = k ? p.st[1].rs : p.st[0].rs;
  const int g0 = (c_off + n_lo) / cg, g1 = (c_off + n_hi - 1) / cg;
  const int g = g0 + gl;
  if (g > g1 || g >= G) return;
  double* dst = acc + (size_t)rep * rs + ((size_t)b * G + g) * 2;
  unsafeAtomicAdd(dst, red[(k * STAT_NG + gl) * 2]);
  unsafeAtomicAdd(dst + 1, red[(k * STAT_NG + gl) * 2 + 1]);
}

// ---- LDS-staged tile epilogue --------------------------------------------------------------
// After the main loop the fp32 accumulator tile is written to LDS ([row][col], rows padded by 16 B:
// conflict-free ds_write_b128 of the fragments, ds_read_b128 of row vectors) in column passes that
// fit the kernel's LDS, and every thread then walks "items" = 8 consecutive channels of one row:
// bias / time-embedding / residual loads and the output stores are 16-byte vectors along full rows
// (coalesced lines instead of 16 rows x 32 B per fragment store), U items' loads are in flight
// together, and one compact loop body serves every fragment (the per-fragment unrolled epilogue
// serialised one memory latency per fragment and cost 40-50% of the batched short-K GEMMs:
// profiles/r03_gemm_probe_epilogue_b16.log).  The same pass writes split-K fp32 slabs as full rows.
#ifndef TAIR_EPI_U_SMALL
#define TAIR_EPI_U_SMALL 1
#endif
#ifndef TAIR_EPI_U_BIG
#define TAIR_EPI_U_BIG 1
#endif
constexpr int epi_q(int BM, int WN, int WNW, int cap) {
  for (int q = WNW; q >= 1; --q)
    if (WNW % q == 0 && BM * (WN * q + 4) * 4 <= cap) return q;
  return 0;
}

TAIR_DEV bool al16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

// 8-channel statistics accumulator: channels before `bnd` belong to group gA, the rest to gA + 1
// (8 aligned channels touch at most two groups: host-checked cg >= 8, or cg % 4 == 0 with 4-aligned
// offsets)
struct Stat8 {
  double sa, qa, sb, qb;
};
TAIR_DEV void stat8_add(const StatTgt& t, int n, const float (&v)[8], Stat8& a) {
  const int c = t.c_off + n;
  const int bnd = (c / t.cg + 1) * t.cg - c;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const double d = v[e];
    if (e < bnd) { a.sa += d; a.qa += d * d; }
    else { a.sb += d; a.qb += d * d; }
  }
}
TAIR_DEV void stat8_flush(double* red, const StatTgt& t, int n, int gbase, Stat8& a) {
  const int gA = (t.c_off + n) / t.cg - gbase;
  if (a.sa != 0.0 || a.qa != 0.0) {
    atomicAdd(red + 2 * gA, a.sa);
    atomicAdd(red + 2 * gA + 1, a.qa);
  }
  if (a.sb != 0.0 || a.qb != 0.0) {
    atomicAdd(red + 2 * gA + 2, a.sb);
    atomicAdd(red + 2 * gA + 3, a.qb);
  }
  a = Stat8{0.0, 0.0, 0.0, 0.0};
}

// Operands of one item, loaded before any item of the batch is finished (latency overlap).
struct EpiIn {
  float a[8];       // alpha * acc (bias etc. added in epilogue8)
  float4 b0, b1;    // bias
  float4 e0, e1;    // time embedding
  uint4 r, rl;      // residual hi / lo (bf16 x 8)
  float lmu, lrs;   // folded LayerNorm: the row's mean and rstd
  float4 c0, c1;    // folded LayerNorm: column sums of W'
};

// Epilogue feature sets: the items loop of epilogue_tile is compiled per set F, whose bits stand for the
// GemmArgs features of a tile (epi_mask); E_GENERIC compiles every feature as a runtime test.
constexpr unsigned E_BIAS = 1, E_EMB = 2, E_RES = 4, E_RESLO = 8, E_OUTLO = 16, E_STATS = 32, E_STATS2 = 64,
                   E_ROWST = 128, E_LNC = 256, E_SILU = 512, E_GEGLU = 1024, E_GENERIC = 1u << 31;
// (F, runtime test): the test in the generic loop, the set's bit in a listed one
#define TAIR_EH(F, BIT, RT) (((F) & E_GENERIC) ? (bool)(RT) : (((F) & (BIT)) != 0))

template <unsigned F = E_GENERIC, class PA>
TAIR_DEV void epi_load(const PA& p, int m, int n, bool vec, EpiIn& in) {
  if (!vec) return;  // the scalar tail path loads its operands itself
  if (TAIR_EH(F, E_LNC, p.lnst)) {
    in.c0 = *(const float4*)(p.lncs + n);
    in.c1 = *(const float4*)(p.lncs + n + 4);
  }
  if (TAIR_EH(F, E_BIAS, p.bias)) {
    const float* bp = p.bias + n;
    in.b0 = *(const float4*)bp;
    in.b1 = *(const float4*)(bp + 4);
  }
  if (TAIR_EH(F, E_EMB, p.emb)) {
    const float* ep = p.emb + (size_t)p.emb_row[m / p.rows_per_b] * p.ld_emb + n;
    in.e0 = *(const float4*)ep;
    in.e1 = *(const float4*)(ep + 4);
  }
  if (TAIR_EH(F, E_RES, p.res)) {
    const bf16* rp = p.res + (size_t)m * p.ld_res + n;
    in.r = *(const uint4*)rp;
    if (TAIR_EH(F, E_RESLO, p.res_lo)) in.rl = *(const uint4*)(rp + p.res_lo);
  }
}

// The epilogue of 8 channels n..n+7 of row m (same arithmetic and order as epilogue4); `vec`: the
// 16-byte vector path (n + 8 <= N, aligned operands), else element-wise with bounds.  stored[] gets the
// values the GroupNorm statistics see (the rounded bf16 output, or v for two-plane / split outputs).
template <unsigned F = E_GENERIC, class PA>
TAIR_DEV void epilogue8(const PA& p, int m, int n, bool vec_rt, const EpiIn& in, float (&stored)[8]) {
  constexpr bool GEN = (F & E_GENERIC) != 0;
  const bool vec = GEN ? vec_rt : true;  // (listed sets: full aligned 8-channel items)
  float v[8];
  const float bscale = p.scale_bias ? p.alpha : 1.f;
  const int ne = vec ? 8 : max(0, min(8, p.N - n));
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = in.a[e];
  if (GEN && (p.row_scale || p.col_scale)) {  // fp8 dequantisation: token scale (or 1) x channel scale
    const float rs = p.row_scale ? p.row_scale[m] : 1.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= rs * (e < ne ? p.col_scale[n + e] : 0.f);
  }
  if (TAIR_EH(F, E_LNC, p.lnst)) {  // folded LayerNorm: v = rstd (acc - mean * colsum), the row's mean / rstd from the tile's LDS
    if (vec) {
      const float cc[8] = {in.c0.x, in.c0.y, in.c0.z, in.c0.w, in.c1.x, in.c1.y, in.c1.z, in.c1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = epi_lnfold(v[e], in.lmu, in.lrs, cc[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = e < ne ? epi_lnfold(v[e], in.lmu, in.lrs, p.lncs[n + e]) : 0.f;
    }
  }
  if (vec) {
    if (TAIR_EH(F, E_BIAS, p.bias)) {
      const float bb[8] = {in.b0.x, in.b0.y, in.b0.z, in.b0.w, in.b1.x, in.b1.y, in.b1.z, in.b1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = epi_bias(v[e], bscale, bb[e]);
    }
    if (TAIR_EH(F, E_EMB, p.emb)) {
      const float ee[8] = {in.e0.x, in.e0.y, in.e0.z, in.e0.w, in.e1.x, in.e1.y, in.e1.z, in.e1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += ee[e];
    }
    if (TAIR_EH(F, E_RES, p.res)) {
      union { uint4 u; bf16 h[8]; } r, rl;
      r.u = in.r;
      rl.u = in.rl;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += TAIR_EH(F, E_RESLO, p.res_lo) ? bf2f(r.h[e]) + bf2f(rl.h[e]) : bf2f(r.h[e]);
    }
  } else {
    const float* embrow = p.emb ? p.emb + (size_t)p.emb_row[m / p.rows_per_b] * p.ld_emb : nullptr;
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // (compile-time indices everywhere: a runtime-indexed array goes to scratch)
      if (e >= ne) continue;
      if (p.bias) v[e] = epi_bias(v[e], bscale, p.bias[n + e]);
      if (embrow) v[e] += embrow[n + e];
      if (p.res) {
        const bf16* rp = p.res + (size_t)m * p.ld_res + n + e;
        v[e] += p.res_lo ? bf2f(rp[0]) + bf2f(rp[p.res_lo]) : bf2f(rp[0]);
      }
    }
  }
  if (TAIR_EH(F, E_SILU, p.act == 1)) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = silu_f(v[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) stored[e] = 0.f;
  if (TAIR_EH(F, E_GEGLU, p.act == 2)) {  // GEGLU pairs (x_2q, x_2q+1, gate_2q, gate_2q+1) -> out columns 2q, 2q+1 (N % 4 == 0)
    const bf16x4 y = {f2bf(v[0] * gelu_erf(v[2])), f2bf(v[1] * gelu_erf(v[3])), f2bf(v[4] * gelu_erf(v[6])),
                      f2bf(v[5] * gelu_erf(v[7]))};
    if (GEN && (p.probe & 1)) {
      asm volatile("" ::"v"(y));
      return;
    }
    bf16* o = (bf16*)p.out + (size_t)m * p.ldo + (n >> 1);
    if (!GEN || (ne == 8 && (((uintptr_t)o) & 7) == 0)) {
      *(bf16x4*)o = y;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (2 * e < ne) o[e] = y[e];
    }
    return;
  }
  if (GEN && p.out_split) {  // 3-plane split output (the statistics see the fp32 value)
    union { uint4 u; bf16 h[8]; } hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      hi.h[e] = f2bf(v[e]);
      lo.h[e] = f2bf(v[e] - bf2f(hi.h[e]));
      stored[e] = e < ne ? v[e] : 0.f;
    }
    bf16* o = (bf16*)p.out + (size_t)m * p.ldo + n;
    bf16* o1 = o + p.N;
    bf16* o2 = o + 2 * p.N;
    const uint4 second = p.out_split == 1 ? lo.u : hi.u, third = p.out_split == 1 ? hi.u : lo.u;
    if (ne == 8 && al16(o) && al16(o1) && al16(o2)) {
      *(uint4*)o = hi.u;
      *(uint4*)o1 = second;
      *(uint4*)o2 = third;
    } else {
      union { uint4 u; bf16 h[8]; } s2, s3;
      s2.u = second;
      s3.u = third;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (e >= ne) continue;
        o[e] = hi.h[e];
        o1[e] = s2.h[e];
        o2[e] = s3.h[e];
      }
    }
    return;
  }
  if (GEN && p.out_f32) {
    float* o = (float*)p.out + (size_t)m * p.ldo + n;
    if (p.probe & 1) {
      asm volatile("" ::"v"(v[0]), "v"(v[7]));
      return;
    }
    if (ne == 8 && al16(o)) {
      *(float4*)o = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < ne) o[e] = v[e];
    }
    return;
  }
  bf16* o = (bf16*)p.out + (size_t)m * p.ldo + n;
  union { uint4 u; bf16 h[8]; } w, lo;
#pragma unroll
  for (int e = 0; e < 8; ++e) w.h[e] = f2bf(v[e]);
  if (GEN && (p.probe & 1)) {  // measurement probe: the values are formed but not stored
    asm volatile("" ::"v"(w.u.x), "v"(w.u.w));
    return;
  }
  if (TAIR_EH(F, E_OUTLO, p.out_lo)) {  // two-plane storage: hi + lo carries v to ~2^-16; consumers (and the statistics) see v
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      lo.h[e] = f2bf(v[e] - bf2f(w.h[e]));
      stored[e] = e < ne ? v[e] : 0.f;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) stored[e] = e < ne ? bf2f(w.h[e]) : 0.f;
  }
  if (!GEN || (ne == 8 && al16(o) && (!p.out_lo || al16(o + p.out_lo)))) {
    *(uint4*)o = w.u;
    if (TAIR_EH(F, E_OUTLO, p.out_lo)) *(uint4*)(o + p.out_lo) = lo.u;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (e >= ne) continue;
      o[e] = w.h[e];
      if (p.out_lo) o[p.out_lo + e] = lo.h[e];
    }
  }
}

// Epilogue of a finished tile: the wave owns FM x FN 16x16 fragments at rows m0 + wm*WM + 16i, columns
// n0 + wn*WN + 16j (lane: 4 consecutive columns of one row).  Non-split: the full epilogue + GroupNorm
// statistics; split-K (p.splits > 1): this K slice's fp32 slab, summed by splitk_reduce_kernel.
// `smem`: the kernel's LDS (LDS_CAP bytes), free once every wave passed the barrier below (each wave
// drained its own LDS-DMA copies before calling).
// ---- in-kernel split-K combine ---------------------------------------------------------------
// Every K slice stores its accumulator fragments write-through (sc1, fragment-native layout: lane-
// linear 16-byte pieces, so every store and load is a full 1 KiB wave line), drains them, and one lane
// takes the tile's arrival ticket (agent-scope atomic); the slice that draws splits - 1 adds the other
// slabs (sc1 loads: no acquire fence needed, cdna_hip_programming.md Guideline 16 R1) and goes on to
// the full epilogue.  It resets the ticket for the next launch.  Returns false for the other slices.
constexpr int INK_SMAX_BUILT = 16;  // largest split count the launcher combines in-kernel
template <int BM, int BN, int FM, int FN, class PA>
TAIR_DEV bool splitk_combine(const PA& p, f32x4 (&acc)[FN][FM], int m0, int n0, int lane, char* smem,
                             int bz) {
  constexpr int TILE = BM * BN;  // floats per slab
  const int S = p.splits;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = (m0 / BM) * ((p.N + BN - 1) / BN) + n0 / BN;
  float* base = p.partial + (size_t)tile * S * TILE;
  const __amdgpu_buffer_rsrc_t mine = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)bz * TILE, 0, TILE * 4,
                                                                        0x00020000);
  static_for<0, FN>([&](auto J) {
    constexpr int j = decltype(J)::value;
    static_for<0, FM>([&](auto I) {
      constexpr int i = decltype(I)::value;
      __builtin_amdgcn_raw_buffer_store_b128(acc[j][i], mine, (((wid * FN + j) * FM + i) * 64 + lane) * 16, 0,
                                             16 /* sc1 */);
    });
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its slab stores
  __syncthreads();
  int* flag = (int*)smem;
  if (threadIdx.x == 0)
    *flag = __hip_atomic_fetch_add(p.tile_sem + tile * p.sem_stride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            S - 1;
  __syncthreads();
  const bool last = *flag;
  __syncthreads();  // the flag is read before the epilogue's staging reuses the LDS
  if (!last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the ticket)
  // sum in slice order 0 + s_0 + s_1 + ... (splitk_reduce_kernel's order: both paths give the same bits,
  // whichever slice arrives last).  Every slab, this slice's own included, is read back (the own slab's
  // values are its fragments, drained above), LD slabs in flight per batch: the slabs of other XCDs'
  // slices come from beyond this XCD's L2, so one slab at a time would chain S - 1 memory latencies.
  constexpr int LD = FN * FM >= 16 ? 1 : FN * FM >= 8 ? 2 : 4;  // (the launcher combines 64-row tiles only)
  const __amdgpu_buffer_rsrc_t all = __builtin_amdgcn_make_buffer_rsrc(base, 0, S * TILE * 4, 0x00020000);
  static_for<0, FN>([&](auto J) {
    static_for<0, FM>([&](auto I) { acc[decltype(J)::value][decltype(I)::value] = f32x4{0.f, 0.f, 0.f, 0.f}; });
  });
  for (int z0 = 0; z0 < S; z0 += LD) {
    f32x4 t[LD][FN][FM];
    static_for<0, LD>([&](auto Z) {
      constexpr int zz = decltype(Z)::value;
      if (z0 + zz < S) {
        static_for<0, FN>([&](auto J) {
          constexpr int j = decltype(J)::value;
          static_for<0, FM>([&](auto I) {
            constexpr int i = decltype(I)::value;
            t[zz][j][i] = __builtin_amdgcn_raw_buffer_load_b128(all, (((wid * FN + j) * FM + i) * 64 + lane) * 16,
                                                                (z0 + zz) * TILE * 4, 16 /* sc1 */);
          });
        });
      }
    });
    static_for<0, LD>([&](auto Z) {
      constexpr int zz = decltype(Z)::value;
      if (z0 + zz < S) {
        static_for<0, FN>([&](auto J) {
          static_for<0, FM>([&](auto I) {
            acc[decltype(J)::value][decltype(I)::value] += t[zz][decltype(J)::value][decltype(I)::value];
          });
        });
      }
    });
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(p.tile_sem + tile * p.sem_stride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// ---- cooperative split-K combine -------------------------------------------------------------
// Every K slice stores its accumulator tile row-major ([BM][BN] fp32 slab, write-through sc1 stores),
// drains them and takes the tile's arrival ticket; one lane then polls the ticket word (relaxed agent-scope
// loads + s_sleep) until all `splits` slices have arrived.  The last to arrive resets the word: within a
// launch it only counts up, so a poller that reads a value at or below its own ticket saw the reset and
// knows every slice arrived.  Slice z then sums rows [z BM / S, (z + 1) BM / S) of every slab in slice order
// 0, 1, ..., S - 1 (splitk_reduce_kernel's order: the same bits) with sc1 loads (Guideline 16 R1) into the
// LDS stage, and epilogue_tile finishes those rows.  The launcher puts a tile's slices on consecutive
// workgroups (xcd_remap 3 / 4) and uses it only on grids the chip holds at once, so every slice a tile
// waits for is resident or next in dispatch order.
template <int BM, int BN, int FM, int FN, int WM, int WN, int LDR, int NT, class PA>
TAIR_DEV void splitk_coop(const PA& p, f32x4 (&acc)[FN][FM], int m0, int n0, int wm, int wn, int lane, float* stage,
                          int bz, int& r_lo, int& r_hi) {
  constexpr int TILE = BM * BN;  // floats per slab
  constexpr int PR = BN / 4;     // 16-byte pieces per row
  const int S = p.splits;
  const int tile = (m0 / BM) * ((p.N + BN - 1) / BN) + n0 / BN;
  float* base = p.partial + (size_t)tile * S * TILE;
  const __amdgpu_buffer_rsrc_t mine = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)bz * TILE, 0, TILE * 4,
                                                                        0x00020000);
  static_for<0, FN>([&](auto J) {
    constexpr int j = decltype(J)::value;
    static_for<0, FM>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int row = wm * WM + 16 * i + (lane & 15), col = wn * WN + 16 * j + 4 * (lane >> 4);
      __builtin_amdgcn_raw_buffer_store_b128(acc[j][i], mine, (row * BN + col) * 4, 0, 16 /* sc1 */);
    });
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its slab stores
  __syncthreads();
  if (threadIdx.x == 0) {
    int* sem = p.tile_sem + tile * p.sem_stride;
    const int t = __hip_atomic_fetch_add(sem, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == S - 1) {
      __hip_atomic_store(sem, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      // bounded, so a protocol fault never hangs the queue; a wait that runs out is counted in the launch's
      // fault word (vector atomic), which the host reads (gemm_fault_count) and reports as an error instead of
      // returning the sums of incomplete slabs as a result
      bool done = false;
      for (int spin = 0; spin < (1 << 24) && !done; ++spin) {
        const int v = __hip_atomic_load(sem, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done = v >= S || v <= t;
        if (!done) __builtin_amdgcn_s_sleep(2);
      }
      int* fault = kernarg0<GemmGroup>().fault;  // (cooperative plans run only in gemm_tile_kernel)
      if (!done && fault) __hip_atomic_fetch_add(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the wait)
  r_lo = bz * BM / S;
  r_hi = (bz + 1) * BM / S;
  const __amdgpu_buffer_rsrc_t all = __builtin_amdgcn_make_buffer_rsrc(base, 0, S * TILE * 4, 0x00020000);
  for (int pc = threadIdx.x; pc < (r_hi - r_lo) * PR; pc += NT) {
    const int r = r_lo + pc / PR, c = (pc % PR) * 4;
    f32x4 x[INK_SMAX_BUILT];
    static_for<0, INK_SMAX_BUILT>([&](auto Z) {  // every slab's piece in flight before the first add
      constexpr int z = decltype(Z)::value;
      if (z < S) x[z] = __builtin_amdgcn_raw_buffer_load_b128(all, (r * BN + c) * 4, z * TILE * 4, 16 /* sc1 */);
    });
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    static_for<0, INK_SMAX_BUILT>([&](auto Z) {
      if (decltype(Z)::value < S) sum += x[decltype(Z)::value];
    });
    *(f32x4*)(stage + r * LDR + c) = sum;
  }
  __syncthreads();
}

// Item geometry of epilogue_tile: the column pass width CP, NV items of 8 channels per row, U items per
// thread in flight.
template <int BM, int BN, int FM, int FN, int WN, int NT, int LDS_CAP>
struct EpiGeom {
  static constexpr int WNW = BN / WN;
  static constexpr int RED_BYTES = 4 * STAT_NG * (int)sizeof(double);
  static constexpr int Q = epi_q(BM, WN, WNW, LDS_CAP - RED_BYTES);
  static constexpr int CP = WN * Q, LDR = CP + 4, NV = CP / 8, ITEMS = BM * NV;
  // items per thread in flight (2 measured slower on the batched tiles; beside the 128x320 tile it spilled).
  // TAIR_EPI_U_SMALL (A/B experiment): U for the 4-wave 64x64 tiles of >= 3-deep rings (the B = 1 plans)
  // TAIR_EPI_U_BIG (A/B experiment): U for the 8-wave tiles (one workgroup per CU: nothing else on the CU
  // hides the items' memory latency)
  static constexpr int U = (TAIR_EPI_U_SMALL > 1 && FM * FN <= 4 && NT == 256 && LDS_CAP >= 3 * (BM + BN) * 128)
                               ? TAIR_EPI_U_SMALL
                               : (TAIR_EPI_U_BIG > 1 && NT == 512 && FM * FN <= 16 && ITEMS >= NT * TAIR_EPI_U_BIG)
                                     ? TAIR_EPI_U_BIG : 1;
};

// The feature set of a finished tile (uniform): a listed set needs full aligned 8-channel items and no
// slab / split / fp32 / fp8-scaled output; anything else takes the generic loop.
TAIR_DEV unsigned epi_mask(const EpiArgs& p, bool slab, bool stats, bool stats2, bool rowst, bool lnc,
                           bool vec_base) {
  if (slab || p.out_split || p.out_f32 || p.row_scale || p.col_scale || (p.probe & ~128) || !vec_base || p.act > 2 ||
      !al16(p.out) || (p.ldo & 7) || (p.out_lo & 7) || (p.bias && !al16(p.bias)) ||
      (p.emb && (!al16(p.emb) || (p.ld_emb & 3))) || (p.res && (!al16(p.res) || (p.ld_res & 7) || (p.res_lo & 7))) ||
      (p.lnst && (!lnc || !al16(p.lncs))) || (p.rst && !rowst))
    return E_GENERIC;
  return (p.bias ? E_BIAS : 0u) | (p.emb ? E_EMB : 0u) | (p.res ? E_RES : 0u) | (p.res && p.res_lo ? E_RESLO : 0u) |
         (p.out_lo ? E_OUTLO : 0u) | (stats ? E_STATS : 0u) | (stats2 ? E_STATS2 : 0u) | (rowst ? E_ROWST : 0u) |
         (lnc ? E_LNC : 0u) | (p.act == 1 ? E_SILU : 0u) | (p.act == 2 ? E_GEGLU : 0u);
}
// The listed sets: the epilogues of the denoise step (cldm.cpp: ResBlock conv1 / conv2 with and without the
// trunk residual, the transformer's proj_in, LayerNorm-folded q|k|v, q and GEGLU-in, the out-projections,
// FF-out, proj_out, zero-convs, resamplers)
#ifndef TAIR_EPI_SETS
#define TAIR_EPI_SETS 1
#endif
#define TAIR_EPI_LISTED(X)                                                                        \
  X(E_BIAS | E_EMB | E_STATS)                                                                     \
  X(E_BIAS | E_RES | E_RESLO | E_OUTLO) X(E_BIAS | E_RES | E_RESLO | E_OUTLO | E_STATS)           \
  X(E_BIAS | E_RES | E_RESLO | E_OUTLO | E_STATS | E_STATS2)                                      \
  X(E_BIAS | E_OUTLO) X(E_BIAS | E_OUTLO | E_STATS) X(E_BIAS | E_OUTLO | E_STATS | E_STATS2)      \
  X(E_BIAS | E_ROWST) X(E_BIAS | E_LNC) X(E_BIAS | E_RES | E_ROWST) X(E_BIAS | E_LNC | E_GEGLU)    \
  X(E_BIAS | E_RES) X(E_BIAS)

// COMBINE: the kernel may combine K slices in-kernel (splitk_coop / splitk_combine): the launcher does that only
// for the 64-row tile kernels with >= 3-deep rings (gemm_grouped `ink`), so the other instances compile without
// the combine paths (the 2-stage 64x64 tile spilled 27 VGPRs at its 4-waves-per-SIMD bound for code it never runs)
// SLAB: the kernel may store fp32 K-slice slabs for splitk_reduce_kernel (all but the 2-stage 64-row tiles, which
// the launcher never splits)
template <int BM, int BN, int FM, int FN, int WM, int WN, int NT, int LDS_CAP, bool COMBINE = true, bool SLAB = true>
TAIR_DEV void epilogue_tile(const GemmArgs& pk, f32x4 (&acc)[FN][FM], int m0, int n0, int wm, int wn, int lane,
                            char* smem, int bz) {
  constexpr bool COMBINE_OR_SLAB = COMBINE || SLAB;
  const EpiArgs p = epi_args(pk);  // one batch of kernel-argument loads, kept in registers
  using G = EpiGeom<BM, BN, FM, FN, WN, NT, LDS_CAP>;
  constexpr int WNW = G::WNW;
  constexpr int RED_BYTES = G::RED_BYTES;
  constexpr int Q = G::Q;
  static_assert(Q > 0 && WN % 8 == 0, "epilogue staging does not fit the kernel's LDS");
  constexpr int CP = G::CP, LDR = G::LDR, NV = G::NV, ITEMS = G::ITEMS;
  constexpr int U = G::U;
  constexpr bool FIXED_COL = (NT % NV) == 0;  // a thread's items share one column vector
  if (p.probe & 2) {  // measurement probe: no epilogue at all (the accumulators kept live)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(acc[j][i]));
    return;
  }
  float* stage = (float*)smem;
  double* red = (double*)(smem + BM * LDR * 4);
  bool slab = COMBINE_OR_SLAB && p.splits > 1;  // (2-stage 64-row tiles: never split, host-checked)
  const int tid = threadIdx.x;
  __syncthreads();  // every wave is done reading the main loop's LDS
  int r_lo = 0, r_hi = BM;  // the rows this workgroup finishes (cooperative split-K: 1/splits of them)
  bool coop = false;
  if constexpr (Q == WNW && COMBINE) {  // (one-pass stage: the cooperative combine fills it)
    if (slab && p.tile_sem && p.coop) {
      splitk_coop<BM, BN, FM, FN, WM, WN, LDR, NT>(p, acc, m0, n0, wm, wn, lane, stage, bz, r_lo, r_hi);
      slab = false;
      coop = true;
    }
  }
  if constexpr (COMBINE) {
    if (slab && p.tile_sem) {  // in-kernel combine (gemm_grouped picked it): only the last slice goes on
      if (!splitk_combine<BM, BN, FM, FN>(p, acc, m0, n0, lane, smem, bz)) {
        stamp(p, 7);
        return;
      }
      slab = false;
    }
  }
  stamp(p, 4);
  const bool stats = !slab && p.st[0].acc != nullptr;
  const bool stats2 = stats && p.st[1].acc != nullptr;
  // LayerNorm row statistics of the output (host: BM <= 128, no GroupNorm targets): [BM][2] doubles in
  // the reduction area, one fp64 atomic pair per row per tile at the end
  const bool rowst = BM * 16 <= RED_BYTES && !slab && p.rst != nullptr;
  if (rowst)
    for (int i = tid; i < 2 * BM; i += NT) red[i] = 0.0;
  // folded-LayerNorm consumer: every row's (mean, rstd) once per tile, into the reduction area (host:
  // no GroupNorm / row-statistics targets beside it); read by the items after the pass barrier
  float2* const lrow = (float2*)red;
  const bool lnc = BM * 8 <= RED_BYTES && !slab && p.lnst != nullptr;
  if (lnc)
    for (int r = tid; r < BM; r += NT)
      if (m0 + r < p.M) {
        float mu, rstd;
        ln_row(p, m0 + r, mu, rstd);
        lrow[r] = make_float2(mu, rstd);
      }
  if (stats)
    for (int i = tid; i < 4 * STAT_NG; i += NT) red[i] = 0.0;
  const int gb0 = stats ? (p.st[0].c_off + n0) / p.st[0].cg : 0;
  const int gb1 = stats2 ? (p.st[1].c_off + n0) / p.st[1].cg : 0;
  const bool vec_base = (p.N & 7) == 0;
  // the items loop is compiled once per epilogue feature set F (epi_mask): a tile whose features match a
  // listed set runs a loop without per-feature branches (the generic loop's branches cost ~1 us per B = 1
  // launch, tools/b1_probe.py), any other runs the generic loop (F = E_GENERIC: every feature a runtime test)
  const unsigned mask = epi_mask(p, slab, stats, stats2, rowst, lnc, vec_base);
  const int it_lo = r_lo * NV, it_hi = r_hi * NV;  // the items of those rows
  auto run_items = [&](auto FC, int pass) {
    constexpr unsigned F = decltype(FC)::value;
    constexpr bool GEN = (F & E_GENERIC) != 0;
    const bool f_slab = GEN && slab;
    const bool f_stats = GEN ? stats : (F & E_STATS) != 0;
    const bool f_stats2 = GEN ? stats2 : (F & E_STATS2) != 0;
    const bool f_rowst = GEN ? rowst : (F & E_ROWST) != 0;
    const bool f_lnc = GEN ? lnc : (F & E_LNC) != 0;
    Stat8 s0{0.0, 0.0, 0.0, 0.0}, s1{0.0, 0.0, 0.0, 0.0};
    int stat_n = -1;
    for (int it0 = it_lo + tid; it0 < it_hi; it0 += NT * U) {
      stamp_it(p.stamps, 48 + 2 * pass + 8 * ((it0 - it_lo - tid) / (NT * U)), 0);  // (TAIR_STAMPS >= 2: items)
      EpiIn in[U];
      int mm[U], nn[U];
      bool ok[U], vec[U];
      static_for<0, U>([&](auto UU) {  // operands of all U items first: their latencies overlap
        constexpr int u = decltype(UU)::value;
        const int it = it0 + u * NT;
        const int row = it / NV, col = (it - row * NV) * 8;
        mm[u] = m0 + row;
        nn[u] = n0 + pass * CP + col;
        ok[u] = it < it_hi && mm[u] < p.M && nn[u] < p.N;
        vec[u] = GEN ? ok[u] && vec_base && nn[u] + 8 <= p.N : ok[u];  // (listed sets: N % 8 == 0)
        if (ok[u]) {
          const float4 x0 = *(const float4*)(stage + row * LDR + col);
          const float4 x1 = *(const float4*)(stage + row * LDR + col + 4);
          const float al = f_slab ? 1.f : p.alpha;
          in[u].a[0] = epi_alpha(x0.x, al); in[u].a[1] = epi_alpha(x0.y, al);
          in[u].a[2] = epi_alpha(x0.z, al); in[u].a[3] = epi_alpha(x0.w, al);
          in[u].a[4] = epi_alpha(x1.x, al); in[u].a[5] = epi_alpha(x1.y, al);
          in[u].a[6] = epi_alpha(x1.z, al); in[u].a[7] = epi_alpha(x1.w, al);
          if (!f_slab) epi_load<F>(p, mm[u], nn[u], vec[u], in[u]);
          if (f_lnc) {
            const float2 lr = lrow[row];
            in[u].lmu = lr.x;
            in[u].lrs = lr.y;
          }
        }
      });
      stamp_it(p.stamps, 48 + 2 * pass + 8 * ((it0 - it_lo - tid) / (NT * U)), 1);
      double rsu[U], rqu[U];  // LayerNorm row statistics of the items' stored values
      static_for<0, U>([&](auto UU) {
        constexpr int u = decltype(UU)::value;
        rsu[u] = 0.0;
        rqu[u] = 0.0;
        if (!ok[u]) return;
        const int m = mm[u], n = nn[u];
        if (f_slab) {  // this K slice's partial sums, one fp32 row segment per item
          float* dst = p.partial + ((size_t)bz * p.M + m) * p.N + n;
          if (vec[u] && al16(dst)) {
            *(float4*)dst = make_float4(in[u].a[0], in[u].a[1], in[u].a[2], in[u].a[3]);
            *(float4*)(dst + 4) = make_float4(in[u].a[4], in[u].a[5], in[u].a[6], in[u].a[7]);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (n + e < p.N) dst[e] = in[u].a[e];
          }
          return;
        }
        float st[8];
        epilogue8<F>(p, m, n, vec[u], in[u], st);
        if (f_rowst) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            rsu[u] += st[e];
            rqu[u] += (double)st[e] * st[e];
          }
        }
        if (f_stats) {
          if (!FIXED_COL && stat_n >= 0 && stat_n != n) {
            stat8_flush(red, p.st[0], stat_n, gb0, s0);
            if (f_stats2) stat8_flush(red + 2 * STAT_NG, p.st[1], stat_n, gb1, s1);
          }
          stat_n = n;
          stat8_add(p.st[0], n, st, s0);
          if (f_stats2) stat8_add(p.st[1], n, st, s1);
        }
      });
      stamp_it(p.stamps, 48 + 2 * pass + 8 * ((it0 - it_lo - tid) / (NT * U)), 2);
      if (f_rowst) {
        static_for<0, U>([&](auto UU) {  // the NV lanes of a row reduce by shuffles, one LDS add per row
          constexpr int u = decltype(UU)::value;
          const int row = (it0 + u * NT) / NV;
          double rs = rsu[u], rq = rqu[u];
          if constexpr (FIXED_COL && NV <= 64 && 64 % NV == 0) {
#pragma unroll
            for (int o = 1; o < NV; o <<= 1) {
              rs += __shfl_xor(rs, o, 64);
              rq += __shfl_xor(rq, o, 64);
            }
            if (lane % NV == 0 && row < BM) {
              atomicAdd(red + 2 * row, rs);
              atomicAdd(red + 2 * row + 1, rq);
            }
          } else if (row < BM && (rs != 0.0 || rq != 0.0)) {
            atomicAdd(red + 2 * row, rs);
            atomicAdd(red + 2 * row + 1, rq);
          }
        });
      }
    }
    if (f_stats && stat_n >= 0) {
      stat8_flush(red, p.st[0], stat_n, gb0, s0);
      if (f_stats2) stat8_flush(red + 2 * STAT_NG, p.st[1], stat_n, gb1, s1);
    }
  };
  for (int pass = 0; pass < WNW / Q; ++pass) {
    if (!coop && wn / Q == pass) {
      const int cb = (wn - pass * Q) * WN + 4 * (lane >> 4);
      static_for<0, FN>([&](auto J) {
        constexpr int j = decltype(J)::value;
        static_for<0, FM>([&](auto I) {
          constexpr int i = decltype(I)::value;
          *(f32x4*)(stage + (wm * WM + 16 * i + (lane & 15)) * LDR + cb + 16 * j) = acc[j][i];
        });
      });
    }
    __syncthreads();
    if (pass == 0) stamp(p, 5);
    switch (mask) {  // (TAIR_EPI_SETS=0: the generic loop only, A/B builds)
#if TAIR_EPI_SETS
#define TAIR_EPI_CASE(S) \
      case (S): run_items(std::integral_constant<unsigned, (S)>{}, pass); break;
      TAIR_EPI_LISTED(TAIR_EPI_CASE)
#undef TAIR_EPI_CASE
#endif
      default: run_items(std::integral_constant<unsigned, E_GENERIC>{}, pass); break;
    }
    __syncthreads();  // the stage is rewritten by the next pass / the statistics are complete
  }
  stamp(p, 6);
  if (stats) {
    const int b = m0 / p.st[0].hw;
    stat_flush(p, red, b, n0, min(p.N, n0 + BN), (blockIdx.x + blockIdx.y + blockIdx.z) & (STAT_REPL - 1));
  }
  if (rowst)  // (every item's LDS adds precede the pass's closing barrier; a cooperative slice: its own rows)
    for (int r = r_lo + tid; r < r_hi; r += NT)
      if (m0 + r < p.M) {
        unsafeAtomicAdd(p.rst + 2 * (size_t)(m0 + r), red[2 * r]);
        unsafeAtomicAdd(p.rst + 2 * (size_t)(m0 + r) + 1, red[2 * r + 1]);
      }
  stamp(p, 7);
}

// ---- register-staged epilogue of the wide tiles and the 64-row B = 1 tiles (round 6) ---------------------
// The LDS-staged epilogue_tile moves a 256-row tile's fp32 accumulators through the LDS in WNW column passes
// (only the waves of the pass's columns storing, a barrier pair per pass, each item then re-loading its
// column operands): on the batched GEGLU-in linear (64^2 level, M = 262144, N = 2560, K = 320) it took 590 of
// 1053 us, and 480 us with a bias-only epilogue, against 410 us for the whole main loop
// (profiles/r06_geglu_probe*.log).  For the feature sets without GroupNorm statistics or split outputs -- bias,
// folded LayerNorm, GEGLU, a bf16 / hi + lo residual, LayerNorm row statistics of the output: FF-in, the
// LayerNorm-fed projections, proj_in, the out-projections, FF-out -- every wave forms its values
// straight from its accumulator fragments (same arithmetic and order as epilogue8, so the bits are the same),
// writes them as bf16 into an LDS image of the output tile (all waves at once, one barrier), and the
// workgroup copies that image out in 16-byte row-contiguous pieces.  The 3-deep 64-row tiles of the B = 1 plans
// take it too (GEGLU-in 39.2 -> 33.9 us at 64^2, B = 1 step +2.0% paired, profiles/r06_b1_geglu_probe.log,
// r06_b1_epireg_*.log).
template <int BM, int BN, int LDS_CAP>
struct RegStage {
  static constexpr int ROWB_GEGLU = BN + 16;      // BN / 2 bf16 output columns + 16 B of bank padding
  static constexpr int ROWB_PLAIN = 2 * BN + 16;
  // + per row: (mean, rstd) of a folded LayerNorm (8 B) and the LayerNorm row-statistics partials (16 B)
  static constexpr bool GEGLU_FITS = BM * ROWB_GEGLU + BM * 24 <= LDS_CAP;
  static constexpr bool PLAIN_FITS = BM * ROWB_PLAIN + BM * 24 <= LDS_CAP;
};
#ifndef TAIR_EPI_REG
#define TAIR_EPI_REG 1
#endif
// the register-staged feature set of a finished tile, or 0 (epilogue_tile); GemmArgs.probe bit 7 (128) turns it off
// (A/B measurements: tools/geglu_probe.py "e128:")
template <int BM, int BN, int LDS_CAP>
TAIR_DEV unsigned regstage_set(const EpiArgs& p) {
  if (!TAIR_EPI_REG || p.splits > 1 || p.probe || p.st[0].acc || p.emb || p.out_lo || p.out_split || p.out_f32 ||
      p.row_scale || p.col_scale || (p.act != 0 && p.act != 2) || (p.ldo & 7) || !al16(p.out) ||
      (p.bias && !al16(p.bias)) || (p.lnst && !al16(p.lncs)) ||
      (p.res && ((((uintptr_t)p.res) & 7) || (p.ld_res & 3) || (p.res_lo & 3))) || (BM > 128 && p.rst))
    return 0;
  if (p.act == 2 && (!RegStage<BM, BN, LDS_CAP>::GEGLU_FITS || (p.N & 15) || p.res || p.rst)) return 0;
  if (p.act == 0 && (!RegStage<BM, BN, LDS_CAP>::PLAIN_FITS || (p.N & 7))) return 0;
  return (p.bias ? E_BIAS : 0u) | (p.lnst ? E_LNC : 0u) | (p.act == 2 ? E_GEGLU : 0u) | (p.res ? E_RES : 0u) |
         (p.res && p.res_lo ? E_RESLO : 0u) | (p.rst ? E_ROWST : 0u);
}
template <unsigned F, int BM, int BN, int FM, int FN, int WM, int WN, int NT, int LDS_CAP>
TAIR_DEV void epilogue_regstage(const EpiArgs& p, f32x4 (&acc)[FN][FM], int m0, int n0, int wm, int wn, int lane,
                                char* smem) {
  constexpr bool GEGLU = (F & E_GEGLU) != 0, LNC = (F & E_LNC) != 0, BIAS = (F & E_BIAS) != 0;
  constexpr bool RES = (F & E_RES) != 0, RESLO = (F & E_RESLO) != 0, ROWST = (F & E_ROWST) != 0;
  constexpr int OUTC = GEGLU ? BN / 2 : BN;  // output columns of the tile
  constexpr int ROWB = GEGLU ? RegStage<BM, BN, LDS_CAP>::ROWB_GEGLU : RegStage<BM, BN, LDS_CAP>::ROWB_PLAIN;
  float2* const lrow = (float2*)(smem + BM * ROWB);
  double* const rred = (double*)(smem + BM * ROWB + BM * 8);  // [BM][2] row (sum, sum^2) of the stored values
  const int tid = threadIdx.x;
  __syncthreads();  // every wave is done reading the main loop's LDS
  if constexpr (LNC) {
    for (int r = tid; r < BM; r += NT) {
      float mu = 0.f, rstd = 0.f;
      if (m0 + r < p.M) ln_row(p, m0 + r, mu, rstd);
      lrow[r] = make_float2(mu, rstd);
    }
  }
  if constexpr (ROWST)
    for (int i = tid; i < 2 * BM; i += NT) rred[i] = 0.0;
  if constexpr (LNC || ROWST) __syncthreads();
  double rs[FM], rq[FM];  // this lane's row partials (row wm WM + 16 i + lane % 16, its 4 x FN columns)
#pragma unroll
  for (int i = 0; i < FM; ++i) rs[i] = rq[i] = 0.0;
  const float al = p.alpha, bscale = p.scale_bias ? p.alpha : 1.f;
  static_for<0, FN>([&](auto J) {
    constexpr int j = decltype(J)::value;
    const int cl = wn * WN + 16 * j + 4 * (lane >> 4);  // tile column of the lane's 4 values (N % 8 == 0)
    const int n = n0 + cl;
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f), bb = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n < p.N) {
      if constexpr (LNC) cs = *(const float4*)(p.lncs + n);
      if constexpr (BIAS) bb = *(const float4*)(p.bias + n);
    }
    const float cc[4] = {cs.x, cs.y, cs.z, cs.w}, bv[4] = {bb.x, bb.y, bb.z, bb.w};
    static_for<0, FM>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int r = wm * WM + 16 * i + (lane & 15);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = epi_alpha(acc[j][i][e], al);
      if constexpr (LNC) {
        const float2 lr = lrow[r];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = epi_lnfold(v[e], lr.x, lr.y, cc[e]);
      }
      if constexpr (BIAS) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = epi_bias(v[e], bscale, bv[e]);
      }
      if constexpr (RES) {  // residual (may alias the output: read before this tile's copy-out), hi + lo exact in fp32
        const int m = m0 + r;
        if (m < p.M && n < p.N) {
          const bf16* rp = p.res + (size_t)m * p.ld_res + n;
          const bf16x4 h4 = *(const bf16x4*)rp;
          if constexpr (RESLO) {
            const bf16x4 l4 = *(const bf16x4*)(rp + p.res_lo);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += bf2f(h4[e]) + bf2f(l4[e]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += bf2f(h4[e]);
          }
        }
      }
      if constexpr (GEGLU) {  // (x_2q, x_2q+1, gate_2q, gate_2q+1) -> output columns 2q, 2q+1
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        const bf16x2 y = {f2bf(v[0] * gelu_erf(v[2])), f2bf(v[1] * gelu_erf(v[3]))};
        *(bf16x2*)(smem + r * ROWB + cl) = y;  // output column cl / 2, 2 bytes each
      } else {
        const bf16x4 w = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
        *(bf16x4*)(smem + r * ROWB + 2 * cl) = w;
        if constexpr (ROWST) {  // the statistics see the stored (rounded) values, as epilogue8's
          if (n < p.N) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float st = bf2f(w[e]);
              rs[i] += st;
              rq[i] += (double)st * st;
            }
          }
        }
      }
    });
  });
  if constexpr (ROWST) {  // the 4 lane groups of a row, then the WNW waves of its row range through the LDS
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      double a = rs[i], b = rq[i];
      a += __shfl_xor(a, 16, 64);
      b += __shfl_xor(b, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b += __shfl_xor(b, 32, 64);
      if (lane < 16) {
        const int r = wm * WM + 16 * i + lane;
        atomicAdd(rred + 2 * r, a);
        atomicAdd(rred + 2 * r + 1, b);
      }
    }
  }
  __syncthreads();
  if constexpr (ROWST)
    for (int r = tid; r < BM; r += NT)
      if (m0 + r < p.M) {
        unsafeAtomicAdd(p.rst + 2 * (size_t)(m0 + r), rred[2 * r]);
        unsafeAtomicAdd(p.rst + 2 * (size_t)(m0 + r) + 1, rred[2 * r + 1]);
      }
  // (ordinary stores: non-temporal ones were 0-13% slower, profiles/r06_geglu_probe6.log)
  constexpr int CPR = OUTC * 2 / 16;  // 16-byte pieces per output row
  const int oc0 = GEGLU ? n0 / 2 : n0, no = GEGLU ? p.N / 2 : p.N;
  bf16* const out = (bf16*)p.out;
#pragma unroll 4
  for (int c = tid; c < BM * CPR; c += NT) {
    const int r = c / CPR, k = c - r * CPR;
    const int m = m0 + r, col = oc0 + 8 * k;
    if (m < p.M && col < no) *(uint4*)(out + (size_t)m * p.ldo + col) = *(const uint4*)(smem + r * ROWB + 16 * k);
  }
}

// Direct (register) epilogue of a finished, unsplit tile + its GroupNorm statistics, one fragment at a
// time: for the 256-row phase kernel, whose 160-register accumulator tile cannot stay live beside the
// LDS-staged epilogue's items (epilogue_tile spilled it: 932 bytes of scratch per lane).  The wave owns
// FM x FN 16x16 fragments at rows m0 + wm*WM + 16i, columns n0 + wn*WN + 16j.  `red`: LDS that every
// wave is done reading.
template <int FM, int FN, int WM, int WN>
TAIR_DEV void epilogue_direct(const GemmArgs& pk, f32x4 (&acc)[FN][FM], int m0, int n0, int wm, int wn, int lane,
                              double* red, int bn_tile) {
  const EpiArgs p = epi_args(pk);  // one batch of kernel-argument loads, kept in registers
  const bool stats = p.st[0].acc != nullptr;
  if (p.probe & 2) {  // measurement probe: no epilogue at all (the accumulators kept live)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(acc[j][i]));
    return;
  }
  if (stats) {
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * STAT_NG; i += blockDim.x) red[i] = 0.0;
    __syncthreads();
  }
  static_for<0, FN>([&](auto J) {
    constexpr int j = decltype(J)::value;
    const int n = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
    Stat4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
    static_for<0, FM>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int m = m0 + wm * WM + i * 16 + (lane & 15);
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (m < p.M && n < p.N) {
        epilogue4(p, m, n, acc[j][i], v);
        if (stats) {
          stat_add(p.st[0], n, v, a0);
          if (p.st[1].acc) stat_add(p.st[1], n, v, a1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one fragment's operands live at a time
    });
    if (stats) {  // the 16 lanes (pixels) that share these 4 channels
      stat_shfl16(a0);
      if (p.st[1].acc) stat_shfl16(a1);
      if ((lane & 15) == 0 && n < p.N) {
        lds_stat_add(red, p.st[0], n, (p.st[0].c_off + n0) / p.st[0].cg, a0);
        if (p.st[1].acc) lds_stat_add(red + 2 * STAT_NG, p.st[1], n, (p.st[1].c_off + n0) / p.st[1].cg, a1);
      }
    }
  });
  if (stats) {
    __syncthreads();
    stat_flush(p, red, m0 / p.st[0].hw, n0, min(p.N, n0 + bn_tile), (blockIdx.x + blockIdx.y + blockIdx.z) & (STAT_REPL - 1));
  }
}

// ---------------------------------------------------------------------------------------------
// Register-staged kernel (2x2 waves, BK = 64): only for A_CONV3_SMALLC, the first convs with 4 / 8
// input channels whose activation chunks are element gathers (no 16-byte LDS-DMA source).
// Global -> register staging runs two K-tiles ahead in two named register sets, LDS double
// buffered, one barrier per K-tile, every load unconditional (zero-page pointer select).
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int AMODE>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmGroup P_arg) {
  const GemmGroup& P = kernarg0<GemmGroup>();
  int bxl, by, bz;
  xcd_remap(bxl, by, bz, P.xcd);
  const int grp = bxl / P.tiles_m;  // grouped launch: which independent GEMM
  const int bx = bxl - grp * P.tiles_m;
  const GemmArgs& p = P.g[grp];
  constexpr int WM = BM / 2, WN = BN / 2;    // per-wave tile (2x2 waves)
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int LA = BM / 32, LB = BN / 32;  // 16-byte loads per thread per K-tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sA = (bf16*)smem;          // [2][BM][BK] activations
  bf16* sB = sA + 2 * BM * BK;     // [2][BN][BK] weights

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wn = wid >> 1, wm = wid & 1;
  const int m0 = bx * BM, n0 = by * BN;

  const int ktot = (p.K + p.Kx) / BK;
  const int per = (ktot + p.splits - 1) / p.splits;
  const int kt0 = bz * per;
  const int kt1 = min(ktot, kt0 + per);

  const int lrow = tid >> 3, chunk = tid & 7;
  RowInfo<AMODE> rows[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) rows[i] = row_info<AMODE>(p, m0 + lrow + 32 * i, chunk);
  const bf16* wrow[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int n = n0 + lrow + 32 * i;
    wrow[i] = n < p.N ? p.Wt + (size_t)n * p.ldw + chunk * 8 : nullptr;
  }
  const bf16* zp = (const bf16*)g_zero_page;

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra0[LA], rb0[LB], ra1[LA], rb1[LB];
  // Staging as macros over fixed local arrays (lambdas taking array references made hipcc keep the
  // prefetch registers in scratch).
#define TAIR_GLOAD(RA, RB, KT)                                                              \
  do {                                                                                      \
    const int k0_ = (KT) * BK;                                                              \
    _Pragma("unroll") for (int i = 0; i < LA; ++i) RA[i] = load_act<AMODE>(p, rows[i], k0_, chunk); \
    _Pragma("unroll") for (int i = 0; i < LB; ++i)                                          \
      RB[i] = *(const u32x4*)(wrow[i] ? wrow[i] + k0_ : zp);                                \
  } while (0)
#define TAIR_SSTORE(RA, RB, BUF)                                                            \
  do {                                                                                      \
    _Pragma("unroll") for (int i = 0; i < LA; ++i)                                          \
      *(u32x4*)(sA + (BUF) * BM * BK + swz(lrow + 32 * i, chunk)) = RA[i];                  \
    _Pragma("unroll") for (int i = 0; i < LB; ++i)                                          \
      *(u32x4*)(sB + (BUF) * BN * BK + swz(lrow + 32 * i, chunk)) = RB[i];                  \
  } while (0)
#define TAIR_COMPUTE(BUF)                                                                   \
  do {                                                                                      \
    const bf16* a_s = sA + (BUF) * BM * BK;                                                 \
    const bf16* b_s = sB + (BUF) * BN * BK;                                                 \
    _Pragma("unroll") for (int s = 0; s < 2; ++s) {                                         \
      const int ch = 4 * s + (lane >> 4);                                                   \
      bf16x8 wf[FN], xf[FM];                                                                \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                        \
        wf[j] = *(const bf16x8*)(b_s + swz(wn * WN + j * 16 + (lane & 15), ch));            \
      _Pragma("unroll") for (int i = 0; i < FM; ++i)                                        \
        xf[i] = *(const bf16x8*)(a_s + swz(wm * WM + i * 16 + (lane & 15), ch));            \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                        \
        _Pragma("unroll") for (int i = 0; i < FM; ++i)                                      \
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0); \
    }                                                                                       \
  } while (0)

  if (kt0 < kt1) {
    const int kl = kt1 - 1;
    TAIR_GLOAD(ra0, rb0, kt0);
    TAIR_GLOAD(ra1, rb1, min(kt0 + 1, kl));
    TAIR_SSTORE(ra0, rb0, 0);
    __syncthreads();
    TAIR_GLOAD(ra0, rb0, min(kt0 + 2, kl));
    int t = kt0;
    for (; t + 1 < kt1; t += 2) {                  // no exit inside the body: exact vmcnt counts
      TAIR_COMPUTE(0);                             // tile t (set1: t+1, set0: t+2 in flight)
      TAIR_SSTORE(ra1, rb1, 1);
      __syncthreads();
      TAIR_GLOAD(ra1, rb1, min(t + 3, kl));
      TAIR_COMPUTE(1);                             // tile t+1
      TAIR_SSTORE(ra0, rb0, 0);
      __syncthreads();
      TAIR_GLOAD(ra0, rb0, min(t + 4, kl));
    }
    if (t < kt1) TAIR_COMPUTE(0);                  // odd tail: last tile already in buffer 0
  }
#undef TAIR_GLOAD
#undef TAIR_SSTORE
#undef TAIR_COMPUTE

  epilogue_tile<BM, BN, FM, FN, WM, WN, 256, 2 * (BM + BN) * BK * 2>(p, acc, m0, n0, wm, wn, lane, smem, bz);
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA ring kernel, any tile: BM x BN output tile, WMW x WNW waves (4 or 8), BK = 64, STAGES-deep
// ring.  Every K-tile is copied global -> LDS by global_load_lds_dwordx4 (no VGPR staging, no
// ds_write), STAGES-1 tiles in flight; the 128-byte LDS rows keep the XOR swizzle by permuting
// each lane's SOURCE chunk (the DMA destination is lane-linear).  One DMA instruction moves 8 rows
// x 128 B; instruction q of wave w covers rows 8(q*NW + w) .. +7 of the A tile, then of the B tile.
// Fragments are read with inline-asm ds_read_b128 (immediate offsets: rows 16 apart = 2048 B) so
// hipcc inserts no conservative "LDS DMA pending" vmcnt(0); the only vmcnt waits are ours: one
// counted vmcnt((STAGES-2)*G) + raw s_barrier per K-tile (G = DMA instructions per wave per tile).
// The prefetch index is clamped so every iteration issues exactly G DMAs (constant counts); the
// clamped tail copies land in a buffer that is never read again.  Per K-tile each wave reads the
// fragments of one 32-deep half, waits, issues the second half's reads and runs the first half's
// MFMAs over them, then the second half's: with two waves per SIMD (8-wave tiles) the partner's
// MFMAs cover this wave's LDS reads and barrier.
// Tiles built (tile, waves, ring): 64x64 / 64x128 / 128x64 / 128x128 (2x2, 3), 128x256 (2x4, 3),
// 256x256 (2x4, 2), 128x320 / 256x320 (2x4, 2), 256x160 (2x2, 3), 256x128 (4x2, 3): 320 divides every
// channel count of the UNet, 128 every channel count of the VAE.
// ---------------------------------------------------------------------------------------------
TAIR_DEV uint32_t lds_u32(const void* ptr) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)ptr;
}
#define TAIR_LDS(ptr) ((__attribute__((address_space(3))) void*)(ptr))

typedef int i32x8 __attribute__((ext_vector_type(8)));
TAIR_DEV i32x8 cat8(bf16x8 a, bf16x8 b) {  // two 16-byte chunks as one 32-byte MFMA operand
  const u32x4 x = __builtin_bit_cast(u32x4, a), y = __builtin_bit_cast(u32x4, b);
  return i32x8{(int)x[0], (int)x[1], (int)x[2], (int)x[3], (int)y[0], (int)y[1], (int)y[2], (int)y[3]};
}

template <int N>
TAIR_DEV void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <int N>
TAIR_DEV void wait_lgkmcnt() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }
template <int OFF>
TAIR_DEV void ds_read16(bf16x8& o, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o) : "v"(addr), "n"(OFF));
}
template <int F, int I = 0>
TAIR_DEV void ds_read_frags(bf16x8 (&o)[F], uint32_t addr) {  // fragment rows 16 apart = 2048 B apart
  if constexpr (I < F) {
    ds_read16<I * 2048>(o[I], addr);
    ds_read_frags<F, I + 1>(o, addr);
  }
}
template <int F>
TAIR_DEV void touch(bf16x8 (&o)[F]) {
#pragma unroll
  for (int i = 0; i < F; ++i) asm volatile("" : "+v"(o[i]));
}

// ---- GroupNorm(+SiLU) on load (GemmArgs.gn_st) ------------------------------------------------------
// LDS region behind the kernel's staging memory: mean / rstd of up to 64 groups (512 B), then (scale, shift)
// per channel of the workgroup's channel range.  Arithmetic as gn_apply_kernel (norm.hip), so the fused
// operand is bitwise the separate apply's output.
constexpr int GN_MR_BYTES = 512;
__host__ __device__ inline size_t gn_lds_bytes(int nch) { return GN_MR_BYTES + (size_t)nch * 8; }
TAIR_DEV void gn_table(const GemmArgs& p, int b, int hw, int cin, int ch0, int nch, char* lds) {
  float* mr = (float*)lds;
  float* tab = (float*)(lds + GN_MR_BYTES);
  const int nthr = blockDim.x, tid = threadIdx.x;
  const int cg = cin / p.gn_G;
  const int g0 = ch0 / cg, g1 = (ch0 + nch - 1) / cg;
  for (int g = g0 + tid; g <= g1; g += nthr) {
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int r = 0; r < STAT_REPL; ++r) {
      const double* q = p.gn_st + (size_t)r * p.gn_rs + ((size_t)b * p.gn_G + g) * 2;
      s1 += q[0];
      s2 += q[1];
    }
    const double cnt = (double)hw * cg;
    const double mean = s1 / cnt;
    const double var = fmax(s2 / cnt - mean * mean, 0.0);
    mr[2 * (g - g0)] = (float)mean;
    mr[2 * (g - g0) + 1] = (float)(1.0 / sqrt(var + (double)p.gn_eps));
  }
  __syncthreads();
  for (int c = tid; c < nch; c += nthr) {
    const int ch = ch0 + c, g = ch / cg - g0;
    const float sc = p.gn_gamma[ch] * mr[2 * g + 1];
    tab[2 * c] = sc;
    tab[2 * c + 1] = p.gn_beta[ch] - mr[2 * g] * sc;
  }
  __syncthreads();
}
// the lane's 8 channels (c .. c + 7 of the table) of one chunk
TAIR_DEV void gn_coeffs(const char* lds, int c, float (&sc)[8], float (&sh)[8]) {
  const float4* t = (const float4*)(lds + GN_MR_BYTES + (size_t)c * 8);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 v = t[i];
    sc[2 * i] = v.x;
    sh[2 * i] = v.y;
    sc[2 * i + 1] = v.z;
    sh[2 * i + 1] = v.w;
  }
}
// normalise the 16 bytes (8 channels) at LDS address ptr in place
TAIR_DEV void gn_apply16(char* ptr, const float (&sc)[8], const float (&sh)[8], int silu) {
  typedef union { uint4 u; bf16 h[8]; } V8;
  V8 v;
  v.u = *(const uint4*)ptr;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float a = bf2f(v.h[e]) * sc[e] + sh[e];
    if (silu) a = silu_gn(a);
    v.h[e] = f2bf(a);
  }
  *(uint4*)ptr = v.u;
}

// (the 2-stage 64x64 tiles of the batched short-K linears: 4 waves per SIMD, so 4 workgroups per CU hide one
// another's epilogue -- B = 16 step -3%; 3 waves per SIMD without spills measured slower, r05_sw3_*.log; the
// 3-stage B = 1 tiles measured slower with the same bound)
template <int BM, int BN, int STAGES>
constexpr int tile_min_waves() { return (BM * BN <= 64 * 64 && STAGES == 2) ? 4 : 1; }
template <int BM, int BN, int WMW, int WNW, int STAGES, int AMODE, int F8 = 0>
__global__ __launch_bounds__(WMW * WNW * 64, (tile_min_waves<BM, BN, STAGES>())) void gemm_tile_kernel(const GemmGroup P_arg) {
  constexpr int NW = WMW * WNW;
  constexpr int WM = BM / WMW, WN = BN / WNW;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int NA = BM / (8 * NW), NB = BN / (8 * NW);  // DMA instructions per wave per K-tile
  constexpr int G = NA + NB;
  constexpr int STAGE_BYTES = (BM + BN) * BK * 2;
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "DMA rows per wave");
  static_assert(WM % 16 == 0 && WN % 16 == 0 && FM + FN <= 15, "wave tile");
  static_assert(STAGES >= 2 && STAGES * STAGE_BYTES <= 160 * 1024, "LDS");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const GemmGroup& P = kernarg0<GemmGroup>();
  int xcd = P.xcd, tiles_m = P.tiles_m;
  TAIR_PIN_ASM("" : "+s"(xcd), "+s"(tiles_m));  // (one round trip for both; see pin)
  int bxl, by, bz;
  xcd_remap(bxl, by, bz, xcd);
  const int grp = bxl / tiles_m;  // grouped launch: which independent GEMM
  const int bx = bxl - grp * tiles_m;
  const GemmArgs& p = P.g[grp];
  stamp(p, 0);
  const MainArgs ma = main_args(p);  // the prologue / main-loop fields as one batch of loads

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid % WMW, wn = wid / WMW;
  const int m0 = bx * BM, n0 = by * BN;
  const int ktot = (ma.K + ma.Kx) / BK;
  const int per = (ktot + ma.splits - 1) / ma.splits;
  const int kt0 = bz * per;
  const int kt1 = min(ktot, kt0 + per);

  // DMA lane mapping: lane l -> row (l>>3) of the instruction's 8, LDS slot l&7, which must hold
  // logical chunk (l&7) ^ (row&7) = (l&7) ^ (l>>3).
  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ drow;
  RowInfo<AMODE> rows[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) rows[i] = row_info<AMODE>(ma, m0 + (i * NW + wid) * 8 + drow, dchunk);
  const bf16* wrow[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + (i * NW + wid) * 8 + drow;
    wrow[i] = n < ma.N ? ma.Wt + (size_t)n * ma.ldw + dchunk * 8 : nullptr;
  }
  const bf16* zp = (const bf16*)g_zero_page;
  const ActArgs pa = act_args(ma);

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#define TAIR_ISSUE(KT, STG)                                                                       \
  do {                                                                                            \
    const int k0_ = (KT) * BK;                                                                    \
    char* sb_ = smem + (STG) * STAGE_BYTES;                                                       \
    _Pragma("unroll") for (int i = 0; i < NA; ++i)                                                \
      __builtin_amdgcn_global_load_lds((const void*)(F8 && AMODE != A_DENSE                       \
                                                         ? act_src_f8<AMODE>(pa, rows[i], k0_, dchunk) \
                                                         : act_src<AMODE>(pa, rows[i], k0_)),     \
                                       TAIR_LDS(sb_ + (i * NW + wid) * 8 * 128), 16, 0, 0);       \
    _Pragma("unroll") for (int i = 0; i < NB; ++i)                                                \
      __builtin_amdgcn_global_load_lds((const void*)(wrow[i] ? wrow[i] + k0_ : zp),              \
                                       TAIR_LDS(sb_ + BM * 128 + (i * NW + wid) * 8 * 128), 16, 0, 0); \
  } while (0)

  const int kt_f8 = F8 ? ma.K / BK : 0;  // fp8 K-tiles (then the bf16 K-extension's, if any)
  const uint32_t lds0 = lds_u32(smem);
  const int ra = wm * WM + (lane & 15), rb = wn * WN + (lane & 15);
  const uint32_t aoff0 = ra * 128 + ((((lane >> 4)) ^ (ra & 7)) << 4);
  const uint32_t aoff1 = ra * 128 + (((4 + (lane >> 4)) ^ (ra & 7)) << 4);
  const uint32_t boff0 = BM * 128 + rb * 128 + ((((lane >> 4)) ^ (rb & 7)) << 4);
  const uint32_t boff1 = BM * 128 + rb * 128 + (((4 + (lane >> 4)) ^ (rb & 7)) << 4);
  // fp8: the lane's two consecutive chunks 2h, 2h + 1 (h = lane >> 4) of its row
  const uint32_t f8a0 = ra * 128 + (((2 * (lane >> 4)) ^ (ra & 7)) << 4);
  const uint32_t f8a1 = ra * 128 + (((2 * (lane >> 4) + 1) ^ (ra & 7)) << 4);
  const uint32_t f8b0 = BM * 128 + rb * 128 + (((2 * (lane >> 4)) ^ (rb & 7)) << 4);
  const uint32_t f8b1 = BM * 128 + rb * 128 + (((2 * (lane >> 4) + 1) ^ (rb & 7)) << 4);

  // Software-pipelined bf16 main loop (register double buffer; ring of STAGES K-tiles all in flight):
  // per K-tile, the second half's fragment reads run under the first half's MFMAs, and the next K-tile's
  // first-half reads under the second half's; the barrier sits between the two MFMA groups, after each
  // wave has all of this K-tile's fragments in registers, so the tile's stage is refilled right away.
  // Taken where both fragment sets fit beside the accumulators.
  // (not the 4-wave 3-stage tiles of the latency-bound B = 1 plans: there the deeper prologue cost ~3%,
  // profiles/r04_bench_b1_pipe_nohalo.log vs r04_early_r4_bench_b1.log)
  constexpr bool PIPE = gemm_tile_pipe(WMW * WNW, STAGES) && !F8 && (FM * FN * 4 + 2 * (FM + FN) * 4 <= 200);
  // GroupNorm on load (conv / dense, PIPE plans; the host keeps a tile inside one batch element): each
  // lane normalises the 16-byte pieces its own DMA brought, after they land and before the barrier that
  // publishes the K-tile; padding taps (zero page) and the K-extension stay as loaded
  constexpr bool GNOK = PIPE && (AMODE == A_CONV3 || AMODE == A_DENSE);
  const bool gn = GNOK && ma.gn_st != nullptr;
  const int kreal = ma.K / BK;
  const int gch0 = AMODE == A_DENSE ? kt0 : kt0 / 9;  // first 64-channel chunk of the slice
  char* gnl = smem + STAGES * STAGE_BYTES;
  auto gn_tile = [&](int t, int stg) {
    if (t >= kreal) return;
    const int chunk = AMODE == A_DENSE ? t : t / 9;
    float sc[8], sh[8];
    gn_coeffs(gnl, (chunk - gch0) * 64 + dchunk * 8, sc, sh);
#pragma unroll
    for (int i = 0; i < NA; ++i)
      if (act_src<AMODE>(pa, rows[i], t * BK) != zp)
        gn_apply16(smem + stg * STAGE_BYTES + (i * NW + wid) * 8 * 128 + lane * 16, sc, sh, p.gn_silu);
  };
  if constexpr (PIPE) {
    if (kt0 < kt1) {
      const int kl = kt1 - 1;
#pragma unroll
      for (int s = 0; s < STAGES; ++s) TAIR_ISSUE(min(kt0 + s, kl), s);
      bf16x8 x0[FM], w0[FN], x1[FM], w1[FN];
      if (gn) {
        const int hw = AMODE == A_DENSE ? p.rows_per_b : p.H * p.W;
        const int cin = AMODE == A_DENSE ? p.K : p.C;
        const int ch1 = AMODE == A_DENSE ? min(kt1, kreal) : (min(kt1, kreal) - 1) / 9 + 1;
        gn_table(p, m0 / p.rows_per_b, hw, cin, gch0 * 64, (ch1 - gch0) * 64, gnl);
      }
      stamp(p, 1);
      wait_vmcnt<(STAGES - 1) * G>();
      if (gn) {
        gn_tile(kt0, 0);
        wait_lgkmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
      stamp(p, 2);
      ds_read_frags<FM>(x0, lds0 + aoff0);
      ds_read_frags<FN>(w0, lds0 + boff0);
      int stage = 0;
      for (int t = kt0; t < kt1; ++t) {
        const uint32_t sb = lds0 + stage * STAGE_BYTES;
        ds_read_frags<FM>(x1, sb + aoff1);
        ds_read_frags<FN>(w1, sb + boff1);
        wait_lgkmcnt<FM + FN>();  // this half's reads (issued before the other half's) have landed
        touch<FM>(x0);
        touch<FN>(w0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[j], x0[i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        wait_lgkmcnt<0>();
        touch<FM>(x1);
        touch<FN>(w1);
        wait_vmcnt<(STAGES - 2) * G>();  // K-tile t + 1 has landed (this wave's copies) ...
        const int nst = (stage + 1 == STAGES) ? 0 : stage + 1;
        if (gn && t + 1 < kt1) {
          gn_tile(t + 1, nst);
          wait_lgkmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();    // ... every wave's, and every wave holds K-tile t in registers
        TAIR_ISSUE(min(t + STAGES, kl), stage);
        ds_read_frags<FM>(x0, lds0 + nst * STAGE_BYTES + aoff0);
        ds_read_frags<FN>(w0, lds0 + nst * STAGE_BYTES + boff0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[j], x1[i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        stage = nst;
      }
      wait_lgkmcnt<0>();
      wait_vmcnt<0>();  // drain the clamped tail copies before the wave can exit
      stamp(p, 3);
    }
  } else if (kt0 < kt1) {
    const int kl = kt1 - 1;
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) TAIR_ISSUE(min(kt0 + s, kl), s);
    stamp(p, 1);
    int stage = 0;
    for (int t = kt0; t < kt1; ++t) {
      stamp_it(ma.stamps, t - kt0, 0);
      wait_vmcnt<(STAGES - 2) * G>();  // this wave's copies of tile t have landed
      __builtin_amdgcn_s_barrier();    // ... and every wave's; tile t-1's buffer is free
      if (t == kt0) stamp(p, 2);
      stamp_it(ma.stamps, t - kt0, 1);
      int ps = stage + STAGES - 1;
      if (ps >= STAGES) ps -= STAGES;
      TAIR_ISSUE(min(t + STAGES - 1, kl), ps);
      stamp_it(ma.stamps, t - kt0, 2);
      const uint32_t sb = lds0 + stage * STAGE_BYTES;
      if (F8 && t < kt_f8) {
        // one 16x16x128 e4m3 MFMA per fragment pair: a lane brings 32 bytes (two 16-byte chunks) of
        // its row; A and B use the same chunk order, so the k pairing is consistent (scales = 2^0)
        // wide tiles (FM + FN > 8, e.g. 128x320: 4 + 5 fragments) take the weight fragments in two groups,
        // the second group's reads under the first group's MFMAs (18 live fragments spilled)
        constexpr int JA = (FM + FN > 8) ? (FN + 1) / 2 : FN;
        bf16x8 xa[FM], xb[FM], wa[JA], wb[JA];
        ds_read_frags<FM>(xa, sb + f8a0);
        ds_read_frags<FM>(xb, sb + f8a1);
        ds_read_frags<JA>(wa, sb + f8b0);
        ds_read_frags<JA>(wb, sb + f8b1);
        wait_lgkmcnt<0>();
        touch<FM>(xa);
        touch<FM>(xb);
        touch<JA>(wa);
        touch<JA>(wb);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < JA; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(cat8(wa[j], wb[j]), cat8(xa[i], xb[i]),
                                                                        acc[j][i], 0, 0, 0, 127, 0, 127);
        if constexpr (JA < FN) {
          constexpr int JB = FN - JA;
          bf16x8 wc[JB], wd[JB];
          __builtin_amdgcn_sched_barrier(0);
          ds_read_frags<JB>(wc, sb + f8b0 + JA * 2048);
          ds_read_frags<JB>(wd, sb + f8b1 + JA * 2048);
          wait_lgkmcnt<0>();
          touch<JB>(wc);
          touch<JB>(wd);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < JB; ++j)
#pragma unroll
            for (int i = 0; i < FM; ++i)
              acc[JA + j][i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                  cat8(wc[j], wd[j]), cat8(xa[i], xb[i]), acc[JA + j][i], 0, 0, 0, 127, 0, 127);
        }
        stage = (stage + 1 == STAGES) ? 0 : stage + 1;
        continue;
      }
      bf16x8 xf[FM], wf[FN];
      ds_read_frags<FM>(xf, sb + aoff0);
      ds_read_frags<FN>(wf, sb + boff0);
      wait_lgkmcnt<0>();
      touch<FM>(xf);
      touch<FN>(wf);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // first-half MFMAs issue before the second half's reads
      ds_read_frags<FM>(xf, sb + aoff1);
      ds_read_frags<FN>(wf, sb + boff1);
      wait_lgkmcnt<0>();
      touch<FM>(xf);
      touch<FN>(wf);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[j][i], 0, 0, 0);
      stamp_it(ma.stamps, t - kt0, 3);
      stage = (stage + 1 == STAGES) ? 0 : stage + 1;
    }
    wait_vmcnt<0>();  // drain the clamped tail copies before the wave can exit
    stamp(p, 3);
  }
#undef TAIR_ISSUE

  // the wide tiles, and the 64-row B = 1 tiles (3-deep rings): register-staged epilogue where it applies
  if constexpr (!F8 && (BM * BN >= 128 * 256 || (BM == 64 && STAGES >= 3))) {
    constexpr int CAP = STAGES * STAGE_BYTES;
    const EpiArgs ep = epi_args(p);
    switch (regstage_set<BM, BN, CAP>(ep)) {
#define TAIR_RS_CASE(S)                                                                 \
      case (S): epilogue_regstage<(S), BM, BN, FM, FN, WM, WN, NW * 64, CAP>(ep, acc, m0, n0, wm, wn, lane, smem); \
        return;
      TAIR_RS_CASE(E_BIAS | E_LNC | E_GEGLU)
      TAIR_RS_CASE(E_BIAS | E_GEGLU)
      TAIR_RS_CASE(E_BIAS | E_LNC)
      TAIR_RS_CASE(E_BIAS)
      TAIR_RS_CASE(E_BIAS | E_ROWST)
      TAIR_RS_CASE(E_BIAS | E_RES | E_ROWST)
      TAIR_RS_CASE(E_BIAS | E_RES)
#undef TAIR_RS_CASE
      default: break;
    }
  }
  epilogue_tile<BM, BN, FM, FN, WM, WN, NW * 64, STAGES * STAGE_BYTES, (BM == 64 && STAGES >= 3),
                !(BM == 64 && STAGES == 2)>(p, acc, m0, n0, wm, wn, lane, smem, bz);
}

// ---------------------------------------------------------------------------------------------
// Halo-tile 3x3 convolution (stride 1, pad 1; unet.py:203-223 ResBlock convs), BM = 256 output pixels =
// R = 256 / W whole image rows of one batch element (W in {16, 32, 64}), BN output channels, 8 waves
// (4 m x 2 n, 64 x BN/2 each).  The implicit GEMM of gemm_tile_kernel streams one (64-channel chunk,
// tap) K-tile of activations per weight K-tile: every input pixel is copied into LDS nine times, and
// at the batched sizes these copies (beside the weight tile every M-tile re-streams) keep the
// LDS-DMA path busy (~5-6 TB/s chip-wide: the conv kernels are copy-bound, not MFMA-bound;
// profiles/r04_*).  Here the (R + 2) x (W + 2) halo block of a chunk is copied ONCE and the nine taps
// read it at shifted rows; only the weights stream per tap.
// * LDS: two halo buffers of HRP rows (128 B each: 64 bf16 channels, XOR swizzle chunk ^ (row & 7)
//   carried by the DMA source as everywhere) + a STAGES-deep ring of BN-row weight K-tiles.
// * Order: K-tile t = (chunk, tap), chunk-major like the packed weights ((c/64 * 9 + tap) * 64 + c%64).
//   At tap 0 of chunk c the halo of c + 1 is issued into the other buffer (9 K-tiles ahead); the
//   weight ring runs STAGES - 1 K-tiles ahead.  Both prefetches are clamped at the end so every
//   iteration issues the same DMA counts: the counted vmcnt of K-tile t is (STAGES - 2) G_W, plus the
//   G_H halo copies when the next chunk's halo was issued after weight tile t (taps 1 .. STAGES - 2).
// * A fragments: lane row = output pixel (r, x) -> halo row (r + ky) (W + 2) + x + kx, per-lane
//   addresses (rows of one fragment are consecutive pixels: conflict-free as in the tile kernel).
// Split-K over chunks (blockIdx.z); epilogue_tile as every GEMM (bias, emb, residual, statistics).
// No K-extension, no fp8 (the planner keeps those convs on gemm_tile_kernel).
// ---------------------------------------------------------------------------------------------
// The counted wait of conv_halo_kernel: a wave issues GW weight copies per K-tile (GW - 1 for waves >= WX
// when BN is not a multiple of 64) and GH halo copies per chunk (GH + 1 for waves < HX); `pend`: the next
// chunk's halo was issued after the weight tile being waited for.
template <int S, int GW, int WX, int GH, int HX>
TAIR_DEV void halo_wait(int wid, bool pend) {
  const bool wf = WX == 0 || wid < WX, hx = HX != 0 && wid < HX;
  if (pend) {
    if (wf) {
      if (hx) wait_vmcnt<(S - 2) * GW + GH + 1>();
      else wait_vmcnt<(S - 2) * GW + GH>();
    } else {
      if (hx) wait_vmcnt<(S - 2) * (GW - 1) + GH + 1>();
      else wait_vmcnt<(S - 2) * (GW - 1) + GH>();
    }
  } else {
    if (wf) wait_vmcnt<(S - 2) * GW>();
    else wait_vmcnt<(S - 2) * (GW - 1)>();
  }
}

template <int BN, int HRP, int STAGES, int ABL = 0>  // ABL: ablation probes (tools/conv_probe.py --ablate)
__global__ __launch_bounds__(512) void conv_halo_kernel(const GemmGroup P_arg) {
  constexpr int BM = 256, WMW = 4, WNW = 2, NW = 8;
  constexpr int WM = BM / WMW, WN = BN / WNW;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int GW = (BN + 8 * NW - 1) / (8 * NW);  // weight DMA instructions per wave per K-tile
  constexpr int WX = (BN % (8 * NW)) / 8;            // waves that issue the last (partial) weight round
  constexpr int GH = HRP / (8 * NW);                 // full halo DMA rounds per chunk
  constexpr int HX = (HRP % (8 * NW)) / 8;           // waves that issue one more halo round
  constexpr int HBYTES = HRP * 128, WBYTES = BN * 128;
  static_assert(BN % 8 == 0 && HRP % 8 == 0 && STAGES >= 2 && STAGES <= 9, "halo tile");
  static_assert(2 * HBYTES + STAGES * WBYTES <= 160 * 1024, "LDS");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const GemmGroup& P = kernarg0<GemmGroup>();
  int xcd = P.xcd, tiles_m = P.tiles_m;
  TAIR_PIN_ASM("" : "+s"(xcd), "+s"(tiles_m));  // (one round trip for both; see pin)
  int bxl, by, bz;
  xcd_remap(bxl, by, bz, xcd);
  const int grp = bxl / tiles_m;
  const int bx = bxl - grp * tiles_m;
  const GemmArgs& p = P.g[grp];
  stamp(p, 0);
  const MainArgs ma = main_args(p);  // the prologue / main-loop fields as one batch of loads

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid % WMW, wn = wid / WMW;
  const int m0 = bx * BM, n0 = by * BN;
  const int W = ma.W, H = ma.H, W2 = W + 2;
  const int HW = H * W;
  const int bimg = m0 / HW, y0 = (m0 - bimg * HW) / W;
  const int R = BM / W;
  const int hrows = (R + 2) * W2;
  const int nchunk = ma.C / 64;
  const int per = (nchunk + ma.splits - 1) / ma.splits;
  const int c0 = bz * per, c1 = min(nchunk, c0 + per);

  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ drow;
  // halo DMA rows of this wave: hr = (q * NW + wid) * 8 + drow -> source pixel offset (elements) or -1
  int hsrc[GH + 1];
#pragma unroll
  for (int q = 0; q < GH + 1; ++q) {
    const int hr = (q * NW + wid) * 8 + drow;
    const int hy = hr / W2, hx = hr - hy * W2;
    const int y = y0 + hy - 1, x = hx - 1;
    const bool ok = hr < hrows && y >= 0 && y < H && x >= 0 && x < W;
    hsrc[q] = ok ? (int)((uint32_t)((bimg * HW + y * W + x)) * (uint32_t)ma.lda) + dchunk * 8 : -1;
  }
  const bf16* wrow[GW];
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int n = n0 + (i * NW + wid) * 8 + drow;
    wrow[i] = n < ma.N ? ma.Wt + (size_t)n * ma.ldw + dchunk * 8 : nullptr;
  }
  const bf16* zp = (const bf16*)g_zero_page;
  // the activation base once, in registers (read through P inside the issue macro it was re-loaded from the
  // kernel arguments, behind an lgkmcnt(0), for every halo DMA round)
  const bf16* const Ah = ma.A;

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#define TAIR_HALO_ISSUE(C, HB)                                                                    \
  do {                                                                                            \
    char* hb_ = smem + (HB) * HBYTES;                                                             \
    _Pragma("unroll") for (int q = 0; q < GH; ++q)                                                \
      __builtin_amdgcn_global_load_lds((const void*)(hsrc[q] >= 0 ? Ah + hsrc[q] + (C) * 64 : zp), \
                                       TAIR_LDS(hb_ + (q * NW + wid) * 8 * 128), 16, 0, 0);       \
    if (HX && wid < HX)                                                                           \
      __builtin_amdgcn_global_load_lds((const void*)(hsrc[GH] >= 0 ? Ah + hsrc[GH] + (C) * 64 : zp), \
                                       TAIR_LDS(hb_ + (GH * NW + wid) * 8 * 128), 16, 0, 0);      \
  } while (0)
#define TAIR_W_ISSUE(KT, STG)                                                                     \
  do {                                                                                            \
    char* sb_ = smem + 2 * HBYTES + (STG) * WBYTES;                                               \
    _Pragma("unroll") for (int i = 0; i < GW; ++i)                                                \
      if (i < GW - 1 || WX == 0 || wid < WX)                                                      \
        __builtin_amdgcn_global_load_lds((const void*)(wrow[i] ? wrow[i] + (KT) * 64 : zp),      \
                                         TAIR_LDS(sb_ + (i * NW + wid) * 8 * 128), 16, 0, 0);     \
  } while (0)

  const uint32_t lds0 = lds_u32(smem);
  // A fragment rows: output pixel pl = wm * 64 + 16 i + (lane & 15) -> halo row at tap (0, 0)
  int hbase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pl = wm * WM + 16 * i + (lane & 15);
    const int r = pl / W, x = pl - r * W;
    hbase[i] = r * W2 + x;
  }
  const int rb = wn * WN + (lane & 15);
  const uint32_t boff0 = 2 * HBYTES + rb * 128 + ((((lane >> 4)) ^ (rb & 7)) << 4);
  const uint32_t boff1 = 2 * HBYTES + rb * 128 + (((4 + (lane >> 4)) ^ (rb & 7)) << 4);
  const int cl = lane >> 4;

  // software-pipelined as gemm_tile_kernel's bf16 loop: each half-K's fragment reads run under the
  // previous half's MFMAs, the barrier between the two MFMA groups (every wave holds K-tile t in
  // registers), the weight ring holds STAGES K-tiles in flight
  // A fragment addresses of K-tile t's half-K `half`
  auto aaddr = [&](uint32_t (&xa)[FM], int t, int half) {
    const int cc = t / 9, tap = t - 9 * cc;
    const int ky = tap / 3, kx = tap - 3 * ky;
    const uint32_t hb = lds0 + (cc & 1) * HBYTES;
    const int dt = ky * W2 + kx;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int hr = hbase[i] + dt;
      xa[i] = hb + hr * 128 + (((half * 4 + cl) ^ (hr & 7)) << 4);
    }
  };
  auto reads = [&](bf16x8 (&xd)[FM], bf16x8 (&wd)[FN], const uint32_t (&xa)[FM], uint32_t wa) {
#pragma unroll
    for (int i = 0; i < FM; ++i) ds_read16<0>(xd[i], xa[i]);
    ds_read_frags<FN>(wd, wa);
  };
  // GroupNorm on load: (scale, shift) of the slice's channels in LDS behind the weight ring; each lane
  // normalises the halo rows its own DMA brought once per chunk (out-of-image rows stay zero)
  const bool gn = ma.gn_st != nullptr;
  char* gnl = smem + 2 * HBYTES + STAGES * WBYTES;
  // rows q = part, part + nparts, ... of the lane's DMA rounds (the whole set when nparts = 1)
  auto gn_halo = [&](int hbuf, int chunk, int part, int nparts) {
    float sc[8], sh[8];
    gn_coeffs(gnl, (chunk - c0) * 64 + dchunk * 8, sc, sh);
    char* hb_ = smem + hbuf * HBYTES;
#pragma unroll
    for (int q = 0; q < GH; ++q)
      if (q % nparts == part && hsrc[q] >= 0) gn_apply16(hb_ + (q * NW + wid) * 8 * 128 + lane * 16, sc, sh, p.gn_silu);
    if (HX && GH % nparts == part && wid < HX && hsrc[GH] >= 0)
      gn_apply16(hb_ + (GH * NW + wid) * 8 * 128 + lane * 16, sc, sh, p.gn_silu);
  };
  if (c0 < c1) {
    const int T = (c1 - c0) * 9;
    TAIR_HALO_ISSUE(c0, 0);
#pragma unroll
    for (int s = 0; s < STAGES; ++s) {
      const int t = min(s, T - 1);
      TAIR_W_ISSUE((c0 + t / 9) * 9 + t % 9, s);
    }
    bf16x8 x0[FM], w0[FN], x1[FM], w1[FN];
    // ablation probes (timing only, results invalid): bit 3 no weight DMA in the loop, bit 4 no MFMA,
    // bit 5 no barrier in the loop
    constexpr int abl = ABL;
    if (gn) gn_table(p, bimg, HW, p.C, c0 * 64, (c1 - c0) * 64, gnl);
    stamp(p, 1);
    halo_wait<STAGES + 1, GW, WX, GH, HX>(wid, false);  // halo(c0) and weight K-tile 0
    if (gn) {
      gn_halo(0, c0, 0, 1);
      wait_lgkmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    stamp(p, 2);
    uint32_t xa[FM];
    aaddr(xa, 0, 0);
    reads(x0, w0, xa, lds0 + boff0);
    // the nine taps of a chunk unrolled: tap, its halo-row offset, the counted wait and
    // the halo / GroupNorm branches are compile-time, and with 9 % STAGES == 0 so is the weight stage
    int stage_rt = 0;
    const int nch = c1 - c0;
    for (int cc = 0; cc < nch; ++cc) {
      const uint32_t hb_cur = lds0 + (cc & 1) * HBYTES;
      const uint32_t hb_nxt = lds0 + (min(cc + 1, nch - 1) & 1) * HBYTES;
      static_for<0, 9>([&](auto TAP) {
        constexpr int tap = decltype(TAP)::value;
        constexpr int ky = tap / 3, kx = tap - 3 * (tap / 3);
        constexpr int tapn = tap == 8 ? 0 : tap + 1;  // the next K-tile's tap
        constexpr int kyn = tapn / 3, kxn = tapn - 3 * (tapn / 3);
        const int t = cc * 9 + tap;
        const int stage = (9 % STAGES == 0) ? tap % STAGES : stage_rt;
        stamp_it(ma.stamps, t, 0);
        const uint32_t sb = lds0 + stage * WBYTES;
        // (the fragment rows' halo bases pass an empty asm per tap: otherwise the compiler hoists all nine
        // taps' addresses out of the chunk loop and the kernel spills)
        int hbt[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          hbt[i] = hbase[i];
          asm volatile("" : "+v"(hbt[i]));
        }
        {
          const int dt = ky * W2 + kx;
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const int hr = hbt[i] + dt;
            xa[i] = hb_cur + hr * 128 + (((4 + cl) ^ (hr & 7)) << 4);
          }
        }
        reads(x1, w1, xa, sb + boff1);
        wait_lgkmcnt<FM + FN>();
        touch<FM>(x0);
        touch<FN>(w0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(abl & 16))
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int i = 0; i < FM; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[j], x0[i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        wait_lgkmcnt<0>();
        touch<FM>(x1);
        touch<FN>(w1);
        // K-tile t + 1 (and, at tap 8, the next chunk's halo, issued before it) has landed; the next chunk's
        // halo was issued after weight K-tile t + 1 when 1 <= tap <= STAGES - 2
        halo_wait<STAGES, GW, WX, GH, HX>(wid, tap >= 1 && tap <= STAGES - 2);
        if constexpr (!(abl & 32)) __builtin_amdgcn_s_barrier();
        stamp_it(ma.stamps, t, 1);
        if constexpr (tap == 0) TAIR_HALO_ISSUE(min(c0 + cc + 1, c1 - 1), (cc + 1) & 1);
        if constexpr (!(abl & 8)) {
          const int tn = min(t + STAGES, T - 1);
          TAIR_W_ISSUE(c0 * 9 + tn, stage);
        }
        stamp_it(ma.stamps, t, 2);
        const int nst = (stage + 1 == STAGES) ? 0 : stage + 1;
        {
          // the next K-tile's first-half fragments: tap + 1 of this chunk, or tap 0 of the next one (the
          // last K-tile re-reads its own tap: clamped as the weight ring)
          const bool last = tap == 8 && cc + 1 == nch;
          const uint32_t hbn = tap == 8 ? hb_nxt : hb_cur;
          const int dtn = last ? 2 * W2 + 2 : kyn * W2 + kxn;
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            const int hr = hbt[i] + dtn;
            xa[i] = (last ? hb_cur : hbn) + hr * 128 + (((cl) ^ (hr & 7)) << 4);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        reads(x0, w0, xa, lds0 + nst * WBYTES + boff0);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(abl & 16))
#pragma unroll
          for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int i = 0; i < FM; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[j], x1[i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        // GroupNorm of the next chunk's halo, spread over taps STAGES - 1 .. 7 behind the MFMAs (it has landed
        // for this wave from tap STAGES - 1 on: issued before weight K-tile 9 cc + STAGES); the ds_writes are
        // drained by tap 8's lgkmcnt(0), ahead of the barrier that publishes the chunk
        if constexpr (tap >= STAGES - 1 && tap <= 7)
          if (gn && cc + 1 < nch) gn_halo((cc + 1) & 1, c0 + cc + 1, tap - (STAGES - 1), 9 - STAGES);
        stamp_it(ma.stamps, t, 3);
        stage_rt = nst;
      });
    }
    wait_lgkmcnt<0>();
    wait_vmcnt<0>();  // drain the clamped tail copies before the LDS is reused / the wave exits
    stamp(p, 3);
  }
#undef TAIR_HALO_ISSUE
#undef TAIR_W_ISSUE

  epilogue_tile<BM, BN, FM, FN, WM, WN, NW * 64, 2 * HBYTES + STAGES * WBYTES>(p, acc, m0, n0, wm, wn, lane, smem,
                                                                               bz);
}

// halo tile configurations: halo rows (R + 2) (W + 2) rounded up to 8 (W = 64: 396 -> 400, W = 32: 340 -> 344,
// W = 16: 324 -> 328), BN output channels (a multiple of 64: the weight rounds are equal per wave)
template <int BN_, int HRP_, int STAGES_>
struct HaloCfg {
  static constexpr int BN = BN_, HRP = HRP_, STAGES = STAGES_;
  static constexpr size_t LDS = (size_t)2 * HRP * 128 + (size_t)STAGES * BN * 128;
};
using H64x448 = HaloCfg<64, 448, 4>;
using H128x384 = HaloCfg<128, 384, 3>;
using H128W64 = HaloCfg<128, 400, 3>;
using H160W64 = HaloCfg<160, 400, 3>;
using H160W32 = HaloCfg<160, 344, 3>;
using H160W16 = HaloCfg<160, 328, 3>;
using H192W32 = HaloCfg<192, 344, 3>;
using H192W16 = HaloCfg<192, 328, 3>;
using H160W64S2 = HaloCfg<160, 400, 2>;
using H160W32S2 = HaloCfg<160, 344, 2>;
using H160W16S2 = HaloCfg<160, 328, 2>;

template <class T, int AMODE>
hipError_t set_attr_halo() {
  TAIR_HIP_CHECK(hipFuncSetAttribute((const void*)conv_halo_kernel<T::BN, T::HRP, T::STAGES>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  return hipSuccess;
}
template <int AMODE>
hipError_t set_attrs_halo() {
  static_assert(AMODE == A_CONV3, "halo tiles: stride-1 3x3 convs");
  TAIR_HIP_CHECK((set_attr_halo<H64x448, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H128x384, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H128W64, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H160W64, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H160W32, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H160W16, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H192W32, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H160W64S2, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H160W32S2, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H160W16S2, AMODE>()));
  TAIR_HIP_CHECK((set_attr_halo<H192W16, AMODE>()));
  return hipSuccess;
}
// extra dynamic LDS of a GroupNorm-on-load plan: the table of one K slice's channels
inline size_t gn_extra_lds(const GemmArgs& g, int splits) {
  if (!g.gn_st) return 0;
  const int cin = g.amode == A_DENSE ? g.K : g.C;
  const int per = cdiv((g.K + g.Kx) / BK, splits);             // K-tiles of one slice
  const int nch = g.amode == A_DENSE ? per : per / 9 + 2;     // 64-channel chunks it can touch
  return gn_lds_bytes(64 * std::min(nch, cin / 64));
}
template <class T, int ABL = 0>
hipError_t launch_halo_tile(GemmGroup& a, int n, int splits, hipStream_t s) {
  a.tiles_m = cdiv(a.g[0].M, 256);
  dim3 grid(a.tiles_m * n, cdiv(a.g[0].N, T::BN), splits);
  if constexpr (ABL != 0)
    TAIR_HIP_CHECK(hipFuncSetAttribute((const void*)conv_halo_kernel<T::BN, T::HRP, T::STAGES, ABL>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipLaunchKernelGGL((conv_halo_kernel<T::BN, T::HRP, T::STAGES, ABL>), grid, dim3(512),
                     T::LDS + gn_extra_lds(a.g[0], splits), s, a);
  return hipGetLastError();
}
// ablation-probe instances of the 256x160 tiles (timing only; GemmArgs.probe bits 3-5)
template <class T>
hipError_t launch_halo_abl(GemmGroup& a, int n, int splits, hipStream_t s) {
  switch (a.g[0].probe & 56) {
    case 8: return launch_halo_tile<T, 8>(a, n, splits, s);
    case 16: return launch_halo_tile<T, 16>(a, n, splits, s);
    case 24: return launch_halo_tile<T, 24>(a, n, splits, s);
    case 32: return launch_halo_tile<T, 32>(a, n, splits, s);
    case 40: return launch_halo_tile<T, 40>(a, n, splits, s);
    case 56: return launch_halo_tile<T, 56>(a, n, splits, s);
    default: return launch_halo_tile<T>(a, n, splits, s);
  }
}
template <int AMODE>
hipError_t launch_halo(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s) {
  if (bm != 256) return hipErrorInvalidValue;
  const int W = a.g[0].W;
  if (a.g[0].halo_s2) {  // 2-stage weight ring (LDS room for a fused GroupNorm table)
    if (bn == 160 && W == 64) return launch_halo_tile<H160W64S2>(a, n, splits, s);
    if (bn == 160 && W == 32) return launch_halo_tile<H160W32S2>(a, n, splits, s);
    if (bn == 160 && W == 16) return launch_halo_tile<H160W16S2>(a, n, splits, s);
    return hipErrorInvalidValue;
  }
  if (bn == 64 && W == 64) return launch_halo_tile<H64x448>(a, n, splits, s);
  if (bn == 128 && W == 64) return launch_halo_tile<H128W64>(a, n, splits, s);
  if (bn == 128 && (W == 32 || W == 16)) return launch_halo_tile<H128x384>(a, n, splits, s);
  if (bn == 160 && W == 64) return launch_halo_abl<H160W64>(a, n, splits, s);
  if (bn == 160 && W == 32) return launch_halo_abl<H160W32>(a, n, splits, s);
  if (bn == 160 && W == 16) return launch_halo_abl<H160W16>(a, n, splits, s);
  if (bn == 192 && W == 32) return launch_halo_tile<H192W32>(a, n, splits, s);
  if (bn == 192 && W == 16) return launch_halo_tile<H192W16>(a, n, splits, s);
  return hipErrorInvalidValue;
}

// ---- launchers ----------------------------------------------------------------------------------
template <int BM, int BN, int AMODE>
hipError_t set_attr_reg() {
  const size_t lds = (size_t)2 * (BM + BN) * BK * sizeof(bf16);
  TAIR_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, AMODE>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  return hipSuccess;
}

template <int AMODE>
hipError_t set_attrs_reg() {
  TAIR_HIP_CHECK((set_attr_reg<64, 128, AMODE>()));
  TAIR_HIP_CHECK((set_attr_reg<64, 64, AMODE>()));
  return hipSuccess;
}

template <int AMODE>
hipError_t launch_reg(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s) {
  auto go = [&](auto kern, int BM, int BN) {
    const size_t lds = (size_t)2 * (BM + BN) * BK * sizeof(bf16);
    a.tiles_m = cdiv(a.g[0].M, BM);
    dim3 grid(a.tiles_m * n, cdiv(a.g[0].N, BN), splits);
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a);
    return hipGetLastError();
  };
  if (bn == 128) return go(gemm_kernel<64, 128, AMODE>, 64, 128);
  return go(gemm_kernel<64, 64, AMODE>, 64, 64);
}

// ---------------------------------------------------------------------------------------------
// Deep-ring kernel: BK = 32 (64-byte LDS rows), STAGES-deep LDS-DMA ring with STAGES-1 K-tiles in
// flight.  A 2-stage ring of 64-deep K-tiles keeps only one 28-57 KB tile in flight per CU, which
// at L2/MALL latency caps a CU at ~30 GB/s (Little's law; measured 2 us per 128x320x64 K-tile);
// halving the K-tile doubles the depth that fits in LDS.  One DMA instruction moves 16 rows x 64 B.
// 64-byte rows break the 128-byte XOR swizzle, so chunks are permuted by h((row >> 2) & 3) with
// h = (0, 3, 2, 1): for every ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...)
// the 16 lanes then hit 16 distinct 16-byte bank slots (checked per group, one 16-row fragment =
// four 4-row blocks).  The DMA writes lane-linear and the SOURCE chunk carries the permutation.
// Per K-tile each wave reads one 16x16x32 fragment set; with DBUF the next K-tile's fragments are
// read right after its barrier, under the tail of this K-tile's MFMAs (1 wave per SIMD configs).
// ---------------------------------------------------------------------------------------------
TAIR_DEV int ring_h(int g) { return (4 - g) & 3; }

template <int F, int I = 0>
TAIR_DEV void ds_read_frags64(bf16x8 (&o)[F], uint32_t addr) {  // fragment rows 16 apart = 1024 B apart
  if constexpr (I < F) {
    ds_read16<I * 1024>(o[I], addr);
    ds_read_frags64<F, I + 1>(o, addr);
  }
}

template <int BM, int BN, int WMW, int WNW, int STAGES, int DBUF, int AMODE>
__global__ __launch_bounds__(WMW * WNW * 64) void gemm_ring_kernel(const GemmGroup P_arg) {
  constexpr int BKS = 32;
  constexpr int NW = WMW * WNW;
  constexpr int WM = BM / WMW, WN = BN / WNW;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int NA = BM / (16 * NW), NB = BN / (16 * NW);  // DMA instructions per wave per K-tile
  constexpr int G = NA + NB;
  constexpr int STAGE_BYTES = (BM + BN) * BKS * 2;
  static_assert(BM % (16 * NW) == 0 && BN % (16 * NW) == 0, "DMA rows per wave");
  static_assert(WM % 16 == 0 && WN % 16 == 0 && FM + FN <= 15, "wave tile");
  static_assert(STAGES >= 3 && STAGES * STAGE_BYTES + 2048 + 64 <= 160 * 1024, "LDS");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const GemmGroup& P = kernarg0<GemmGroup>();
  int bxl, by, bz;
  xcd_remap(bxl, by, bz, P.xcd);
  const int grp = bxl / P.tiles_m;
  const int bx = bxl - grp * P.tiles_m;
  const GemmArgs& p = P.g[grp];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid % WMW, wn = wid / WMW;
  const int m0 = bx * BM, n0 = by * BN;
  const int ktot = (p.K + p.Kx) / BKS;
  const int per = (ktot + p.splits - 1) / p.splits;
  const int kt0 = bz * per;
  const int kt1 = min(ktot, kt0 + per);

  // DMA lane mapping: lane l -> row (l>>2) of the instruction's 16, LDS slot l&3, which must hold
  // logical chunk (l&3) ^ h((l>>4) & 3)
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ ring_h((lane >> 4) & 3);
  RowInfo<AMODE> rows[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) rows[i] = row_info<AMODE>(p, m0 + (i * NW + wid) * 16 + drow, dchunk);
  const bf16* wrow[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + (i * NW + wid) * 16 + drow;
    wrow[i] = n < p.N ? p.Wt + (size_t)n * p.ldw + dchunk * 8 : nullptr;
  }
  const bf16* zp = (const bf16*)g_zero_page;

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#define TAIR_ISSUE32(KT, STG)                                                                     \
  do {                                                                                            \
    const int k0_ = (KT) * BKS;                                                                   \
    char* sb_ = smem + (STG) * STAGE_BYTES;                                                       \
    _Pragma("unroll") for (int i = 0; i < NA; ++i)                                                \
      __builtin_amdgcn_global_load_lds((const void*)act_src<AMODE>(p, rows[i], k0_),             \
                                       TAIR_LDS(sb_ + (i * NW + wid) * 16 * 64), 16, 0, 0);       \
    _Pragma("unroll") for (int i = 0; i < NB; ++i)                                                \
      __builtin_amdgcn_global_load_lds((const void*)(wrow[i] ? wrow[i] + k0_ : zp),              \
                                       TAIR_LDS(sb_ + BM * 64 + (i * NW + wid) * 16 * 64), 16, 0, 0); \
  } while (0)

  const uint32_t lds0 = lds_u32(smem);
  const int r16 = lane & 15;
  const int cq = (lane >> 4) ^ ring_h(r16 >> 2);  // permuted chunk of this lane's fragment row
  const uint32_t aoff = (wm * WM + r16) * 64 + cq * 16;
  const uint32_t boff = BM * 64 + (wn * WN + r16) * 64 + cq * 16;

  if (kt0 < kt1) {
    const int kl = kt1 - 1;
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) TAIR_ISSUE32(min(kt0 + s, kl), s);
    int stage = 0;
    bf16x8 xf[FM], wf[FN];
    if constexpr (DBUF) {  // fragments of the first K-tile
      wait_vmcnt<(STAGES - 2) * G>();
      __builtin_amdgcn_s_barrier();
      ds_read_frags64<FM>(xf, lds0 + aoff);
      ds_read_frags64<FN>(wf, lds0 + boff);
    }
    for (int t = kt0; t < kt1; ++t) {
      if constexpr (!DBUF) {
        wait_vmcnt<(STAGES - 2) * G>();  // this wave's copies of tile t have landed
        __builtin_amdgcn_s_barrier();    // ... and every wave's; tile t-1's buffer is free
      }
      int ps = stage + STAGES - 1;
      if (ps >= STAGES) ps -= STAGES;
      TAIR_ISSUE32(min(t + STAGES - 1, kl), ps);  // into the buffer of tile t-1
      if constexpr (!DBUF) {
        const uint32_t sb = lds0 + stage * STAGE_BYTES;
        ds_read_frags64<FM>(xf, sb + aoff);
        ds_read_frags64<FN>(wf, sb + boff);
      }
      wait_lgkmcnt<0>();
      touch<FM>(xf);
      touch<FN>(wf);
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 cx[FM], cw[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) cx[i] = xf[i];
#pragma unroll
      for (int j = 0; j < FN; ++j) cw[j] = wf[j];
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[j], cx[i], acc[j][i], 0, 0, 0);
      stage = (stage + 1 == STAGES) ? 0 : stage + 1;
      if constexpr (DBUF) {
        // next K-tile: wait + barrier, then its fragment reads run under this tile's MFMA tail
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < kt1) {
          wait_vmcnt<(STAGES - 2) * G>();
          __builtin_amdgcn_s_barrier();
          const uint32_t sb = lds0 + stage * STAGE_BYTES;
          ds_read_frags64<FM>(xf, sb + aoff);
          ds_read_frags64<FN>(wf, sb + boff);
        }
      }
    }
    wait_vmcnt<0>();  // drain the clamped tail copies before the wave can exit
  }
#undef TAIR_ISSUE32

  epilogue_tile<BM, BN, FM, FN, WM, WN, NW * 64, STAGES * STAGE_BYTES + 2048 + 64>(p, acc, m0, n0, wm, wn, lane,
                                                                                smem, bz);
}

template <int BM_, int BN_, int WMW_, int WNW_, int STAGES_, int DBUF_>
struct RingCfg {
  static constexpr int BM = BM_, BN = BN_, WMW = WMW_, WNW = WNW_, STAGES = STAGES_, DBUF = DBUF_;
  static constexpr size_t LDS = (size_t)STAGES * (BM + BN) * 32 * sizeof(bf16) + 2048 + 64;
  static constexpr int THREADS = WMW * WNW * 64;
};
using R128x320 = RingCfg<128, 320, 2, 2, 5, 1>;  // 1 wave / SIMD, fragments double-buffered
using R256x256 = RingCfg<256, 256, 2, 4, 4, 0>;  // 2 waves / SIMD
using R256x128 = RingCfg<256, 128, 4, 2, 6, 0>;
using R128x256 = RingCfg<128, 256, 2, 4, 6, 0>;
using R128x128 = RingCfg<128, 128, 2, 2, 8, 1>;
using R64x128 = RingCfg<64, 128, 2, 2, 8, 1>;
using R64x64 = RingCfg<64, 64, 2, 2, 8, 1>;

template <class T, int AMODE>
hipError_t set_attr_ring() {
  TAIR_HIP_CHECK(hipFuncSetAttribute(
      (const void*)gemm_ring_kernel<T::BM, T::BN, T::WMW, T::WNW, T::STAGES, T::DBUF, AMODE>,
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)T::LDS));
  return hipSuccess;
}
template <class T, int AMODE>
hipError_t launch_ring_tile(GemmGroup& a, int n, int splits, hipStream_t s) {
  a.tiles_m = cdiv(a.g[0].M, T::BM);
  dim3 grid(a.tiles_m * n, cdiv(a.g[0].N, T::BN), splits);
  hipLaunchKernelGGL((gemm_ring_kernel<T::BM, T::BN, T::WMW, T::WNW, T::STAGES, T::DBUF, AMODE>), grid,
                     dim3(T::THREADS), T::LDS, s, a);
  return hipGetLastError();
}
template <int AMODE>
hipError_t set_attrs_ring() {
  TAIR_HIP_CHECK((set_attr_ring<R128x320, AMODE>()));
  TAIR_HIP_CHECK((set_attr_ring<R256x256, AMODE>()));
  TAIR_HIP_CHECK((set_attr_ring<R256x128, AMODE>()));
  TAIR_HIP_CHECK((set_attr_ring<R128x256, AMODE>()));
  TAIR_HIP_CHECK((set_attr_ring<R128x128, AMODE>()));
  TAIR_HIP_CHECK((set_attr_ring<R64x128, AMODE>()));
  TAIR_HIP_CHECK((set_attr_ring<R64x64, AMODE>()));
  return hipSuccess;
}
template <int AMODE>
hipError_t launch_ring(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s) {
  if (bm == 128 && bn == 320) return launch_ring_tile<R128x320, AMODE>(a, n, splits, s);
  if (bm == 256 && bn == 256) return launch_ring_tile<R256x256, AMODE>(a, n, splits, s);
  if (bm == 256 && bn == 128) return launch_ring_tile<R256x128, AMODE>(a, n, splits, s);
  if (bm == 128 && bn == 256) return launch_ring_tile<R128x256, AMODE>(a, n, splits, s);
  if (bm == 128 && bn == 128) return launch_ring_tile<R128x128, AMODE>(a, n, splits, s);
  if (bm == 64 && bn == 128) return launch_ring_tile<R64x128, AMODE>(a, n, splits, s);
  if (bm == 64 && bn == 64) return launch_ring_tile<R64x64, AMODE>(a, n, splits, s);
  return hipErrorInvalidValue;
}

// A tile configuration of gemm_tile_kernel: tile, wave grid, ring depth.
template <int BM_, int BN_, int WMW_, int WNW_, int STAGES_>
struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, WMW = WMW_, WNW = WNW_, STAGES = STAGES_;
  static constexpr size_t LDS = (size_t)STAGES * (BM + BN) * BK * sizeof(bf16);
  static constexpr int THREADS = WMW * WNW * 64;
};
// small tiles (B = 1 shapes): 4 waves, 3-deep ring
using T64x64 = TileCfg<64, 64, 2, 2, 3>;
using T64x128 = TileCfg<64, 128, 2, 2, 3>;
using T128x64 = TileCfg<128, 64, 2, 2, 3>;
using T128x128 = TileCfg<128, 128, 2, 2, 3>;
// "shallow" 2-stage 64-row tiles: 32 / 48 KiB of LDS, so 4-5 workgroups share a CU and overlap one
// another's prologue / epilogue -- the short-K linears of the batched network (B = 16: proj 79 -> 62 us,
// qkv 160 -> 130, ff1 389 -> 318); the latency-bound B = 1 plans keep the 3-deep ring
using T64x64S = TileCfg<64, 64, 2, 2, 2>;
using T64x128S = TileCfg<64, 128, 2, 2, 2>;
// "deep" 64-row tiles (B = 1, latency-bound): more K-tiles in flight per workgroup where the grid still fits
// the CUs in the same number of rounds as with the 3-deep ring (gemm_grouped picks the depth: GemmArgs.tile_stages)
using T64x64D4 = TileCfg<64, 64, 2, 2, 4>;
using T64x64D5 = TileCfg<64, 64, 2, 2, 5>;
using T64x64D6 = TileCfg<64, 64, 2, 2, 6>;
using T64x64D8 = TileCfg<64, 64, 2, 2, 8>;
using T64x128D4 = TileCfg<64, 128, 2, 2, 4>;
using T64x128D5 = TileCfg<64, 128, 2, 2, 5>;
using T64x128D6 = TileCfg<64, 128, 2, 2, 6>;
// large tiles (batched tiles): 8 waves
using T128x256 = TileCfg<128, 256, 2, 4, 3>;
using T256x256 = TileCfg<256, 256, 2, 4, 2>;
using T128x320 = TileCfg<128, 320, 2, 4, 2>;
using T256x320 = TileCfg<256, 320, 2, 4, 2>;
using T256x160 = TileCfg<256, 160, 2, 2, 3>;  // 3-deep ring at half the 320-column tile
using T256x128 = TileCfg<256, 128, 4, 2, 3>;

template <class T, int AMODE, int F8 = 0>
hipError_t set_attr_tile() {
  TAIR_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_tile_kernel<T::BM, T::BN, T::WMW, T::WNW, T::STAGES, AMODE, F8>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  return hipSuccess;
}

// Workgroups of one kernel the device holds at once: CUs x the kernel's occupancy at this LDS size (cached per
// device and LDS size).  0 when it cannot be queried.
template <class KernT>
long resident_wgs(KernT kern, int threads, size_t lds) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
      hipSuccess)
    return 0;
  static thread_local struct { const void* k; int dev; size_t lds; long v; } memo[8] = {};
  for (auto& m : memo)
    if (m.k == (const void*)kern && m.dev == dev && m.lds == lds) return m.v;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, threads, lds) != hipSuccess) return 0;
  static thread_local int next = 0;
  memo[next] = {(const void*)kern, dev, lds, (long)cus * per};
  next = (next + 1) % 8;
  return (long)cus * per;
}

template <class T, int AMODE, int F8 = 0>
hipError_t launch_tile(GemmGroup& a, int n, int splits, hipStream_t s) {
  a.tiles_m = cdiv(a.g[0].M, T::BM);
  dim3 grid(a.tiles_m * n, cdiv(a.g[0].N, T::BN), splits);
  if (a.g[0].coop) {
    // the cooperative combine makes a tile's K slices wait for one another: only on grids the device holds at
    // once (device CU count x this kernel's occupancy); otherwise the last-arriving slice combines (no waits)
    const long cap = resident_wgs(gemm_tile_kernel<T::BM, T::BN, T::WMW, T::WNW, T::STAGES, AMODE, F8>, T::THREADS,
                                  T::LDS + gn_extra_lds(a.g[0], splits));
    if ((long)grid.x * grid.y * grid.z > cap)
      for (int i = 0; i < MAX_GROUP; ++i) a.g[i].coop = 0;
  }
  hipLaunchKernelGGL((gemm_tile_kernel<T::BM, T::BN, T::WMW, T::WNW, T::STAGES, AMODE, F8>), grid, dim3(T::THREADS),
                     T::LDS + gn_extra_lds(a.g[0], splits), s, a);
  return hipGetLastError();
}

// fp8 (e4m3 x e4m3, 16x16x128 MFMA) dense tiles: the B = 1 64-row tiles and the batched 128-row tiles
template <int AMODE>
hipError_t set_attrs_f8() {
  TAIR_HIP_CHECK((set_attr_tile<T64x64, AMODE, 1>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x128, AMODE, 1>()));
  TAIR_HIP_CHECK((set_attr_tile<T128x128, AMODE, 1>()));
  TAIR_HIP_CHECK((set_attr_tile<T128x256, AMODE, 1>()));
  TAIR_HIP_CHECK((set_attr_tile<T128x320, AMODE, 1>()));
  if constexpr (AMODE == A_DENSE) {  // the 2-stage 64-row tiles of the batched short-K linears
    TAIR_HIP_CHECK((set_attr_tile<T64x64S, AMODE, 1>()));
    TAIR_HIP_CHECK((set_attr_tile<T64x128S, AMODE, 1>()));
  }
  return hipSuccess;
}
template <int AMODE>
hipError_t launch_f8(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s, bool shallow = false) {
  if constexpr (AMODE == A_DENSE) {
    if (shallow && bm == 64 && bn == 64) return launch_tile<T64x64S, AMODE, 1>(a, n, splits, s);
    if (shallow && bm == 64 && bn == 128) return launch_tile<T64x128S, AMODE, 1>(a, n, splits, s);
  }
  if (bm == 64 && bn == 64) return launch_tile<T64x64, AMODE, 1>(a, n, splits, s);
  if (bm == 64 && bn == 128) return launch_tile<T64x128, AMODE, 1>(a, n, splits, s);
  if (bm == 128 && bn == 128) return launch_tile<T128x128, AMODE, 1>(a, n, splits, s);
  if (bm == 128 && bn == 256) return launch_tile<T128x256, AMODE, 1>(a, n, splits, s);
  if (bm == 128 && bn == 320) return launch_tile<T128x320, AMODE, 1>(a, n, splits, s);
  return hipErrorInvalidValue;
}

template <int AMODE>
hipError_t set_attrs_shallow() {
  TAIR_HIP_CHECK((set_attr_tile<T64x64S, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x128S, AMODE>()));
  return hipSuccess;
}
template <int AMODE>
hipError_t launch_shallow(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s) {
  if (bm == 64 && bn == 64) return launch_tile<T64x64S, AMODE>(a, n, splits, s);
  if (bm == 64 && bn == 128) return launch_tile<T64x128S, AMODE>(a, n, splits, s);
  return hipErrorInvalidValue;
}

// "small" tile set (4 waves) and "big" tile set (8 waves): separate translation units per mode
template <int AMODE>
hipError_t set_attrs_small() {
  TAIR_HIP_CHECK((set_attr_tile<T64x64, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x128, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T128x64, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T128x128, AMODE>()));
  return hipSuccess;
}
template <int AMODE>
hipError_t launch_small(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s) {
  if (bm == 64 && bn == 64) return launch_tile<T64x64, AMODE>(a, n, splits, s);
  if (bm == 64 && bn == 128) return launch_tile<T64x128, AMODE>(a, n, splits, s);
  if (bm == 128 && bn == 64) return launch_tile<T128x64, AMODE>(a, n, splits, s);
  if (bm == 128 && bn == 128) return launch_tile<T128x128, AMODE>(a, n, splits, s);
  return hipErrorInvalidValue;
}
template <int AMODE>
hipError_t set_attrs_deep() {
  TAIR_HIP_CHECK((set_attr_tile<T64x64D4, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x64D5, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x64D6, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x64D8, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x128D4, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x128D5, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T64x128D6, AMODE>()));
  return hipSuccess;
}
template <int AMODE>
hipError_t launch_deep(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s) {
  const int st = a.g[0].tile_stages;
  if (bm == 64 && bn == 64) {
    if (st == 4) return launch_tile<T64x64D4, AMODE>(a, n, splits, s);
    if (st == 5) return launch_tile<T64x64D5, AMODE>(a, n, splits, s);
    if (st == 6) return launch_tile<T64x64D6, AMODE>(a, n, splits, s);
    if (st == 8) return launch_tile<T64x64D8, AMODE>(a, n, splits, s);
  }
  if (bm == 64 && bn == 128) {
    if (st == 4) return launch_tile<T64x128D4, AMODE>(a, n, splits, s);
    if (st == 5) return launch_tile<T64x128D5, AMODE>(a, n, splits, s);
    if (st == 6) return launch_tile<T64x128D6, AMODE>(a, n, splits, s);
  }
  return hipErrorInvalidValue;
}
template <int AMODE>
hipError_t set_attrs_big() {
  TAIR_HIP_CHECK((set_attr_tile<T128x256, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T256x256, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T128x320, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T256x320, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T256x160, AMODE>()));
  TAIR_HIP_CHECK((set_attr_tile<T256x128, AMODE>()));
  return hipSuccess;
}
template <int AMODE>
hipError_t launch_big(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s) {
  if (bm == 128 && bn == 256) return launch_tile<T128x256, AMODE>(a, n, splits, s);
  if (bm == 256 && bn == 256) return launch_tile<T256x256, AMODE>(a, n, splits, s);
  if (bm == 128 && bn == 320) return launch_tile<T128x320, AMODE>(a, n, splits, s);
  if (bm == 256 && bn == 320) return launch_tile<T256x320, AMODE>(a, n, splits, s);
  if (bm == 256 && bn == 160) return launch_tile<T256x160, AMODE>(a, n, splits, s);
  if (bm == 256 && bn == 128) return launch_tile<T256x128, AMODE>(a, n, splits, s);
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------
// 4-phase ping-pong kernel for large grids: 256 x BN tile (BN = 256 | 320), 8 waves as 2 (m) x 4 (n),
// each wave 128 pixels x BN/4 channels, BK = 64, two LDS buffers.
// * Phases.  A K-tile is 4 phases; in phase q a wave multiplies its A-quarter q (2 x 16 pixel rows)
//   by all its weight fragments (read into registers once per K-tile, in phase 0): 2 x FN x 2 MFMAs.
// * Ping-pong (cdna_hip_programming.md, 8-phase template): every phase is
//     ds_read (this phase's fragments) ; LDS-DMA issue ; vmcnt wait ; s_barrier R ;
//     lgkmcnt(0) ; MFMAs (s_setprio 1) ; s_barrier M
//   and waves 4-7 (one per SIMD) run ONE barrier behind waves 0-3: each SIMD's matrix pipe alternates
//   between one wave's MFMA section and the other's read/DMA section.
// * Quarters.  Each A quarter / the W tile of a buffer is re-staged by LDS-DMA (with the data of the
//   K-tile two ahead) two phases after its last read (the lagging group's reads of phase P are done
//   by barrier 2P+2, the leading group issues phase P+2's copies after barrier 2P+3), and read six
//   phases after it was issued: about 1.5 K-tiles of copies stay in flight across every barrier.
//   Phase issue list of K-tile t: q0 A-q2 (t+1) | q1 A-q3 (t+1) | q2 W + A-q0 (t+2) | q3 A-q1 (t+2).
// * Waits.  In phase P a wave waits for its own copies of the regions read in P+1 (issued in P-5),
//   letting the copies of phases P-4..P stay in flight: GW + 5, or 2 GW + 5 at q = 2 (GW = BN/64 W
//   copies per wave per K-tile, 1 per A quarter).  The wait precedes barrier R of phase P, which for
//   the lagging group is barrier 2P+1, the one the leading group passes before reading phase P+1.
// LDS A row of logical tile row m = 128 wm + 32 q + rr (rr < 32) is 64 q + 32 wm + rr; rows are 128 B
// with the chunk ^ (row & 7) swizzle carried by the DMA source chunk (lane-linear DMA destination).
// ---------------------------------------------------------------------------------------------
template <int BN, int AMODE, int ABL = 0>  // ABL (ablation probes, tools/gemm_probe.py): 1 no DMA in the loop, 2 no MFMA
__global__ __launch_bounds__(512) void gemm_phase_kernel(const GemmGroup P_arg) {
  constexpr int BM = 256, NW = 8, WM = 128, WN = BN / 4;
  constexpr int FM = 8, FN = WN / 16;
  constexpr int GW = BN / 64;                      // W DMA instructions per wave per K-tile
  constexpr int SA = BM * 128, SBUF = (BM + BN) * 128;
  static_assert(WN % 16 == 0 && (BN % 64) == 0, "tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const GemmGroup& P = kernarg0<GemmGroup>();
  int bxl, by, bz;
  xcd_remap(bxl, by, bz, P.xcd);
  const int grp = bxl / P.tiles_m;
  const int bx = bxl - grp * P.tiles_m;
  const GemmArgs& p = P.g[grp];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid & 1, wn = wid >> 1;
  const bool lag = wid >= 4;  // waves 4-7: one barrier behind (one wave of each group per SIMD)
  const int m0 = bx * BM, n0 = by * BN;
  const int ktot = (p.K + p.Kx) / BK;
  const int per = (ktot + p.splits - 1) / p.splits;
  const int kt0 = bz * per;
  const int kt1 = min(ktot, kt0 + per);

  const int drow = lane >> 3;
  const int dchunk = (lane & 7) ^ drow;
  // DMA rows of this wave: A quarter q -> LDS rows 64q + 8 wid + drow = tile row 128 (wid >> 2) + 32 q +
  // 8 (wid & 3) + drow; W -> rows (i*8 + wid)*8 + drow
  RowInfo<AMODE> rows[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    rows[q] = row_info<AMODE>(p, m0 + 128 * (wid >> 2) + 32 * q + 8 * (wid & 3) + drow, dchunk);
  const bf16* wrow[GW];
#pragma unroll
  for (int i = 0; i < GW; ++i) {
    const int n = n0 + (i * NW + wid) * 8 + drow;
    wrow[i] = n < p.N ? p.Wt + (size_t)n * p.ldw + dchunk * 8 : nullptr;
  }
  const bf16* zp = (const bf16*)g_zero_page;

  f32x4 acc[FN][FM];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

#define TAIR_PH_A(KT, BUF, Q)                                                                     \
  __builtin_amdgcn_global_load_lds((const void*)act_src<AMODE>(p, rows[Q], (KT) * BK),           \
                                   TAIR_LDS(smem + (BUF) * SBUF + (64 * (Q) + 8 * wid) * 128), 16, 0, 0)
#define TAIR_PH_W(KT, BUF)                                                                        \
  do {                                                                                            \
    _Pragma("unroll") for (int i = 0; i < GW; ++i)                                                \
      __builtin_amdgcn_global_load_lds((const void*)(wrow[i] ? wrow[i] + (KT) * BK : zp),        \
                                       TAIR_LDS(smem + (BUF) * SBUF + SA + (i * NW + wid) * 8 * 128), 16, 0, 0); \
  } while (0)

  const uint32_t lds0 = lds_u32(smem);
  // fragment read offsets within a buffer: A rows 64q + 32 wm + 16 i' + (lane & 15); W rows
  // wn*WN + 16 j + (lane & 15); (row & 7) == (lane & 7) for both
  const int r16 = lane & 15;
  const uint32_t c0 = (((lane >> 4)) ^ (lane & 7)) << 4, c1 = (((4 + (lane >> 4))) ^ (lane & 7)) << 4;
  const uint32_t a_row = (32 * wm + r16) * 128, w_row = SA + (wn * WN + r16) * 128;

  if (kt0 < kt1) {
    const int kl = kt1 - 1;
    // prologue: the copies the steady state issues in the six phases before K-tile kt0
    const int k1 = min(kt0 + 1, kl);
    TAIR_PH_W(kt0, 0);
    TAIR_PH_A(kt0, 0, 0);
    TAIR_PH_A(kt0, 0, 1);
    TAIR_PH_A(kt0, 0, 2);
    TAIR_PH_A(kt0, 0, 3);
    TAIR_PH_W(k1, 1);
    TAIR_PH_A(k1, 1, 0);
    TAIR_PH_A(k1, 1, 1);
    wait_vmcnt<GW + 5>();  // own copies of W(kt0), A-q0(kt0) landed
    __builtin_amdgcn_s_barrier();
    if (lag) __builtin_amdgcn_s_barrier();  // the stagger (pairs with the leaders' first barrier R)
    bf16x8 wf0[FN], wf1[FN];  // weight fragments of the K-tile: K halves 0 / 1
    int buf = 0;
    for (int t = kt0; t < kt1; ++t) {
      const int t1 = min(t + 1, kl), t2 = min(t + 2, kl);
      const uint32_t sb = lds0 + buf * SBUF;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x8 xf0[2], xf1[2];
        const uint32_t aq = sb + a_row + q * 64 * 128;
        if (q == 0) {
          ds_read_frags<FN>(wf0, sb + w_row + c0);
          ds_read_frags<FN>(wf1, sb + w_row + c1);
        }
        ds_read16<0>(xf0[0], aq + c0);
        ds_read16<2048>(xf0[1], aq + c0);
        ds_read16<0>(xf1[0], aq + c1);
        ds_read16<2048>(xf1[1], aq + c1);
        if (ABL != 1) {
          if (q == 0) TAIR_PH_A(t1, buf ^ 1, 2);
          if (q == 1) TAIR_PH_A(t1, buf ^ 1, 3);
          if (q == 2) {
            TAIR_PH_W(t2, buf);
            TAIR_PH_A(t2, buf, 0);
          }
          if (q == 3) TAIR_PH_A(t2, buf, 1);
        }
        if (q == 2) wait_vmcnt<2 * GW + 5>();
        else wait_vmcnt<GW + 5>();
        __builtin_amdgcn_s_barrier();  // R
        wait_lgkmcnt<0>();
        touch<2>(xf0);
        touch<2>(xf1);
        touch<FN>(wf0);
        touch<FN>(wf1);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            if (ABL != 2)
              acc[j][2 * q + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf0[j], xf0[i], acc[j][2 * q + i], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            if (ABL != 2)
              acc[j][2 * q + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf1[j], xf1[i], acc[j][2 * q + i], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();  // M
      }
      buf ^= 1;
    }
    if (!lag) __builtin_amdgcn_s_barrier();  // the leaders' last barrier pairs with the laggards' M
    wait_vmcnt<0>();  // drain the clamped tail copies before LDS reuse / exit
    __builtin_amdgcn_s_barrier();
  }
#undef TAIR_PH_A
#undef TAIR_PH_W
  epilogue_direct<FM, FN, WM, WN>(p, acc, m0, n0, wm, wn, lane, (double*)smem, BN);
}

template <int BN>
struct PhaseCfg {
  static constexpr size_t LDS = (size_t)2 * (256 + BN) * BK * sizeof(bf16);
};
template <int BN, int AMODE, int ABL = 0>
hipError_t set_attr_phase() {
  TAIR_HIP_CHECK(hipFuncSetAttribute((const void*)gemm_phase_kernel<BN, AMODE, ABL>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)PhaseCfg<BN>::LDS));
  return hipSuccess;
}
template <int AMODE>
hipError_t set_attrs_phase() {
  TAIR_HIP_CHECK((set_attr_phase<256, AMODE>()));
  TAIR_HIP_CHECK((set_attr_phase<320, AMODE>()));
  if constexpr (AMODE == A_CONV3) {  // ablation probes (force_stages 5 / 6)
    TAIR_HIP_CHECK((set_attr_phase<256, AMODE, 1>()));
    TAIR_HIP_CHECK((set_attr_phase<256, AMODE, 2>()));
  }
  return hipSuccess;
}
template <int BN, int AMODE, int ABL = 0>
hipError_t launch_phase_tile(GemmGroup& a, int n, int splits, hipStream_t s) {
  a.tiles_m = cdiv(a.g[0].M, 256);
  dim3 grid(a.tiles_m * n, cdiv(a.g[0].N, BN), splits);
  hipLaunchKernelGGL((gemm_phase_kernel<BN, AMODE, ABL>), grid, dim3(512), PhaseCfg<BN>::LDS, s, a);
  return hipGetLastError();
}
template <int AMODE>
hipError_t launch_phase(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s) {
  if constexpr (AMODE == A_CONV3) {
    if (a.g[0].force_stages == 5 && bn == 256) return launch_phase_tile<256, AMODE, 1>(a, n, splits, s);
    if (a.g[0].force_stages == 6 && bn == 256) return launch_phase_tile<256, AMODE, 2>(a, n, splits, s);
  }
  if (bm != 256) return hipErrorInvalidValue;
  if (bn == 256) return launch_phase_tile<256, AMODE>(a, n, splits, s);
  if (bn == 320) return launch_phase_tile<320, AMODE>(a, n, splits, s);
  return hipErrorInvalidValue;
}

}  // namespace

// Per-mode, per-tile-set translation units: gemm_mode_attrs / gemm_mode_launch for AMODE and SET
// (small | big | reg).
template <int AMODE, int SET> hipError_t gemm_set_attrs();
template <int AMODE, int SET> hipError_t gemm_set_launch(GemmGroup& a, int n, int bm, int bn, int splits, hipStream_t s);
constexpr int SET_SMALL = 0, SET_BIG = 1, SET_REG = 2, SET_RING = 3, SET_PHASE = 4, SET_SHALLOW = 5, SET_F8 = 6,
              SET_HALO = 7, SET_DEEP = 8;

}  // namespace tair

#define TAIR_GEMM_SET_TU(AMODE, SET, KIND)                                                             \
  namespace tair {                                                                                     \
  template <>                                                                                          \
  hipError_t gemm_set_attrs<AMODE, SET>() {                                                            \
    return set_attrs_##KIND<AMODE>();                                                                  \
  }                                                                                                    \
  template <>                                                                                          \
  hipError_t gemm_set_launch<AMODE, SET>(GemmGroup & a, int n, int bm, int bn, int splits, hipStream_t s) { \
    return launch_##KIND<AMODE>(a, n, bm, bn, splits, s);                                              \
  }                                                                                                    \
  }
