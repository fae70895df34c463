// Tile stitching on the device (reference: val_patches.py:114-206 merge_patches_with_overlap,
// image_splitter.py:23-51): the decoded 512^2 tiles of an image -- gathered across ranks by the
// RCCL all-gather -- are blended into the output in one pass, instead of a host loop of
// per-tile slice-adds (2 launches per tile, serialised on the weight map).
//
// Each output pixel (cropped to scale * LQ size) visits the tiles that cover it IN RASTER ORDER,
// exactly as the reference's loop accumulates them, with the same fp32 operations:
//   w   = r(a) * r(b)                  ramp window, r(i) = fp32((i + 1) / overlap) at the borders
//   acc = acc + tile * w               (two roundings: no fma contraction)
//   sum = sum + w
//   out = acc / max(sum, 1e-8)         (correctly rounded division)
// so the result is bitwise the reference loop's (tests/test_val_patches_gpu.py).  The stride is a
// parameter (the reference hard-codes 112 / 448, val_patches.py:134-138).  Memory-bound: each output
// element reads the covering tiles' elements once (<= 4 for overlap < stride) and writes once.
#include "kernels.h"

namespace tair {
namespace {

TAIR_DEV float ramp(int i, int patch, int overlap, const float* rtab) {
  // rtab[i] = fp32((i + 1) / overlap), i < overlap (computed on the host in double, then rounded)
  if (i < overlap) return rtab[i];
  if (i >= patch - overlap) return rtab[patch - 1 - i];
  return 1.f;
}

__global__ __launch_bounds__(256) void merge_overlap_kernel(const float* __restrict__ tiles, int n_tiles, int nh,
                                                            int nw, int patch, int overlap, int stride,
                                                            float* __restrict__ out, int C, int H, int W,
                                                            const float* __restrict__ rtab) {
#pragma clang fp contract(off)  // hipcc contracts a*b+c into fma by default: keep the two roundings
  // (plain operators in this scope: the pragma does not reach the fmul/fadd of inlined intrinsics)
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)H * W) return;
  const int y = (int)(idx / W), x = (int)(idx - (long)y * W);
  // tiles covering row y: i*stride <= y < i*stride + patch
  const int span = (patch + stride - 1) / stride;  // tiles that can cover one coordinate
  const int i_hi = min(nh - 1, y / stride), i_lo = max(0, y / stride - span);
  const int j_hi = min(nw - 1, x / stride), j_lo = max(0, x / stride - span);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float wsum = 0.f;
  const size_t plane = (size_t)patch * patch;
  for (int i = i_lo; i <= i_hi; ++i) {
    const int a = y - i * stride;
    if (a < 0 || a >= patch) continue;
    const float ra = ramp(a, patch, overlap, rtab);
    for (int j = j_lo; j <= j_hi; ++j) {
      const int b = x - j * stride;
      if (b < 0 || b >= patch) continue;
      const int k = i * nw + j;
      if (k >= n_tiles) continue;
      const float w = ra * ramp(b, patch, overlap, rtab);
      const float* t = tiles + (size_t)k * C * plane + (size_t)a * patch + b;
      for (int c = 0; c < C && c < 4; ++c) {
        const float tw = t[c * plane] * w;
        acc[c] = acc[c] + tw;
      }
      wsum = wsum + w;
    }
  }
  const float den = fmaxf(wsum, 1e-8f);
  for (int c = 0; c < C && c < 4; ++c) out[(size_t)c * H * W + idx] = __fdiv_rn(acc[c], den);
}

// ---- stitch fused with the tile exchange ------------------------------------------
// configs[3]: the global tile list (image-major, raster inside an image) is sharded into contiguous
// per-rank blocks of `per_rank` tiles [C][patch][patch] fp32.  Instead of an RCCL all-gather into one
// buffer followed by the blend, every rank's kernel reads the covering tiles straight out of the owning
// rank's block (src[r]: that rank's buffer, mapped into this process by IPC; over xGMI for a peer GPU)
// and writes the stitched images: one pass, no gathered copy.  blockIdx.y = image - img0 (a rank stitches
// only the images it owns, reading just the tiles that cover them: img0 = its first image).  mode 0: the
// image_splitter.py placement (each output pixel from exactly one tile, H = nh * patch); mode 1: the
// overlap blend above, bitwise the reference merge loop (same visiting order and fp32 operations).
TAIR_DEV const float* peer_tile(const float* const* src, int per_rank, int g, size_t tile_elems) {
  const int r = g / per_rank;
  return src[r] + (size_t)(g - r * per_rank) * tile_elems;
}

__global__ __launch_bounds__(256) void stitch_peers_kernel(const float* const* __restrict__ src, int per_rank,
                                                           int img0, int tiles_per_image, int nh, int nw, int mode,
                                                           int patch, int overlap, int stride,
                                                           float* __restrict__ out, int C, int H, int W,
                                                           const float* __restrict__ rtab) {
#pragma clang fp contract(off)
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)H * W) return;
  const int img = blockIdx.y;
  const int y = (int)(idx / W), x = (int)(idx - (long)y * W);
  const size_t plane = (size_t)patch * patch, tile_elems = (size_t)C * plane;
  float* o = out + (size_t)img * C * H * W + idx;
  const int g0 = (img0 + img) * tiles_per_image;
  if (mode == 0) {
    const int i = y / patch, j = x / patch;
    const float* t = peer_tile(src, per_rank, g0 + i * nw + j, tile_elems) + (size_t)(y - i * patch) * patch +
                     (x - j * patch);
    for (int c = 0; c < C && c < 4; ++c) o[(size_t)c * H * W] = t[c * plane];
    return;
  }
  const int span = (patch + stride - 1) / stride;
  const int i_hi = min(nh - 1, y / stride), i_lo = max(0, y / stride - span);
  const int j_hi = min(nw - 1, x / stride), j_lo = max(0, x / stride - span);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float wsum = 0.f;
  for (int i = i_lo; i <= i_hi; ++i) {
    const int a = y - i * stride;
    if (a < 0 || a >= patch) continue;
    const float ra = ramp(a, patch, overlap, rtab);
    for (int j = j_lo; j <= j_hi; ++j) {
      const int b = x - j * stride;
      if (b < 0 || b >= patch) continue;
      const int k = i * nw + j;
      if (k >= tiles_per_image) continue;
      const float w = ra * ramp(b, patch, overlap, rtab);
      const float* t = peer_tile(src, per_rank, g0 + k, tile_elems) + (size_t)a * patch + b;
      for (int c = 0; c < C && c < 4; ++c) {
        const float tw = t[c * plane] * w;
        acc[c] = acc[c] + tw;
      }
      wsum = wsum + w;
    }
  }
  const float den = fmaxf(wsum, 1e-8f);
  for (int c = 0; c < C && c < 4; ++c) o[(size_t)c * H * W] = __fdiv_rn(acc[c], den);
}

}  // namespace

hipError_t stitch_peers(const float* const* src, int per_rank, int first_image, int n_images, int tiles_per_image,
                        int nh, int nw,
                        int mode, int patch, int overlap, int stride, float* out, int C, int H, int W,
                        const float* rtab, hipStream_t s) {
  const bool geom = mode == 0 ? (H == nh * patch && W == nw * patch && tiles_per_image == nh * nw)
                              : (stride >= 1 && overlap >= 1 && 2 * overlap <= patch && stride <= patch && rtab);
  if (C < 1 || C > 4 || n_images < 1 || first_image < 0 || per_rank < 1 || tiles_per_image < 1 || (mode != 0 && mode != 1) || !geom ||
      n_images > 65535) {
    set_error("stitch_peers: unsupported geometry (mode %d, C %d, patch %d, overlap %d, stride %d, %dx%d tiles, %dx%d)",
              mode, C, patch, overlap, stride, nh, nw, H, W);
    return hipErrorInvalidValue;
  }
  const long total = (long)H * W;
  hipLaunchKernelGGL(stitch_peers_kernel, dim3((unsigned)((total + 255) / 256), n_images), dim3(256), 0, s, src,
                     per_rank, first_image, tiles_per_image, nh, nw, mode, patch, overlap, stride, out, C, H, W, rtab);
  return hipGetLastError();
}

hipError_t merge_overlap(const float* tiles, int n_tiles, int nh, int nw, int patch, int overlap, int stride,
                         float* out, int C, int H, int W, const float* rtab, hipStream_t s) {
  if (C < 1 || C > 4 || stride < 1 || overlap < 1 || 2 * overlap > patch || stride > patch) {
    set_error("merge_overlap: unsupported geometry (C %d, patch %d, overlap %d, stride %d)", C, patch, overlap,
              stride);
    return hipErrorInvalidValue;
  }
  const long total = (long)H * W;
  hipLaunchKernelGGL(merge_overlap_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, tiles, n_tiles,
                     nh, nw, patch, overlap, stride, out, C, H, W, rtab);
  return hipGetLastError();
}

}  // namespace tair
