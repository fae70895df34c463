// Launcher interfaces for the gfx950 kernels (host side).  All launchers are asynchronous on the
// given stream, allocate nothing and never synchronise, so every forward is hipGraph-capturable.
#pragma once
#include "common.h"

namespace tair {

// How the GEMM kernel forms its activation operand X[m][k] (m = output pixel / token).
enum AMode : int {
  A_DENSE = 0,     // X[m][k] = A[m*lda + k]                          (Linear, 1x1 conv)
  A_CONV3 = 1,     // 3x3, stride 1, pad 1 implicit im2col (C % 64 == 0), channel-chunk-major K:
                   // k = (c/64 * 9 + tap) * 64 + c%64, so the 9 taps of a 64-channel slice are
                   // consecutive K-tiles and a tile's halo rows stay in L2 across them
  A_CONV3_S2 = 2,  // 3x3, stride 2, pad 1 (Downsample, unet.py:82-108)
  A_CONV3_UP = 3,  // 3x3 over the nearest-x2-upsampled input (Upsample, unet.py:51-79)
  A_CONV3_SMALLC = 4,  // 3x3 stride 1 for C % 64 != 0 (first convs: 4 / 8 input channels), k = tap*C + c
};

// GroupNorm statistics of a GEMM's output, accumulated in its epilogue for the GroupNorm that will
// consume that tensor (unet.py:203-223 in_layers/out_layers, attention.py:343): per (batch, group)
// running sums (sum x, sum x^2) in fp64, kept in 8 replicas (block id % 8) to spread the atomics.
// The consumer normalises channel c of the GEMM's output column n as channel c_off + n of a
// C-channel tensor split into G groups of cg = C / G channels.  Requires hw % BM == 0 (a tile never
// straddles two batch elements).
constexpr int STAT_REPL = 8;
struct StatTgt {
  double* acc;  // [STAT_REPL][rs] with index (b*G + g)*2 (+1 for sum x^2); null = no statistics
  int rs;       // replica stride (doubles)
  int cg, G;    // channels per group / groups of the consumer
  int c_off;    // channel offset of output column 0 in the consumer's channel space
  int hw;       // pixels per batch element
};

// out[m][n] = alpha * sum_k X[m][k] * W[n][k] + bias[n] + emb[row(b)][n] + res[m][n]
struct GemmArgs {
  int M, N, K;          // K = reduction length of the main operand (9*C for convs)
  int amode;
  // activation operand
  const bf16* A; int lda;   // NHWC input, row (pixel) stride in elements
  int C;                    // input channels (conv modes)
  int Bn, H, W;             // input batch / spatial size (conv modes)
  int Ho, Wo;               // output spatial size (conv modes)
  // fused 1x1 skip conv appended to K (ResBlock skip_connection, unet.py:182-189)
  const bf16* X; int ldx; int Kx;
  // weights, packed [N][ldw] bf16, K-contiguous (ldw >= K + Kx, multiple of 64)
  const bf16* Wt; int ldw;
  // epilogue: v = alpha*acc + (scale_bias ? alpha : 1)*bias + emb + res; v = act(v)
  float alpha;
  int scale_bias;                             // ControlNet zero-conv: (W h + b) * control_scale
  int act;                                    // 0 none, 1 SiLU, 2 GEGLU pairs (see epilogue4)
  const float* bias;                          // [N] or null
  const float* emb; int ld_emb; const int* emb_row;  // + emb[emb_row[b]*ld_emb + n], b = m / (Ho*Wo)
  int rows_per_b;                             // pixels per batch element for emb indexing
  const bf16* res; int ld_res;                // + res[m*ld_res + n] (may alias out)
  void* out; int ldo; int out_f32;            // out[m*ldo + n]
  // split-K (fp32 partial slabs [splits][M][N] then a reduce+epilogue pass)
  int splits; float* partial; size_t partial_cap;
  int force_bm, force_bn, force_splits;       // test overrides (0 = heuristic)
  int force_stages;                           // 4: the 4-phase 256-row kernel; 2: 2-stage 64-row tiles (dense)
  // Split-K arrival tickets (zeroed, self-resetting), one per output tile; null = slabs always summed
  // by splitk_reduce_kernel.  With tickets, plans of at most ink_smax() slices combine in-kernel: each
  // slice stores its accumulators write-through, the last to arrive adds the others' and runs the
  // epilogue (gemm_kern.h splitk_combine).
  int* tile_sem; int sem_cap;
  StatTgt st[2];  // GroupNorm statistics of the output for up to two consumers (bf16 outputs only)
  // Split-precision ("3-plane") operands of the fp32-accurate VAE decoder: a value x is held as
  // hi = bf16(x), lo = bf16(x - hi) in three bf16 planes of width P along the channel axis, in
  // "activation" order (hi, lo, hi) or "weight" order (hi, hi, lo), so one bf16 GEMM over 3K gives
  // hi*hi + lo*hi + hi*lo (the product to ~2^-16 relative).
  int out_split;  // 0: plain; 1: write activation order (hi, lo, hi); 2: weight order (hi, hi, lo);
                  // planes at columns n, n + N, n + 2N of row m (ldo >= 3N)
  int res_lo;     // > 0: the residual is split, res = res[m*ld_res + n] + res[m*ld_res + res_lo + n]
  // Two-plane ("hi + lo") storage of the UNet / ControlNet residual stream: a bf16
  // output with out_lo > 0 also writes its rounding residual lo = bf16(v - bf16(v)) at element
  // offset out_lo (a second plane of the same layout), so consumers that read hi + lo see v to ~2^-16.
  int out_lo;
  // x_wrap > 0: the K-extension reads X channel (k - K) mod x_wrap, i.e. Kx = 2 * x_wrap runs the same
  // activation against weight columns [W_hi | W_lo] (the ResBlock skip conv at fp32-accurate weights)
  int x_wrap;
  // host-only: the activation operand carries `kplanes` split planes of the logical channels
  // (3 = hi/lo/hi for an fp32-accurate conv); FLOP counting divides K by it (0 or 1 = plain)
  int kplanes;
  int flop_k;   // host-only: the logical reduction length for FLOP counting when K carries padding (0 = K / kplanes)
  // measurement probes (tools/gemm_probe.py; 0 in the product): bit 0 skips the epilogue's output
  // stores (values kept live), bit 1 skips the whole epilogue; bit 2 (host) combines K slices in-kernel
  // at any split count when tile_sem is given (tests of the in-kernel combine beyond ink_smax); bits 3-5
  // select conv_halo_kernel ablation variants of the 256x160 tiles (timing only: no weight DMA / no MFMA /
  // no loop barrier; tools/conv_probe.py --ablate); bit 7 keeps the wide tiles on the LDS-staged epilogue
  // (TAIR_EPI_REG=0 A/B measurements; gemm_kern.h epilogue_regstage)
  int probe;
  // fp8 operands (configs[4]): A and Wt hold OCP e4m3 bytes, K-major; M/N as usual, while K, lda and
  // ldw count PAIRS of bytes (the bf16 loader moves the same 128-byte K-tile rows: one K-tile = 128
  // fp8 values = one v_mfma_scale_f32_16x16x128_f8f6f4 per fragment pair, 2x the bf16 MFMA rate).
  // Dense mode only, no K-extension.  The epilogue dequantises: acc * row_scale[m] * col_scale[n].
  int f8;
  const float* row_scale;  // per output row (token) or null
  const float* col_scale;  // per output column (channel) or null
  // LayerNorm folded into its consuming linear (attention.py:265-274 norm1/2/3 -> to_qkv / to_q / GEGLU
  // proj).  Producer: rst != null accumulates per output row the fp64 (sum, sum of
  // squares) of the stored (bf16-rounded) values into rst[2m], rst[2m + 1] -- the LayerNorm statistics
  // of the tensor it writes.  Consumer: the GEMM runs on the raw LayerNorm input against
  // W' = W diag(gamma), and the epilogue first forms v = rstd_m (acc - mean_m lncs[n]) with mean / rstd
  // from lnst (C = ln_c, eps ln_eps) and lncs[n] = sum_k W'[n][k]; bias' = bias + W beta.
  double* rst;
  const double* lnst; const float* lncs; float ln_c; float ln_eps;
  // A_CONV3_S2 input row/col offset: 0 = symmetric pad 1 (UNet Downsample), 1 = pad (0, 1, 0, 1) then
  // pad 0 (the SD VAE encoder's Downsample, vae.py:85-105): input pixel 2 yo + ky - 1 + s2_shift
  int s2_shift;
  // GroupNorm(+SiLU) applied to the activation operand as it is loaded (unet.py:203-223 in_layers /
  // out_layers, attention.py:305 norm -> proj_in): gn_st != null replaces A by y = bf16(act(A sc + sh)),
  // sc = gamma rstd, sh = beta - mean sc per (batch element, channel), mean / rstd of the producer's
  // fp64 statistics (StatTgt layout: STAT_REPL replicas gn_rs doubles apart, (b * gn_G + g) * 2) over
  // rows_per_b pixels; conv padding taps stay zero, the K-extension is not normalised.  For a one-plane
  // input, bitwise the separate gn_apply_kernel + GEMM; a residual-stream (hi + lo) input is read as its
  // hi plane alone, which differs from the apply's hi + lo (v rel-L2 2.44e-3 -> 2.47e-3).
  const double* gn_st; int gn_rs; int gn_G; float gn_eps; const float* gn_gamma; const float* gn_beta;
  int gn_silu;
  int halo_s2;  // halo tiles: the 2-stage weight ring variant
  int tile_stages;  // (launcher-set) ring depth of a GEMM_KERN_DEEP plan: 4, 5, 6 or 8 K-tiles
  // (launcher-set) cooperative split-K combine (gemm_kern.h splitk_coop): the K slices of a tile run on
  // consecutive workgroups, each stores its slab, waits for the tile's other slices and sums and finishes
  // 1/splits of the tile's rows (no reduce launch, no single-workgroup combine)
  int coop;
  int sem_stride;  // (launcher-set) ints between two tiles' tickets: 32 (one 128-byte line each) where they fit
  unsigned long long* stamps;  // measurement builds only (TAIR_STAMPS): per-workgroup phase stamps, [block][8]
};

// Grouped launch: up to MAX_GROUP independent GEMMs of identical shape / mode / epilogue kind
// (e.g. a UNet encoder layer and the same ControlNet layer) in ONE kernel launch; block x
// coordinate = group * tiles_m + m-tile.
constexpr int MAX_GROUP = 2;
struct GemmGroup {
  GemmArgs g[MAX_GROUP];
  int tiles_m;
  int xcd;  // XCD-aware block order: 1 m-tiles fastest, 2 n-tiles fastest; 3 / 4: K slices fastest, then
            // m / n (cooperative split-K: a tile's slices on consecutive workgroups of one XCD; gemm_kern.h xcd_remap)
  int* fault;  // device fault counter (gemm_fault_count): a cooperative split-K wait that timed out adds 1
};


// tiles the GEMM launcher accepts (the planner and the tests pick from these)
inline bool gemm_tile_built(int amode, int bm, int bn) {
  if (amode == A_CONV3_SMALLC) return bm == 64 && (bn == 64 || bn == 128);
  const bool small = (bm == 64 || bm == 128) && (bn == 64 || bn == 128);
  const bool big = (bm == 128 && (bn == 256 || bn == 320)) ||
                   (bm == 256 && (bn == 128 || bn == 160 || bn == 256 || bn == 320));
  return small || big;
}
inline bool gemm_tile_is_big(int bm, int bn) { return bn > 128 || bm > 128; }
// gemm_tile_kernel's software-pipelined main loop (and GroupNorm on load): 8-wave tiles and the 2-stage
// shallow tiles (the 4-wave 3-stage B = 1 tiles keep the plain loop)
constexpr bool gemm_tile_pipe(int waves, int stages) { return waves == 8 || stages == 2; }
// BK = 32 deep-ring tiles (gemm_ring_kernel), requested as force_bm = -bm
inline bool gemm_ring_built(int bm, int bn) {
  return (bm == 128 && (bn == 320 || bn == 256 || bn == 128)) || (bm == 256 && (bn == 256 || bn == 128)) ||
         (bm == 64 && (bn == 128 || bn == 64));
}

hipError_t gemm(const GemmArgs& a, hipStream_t s);
void gemm_set_skip_reduce(bool on);  // timing-only ablation: no split-K reduce launches
constexpr int GEMM_TICKETS = 16384;  // split-K tickets per scratch lane (tiles of one GEMM)
constexpr int ATTN_TICKETS = 16384;  // attention key-split tickets per scratch lane (one 128-byte line per block)
hipError_t gemm_grouped(const GemmArgs* a, int n, hipStream_t s);  // n <= MAX_GROUP, same shapes
bool gemm_gn_ok(const GemmArgs& a);  // a GroupNorm-on-load plan exists for a (validation only, no launch)
// the plan gemm_grouped would launch for a (validation only, touches no device)
hipError_t gemm_plan_query(const GemmArgs& a, int* bm, int* bn, int* splits, int* kern);
hipError_t gemm_init();  // one-time kernel attribute setup (call outside stream capture)
// Faults the GEMM kernels detected since the last call (a cooperative split-K slice that gave up waiting for
// its tile's other slices and therefore summed incomplete slabs); reset = true clears the counter.  Host
// synchronous (reads one device int): call outside stream capture, after the work has been synchronised.
hipError_t gemm_fault_count(int* count, bool reset);
// Choose tile / split heuristics for (M, N, K); exposed for tests / the planner.  kern (optional):
// which kernel runs the tile (GEMM_KERN_TILE: the LDS-DMA tile kernels, ring tiles as bm < 0;
// GEMM_KERN_PHASE: the 4-phase 256-row kernel, force_stages == 4 forces it; GEMM_KERN_SHALLOW:
// 2-stage 64-row tiles of the dense mode, force_stages == 2 forces it)
constexpr int GEMM_KERN_TILE = 0, GEMM_KERN_PHASE = 1, GEMM_KERN_SHALLOW = 2;  // SHALLOW: 2-stage 64-row tiles (dense)
// HALO: conv_halo_kernel (stride-1 3x3 convs, 256-pixel halo tiles, image width 16 / 32 / 64; force_stages 9
// forces it); TAIR_HALO=0 keeps every conv on gemm_tile_kernel
constexpr int GEMM_KERN_HALO = 3;
// DEEP: the 64-row tile kernel with a 4-8 deep LDS ring (B = 1 grids, gemm_grouped picks the depth so the grid
// keeps its number of rounds over the CUs); force_stages 100 + S forces depth S
constexpr int GEMM_KERN_DEEP = 4;
bool conv_halo_ok(const GemmArgs& a);
void gemm_plan(const GemmArgs& a, int* bm, int* bn, int* splits, int* kern = nullptr);
size_t gemm_partial_elems(const GemmArgs& a);
// whether a GEMM's plan can produce LayerNorm row statistics (GemmArgs.rst): tile kernels with at
// most 128-row tiles (the statistics live in the epilogue's 2 KiB reduction area)
bool gemm_rowstats_ok(const GemmArgs& a);

// ---- normalisation ----------------------------------------------------------------------
// GroupNorm statistics -> per-(b, channel) scale/shift:  y = x*scale + shift
hipError_t groupnorm_scale_shift(const bf16* x, int ldx, int B, int HW, int C, int G, float eps,
                                 const float* gamma, const float* beta, float* scale_shift,
                                 float* ws, hipStream_t s, int* tickets = nullptr);
// tickets: B*G zeroed ints (left zeroed) -> stats and finalize in one launch; null -> two launches
// grouped forms: up to MAX_GROUP same-shape instances (own tensors / parameters) per launch
struct GnArgs {
  const bf16* x; int ldx;
  const float* gamma; const float* beta;
  float* ss;          // [B][C][2] scale / shift
  float* ws;          // [B*G*64*2] partial sums
  int* tickets;       // [B*G] zeroed ints (fused finalize) or null
  bf16* y; int ldy;   // apply output
  // apply from producer statistics (StatTgt layout) instead of ss: scale/shift finalised in-kernel
  const double* st; int st_rs; float eps;
  // split-precision I/O (VAE): x_lo > 0 -> x = x[c] + x[x_lo + c]; y_split -> y written as the 3
  // planes (hi, lo, hi) at y + c, y + C + c, y + 2C + c
  int x_lo; int y_split;
  // e4m3 output for an fp8 consumer (y unused): y8[row][c] = e4m3(bf16(y) * inv8[c]) (inv8 = 1 / the static
  // per-channel power-of-two activation scale), row stride ld8 bytes, bytes C..ld8 zeroed
  uint8_t* y8 = nullptr; int ld8 = 0; const float* inv8 = nullptr;
};
struct GnGroup { GnArgs g[MAX_GROUP]; };
hipError_t groupnorm_stats_grouped(const GnArgs* a, int n, int B, int HW, int C, int G, float eps,
                                   hipStream_t s);
hipError_t groupnorm_apply_grouped(const GnArgs* a, int n, int B, int HW, int C, int silu, hipStream_t s,
                                   int G = 32);
// row softmax of fp32 scores S [rows][L] (row stride lds) -> P in 3 split planes (hi, lo, hi) [rows][3L]
hipError_t softmax_split(const float* S, int lds, int rows, int L, bf16* P, hipStream_t s);
// [B][L][3C] activation-order planes -> [B][C][3L] weight-order planes (hi, hi, lo): V -> V^T operand
hipError_t transpose_split(const bf16* x, int B, int L, int C, bf16* y, hipStream_t s);
// y8 != null: the output goes out as OCP e4m3 instead (the fp8 linears' activation operand, configs[4]):
// y8[t][c] = e4m3(y[t][c] / s8[t]) with s8[t] = max_c |y[t][c]| / 448 (1 for an all-zero row), bytes
// C..ld8 of the row zeroed (the GEMM's 128-value K-tiles); y may then be null
struct LnArgs {
  const bf16* x; const float* gamma; const float* beta; bf16* y;
  uint8_t* y8 = nullptr; float* s8 = nullptr; int ld8 = 0;
};
struct LnGroup { LnArgs g[MAX_GROUP]; };
hipError_t layernorm_grouped(const LnArgs* a, int n, int T, int C, float eps, hipStream_t s);
// y = act(x*scale + shift), act = SiLU or identity; NHWC bf16 in/out
hipError_t groupnorm_apply(const bf16* x, int ldx, int B, int HW, int C, const float* scale_shift,
                           int silu, bf16* y, int ldy, hipStream_t s);
// LayerNorm over the channel dim of [T, C] tokens (eps 1e-5)
hipError_t layernorm(const bf16* x, int T, int C, const float* gamma, const float* beta, float eps,
                     bf16* y, hipStream_t s);

// Per-row e4m3 quantisation of a packed bf16 weight [rows][ldw] (first K columns): q[r][k] =
// e4m3(w[r][k] / scale[r]), scale[r] = max_k |w[r][k]| / 448 (1 for a zero row), q's bytes K..ldq zeroed
hipError_t quant_rows_fp8(const bf16* w, int rows, int K, int ldw, uint8_t* q, int ldq, float* scale, hipStream_t s);
// fp8 weights of a consumer with static activation scales a[k] (per K column; null = 1): q[r][k] =
// e4m3(w[r][k] a[k] / s[r]) for k < K (zeros to k8), s[r] a power of two >= max |w a| / 448; the Kx bf16
// columns of a K-extension follow as bf16(w[r][K + j] / s[r]) at byte k8 + 2j (rows of ldq bytes)
hipError_t quant_rows_fp8_ex(const bf16* w, int rows, int K, int Kx, int ldw, const float* a, uint8_t* q, int ldq,
                             int k8, float* scale, hipStream_t s);

// ---- attention ---------------------------------------------------------------------------
// O[b, i, h*64:(h+1)*64] = softmax(Q K^T * scale) V for every (b, h); d = 64.
// ws (optional, ws_bytes) holds the per-KV-split partials; without it the keys are not split.
struct AttnPlan {
  int qsets = 1;     // 16-query sets per wave (workgroup = 64 * qsets queries)
  int splits = 1;    // KV splits (blockIdx.z)
  int kv_split = 0;  // keys per split (multiple of 64)
};
AttnPlan attention_plan(int B, int H, int Sq, int Skv, size_t ws_bytes, int force_qsets = 0,
                        int force_splits = 0);
struct AttnArgs {
  const bf16* q; int ldq;
  const bf16* k; int ldk;
  const bf16* v; int ldv;
  bf16* o; int ldo;
  int kv_bstride;
  void* ws; size_t ws_bytes;  // key-split partials (null: keys not split)
  // arrival tickets of the key-split partials (zeroed, self-resetting; null: attn_combine_kernel merges them):
  // the last split of a (query block, head) to arrive merges the others in-kernel (attention.hip)
  int* tickets; int tickets_cap;
};
struct AttnGroup { AttnArgs g[MAX_GROUP]; };
hipError_t attention_grouped(const AttnArgs* a, int n, int B, int H, int Sq, int Skv, float scale, hipStream_t s,
                             int force_qsets = 0, int force_splits = 0);
hipError_t attention(const bf16* q, int ldq, const bf16* k, int ldk, const bf16* v, int ldv,
                     bf16* o, int ldo, int B, int H, int Sq, int Skv, int kv_bstride,
                     float scale, hipStream_t s, void* ws = nullptr, size_t ws_bytes = 0,
                     int force_qsets = 0, int force_splits = 0);

// ---- misc ---------------------------------------------------------------------------------
hipError_t geglu(const bf16* xg, int T, int D, bf16* y, hipStream_t s);
hipError_t timestep_sinusoid(const int64_t* t, int n, int dim, float* out, hipStream_t s);
hipError_t silu_f32(const float* x, int n, float* y, hipStream_t s);
hipError_t f32_to_bf16(const float* x, int n, bf16* y, hipStream_t s);
hipError_t zero_bytes(void* p, size_t bytes, hipStream_t s);  // bytes % 16 == 0
// NCHW fp32 [B, C, H, W] -> NHWC bf16 rows with stride ldy at channel offset c_off
hipError_t nchw_f32_to_nhwc_bf16(const float* x, int B, int C, int HW, bf16* y, int ldy, int c_off,
                                 hipStream_t s);
// NHWC bf16 (row stride ldx) -> NCHW fp32
hipError_t nhwc_bf16_to_nchw_f32(const bf16* x, int ldx, int B, int C, int HW, float* y, hipStream_t s);
// NHWC fp32 [B*HW, C] -> NCHW fp32
hipError_t nhwc_f32_to_nchw_f32(const float* x, int B, int C, int HW, float* y, hipStream_t s);
// Overlap-blend stitch of N decoded tiles [N][C][P][P] fp32 (raster grid nh x nw, stride) into
// out [C][H][W] (cropped), bitwise the reference's merge loop (val_patches.py:114-206); rtab =
// fp32((i+1)/overlap) for i < overlap (device)
hipError_t merge_overlap(const float* tiles, int n_tiles, int nh, int nw, int patch, int overlap, int stride,
                         float* out, int C, int H, int W, const float* rtab, hipStream_t s);
// configs[3] stitch fused with the tile exchange: src[r] = rank r's block of per_rank tiles (IPC-mapped
// peer memory), out [n_images][C][H][W] = global images first_image .. first_image + n_images - 1; mode 0
// non-overlap placement, 1 overlap blend (bitwise merge_overlap)
hipError_t stitch_peers(const float* const* src, int per_rank, int first_image, int n_images, int tiles_per_image,
                        int nh, int nw,
                        int mode, int patch, int overlap, int stride, float* out, int C, int H, int W,
                        const float* rtab, hipStream_t s);
// v-parameterised ancestral step (spaced_sampler.py:141-189), tables indexed on device
hipError_t sampler_step_v(const float* x, const float* v, const float* noise, const float* tabs,
                          const int* step_idx, int n, float* x_out, hipStream_t s);

// Multi-scale deformable attention sampling (TESTR, msda.hip): level shapes by value (capturable)
constexpr int MSDA_MAX_LEVELS = 8;
struct MsdaArgs {
  int N, S, M, D, L, P, Q;
  int h[MSDA_MAX_LEVELS], w[MSDA_MAX_LEVELS], start[MSDA_MAX_LEVELS];
};
hipError_t ms_deform_attn(const MsdaArgs& a, const float* value, const float* loc, const float* attn, float* out,
                          hipStream_t s);

}  // namespace tair
