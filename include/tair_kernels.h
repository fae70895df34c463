/* tair_kernels.h — kernel-level C ABI of libtair_cldm.so (test and integration hooks).
 *
 * These expose the individual gfx950 kernels the ControlLDM runtime is built from, on raw device
 * pointers in the runtime's native layouts (NHWC bf16 activations, [N][ldw] bf16 K-major weights),
 * so each one can be checked in isolation.  The reference has no equivalent FFI; each hook names
 * the reference op it computes.  All are asynchronous on `stream` and allocate nothing.
 */
#ifndef TAIR_KERNELS_H
#define TAIR_KERNELS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Activation operand modes of the MFMA GEMM. */
#define TAIR_A_DENSE 0
#define TAIR_A_CONV3 1
#define TAIR_A_CONV3_S2 2
#define TAIR_A_CONV3_UP 3
#define TAIR_A_CONV3_SMALLC 4

typedef struct {
  int M, N, K, amode;
  const void* A; int lda; int C; int Bn, H, W, Ho, Wo;
  const void* X; int ldx; int Kx;
  const void* Wt; int ldw;
  float alpha; int scale_bias; int act;
  const float* bias;
  const float* emb; int ld_emb; const int* emb_row; int rows_per_b;
  const void* res; int ld_res;
  void* out; int ldo; int out_f32;
  float* partial; int64_t partial_cap; /* split-K workspace (fp32 elements) or NULL */
  int force_bm, force_bn, force_splits;  /* 0 = heuristic */
  int force_stages;                      /* 4: the 4-phase 256-row kernel; 2: 2-stage 64-row dense tiles */
  int* tile_sem; int sem_cap;            /* split-K tickets (zeroed ints, one per output tile) or NULL:
                                            the last K-slice reduces in-kernel, else a reduce kernel */
  /* split-precision operands (the fp32-accurate VAE decoder): out_split 1 writes hi/lo/hi, 2 hi/hi/lo
   * bf16 planes at columns n, N+n, 2N+n (ldo >= 3N); res_lo > 0: residual = res[n] + res[res_lo + n] */
  int out_split; int res_lo;
  /* GroupNorm statistics of the output for the GroupNorm that consumes it (or st_acc = NULL):
   * fp64 (sum, sum^2) per (batch, group) in 8 replicas of st_rs doubles, groups of st_cg channels */
  double* st_acc; int st_rs, st_cg, st_G, st_coff, st_hw;
  /* two-plane residual-stream storage: out_lo > 0 also writes lo = bf16(v - bf16(v)) at element offset
   * out_lo; x_wrap > 0: the K-extension reads X channel (k - K) mod x_wrap (Kx = 2 x_wrap) */
  int out_lo; int x_wrap;
  int probe; /* measurement probes (0): bit 0 no epilogue stores, bit 1 no epilogue, bit 2 in-kernel split-K at any split count */
  /* f8 != 0: A and Wt hold OCP e4m3 bytes; K, lda, ldw count PAIRS of bytes (K % 64 == 0); dense
   * or stride-1 3x3 conv (A operand e4m3 [pixel][C] bytes, lda = row bytes / 2, K order as the bf16 conv
   * at one byte per value: a 128-value K-tile = two (64-channel chunk, tap) slots; an optional bf16
   * K-extension follows the fp8 K-tiles in each weight row); the epilogue first multiplies by
   * (row_scale ? row_scale[m] : 1) * col_scale[n] */
  int f8; const float* row_scale; const float* col_scale;
  /* stride-2 conv only: 1 = the SD VAE Downsample's padding (0, 1, 0, 1) then pad 0 (vae.py:85-105),
   * 0 = symmetric pad 1 (the UNet Downsample, unet.py:82-108) */
  int s2_shift;
  /* GroupNorm(+SiLU) applied to the activation as it is loaded (unet.py:203-223, attention.py:305; replaces a
   * separate apply pass): gn_st != NULL normalises A per (batch element, channel) with the producer's fp64
   * statistics (the st_acc layout: 8 replicas gn_rs doubles apart, (b * gn_G + g) * 2) over rows_per_b
   * pixels, gamma / beta [C], eps; gn_silu 1 adds SiLU.  Stride-1 conv (rows_per_b = H * W) or dense
   * (C = K); conv padding and the K-extension are not normalised.  Bitwise tair_k_gn_apply_stats + GEMM. */
  const double* gn_st; int gn_rs; int gn_G; float gn_eps; const float* gn_gamma; const float* gn_beta; int gn_silu;
  /* measurement only (a library built with -DTAIR_STAMPS=1; ignored otherwise): per workgroup 8 s_memrealtime
   * stamps (100 MHz) of the kernel's phases, [linear block id][8] u64; null = none */
  unsigned long long* stamps;
  /* LayerNorm folded into this linear (attention.py:265-274 norm1/2/3 -> to_qkv / to_q / GEGLU proj):
   * rst != NULL makes the producer accumulate per output row the fp64 (sum, sum of squares) of its stored bf16
   * values into rst[2m], rst[2m + 1]; lnst != NULL makes the consumer, run on the raw LayerNorm input against
   * W' = W diag(gamma), form v = rstd_m (acc - mean_m lncs[n]) + bias' with mean / rstd from lnst over
   * ln_c channels (eps ln_eps), lncs[n] = sum_k W'[n][k], bias' = bias + W beta. */
  double* rst; const double* lnst; const float* lncs; float ln_c; float ln_eps;
} tair_gemm_desc;

/* act: 0 none, 1 SiLU, 2 GEGLU — output channels packed as (x_2q, x_2q+1, gate_2q, gate_2q+1) groups,
 * y[:, 2q+i] = x_2q+i * gelu(gate_2q+i) written to out (N/2 bf16 columns).
 * nn.Linear / nn.Conv2d (3x3 pad 1, stride 1|2, nearest-x2 upsample fused) + bias + time-emb +
 * residual epilogue (unet.py:51-223, attention.py:19-353). */
int tair_k_gemm(const tair_gemm_desc* d, void* stream);
/* Faults the GEMM kernels detected on the current device since the last reset (a cooperative split-K slice
 * that gave up waiting for its tile's other slices, so its sums are incomplete): *count receives the number;
 * reset != 0 clears it.  Synchronous (reads one device int): call after the work is synchronised, outside
 * stream capture.  A non-zero count means the results of that work are invalid. */
int tair_fault_count(int reset, int* count);
/* sizeof(tair_gemm_desc) as compiled into the library (bindings check their struct mirror against it). */
int tair_k_gemm_desc_bytes(void);
/* The plan tair_k_gemm would launch for d, without launching (host only, no device needed): tile bm x bn
 * (bm < 0: the BK = 32 ring tiles), K splits, kernel (0 tile, 1 4-phase, 2 2-stage shallow, 3 halo conv).
 * Returns the validation status tair_k_gemm would report. */
int tair_k_gemm_plan(const tair_gemm_desc* d, int* bm, int* bn, int* splits, int* kern);
/* The plan tair_k_attention would launch (host only, no device needed): queries per wave / 16 (qsets),
 * key splits and keys per split, for a workspace of ws_bytes (< 0: unbounded). 0 on success. */
int tair_k_attention_plan(int B, int H, int Sq, int Skv, int64_t ws_bytes, int* qsets, int* splits, int* kv_split);
/* softmax(Q K^T * scale) V, head dim 64 (attention.py:168-216). */
int tair_k_attention(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                     int B, int H, int Sq, int Skv, int kv_bstride, float scale, void* stream);
/* Same, with a workspace for the key-split (flash-decoding) partials: per split B*Sq*H*136 bytes.
 * force_qsets (1|2 x 16 queries per wave) / force_splits override the heuristic (0 = heuristic). */
int tair_k_attention_ex(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                        int B, int H, int Sq, int Skv, int kv_bstride, float scale, void* ws, int64_t ws_bytes,
                        int force_qsets, int force_splits, void* stream);
/* Same, with arrival tickets (tickets_cap zeroed ints, left zeroed): the key splits of each (query block, head)
 * are merged in-kernel by the last split to arrive (bitwise the separate merge) when tickets_cap covers
 * 32 ints per block, otherwise by the merge kernel as above. */
int tair_k_attention_tk(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                        int B, int H, int Sq, int Skv, int kv_bstride, float scale, void* ws, int64_t ws_bytes,
                        int* tickets, int tickets_cap, int force_qsets, int force_splits, void* stream);
/* GroupNorm(G, eps) [+ SiLU] on NHWC bf16 (util.py:191-193, attention.py:48-51). ss: [B][C][2] fp32,
 * ws: [B*G*64*2] fp32 scratch. */
int tair_k_groupnorm(const void* x, int ldx, int B, int HW, int C, int G, float eps, const float* gamma,
                     const float* beta, int silu, void* y, int ldy, float* ss, float* ws, void* stream);
/* Same; tickets = B*G zeroed ints (left zeroed): the statistics pass also finalizes (one launch less). */
int tair_k_groupnorm_ex(const void* x, int ldx, int B, int HW, int C, int G, float eps, const float* gamma,
                        const float* beta, int silu, void* y, int ldy, float* ss, float* ws, int* tickets,
                        void* stream);
/* LayerNorm over C (attention.py:255-257). */
int tair_k_layernorm(const void* x, int T, int C, const float* gamma, const float* beta, float eps, void* y,
                     void* stream);
/* LayerNorm over C with e4m3 output for the fp8 linears (configs[4]): y8 [T][ld8] bytes (OCP e4m3,
 * bytes C..ld8 zeroed), s8 [T] per-token scale (max |y| / 448): y ~= y8 * s8. */
int tair_k_layernorm_fp8(const void* x, int T, int C, const float* gamma, const float* beta, float eps, void* y8,
                         int ld8, float* s8, void* stream);
/* Per-output-channel e4m3 quantisation of a bf16 weight [rows][ldw] (first K columns) into q [rows][ldq]
 * bytes (zero-padded) and scale [rows] = max |w| / 448. */
int tair_k_quant_rows_fp8(const void* w, int rows, int K, int ldw, void* q, int ldq, float* scale, void* stream);
/* fp8 weights of a GroupNorm-fed consumer (configs[4] ResBlock convs / proj_in, unet.py:203-223): q[r][k] =
 * e4m3(w[r][k] a[k] / s[r]) for k < K (zero to k8), s[r] = the power of two >= max |w a| / 448, a = the
 * static per-K-column activation scale (null = 1), then the Kx bf16 K-extension columns as w[r][K+j] / s[r]
 * at byte k8 + 2j; q rows of ldq bytes. */
int tair_k_quant_rows_fp8_ex(const void* w, int rows, int K, int Kx, int ldw, const float* a, void* q, int ldq, int k8,
                             float* scale, void* stream);
/* GroupNorm(+SiLU) apply from producer statistics with e4m3 output: y8[row][c] = e4m3(bf16(y) * inv8[c])
 * (inv8 = 1 / the consumer's static power-of-two activation scale), rows of ld8 bytes, C..ld8 zeroed. */
int tair_k_gn_apply_fp8(const void* x, int ldx, int x_lo, int B, int HW, int C, int G, float eps, const float* gamma,
                        const float* beta, int silu, const double* st, int st_rs, const float* inv8, void* y8, int ld8,
                        void* stream);
/* GEGLU: [T, 2D] -> x * gelu(gate) (attention.py:19-26). */
int tair_k_geglu(const void* xg, int T, int D, void* y, void* stream);

/* Overlap-blend stitch of decoded tiles on the device (val_patches.py:114-206 merge_patches_with_overlap,
 * stride generalised): tiles [n_tiles][C][patch][patch] fp32 on a raster nh x nw grid, out [C][H][W]
 * fp32 cropped; rtab[i] = fp32((i+1)/overlap), i < overlap (device).  Bitwise the reference loop. */
int tair_k_merge_overlap(const float* tiles, int n_tiles, int nh, int nw, int patch, int overlap, int stride,
                         float* out, int C, int H, int W, const float* rtab, void* stream);

/* configs[3] stitch fused with the tile exchange (replaces the all-gather + merge of
 * val_patches.py:114-206 / image_splitter.py:23-51 across ranks): src_ptrs = device array of `world`
 * pointers, rank r's contiguous block of per_rank tiles [C][patch][patch] fp32 (peer buffers mapped by
 * tair_ipc_open); the image-major global tile list g -> (g / per_rank, g % per_rank).  out
 * [n_images][C][H][W] fp32 = the global images first_image .. first_image + n_images - 1 (a rank stitches
 * the images it owns, reading only the tiles that cover them).  mode 0: non-overlap placement (H = nh * patch); mode 1: overlap blend,
 * bitwise tair_k_merge_overlap (rtab as there). */
int tair_k_stitch_peers(const void* src_ptrs, int per_rank, int first_image, int n_images, int tiles_per_image,
                        int nh, int nw,
                        int mode, int patch, int overlap, int stride, float* out, int C, int H, int W,
                        const float* rtab, void* stream);
/* IPC export / import of a device buffer for peer reads: handle_out receives TAIR_IPC_HANDLE_BYTES
 * (the allocation's handle) and *offset the buffer's byte offset inside that allocation; tair_ipc_open
 * maps a peer's allocation (base pointer; add the exporter's offset), tair_ipc_close unmaps it. */
#define TAIR_IPC_HANDLE_BYTES 64
int tair_ipc_get_handle(const void* dev_ptr, void* handle_out, unsigned long long* offset);
int tair_ipc_open(const void* handle, void** dev_ptr);
int tair_ipc_close(void* dev_ptr);

/* GroupNorm(+SiLU) apply from producer statistics (a GEMM epilogue's st_acc; vae.py:18-21 eps 1e-6,
 * util.py:191-193): x_lo > 0 reads a split input x[c] + x[x_lo + c]; y_split writes hi/lo/hi planes. */
int tair_k_gn_apply_stats(const void* x, int ldx, int x_lo, int B, int HW, int C, int G, float eps, const float* gamma,
                          const float* beta, int silu, const double* st, int st_rs, void* y, int ldy, int y_split,
                          void* stream);
/* Row softmax of fp32 scores (rows x L, row stride lds) into hi/lo/hi bf16 planes [rows][3L]
 * (vae.py:120-180 AttnBlock, softmax over the keys). */
int tair_k_softmax_split(const float* S, int lds, int rows, int L, void* P, void* stream);
/* [B][L][3C] (hi, lo, hi) -> [B][C][3L] (hi, hi, lo): the V^T operand of P.V. */
int tair_k_transpose_split(const void* x, int B, int L, int C, void* y, void* stream);
/* Multi-scale deformable attention sampling of the stage-3 TESTR spotter, replacing the reference's
 * MSDeformAttnFunction / ms_deformable_im2col_gpu_kernel (testr/adet/layers/ms_deform_attn.py:19-37,
 * csrc/DeformAttn/ms_deform_im2col_cuda.cuh:238-299): fp32 value (N, S, M, D), level shapes
 * level_hw[2l] = H_l, [2l+1] = W_l (host array, L <= 8, levels consecutive along S), loc (N, Q, M, L, P, 2)
 * as (x, y) in [0, 1], attn (N, Q, M, L, P) -> out (N, Q, M*D).  grid_sample bilinear semantics
 * (align_corners = False, zero padding). */
int tair_k_ms_deform_attn(const float* value, int N, int S, int M, int D, const int* level_hw, int L, int Q, int P,
                          const float* loc, const float* attn, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TAIR_KERNELS_H */
