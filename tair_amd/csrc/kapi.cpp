// Kernel-level C ABI (include/tair_kernels.h): thin, allocation-free wrappers over the launchers.
#include <cstring>
#include "kernels.h"
#include "tair_kernels.h"

using namespace tair;

extern "C" {

namespace {
GemmArgs gemm_args_of(const tair_gemm_desc* d) {
  GemmArgs a{};
  a.M = d->M; a.N = d->N; a.K = d->K; a.amode = d->amode;
  a.A = (const bf16*)d->A; a.lda = d->lda; a.C = d->C;
  a.Bn = d->Bn; a.H = d->H; a.W = d->W; a.Ho = d->Ho; a.Wo = d->Wo;
  a.X = (const bf16*)d->X; a.ldx = d->ldx; a.Kx = d->Kx;
  a.Wt = (const bf16*)d->Wt; a.ldw = d->ldw;
  a.alpha = d->alpha; a.scale_bias = d->scale_bias; a.act = d->act;
  a.bias = d->bias;
  a.emb = d->emb; a.ld_emb = d->ld_emb; a.emb_row = d->emb_row; a.rows_per_b = d->rows_per_b > 0 ? d->rows_per_b : 1;
  a.res = (const bf16*)d->res; a.ld_res = d->ld_res;
  a.out = d->out; a.ldo = d->ldo; a.out_f32 = d->out_f32;
  a.splits = 1; a.partial = d->partial; a.partial_cap = (size_t)d->partial_cap;
  a.force_bm = d->force_bm; a.force_bn = d->force_bn; a.force_splits = d->force_splits;
  a.force_stages = d->force_stages;
  a.tile_sem = d->tile_sem; a.sem_cap = d->sem_cap;
  a.out_split = d->out_split; a.res_lo = d->res_lo;
  a.out_lo = d->out_lo; a.x_wrap = d->x_wrap; a.probe = d->probe;
  a.f8 = d->f8; a.row_scale = d->row_scale; a.col_scale = d->col_scale;
  a.s2_shift = d->s2_shift;
  a.gn_st = d->gn_st;
  a.gn_rs = d->gn_rs;
  a.gn_G = d->gn_G;
  a.gn_eps = d->gn_eps;
  a.gn_gamma = d->gn_gamma;
  a.gn_beta = d->gn_beta;
  a.gn_silu = d->gn_silu;
  a.stamps = d->stamps;
  a.rst = d->rst; a.lnst = d->lnst; a.lncs = d->lncs; a.ln_c = d->ln_c; a.ln_eps = d->ln_eps;
  if (d->st_acc) {
    a.st[0].acc = d->st_acc; a.st[0].rs = d->st_rs; a.st[0].cg = d->st_cg; a.st[0].G = d->st_G;
    a.st[0].c_off = d->st_coff; a.st[0].hw = d->st_hw;
  }
  return a;
}
}  // namespace

int tair_k_gemm(const tair_gemm_desc* d, void* stream) {
  if (!d) return -1;
  const GemmArgs a = gemm_args_of(d);
  return gemm(a, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

int tair_fault_count(int reset, int* count) {
  if (!count) return -1;
  return gemm_fault_count(count, reset != 0) == hipSuccess ? 0 : -2;
}

int tair_k_gemm_desc_bytes(void) { return (int)sizeof(tair_gemm_desc); }

int tair_k_gemm_plan(const tair_gemm_desc* d, int* bm, int* bn, int* splits, int* kern) {
  if (!d || !bm || !bn || !splits || !kern) return -1;
  const GemmArgs a = gemm_args_of(d);
  return gemm_plan_query(a, bm, bn, splits, kern) == hipSuccess ? 0 : -2;
}

int tair_k_attention_plan(int B, int H, int Sq, int Skv, int64_t ws_bytes, int* qsets, int* splits, int* kv_split) {
  if (!qsets || !splits || !kv_split || B < 1 || H < 1 || Sq < 1 || Skv < 1) return -1;
  const AttnPlan p = attention_plan(B, H, Sq, Skv, ws_bytes < 0 ? (size_t)-1 : (size_t)ws_bytes);
  *qsets = p.qsets;
  *splits = p.splits;
  *kv_split = p.kv_split;
  return 0;
}

int tair_k_attention(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                     int B, int H, int Sq, int Skv, int kv_bstride, float scale, void* stream) {
  return attention((const bf16*)q, ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (bf16*)o, ldo, B, H, Sq, Skv,
                   kv_bstride, scale, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

int tair_k_attention_ex(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                        int B, int H, int Sq, int Skv, int kv_bstride, float scale, void* ws, int64_t ws_bytes,
                        int force_qsets, int force_splits, void* stream) {
  return attention((const bf16*)q, ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (bf16*)o, ldo, B, H, Sq, Skv,
                   kv_bstride, scale, (hipStream_t)stream, ws, ws ? (size_t)ws_bytes : 0, force_qsets,
                   force_splits) == hipSuccess ? 0 : -2;
}

int tair_k_attention_tk(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                        int B, int H, int Sq, int Skv, int kv_bstride, float scale, void* ws, int64_t ws_bytes,
                        int* tickets, int tickets_cap, int force_qsets, int force_splits, void* stream) {
  AttnArgs a{(const bf16*)q, ldq, (const bf16*)k, ldk, (const bf16*)v, ldv, (bf16*)o, ldo, kv_bstride, ws,
             ws ? (size_t)ws_bytes : 0, tickets, tickets_cap};
  return attention_grouped(&a, 1, B, H, Sq, Skv, scale, (hipStream_t)stream, force_qsets, force_splits) ==
                 hipSuccess ? 0 : -2;
}

int tair_k_groupnorm(const void* x, int ldx, int B, int HW, int C, int G, float eps, const float* gamma,
                     const float* beta, int silu, void* y, int ldy, float* ss, float* ws, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (groupnorm_scale_shift((const bf16*)x, ldx, B, HW, C, G, eps, gamma, beta, ss, ws, s) != hipSuccess) return -2;
  return groupnorm_apply((const bf16*)x, ldx, B, HW, C, ss, silu, (bf16*)y, ldy, s) == hipSuccess ? 0 : -2;
}

int tair_k_groupnorm_ex(const void* x, int ldx, int B, int HW, int C, int G, float eps, const float* gamma,
                        const float* beta, int silu, void* y, int ldy, float* ss, float* ws, int* tickets,
                        void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (groupnorm_scale_shift((const bf16*)x, ldx, B, HW, C, G, eps, gamma, beta, ss, ws, s, tickets) != hipSuccess)
    return -2;
  return groupnorm_apply((const bf16*)x, ldx, B, HW, C, ss, silu, (bf16*)y, ldy, s) == hipSuccess ? 0 : -2;
}

int tair_k_layernorm(const void* x, int T, int C, const float* gamma, const float* beta, float eps, void* y,
                     void* stream) {
  return layernorm((const bf16*)x, T, C, gamma, beta, eps, (bf16*)y, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

int tair_k_layernorm_fp8(const void* x, int T, int C, const float* gamma, const float* beta, float eps, void* y8,
                         int ld8, float* s8, void* stream) {
  LnArgs a{(const bf16*)x, gamma, beta, nullptr, (uint8_t*)y8, s8, ld8};
  return layernorm_grouped(&a, 1, T, C, eps, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

int tair_k_quant_rows_fp8(const void* w, int rows, int K, int ldw, void* q, int ldq, float* scale, void* stream) {
  return quant_rows_fp8((const bf16*)w, rows, K, ldw, (uint8_t*)q, ldq, scale, (hipStream_t)stream) == hipSuccess
             ? 0 : -2;
}

int tair_k_quant_rows_fp8_ex(const void* w, int rows, int K, int Kx, int ldw, const float* a, void* q, int ldq, int k8,
                             float* scale, void* stream) {
  return quant_rows_fp8_ex((const bf16*)w, rows, K, Kx, ldw, a, (uint8_t*)q, ldq, k8, scale, (hipStream_t)stream) ==
                 hipSuccess ? 0 : -2;
}

int tair_k_gn_apply_fp8(const void* x, int ldx, int x_lo, int B, int HW, int C, int G, float eps, const float* gamma,
                        const float* beta, int silu, const double* st, int st_rs, const float* inv8, void* y8, int ld8,
                        void* stream) {
  GnArgs g{};
  g.x = (const bf16*)x; g.ldx = ldx; g.gamma = gamma; g.beta = beta;
  g.st = st; g.st_rs = st_rs; g.eps = eps; g.x_lo = x_lo;
  g.y8 = (uint8_t*)y8; g.ld8 = ld8; g.inv8 = inv8;
  return groupnorm_apply_grouped(&g, 1, B, HW, C, silu, (hipStream_t)stream, G) == hipSuccess ? 0 : -2;
}

int tair_k_geglu(const void* xg, int T, int D, void* y, void* stream) {
  return geglu((const bf16*)xg, T, D, (bf16*)y, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

int tair_k_merge_overlap(const float* tiles, int n_tiles, int nh, int nw, int patch, int overlap, int stride,
                         float* out, int C, int H, int W, const float* rtab, void* stream) {
  return merge_overlap(tiles, n_tiles, nh, nw, patch, overlap, stride, out, C, H, W, rtab, (hipStream_t)stream) ==
                 hipSuccess ? 0 : -2;
}

int tair_k_stitch_peers(const void* src_ptrs, int per_rank, int first_image, int n_images, int tiles_per_image,
                        int nh, int nw,
                        int mode, int patch, int overlap, int stride, float* out, int C, int H, int W,
                        const float* rtab, void* stream) {
  return stitch_peers((const float* const*)src_ptrs, per_rank, first_image, n_images, tiles_per_image, nh, nw, mode, patch, overlap,
                      stride, out, C, H, W, rtab, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

// IPC export / import of a device buffer (the peer-read stitch): the handle names the whole allocation,
// so the exporter also reports the buffer's byte offset inside it
int tair_ipc_get_handle(const void* dev_ptr, void* handle_out, unsigned long long* offset) {
  if (!dev_ptr || !handle_out || !offset) {
    set_error("ipc_get_handle: null argument");
    return -1;
  }
  void* base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange((hipDeviceptr_t*)&base, &size, (hipDeviceptr_t)dev_ptr);
  if (e != hipSuccess) {
    set_error("ipc_get_handle: hipMemGetAddressRange: %s", hipGetErrorString(e));
    return -2;
  }
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, base);
  if (e != hipSuccess) {
    set_error("ipc_get_handle: hipIpcGetMemHandle: %s", hipGetErrorString(e));
    return -2;
  }
  static_assert(sizeof(hipIpcMemHandle_t) <= TAIR_IPC_HANDLE_BYTES, "IPC handle size");
  std::memset(handle_out, 0, TAIR_IPC_HANDLE_BYTES);
  std::memcpy(handle_out, &h, sizeof(h));
  *offset = (unsigned long long)((const char*)dev_ptr - (const char*)base);
  return 0;
}

int tair_ipc_open(const void* handle, void** dev_ptr) {
  if (!handle || !dev_ptr) {
    set_error("ipc_open: null argument");
    return -1;
  }
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  hipError_t e = hipIpcOpenMemHandle(dev_ptr, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    set_error("ipc_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
    return -2;
  }
  return 0;
}

int tair_ipc_close(void* dev_ptr) {
  hipError_t e = hipIpcCloseMemHandle(dev_ptr);
  if (e != hipSuccess) {
    set_error("ipc_close: hipIpcCloseMemHandle: %s", hipGetErrorString(e));
    return -2;
  }
  return 0;
}

int tair_k_gn_apply_stats(const void* x, int ldx, int x_lo, int B, int HW, int C, int G, float eps, const float* gamma,
                          const float* beta, int silu, const double* st, int st_rs, void* y, int ldy, int y_split,
                          void* stream) {
  GnArgs g{};
  g.x = (const bf16*)x; g.ldx = ldx; g.gamma = gamma; g.beta = beta; g.y = (bf16*)y; g.ldy = ldy;
  g.st = st; g.st_rs = st_rs; g.eps = eps; g.x_lo = x_lo; g.y_split = y_split;
  return groupnorm_apply_grouped(&g, 1, B, HW, C, silu, (hipStream_t)stream, G) == hipSuccess ? 0 : -2;
}

int tair_k_softmax_split(const float* S, int lds, int rows, int L, void* P, void* stream) {
  return softmax_split(S, lds, rows, L, (bf16*)P, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

int tair_k_transpose_split(const void* x, int B, int L, int C, void* y, void* stream) {
  return transpose_split((const bf16*)x, B, L, C, (bf16*)y, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

int tair_k_ms_deform_attn(const float* value, int N, int S, int M, int D, const int* level_hw, int L, int Q, int P,
                          const float* loc, const float* attn, float* out, void* stream) {
  if (!level_hw || L < 1 || L > MSDA_MAX_LEVELS) {
    set_error("ms_deform_attn: %d levels (1..%d)", L, MSDA_MAX_LEVELS);
    return -1;
  }
  MsdaArgs a{};
  a.N = N; a.S = S; a.M = M; a.D = D; a.L = L; a.P = P; a.Q = Q;
  int start = 0;
  for (int l = 0; l < L; ++l) {
    a.h[l] = level_hw[2 * l];
    a.w[l] = level_hw[2 * l + 1];
    a.start[l] = start;
    start += a.h[l] * a.w[l];
  }
  return ms_deform_attn(a, value, loc, attn, out, (hipStream_t)stream) == hipSuccess ? 0 : -2;
}

}  // extern "C"
