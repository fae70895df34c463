// MI355X-native ControlLDM runtime: builds the SD-2.1 UNet + ControlNet from the yaml
// hyper-parameters (unet.py:391-685, controlnet.py:61-337), owns packed bf16 weights and an
// HBM workspace sized at create, and runs the denoising forward as a straight line of HIP
// kernel launches on the caller's stream (no host sync, no allocation => hipGraph-capturable).
//
// Activation layout: NHWC bf16 rows.  The UNet skip stack is never materialised separately:
// encoder block i writes its output directly into the right-hand channels of the concat buffer of
// decoder block 11-i (torch.cat([h, hs.pop()+control.pop()]) in controlnet.py:50), the ControlNet
// zero-conv epilogue accumulates its control residual into the same columns in place, and each
// decoder block writes its output into the left-hand channels of the next concat buffer.
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "kernels.h"
#include "tair_cldm.h"

namespace tair {

static thread_local char g_err[2048] = "";

// Live handles: every entry point validates its handle against this set, so a stale handle (e.g. an
// integer kept by a caller of torch.ops.tair.cldm_forward after the model was destroyed) is an error
// status, never a use-after-free.
static std::mutex g_live_mu;
static std::set<const void*> g_live;
static void live_add(const void* h) {
  std::lock_guard<std::mutex> l(g_live_mu);
  g_live.insert(h);
}
static void live_remove(const void* h) {
  std::lock_guard<std::mutex> l(g_live_mu);
  g_live.erase(h);
}
static bool live(const void* h) {
  std::lock_guard<std::mutex> l(g_live_mu);
  return g_live.count(h) != 0;
}
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

static uint16_t f2bf_bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return 0x7fc0;  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf_bits2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ------------------------------------------------------------------------------------------
// parameters
// ------------------------------------------------------------------------------------------
struct Weight {          // packed [rows][ldw] bf16, K-contiguous
  bf16* p = nullptr;
  int rows = 0, ldw = 0;
  int K = 0;             // main reduction length (9*C for 3x3 convs, padded for small C)
  int Kx = 0;            // fused skip-conv extension
  // fp8 twin (compute_dtype TAIR_DTYPE_FP8): per-output-channel e4m3 [rows][ld8] bytes, K zero-padded to
  // the 128-value K-tile, and its scales; quantised from the packed bf16 weight at finalize
  uint8_t* p8 = nullptr;
  float* s8 = nullptr;
  int ld8 = 0;
  // GroupNorm-fed fp8 consumers (ResBlock convs, proj_in): the e4m3 activation carries a static
  // per-channel power-of-two scale a_c >= (|gamma_c| * GN_F8_RANGE + |beta_c|) / 448 from the producing
  // GroupNorm's affine parameters (arena offset f8_gn, C = f8_cin channels), folded into the weights at
  // finalize; the GroupNorm apply reads 1 / a_c from the arena at inv8.  Rows are ldb8 bytes: ld8 e4m3
  // bytes, then the bf16 K-extension (skip conv) columns pre-divided by the row scale (a power of two).
  int f8_gn = -1, f8_cin = 0, inv8 = 0, ldb8 = 0;
  bool f8_conv = false;
};
// the fp8 layer set of compute_dtype FP8 (TAIR_FP8_OPS overrides; bits below at f8_ops)
constexpr int F8_DEFAULT_OPS = 18;  // LayerNorm-fed linears + conv2 without a skip conv
// |x_hat| bound of a GroupNorm'd value behind the static fp8 activation scales (e4m3 saturates beyond;
// its 2^-9 .. 448 range leaves the typical |x_hat| ~ 1 values 12 bits above the subnormal floor)
constexpr float GN_F8_RANGE = 64.f;

enum PackKind { PK_CONV3, PK_CONV1, PK_LIN, PK_VEC };

struct ParamDst {
  std::string key;
  int64_t shape[4] = {0, 0, 0, 0};
  int ndim = 0;
  PackKind kind = PK_VEC;
  Weight* w = nullptr;   // weights: destination + placement
  int row_off = 0, col_off = 0;
  int vec_off = 0;       // vectors: offset in the fp32 arena (contributions are summed)
  int geglu_half = 0;    // >0: GEGLU proj rows/entries [x | gate] (each this long) interleaved as
                         // (x_2q, x_2q+1, gate_2q, gate_2q+1) so the GEMM epilogue fuses x*gelu(gate)
  std::vector<float> vec_src;
  bool loaded = false;
  bool dirty = false;     // loaded since the last finalize
  bool keep_src = false;  // weight of a LayerNorm-folded linear: fp32 rows kept until finalize folds them
  std::vector<float> w_src;
  int cpad = 0;          // PK_CONV3: (planed) input channels zero-padded to this count (the first convs: 64,
                         // so they run the channel-chunk-major A_CONV3 path on a 64-wide input row)
  int split = 0;         // weights at fp32 accuracy as bf16 planes: 2 = PK_CONV1 columns [W_hi | W_lo] (read
                         // against the same activation, GemmArgs.x_wrap); 3 = PK_CONV3 input channels in
                         // three planes (hi, hi, lo) against an activation stored (hi, lo, hi)
};

struct ResW {
  int cin = 0, cout = 0;
  int gn1 = 0, gn2 = 0;  // arena offsets: gamma at off, beta at off + C
  Weight c1, c2;
  int b1 = 0, b2 = 0;    // arena offsets
  int emb_off = 0;       // column offset in the network's emb table
  bool skip = false;
};

struct STW {
  int C = 0, heads = 0;
  int gn = 0, ln1 = 0, ln2 = 0, ln3 = 0;
  Weight pin, qkv, o1, q2, kv2, o2, ff1, ff2, pout;
  int pinb = 0, o1b = 0, o2b = 0, ff1b = 0, ff2b = 0, poutb = 0;
  bf16* kvcache = nullptr;  // [max_ctx_rows, 2C]
  // LayerNorm folding (bf16 path): norm1/2/3's gamma folded into the rows of qkv / q2 / ff1 at finalize,
  // beta into the folded biases fb_*, the column sums of the folded rows in cs_* (arena offsets)
  bool fold = false;
  std::string tb;  // state-dict prefix of the transformer block
  int fb_qkv = 0, fb_q2 = 0, fb_ff1 = 0, cs_qkv = 0, cs_q2 = 0, cs_ff1 = 0;
};

struct ConvW {
  Weight w;
  int b = 0;
  int cin = 0, cout = 0;
};

enum BlockKind { BK_CONVIN, BK_RES, BK_DOWN };

struct EncBlock {        // one input block: conv_in | Res(+ST) | Down
  BlockKind kind;
  int level;             // resolution level of the OUTPUT
  ConvW conv;            // conv_in / Down
  ResW res;
  bool has_st = false;
  STW st;
  ConvW zero;            // ControlNet zero conv (CN only)
};

struct DecBlock {
  int level;             // level of the ResBlock (before upsample)
  ResW res;
  bool has_st = false;
  STW st;
  bool has_up = false;
  ConvW up;
  int ch_out = 0;
};

struct Net {                 // one UNet-shaped network (UNet or ControlNet)
  Weight te0, te2;           // time_embed.0 / .2
  int te0b = 0, te2b = 0;
  Weight emb;                // all emb_layers.1 weights stacked [sum Cout][time_dim]
  int embb = 0;
  int emb_total = 0;
  std::deque<EncBlock> enc;  // deque: ParamDst keeps pointers into the blocks (stable on push_back)
  ResW mid1, mid2;
  STW midst;
  ConvW mid_out;             // ControlNet middle_block_out
  std::deque<DecBlock> dec;  // UNet only
  int out_gn = 0;            // UNet out: GN + SiLU + conv
  ConvW out_conv;
};

// ------------------------------------------------------------------------------------------
// profiling records
// ------------------------------------------------------------------------------------------
struct ProfRec {
  int cls;
  double flops;
  hipEvent_t a, b;
  std::string tag;
  double alg;       // algorithmic bytes of the launch: operands read once, outputs written once
  std::string key;  // kernel family key (tools/pmc_summary.py joins it to the PMC rows' kernel names)
};

}  // namespace tair

using namespace tair;

struct tair_cldm {
  tair_cldm_cfg cfg{};
  int time_dim = 0;
  int nlev = 0;
  std::vector<int> lev_ch;      // channels per level (model_channels * mult)
  std::vector<int> lev_h, lev_w;
  Net unet, cn;
  std::vector<std::unique_ptr<ParamDst>> params;
  std::map<std::string, ParamDst*> by_key;
  std::vector<float> arena_host;
  float* arena = nullptr;
  bool finalized = false;
  std::vector<void*> allocs;
  // residual-stream ("trunk") buffers: hi plane followed by a lo plane of the same size
  struct Trunk { const char* base; size_t bytes; int lo; };
  std::vector<Trunk> trunks;

  // workspace
  struct Cat { bf16* p; int ch, cs, level; };
  std::vector<Cat> cat;         // decoder concat buffers
  struct Scratch {              // per-branch scratch (0: UNet / main stream, 1: ControlNet branch)
    bf16 *T = nullptr, *H1 = nullptr, *X0 = nullptr, *QKV = nullptr, *A = nullptr, *G = nullptr, *F = nullptr,
         *R = nullptr;
    float *ss = nullptr, *gnws = nullptr, *partial = nullptr;
    size_t partial_cap = 0;
    uint8_t* T8 = nullptr;  // fp8: LayerNorm output as e4m3 [M][round_up(C, 128)] + per-token scales
    float* ts8 = nullptr;
    int* gn_tickets = nullptr;  // GroupNorm stats->finalize tickets [B*G] (zeroed once, self-resetting)
    int* gemm_tickets = nullptr;  // split-K arrival tickets per output tile (zeroed once, self-resetting)
    // attention key-split tickets per (query block, head), ATTN_TICKETS ints: the in-kernel merge of the key
    // splits is opt-in (TAIR_ATTN_INK=1): bitwise the merge kernel, but the B = 1 step ran 3.5% slower with it
    // (the last split's write-through drain, ticket round trip and merge reads sit on the critical path;
    // 1.014-1.021 vs 0.982-0.984 Mpix/s, profiles/r05_bench_b1_attn_ink*.log)
    int* attn_tickets = nullptr;
  };
  Scratch ws[2];
  // GroupNorm statistics accumulated by the producing GEMM epilogues (StatTgt): per step a fresh
  // slot per normalised tensor, zeroed by one memset at the start of the step
  double* gst = nullptr;
  size_t gst_rs = 0;              // replica stride (doubles) = max_batch * groups * 2
  int gst_slots = 0, gst_next = 0;
  bool gn_fused = false;          // producer statistics enabled (TAIR_GN_FUSED, shape support)
  // LayerNorm folding (bf16 path; TAIR_LN_FOLD=0 disables): per forward a fresh fp64 [M][2] row-statistics
  // slot per LayerNorm, bump-allocated from lst and zeroed with the GroupNorm slots
  bool ln_fold = false;
  size_t ln_slot_rows = 0;        // rows over all slots of one forward (max_batch)
  double* lst = nullptr;
  size_t lst_next = 0;            // doubles handed out this forward
  hipStream_t cstream = nullptr;  // ControlNet stream of the forked schedule
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_zc[16] = {};      // zero conv of encoder block i done (side-stream schedule)
  bf16* Dout = nullptr;
  std::vector<bf16*> cn_out;    // ControlNet block outputs (zero-conv inputs after the join)
  bf16* cn_mid = nullptr;
  bf16 *in_u = nullptr, *in_c = nullptr;  // [M,4] / [M,8] boundary inputs
  bf16* ctx_bf = nullptr;                 // [Bctx*77, context_dim]
  float* v_out = nullptr;                 // [M, out_ch] fp32
  // time embedding tables
  int tab_rows = 0;
  float* tab_u = nullptr;                 // [tab_rows][unet.emb_total]
  float* tab_c = nullptr;
  float* sinus = nullptr;                 // scratch
  bf16* temb_a = nullptr;                 // [tab_rows][time_dim] bf16 scratch
  bf16* temb_b = nullptr;
  int64_t* t_dev = nullptr;               // [tab_rows]
  int* rows_iota = nullptr;               // [max_batch] 0..B-1
  int* rows_step = nullptr;               // [max_batch] current step row
  // sampler state
  int n_steps = 0;
  std::vector<int64_t> sched_t;
  std::vector<float> sched_tabs_host;
  float* sched_tabs = nullptr;            // [5][n_steps]
  int* counter = nullptr;                 // device {i, n_steps}
  float* xs = nullptr;                    // NHWC fp32 [M,4] sampler state
  float* noise = nullptr;                 // [n_steps][M][4]
  int noise_cap_steps = 0;
  int64_t* sched_t_dev = nullptr;         // [n_steps] model timesteps of the schedule
  int s_batch = 0, s_ctx_bstride = 0, s_control = 0;
  float s_scales[13];
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;

  hipStream_t gstream = nullptr;           // own non-blocking stream: the caller's (often the legacy
  hipEvent_t ev_in = nullptr, ev_out = nullptr;  // NULL) stream cannot be captured
  int graph_batch = -1;                   // what the captured step froze: batch, ControlNet on/off,
  int graph_control = -1, graph_ctx_bstride = -1;  // context batch stride and the zero-conv scales
  float graph_scales[13] = {};
  // instrumentation
  bool dry = false;
  // TAIR_ABLATE (timing experiments only, never set in tests or the bench line): bit c skips every
  // launch of kernel class c (0 gemm, 1 attention, 2 GroupNorm, 3 LayerNorm); bit 8 skips the split-K
  // reduce launches.  Outputs are garbage; the step time says what removing those launches could buy.
  int ablate = 0;
  double dry_flops = 0;
  bool prof = false;
  std::vector<ProfRec> prof_recs;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  double prof_flops[5] = {0, 0, 0, 0, 0};
};
static void drop_step_graphs(tair_cldm* h);  // (tair_sampler_run)

namespace {

#define TRY(expr)                              \
  do {                                         \
    hipError_t _e = (expr);                    \
    if (_e != hipSuccess) return _e;           \
  } while (0)

// ------------------------------------------------------------------------------------------
// construction helpers
// ------------------------------------------------------------------------------------------
constexpr int CONVIN_LD = 64;  // conv_in input rows: (hi, lo, hi) planes of the 4 / 8 input channels, zero-padded

void* dmalloc(tair_cldm* h, size_t bytes) {
  void* p = nullptr;
  if (h->cfg.manifest_only) return (void*)16;  // never dereferenced: no forward without a device
  if (bytes == 0) bytes = 16;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  hipMemset(p, 0, bytes);
  h->allocs.push_back(p);
  return p;
}

// A residual-stream buffer of `elems` bf16 values with its lo plane right behind it.
bf16* trunk_alloc(tair_cldm* h, size_t elems) {
  bf16* p = (bf16*)dmalloc(h, elems * 2 * sizeof(bf16));
  if (p && !h->cfg.manifest_only) h->trunks.push_back({(const char*)p, elems * sizeof(bf16), (int)elems});
  return p;
}
// element offset of the lo plane of the trunk buffer that holds p (0: not a trunk buffer)
int lo_of(const tair_cldm* h, const void* p) {
  const char* c = (const char*)p;
  for (const auto& t : h->trunks)
    if (c >= t.base && c < t.base + t.bytes) return t.lo;
  return 0;
}

int vec_alloc(tair_cldm* h, int n) {
  const int off = (int)h->arena_host.size();
  h->arena_host.resize(off + round_up(n, 4), 0.f);
  return off;
}

// packed position of GEGLU proj output r (x_j = r < D, gate_j = r - D): groups of four
// (x_2q, x_2q+1, gate_2q, gate_2q+1), matching the epilogue's 4 consecutive channels per lane
int geglu_row(int r, int D) {
  const int j = r < D ? r : r - D;
  return 4 * (j >> 1) + (r < D ? 0 : 2) + (j & 1);
}

ParamDst* add_param(tair_cldm* h, const std::string& key, std::initializer_list<int64_t> shape, PackKind kind) {
  auto p = std::make_unique<ParamDst>();
  p->key = key;
  int i = 0;
  for (auto s : shape) p->shape[i++] = s;
  p->ndim = i;
  p->kind = kind;
  ParamDst* raw = p.get();
  h->by_key[key] = raw;
  h->params.push_back(std::move(p));
  return raw;
}

void add_vec(tair_cldm* h, const std::string& key, int n, int off) {
  ParamDst* p = add_param(h, key, {n}, PK_VEC);
  p->vec_off = off;
}

void add_w(tair_cldm* h, const std::string& key, std::initializer_list<int64_t> shape, PackKind kind, Weight* w,
           int row_off = 0, int col_off = 0) {
  ParamDst* p = add_param(h, key, shape, kind);
  p->w = w;
  p->row_off = row_off;
  p->col_off = col_off;
}

void alloc_w(tair_cldm* h, Weight& w, int rows, int K, int Kx = 0) {
  w.rows = rows;
  w.K = K;
  w.Kx = Kx;
  w.ldw = round_up(K + Kx, 64);
  w.p = (bf16*)dmalloc(h, (size_t)rows * w.ldw * sizeof(bf16));
}
void alloc_w8(tair_cldm* h, Weight& w) {  // fp8 twin of a dense weight (after alloc_w)
  w.ld8 = round_up(w.K, 128);
  w.ldb8 = w.ld8;
  w.p8 = (uint8_t*)dmalloc(h, (size_t)w.rows * w.ld8);
  w.s8 = (float*)dmalloc(h, (size_t)w.rows * sizeof(float));
}
// fp8 twin of a GroupNorm-fed conv (9 cin values per row in the channel-chunk-major order) or linear,
// with static activation scales from the GroupNorm at arena offset gn (after alloc_w)
void alloc_w8_gn(tair_cldm* h, Weight& w, int gn, int cin, bool conv) {
  w.ld8 = round_up(w.K, 128);
  w.ldb8 = round_up(w.ld8 + 2 * w.Kx, 16);
  w.p8 = (uint8_t*)dmalloc(h, (size_t)w.rows * w.ldb8);
  w.s8 = (float*)dmalloc(h, (size_t)w.rows * sizeof(float));
  w.f8_gn = gn;
  w.f8_cin = cin;
  w.f8_conv = conv;
  w.inv8 = vec_alloc(h, cin);
}
// which layers take e4m3 operands under compute_dtype FP8, TAIR_FP8_OPS bit mask (accuracy
// / speed A/B experiments): 1 ResBlock conv1, 2 conv2 without a skip conv, 4 conv2 with the bf16 skip
// K-extension, 8 proj_in, 16 the LayerNorm-fed linears (attn1 q|k|v, attn2 q, GEGLU proj)
constexpr int F8_CONV1 = 1, F8_CONV2 = 2, F8_CONV2_SKIP = 4, F8_PROJ_IN = 8, F8_LN_LINEAR = 16;
int f8_ops(const tair_cldm* h) {
  if (h->cfg.compute_dtype != TAIR_DTYPE_FP8) return 0;
  static const int v = [] { const char* e = getenv("TAIR_FP8_OPS"); return e ? atoi(e) : F8_DEFAULT_OPS; }();
  return v;
}

// GroupNorm/LayerNorm affine params: gamma at off, beta at off+C
int norm_params(tair_cldm* h, const std::string& pfx, int C) {
  const int off = vec_alloc(h, 2 * C);
  add_vec(h, pfx + ".weight", C, off);
  add_vec(h, pfx + ".bias", C, off + C);
  return off;
}

void build_res(tair_cldm* h, Net& net, ResW& r, const std::string& pfx, int cin, int cout) {
  r.cin = cin;
  r.cout = cout;
  r.skip = cin != cout;
  r.gn1 = norm_params(h, pfx + ".in_layers.0", cin);
  alloc_w(h, r.c1, cout, 9 * cin);
  add_w(h, pfx + ".in_layers.2.weight", {cout, cin, 3, 3}, PK_CONV3, &r.c1);
  r.b1 = vec_alloc(h, cout);
  add_vec(h, pfx + ".in_layers.2.bias", cout, r.b1);
  r.emb_off = net.emb_total;
  net.emb_total += cout;
  r.gn2 = norm_params(h, pfx + ".out_layers.0", cout);
  alloc_w(h, r.c2, cout, 9 * cout, r.skip ? 2 * cin : 0);  // skip conv as [W_hi | W_lo] K-extension
  add_w(h, pfx + ".out_layers.3.weight", {cout, cout, 3, 3}, PK_CONV3, &r.c2);
  r.b2 = vec_alloc(h, cout);
  add_vec(h, pfx + ".out_layers.3.bias", cout, r.b2);
  if (r.skip) {
    add_w(h, pfx + ".skip_connection.weight", {cout, cin, 1, 1}, PK_CONV1, &r.c2, 0, 9 * cout);
    h->by_key[pfx + ".skip_connection.weight"]->split = 2;
    add_vec(h, pfx + ".skip_connection.bias", cout, r.b2);  // summed into conv2's bias
  }
  const int f8 = f8_ops(h);
  if (f8 && cin % 64 == 0 && cout % 64 == 0) {  // configs[4]: e4m3 x e4m3 convs
    if (f8 & F8_CONV1) alloc_w8_gn(h, r.c1, r.gn1, cin, true);
    if (f8 & (r.skip ? F8_CONV2_SKIP : F8_CONV2)) alloc_w8_gn(h, r.c2, r.gn2, cout, true);
  }
}

// emb_layers weights registered after the net's emb matrix is allocated
void register_emb(tair_cldm* h, Net& net, const ResW& r, const std::string& pfx) {
  add_w(h, pfx + ".emb_layers.1.weight", {r.cout, h->time_dim}, PK_LIN, &net.emb, r.emb_off, 0);
  add_vec(h, pfx + ".emb_layers.1.bias", r.cout, net.embb + r.emb_off);
}

void build_st(tair_cldm* h, STW& s, const std::string& pfx, int C, int lvl) {
  const int ctx = h->cfg.context_dim;
  s.C = C;
  s.heads = C / h->cfg.head_channels;
  s.gn = norm_params(h, pfx + ".norm", C);
  alloc_w(h, s.pin, C, C);
  add_w(h, pfx + ".proj_in.weight", {C, C}, PK_LIN, &s.pin);
  s.pinb = vec_alloc(h, C);
  add_vec(h, pfx + ".proj_in.bias", C, s.pinb);
  const std::string tb = pfx + ".transformer_blocks.0";
  alloc_w(h, s.qkv, 3 * C, C);
  add_w(h, tb + ".attn1.to_q.weight", {C, C}, PK_LIN, &s.qkv, 0);
  add_w(h, tb + ".attn1.to_k.weight", {C, C}, PK_LIN, &s.qkv, C);
  add_w(h, tb + ".attn1.to_v.weight", {C, C}, PK_LIN, &s.qkv, 2 * C);
  alloc_w(h, s.o1, C, C);
  add_w(h, tb + ".attn1.to_out.0.weight", {C, C}, PK_LIN, &s.o1);
  s.o1b = vec_alloc(h, C);
  add_vec(h, tb + ".attn1.to_out.0.bias", C, s.o1b);
  alloc_w(h, s.ff1, 8 * C, C);
  add_w(h, tb + ".ff.net.0.proj.weight", {8 * C, C}, PK_LIN, &s.ff1);
  h->by_key[tb + ".ff.net.0.proj.weight"]->geglu_half = 4 * C;
  s.ff1b = vec_alloc(h, 8 * C);
  add_vec(h, tb + ".ff.net.0.proj.bias", 8 * C, s.ff1b);
  h->by_key[tb + ".ff.net.0.proj.bias"]->geglu_half = 4 * C;
  alloc_w(h, s.ff2, C, 4 * C);
  add_w(h, tb + ".ff.net.2.weight", {C, 4 * C}, PK_LIN, &s.ff2);
  s.ff2b = vec_alloc(h, C);
  add_vec(h, tb + ".ff.net.2.bias", C, s.ff2b);
  alloc_w(h, s.q2, C, C);
  add_w(h, tb + ".attn2.to_q.weight", {C, C}, PK_LIN, &s.q2);
  alloc_w(h, s.kv2, 2 * C, ctx);
  add_w(h, tb + ".attn2.to_k.weight", {C, ctx}, PK_LIN, &s.kv2, 0);
  add_w(h, tb + ".attn2.to_v.weight", {C, ctx}, PK_LIN, &s.kv2, C);
  alloc_w(h, s.o2, C, C);
  add_w(h, tb + ".attn2.to_out.0.weight", {C, C}, PK_LIN, &s.o2);
  s.o2b = vec_alloc(h, C);
  add_vec(h, tb + ".attn2.to_out.0.bias", C, s.o2b);
  s.ln1 = norm_params(h, tb + ".norm1", C);
  s.ln2 = norm_params(h, tb + ".norm2", C);
  s.ln3 = norm_params(h, tb + ".norm3", C);
  alloc_w(h, s.pout, C, C);
  add_w(h, pfx + ".proj_out.weight", {C, C}, PK_LIN, &s.pout);
  s.poutb = vec_alloc(h, C);
  add_vec(h, pfx + ".proj_out.bias", C, s.poutb);
  s.kvcache = (bf16*)dmalloc(h, (size_t)h->cfg.max_batch * h->cfg.context_len * 2 * C * sizeof(bf16));
  if (f8_ops(h) & F8_PROJ_IN) alloc_w8_gn(h, s.pin, s.gn, C, false);  // proj_in: on the GroupNorm's e4m3 output
  if (f8_ops(h) & F8_LN_LINEAR) {  // the LayerNorm-fed linears run e4m3 x e4m3
    alloc_w8(h, s.qkv);
    alloc_w8(h, s.q2);
    alloc_w8(h, s.ff1);
  } else if (h->ln_fold) {  // bf16: the LayerNorms fold into their consumers
    s.fold = true;
    s.tb = tb;
    s.fb_qkv = vec_alloc(h, 3 * C);
    s.cs_qkv = vec_alloc(h, 3 * C);
    s.fb_q2 = vec_alloc(h, C);
    s.cs_q2 = vec_alloc(h, C);
    s.fb_ff1 = vec_alloc(h, 8 * C);
    s.cs_ff1 = vec_alloc(h, 8 * C);
    for (const char* k : {".attn1.to_q.weight", ".attn1.to_k.weight", ".attn1.to_v.weight", ".attn2.to_q.weight",
                          ".ff.net.0.proj.weight"})
      h->by_key[tb + k]->keep_src = true;
    h->ln_slot_rows += 3 * (size_t)h->cfg.max_batch * h->lev_h[lvl] * h->lev_w[lvl];
  }
}

// split3: fp32-accurate conv (weights as three planes (hi, hi, lo) over 3*cin input channels, read
// against an activation stored (hi, lo, hi)): the first and last convs of the UNet / ControlNet
// pad64: the (planed) input channels zero-padded to 64 (the first convs: 4 / 8 channels x 3 planes read as a
// 64-channel NHWC row, one channel chunk on the LDS-DMA implicit-GEMM path; tap-major A_CONV3_SMALLC element
// gathers measured 34 us per launch at B = 1 for 0.2 GFLOP)
void build_conv3(tair_cldm* h, ConvW& c, const std::string& pfx, int cin, int cout, bool pad64 = false,
                 bool split3 = false) {
  c.cin = cin;
  c.cout = cout;
  const int kc = split3 ? 3 * cin : cin;
  alloc_w(h, c.w, cout, pad64 ? 9 * round_up(kc, 64) : 9 * kc);
  add_w(h, pfx + ".weight", {cout, cin, 3, 3}, PK_CONV3, &c.w);
  if (split3) h->by_key[pfx + ".weight"]->split = 3;
  if (pad64) h->by_key[pfx + ".weight"]->cpad = round_up(kc, 64);
  c.b = vec_alloc(h, cout);
  add_vec(h, pfx + ".bias", cout, c.b);
}

void build_conv1(tair_cldm* h, ConvW& c, const std::string& pfx, int cin, int cout) {
  c.cin = cin;
  c.cout = cout;
  alloc_w(h, c.w, cout, cin);
  add_w(h, pfx + ".weight", {cout, cin, 1, 1}, PK_CONV1, &c.w);
  c.b = vec_alloc(h, cout);
  add_vec(h, pfx + ".bias", cout, c.b);
}

bool attn_at(const tair_cldm* h, int ds) {
  for (int i = 0; i < h->cfg.num_attention_ds; ++i)
    if (h->cfg.attention_ds[i] == ds) return true;
  return false;
}

// unet.py:491-569 / controlnet.py:168-267
void build_encoder(tair_cldm* h, Net& net, const std::string& root, int in_ch, bool control) {
  const int mc = h->cfg.model_channels;
  net.enc.emplace_back();
  EncBlock& b0 = net.enc.back();
  b0.kind = BK_CONVIN;
  b0.level = 0;
  build_conv3(h, b0.conv, root + ".input_blocks.0.0", in_ch, mc, true, true);
  if (control) build_conv1(h, b0.zero, root + ".zero_convs.0.0", mc, mc);
  int ch = mc, ds = 1, idx = 1;
  for (int lvl = 0; lvl < h->nlev; ++lvl) {
    for (int r = 0; r < h->cfg.num_res_blocks; ++r) {
      net.enc.emplace_back();
      EncBlock& b = net.enc.back();
      b.kind = BK_RES;
      b.level = lvl;
      const int out = h->cfg.channel_mult[lvl] * mc;
      const std::string pfx = root + ".input_blocks." + std::to_string(idx);
      build_res(h, net, b.res, pfx + ".0", ch, out);
      ch = out;
      if (attn_at(h, ds)) {
        b.has_st = true;
        build_st(h, b.st, pfx + ".1", ch, lvl);
      }
      if (control) build_conv1(h, b.zero, root + ".zero_convs." + std::to_string(idx) + ".0", ch, ch);
      ++idx;
    }
    if (lvl != h->nlev - 1) {
      net.enc.emplace_back();
      EncBlock& b = net.enc.back();
      b.kind = BK_DOWN;
      b.level = lvl + 1;
      build_conv3(h, b.conv, root + ".input_blocks." + std::to_string(idx) + ".0.op", ch, ch);
      if (control) build_conv1(h, b.zero, root + ".zero_convs." + std::to_string(idx) + ".0", ch, ch);
      ds *= 2;
      ++idx;
    }
  }
  // middle (unet.py:580-608)
  build_res(h, net, net.mid1, root + ".middle_block.0", ch, ch);
  build_st(h, net.midst, root + ".middle_block.1", ch, h->nlev - 1);
  build_res(h, net, net.mid2, root + ".middle_block.2", ch, ch);
  if (control) build_conv1(h, net.mid_out, root + ".middle_block_out.0", ch, ch);
}

// unet.py:611-679
void build_decoder(tair_cldm* h, Net& net, const std::string& root) {
  const int mc = h->cfg.model_channels;
  std::vector<int> chans;
  chans.push_back(mc);
  {
    int ch = mc;
    for (int lvl = 0; lvl < h->nlev; ++lvl) {
      for (int r = 0; r < h->cfg.num_res_blocks; ++r) {
        ch = h->cfg.channel_mult[lvl] * mc;
        chans.push_back(ch);
      }
      if (lvl != h->nlev - 1) chans.push_back(ch);
    }
  }
  int ch = h->cfg.channel_mult[h->nlev - 1] * mc;
  int ds = 1 << (h->nlev - 1);
  int idx = 0;
  for (int lvl = h->nlev - 1; lvl >= 0; --lvl) {
    for (int i = 0; i <= h->cfg.num_res_blocks; ++i) {
      net.dec.emplace_back();
      DecBlock& d = net.dec.back();
      d.level = lvl;
      const int ich = chans.back();
      chans.pop_back();
      const int out = mc * h->cfg.channel_mult[lvl];
      const std::string pfx = root + ".output_blocks." + std::to_string(idx);
      build_res(h, net, d.res, pfx + ".0", ch + ich, out);
      ch = out;
      int li = 1;
      if (attn_at(h, ds)) {
        d.has_st = true;
        build_st(h, d.st, pfx + "." + std::to_string(li++), ch, lvl);
      }
      if (lvl && i == h->cfg.num_res_blocks) {
        d.has_up = true;
        build_conv3(h, d.up, pfx + "." + std::to_string(li++) + ".conv", ch, ch);
        ds /= 2;
      }
      d.ch_out = ch;
      ++idx;
    }
  }
  net.out_gn = norm_params(h, root + ".out.0", ch);
  build_conv3(h, net.out_conv, root + ".out.2", mc, h->cfg.out_channels, false, true);
}

void build_time(tair_cldm* h, Net& net, const std::string& root) {
  const int mc = h->cfg.model_channels, td = h->time_dim;
  alloc_w(h, net.te0, td, mc);
  add_w(h, root + ".time_embed.0.weight", {td, mc}, PK_LIN, &net.te0);
  net.te0b = vec_alloc(h, td);
  add_vec(h, root + ".time_embed.0.bias", td, net.te0b);
  alloc_w(h, net.te2, td, td);
  add_w(h, root + ".time_embed.2.weight", {td, td}, PK_LIN, &net.te2);
  net.te2b = vec_alloc(h, td);
  add_vec(h, root + ".time_embed.2.bias", td, net.te2b);
}

void finish_emb(tair_cldm* h, Net& net, const std::string& root, bool decoder) {
  alloc_w(h, net.emb, net.emb_total, h->time_dim);
  net.embb = vec_alloc(h, net.emb_total);
  int idx = 0;
  for (auto& b : net.enc) {
    if (b.kind == BK_RES) register_emb(h, net, b.res, root + ".input_blocks." + std::to_string(idx) + ".0");
    ++idx;
  }
  register_emb(h, net, net.mid1, root + ".middle_block.0");
  register_emb(h, net, net.mid2, root + ".middle_block.2");
  if (decoder) {
    idx = 0;
    for (auto& d : net.dec) register_emb(h, net, d.res, root + ".output_blocks." + std::to_string(idx++) + ".0");
  }
}

// ------------------------------------------------------------------------------------------
// launch wrappers (dry-run FLOP counting + optional per-class event timing)
// ------------------------------------------------------------------------------------------
template <class F>
hipError_t launch(tair_cldm* h, int cls, double flops, hipStream_t s, F&& fn, const std::string& tag = "",
                  double alg = 0.0, const std::string& key = "") {
  if (h->dry) {
    h->dry_flops += flops;
    return hipSuccess;
  }
  if (h->ablate & (1 << cls)) return hipSuccess;  // timing-only ablation (TAIR_ABLATE): results are garbage
  if (!h->prof) return fn();
  if (h->ev_used + 2 > h->ev_pool.size()) {
    for (int i = 0; i < 512; ++i) {
      hipEvent_t e;
      TRY(hipEventCreate(&e));
      h->ev_pool.push_back(e);
    }
  }
  ProfRec r{cls, flops, h->ev_pool[h->ev_used], h->ev_pool[h->ev_used + 1], tag, alg, key};
  h->ev_used += 2;
  TRY(hipEventRecord(r.a, s));
  TRY(fn());
  TRY(hipEventRecord(r.b, s));
  h->prof_recs.push_back(r);
  return hipSuccess;
}

const float* V(tair_cldm* h, int off) { return h->arena + off; }

// Forward context.  A step runs one or two "lanes": lane 0 = the UNet, lane 1 = the ControlNet.
// The ControlNet encoder/middle has exactly the UNet encoder/middle's layer shapes, so while both
// are live every layer is issued ONCE as a grouped launch over both networks (own weights, own
// activations, own scratch ws[lane]): half the launches of running the two networks one after the
// other, with twice the workgroups per launch, and no cross-stream dependencies in the step graph.
struct Lane {
  const tair_cldm::Scratch* w;
  const float* tab;  // time-embedding table [rows][tab_ld] of this network
  int tab_ld;
  int net;           // 0 = UNet, 1 = ControlNet
};
struct Fwd {
  hipStream_t s;
  int B;
  const int* emb_row;  // [B] rows into the emb tables
  int ctx_bstride;     // 0 (broadcast c_txt) or context_len
  int n;               // lanes in every launch (1 or 2)
  Lane l[2];
};

GemmArgs gemm_base(int M, const Weight& w) {
  GemmArgs a{};
  a.M = M;
  a.N = w.rows;
  a.K = w.K;
  a.Kx = 0;
  a.Wt = w.p;
  a.ldw = w.ldw;
  a.alpha = 1.f;
  a.rows_per_b = 1;
  a.splits = 1;
  return a;
}

// Algorithmic bytes of one GEMM: every operand read once and every output written once
// -- the activation tensor (a conv's input map, not its nine-tap expansion), the K-extension, the weights,
// the residual and the output planes; split-K slabs, re-reads and statistics are not algorithmic.
double gemm_alg_bytes(const GemmArgs& a) {
  double act;
  if (a.amode == A_DENSE) {
    act = (double)a.M * a.K * 2;  // (fp8: K counts byte pairs)
  } else {
    const int B = a.Bn > 0 ? a.Bn : a.M / std::max(1, a.Ho * a.Wo);
    act = (double)B * a.H * a.W * a.C * (a.f8 ? 1 : 2);
  }
  const double kx = a.x_wrap ? a.x_wrap : a.Kx;
  const double x = (double)a.M * kx * 2;
  const double w = (double)a.N * (a.K + a.Kx) * 2;
  double out = (double)a.M * a.N * (a.out_f32 ? 4 : 2) * (a.out_split ? 3 : 1) * (a.out_lo ? 2 : 1);
  if (a.act == 2) out *= 0.5;  // GEGLU: half the columns
  const double res = a.res ? (double)a.M * a.N * 2 * (a.res_lo ? 2 : 1) : 0.0;
  return act + x + w + out + res;
}

// a[0..f.n): one GEMM per lane (same shape), issued as one grouped launch
hipError_t run_gemm(tair_cldm* h, GemmArgs* a, const Fwd& f, double f8_kfrac = 1.0) {
  // Split-K slices: small split counts are combined inside the GEMM launch by the last-arriving slice
  // (gemm_kern.h splitk_combine), larger ones by splitk_reduce_kernel (gemm_grouped decides).
  for (int i = 0; i < f.n; ++i) {
    a[i].partial = f.l[i].w->partial;
    a[i].partial_cap = f.l[i].w->partial_cap;
    a[i].tile_sem = f.l[i].w->gemm_tickets;  // in-kernel split-K combine where the launcher picks it
    a[i].sem_cap = GEMM_TICKETS;
  }
  // algorithmic FLOPs: the logical reduction length (split planes and the [W_hi | W_lo] K-extension
  // are precision overhead, not work of the reference's layer)
  const double kp = a[0].kplanes > 1 ? a[0].kplanes : 1;
  const double kreal = a[0].flop_k ? (double)a[0].flop_k
                       : a[0].f8 ? 2.0 * a[0].K * f8_kfrac
                       : ((a[0].amode == A_CONV3_SMALLC) ? 9.0 * a[0].C : (double)a[0].K) / kp;
  const double kx = a[0].x_wrap ? 0.5 * a[0].Kx : (double)a[0].Kx;
  const double fl = 2.0 * f.n * a[0].M * a[0].N * (kreal + kx);
  std::string tag, key;
  double alg = 0.0;
  if (h->prof) {
    int bm = 0, bn = 0, sp = 0, kern = 0;
    gemm_plan_query(a[0], &bm, &bn, &sp, &kern);  // the plan gemm_grouped launches
    char buf[200];
    snprintf(buf, sizeof(buf), "gemm mode=%d M=%d N=%d K=%d Kx=%d tile=%dx%d splits=%d kern=%d group=%d", a[0].amode,
             a[0].M, a[0].N, (int)kreal, a[0].Kx, bm, bn, sp, kern, f.n);
    tag = buf;
    const char* fam = kern == GEMM_KERN_HALO ? "halo" : kern == GEMM_KERN_PHASE ? "phase" : bm < 0 ? "ring"
                      : a[0].amode == A_CONV3_SMALLC ? "reg" : "tile";
    snprintf(buf, sizeof(buf), "%s:%dx%d:%d:%d", fam, bm < 0 ? -bm : bm, bn, a[0].amode, a[0].f8 ? 1 : 0);
    key = buf;
    for (int i = 0; i < f.n; ++i) alg += gemm_alg_bytes(a[i]);
  }
  hipStream_t s = f.s;
  const int n = f.n;
  return launch(h, 0, fl, s, [&] { return gemm_grouped(a, n, s); }, tag, alg, key);
}
hipError_t run_gemm1(tair_cldm* h, GemmArgs a, const Fwd& f) {
  Fwd f1 = f;
  f1.n = 1;
  return run_gemm(h, &a, f1);
}

GemmArgs dense(const bf16* A, int lda, int M, const Weight& w) {
  GemmArgs a = gemm_base(M, w);
  a.amode = A_DENSE;
  a.A = A;
  a.lda = lda;
  return a;
}

GemmArgs conv(int mode, const bf16* A, int lda, int C, int B, int Hi, int Wi, int Ho, int Wo, const Weight& w) {
  GemmArgs a = gemm_base(B * Ho * Wo, w);
  a.amode = mode;
  a.A = A;
  a.lda = lda;
  a.C = C;
  a.Bn = B;
  a.H = Hi;
  a.W = Wi;
  a.Ho = Ho;
  a.Wo = Wo;
  a.rows_per_b = Ho * Wo;
  return a;
}

// GroupNorm statistics (+ fused finalize) of x[i] with the parameters at arena offset off[i]
hipError_t run_gn(tair_cldm* h, const Fwd& f, const bf16* const* x, const int* ldx, int HW, int C, float eps,
                  const int* off) {
  GnArgs g[2];
  for (int i = 0; i < f.n; ++i) {
    g[i] = GnArgs{x[i], ldx[i], V(h, off[i]), V(h, off[i] + C), f.l[i].w->ss, f.l[i].w->gnws,
                  f.l[i].w->gn_tickets, nullptr, 0};
    g[i].x_lo = lo_of(h, x[i]);
  }
  double alg = 0.0;
  for (int i = 0; i < f.n; ++i) alg += (double)f.B * HW * C * 2 * (g[i].x_lo ? 2 : 1);
  return launch(h, 2, 0, f.s, [&] { return groupnorm_stats_grouped(g, f.n, f.B, HW, C, h->cfg.groups, eps, f.s); },
                "gn_stats HW=" + std::to_string(HW) + " C=" + std::to_string(C), alg, "gn_stats");
}
// a GroupNorm apply reads the input (hi + lo planes of a residual-stream input) and writes y (split planes,
// or e4m3 bytes for an fp8 consumer)
double gn_alg_bytes(const GnArgs* g, int n, int B, int HW, int C) {
  double t = 0.0;
  for (int i = 0; i < n; ++i) {
    const double px = (double)B * HW * C;
    t += px * 2 * (g[i].x_lo ? 2 : 1);
    t += g[i].y8 ? px : px * 2 * (g[i].y_split ? 3 : 1);
  }
  return t;
}
struct Out8;
void set_out8(tair_cldm* h, GnArgs& g, const Fwd& f, int i, const Out8* o8, int C);
hipError_t run_gn_apply(tair_cldm* h, const Fwd& f, const bf16* const* x, const int* ldx, int HW, int C, int silu,
                        bf16* const* y, const int* ldy, int y_split = 0, const Out8* o8 = nullptr) {
  GnArgs g[2];
  for (int i = 0; i < f.n; ++i) {
    g[i] = GnArgs{x[i], ldx[i], nullptr, nullptr, f.l[i].w->ss, nullptr, nullptr, y[i], ldy[i]};
    g[i].x_lo = lo_of(h, x[i]);
    g[i].y_split = y_split;
    set_out8(h, g[i], f, i, o8, C);
  }
  return launch(h, 2, 0, f.s, [&] { return groupnorm_apply_grouped(g, f.n, f.B, HW, C, silu, f.s); },
                "gn_apply HW=" + std::to_string(HW) + " C=" + std::to_string(C), gn_alg_bytes(g, f.n, f.B, HW, C),
                "gn_apply");
}
hipError_t run_ln(tair_cldm* h, const Fwd& f, const bf16* const* x, int T, int C, const int* off, bf16* const* y) {
  LnArgs g[2];
  for (int i = 0; i < f.n; ++i) g[i] = LnArgs{x[i], V(h, off[i]), V(h, off[i] + C), y[i]};
  return launch(h, 3, 0, f.s, [&] { return layernorm_grouped(g, f.n, T, C, 1e-5f, f.s); },
                "layernorm T=" + std::to_string(T) + " C=" + std::to_string(C), 4.0 * f.n * T * C, "layernorm");
}

// LayerNorm into the e4m3 operand of an fp8 linear (per-token scales in ts8)
hipError_t run_ln8(tair_cldm* h, const Fwd& f, const bf16* const* x, int T, int C, const int* off) {
  LnArgs g[2];
  for (int i = 0; i < f.n; ++i)
    g[i] = LnArgs{x[i], V(h, off[i]), V(h, off[i] + C), nullptr, f.l[i].w->T8, f.l[i].w->ts8, round_up(C, 128)};
  return launch(h, 3, 0, f.s, [&] { return layernorm_grouped(g, f.n, T, C, 1e-5f, f.s); },
                "layernorm_fp8 T=" + std::to_string(T) + " C=" + std::to_string(C), 3.0 * f.n * T * C, "layernorm");
}
// fp8 linear on the LayerNorm's e4m3 output of lane i (w.p8 / w.s8): K and the strides in byte pairs
GemmArgs dense8(const Fwd& f, int i, int M, const Weight& w) {
  GemmArgs a = gemm_base(M, w);
  a.amode = A_DENSE;
  a.f8 = 1;
  a.A = (const bf16*)f.l[i].w->T8;
  a.lda = w.ld8 / 2;
  a.K = w.ld8 / 2;
  a.Wt = (const bf16*)w.p8;
  a.ldw = w.ld8 / 2;
  a.row_scale = f.l[i].w->ts8;
  a.col_scale = w.s8;
  return a;
}

// fp8 3x3 conv / linear on lane i's GroupNorm e4m3 output (static activation scales folded into w.p8)
GemmArgs conv8(const Fwd& f, int i, int cin, int Hh, int Ww, const Weight& w) {
  GemmArgs a = gemm_base(f.B * Hh * Ww, w);
  a.amode = A_CONV3;
  a.f8 = 1;
  a.A = (const bf16*)f.l[i].w->T8;
  a.lda = cin / 2;
  a.C = cin;
  a.Bn = f.B;
  a.H = Hh;
  a.W = Ww;
  a.Ho = Hh;
  a.Wo = Ww;
  a.rows_per_b = Hh * Ww;
  a.K = w.ld8 / 2;
  a.Wt = (const bf16*)w.p8;
  a.ldw = w.ldb8 / 2;
  a.col_scale = w.s8;
  return a;
}
GemmArgs dense8gn(const Fwd& f, int i, int M, const Weight& w) {
  GemmArgs a = dense8(f, i, M, w);
  a.row_scale = nullptr;
  a.ldw = w.ldb8 / 2;
  return a;
}

// ---- GroupNorm statistics produced in GEMM epilogues -------------------------------------
// A tensor that a GroupNorm will consume gets a statistics slot; every GEMM that writes final values
// into it carries a StatTgt for that slot (its channel offset inside the normalised tensor), and
// the GroupNorm then runs as a single apply pass that finalises the statistics itself.
struct Tg {  // statistics targets of one lane's output (up to two consumers)
  StatTgt t[2] = {};
};
// LayerNorm row-statistics slots: each slot [M][2] doubles rounded up to 16 (fresh per forward)
size_t lst_doubles(const tair_cldm* h) { return 2 * h->ln_slot_rows + 16 * 256; }
double* new_lnstat(tair_cldm* h, int M) {
  if (!h->ln_fold || h->dry || !h->lst) return nullptr;
  const size_t need = (size_t)round_up(2 * M, 16);
  if (h->lst_next + need > lst_doubles(h)) return nullptr;
  double* p = h->lst + h->lst_next;
  h->lst_next += need;
  return p;
}
double* new_stat(tair_cldm* h) {
  if (!h->gn_fused || h->dry || h->gst_next >= h->gst_slots) return nullptr;
  return h->gst + (size_t)(h->gst_next++) * STAT_REPL * h->gst_rs;
}
StatTgt stat_tgt(tair_cldm* h, double* acc, int C, int c_off, int hw) {
  StatTgt t{};
  if (!acc) return t;
  t.acc = acc;
  t.rs = (int)h->gst_rs;
  t.G = h->cfg.groups;
  t.cg = C / t.G;
  t.c_off = c_off;
  t.hw = hw;
  return t;
}
void add_tgt(Tg& g, const StatTgt& t) {
  if (!t.acc) return;
  if (!g.t[0].acc) g.t[0] = t;
  else g.t[1] = t;
}
void set_tg(GemmArgs& a, const Tg& g) {
  a.st[0] = g.t[0];
  a.st[1] = g.t[1];
}

// GroupNorm (+ SiLU) of x[i] into y[i]: from producer statistics st[i] when every lane has them,
// else the two-pass statistics + apply kernels.
// e4m3 output of a GroupNorm apply for the fp8 consumer w8[i] (into lane i's T8, rows of w8.ld8 bytes
// for a linear, C bytes for a conv)
struct Out8 {
  const Weight* w8[2] = {nullptr, nullptr};
};
void set_out8(tair_cldm* h, GnArgs& g, const Fwd& f, int i, const Out8* o8, int C) {
  if (!o8 || !o8->w8[i]) return;
  const Weight& w = *o8->w8[i];
  g.y8 = f.l[i].w->T8;
  g.ld8 = w.f8_conv ? C : w.ld8;
  g.inv8 = V(h, w.inv8);
}

// (experiment) TAIR_GN_HI=1: GroupNorm applies read only the hi plane of a residual-stream input
bool gn_hi_only() {
  static const bool on = [] { const char* e = getenv("TAIR_GN_HI"); return e && atoi(e) != 0; }();
  return on;
}
hipError_t run_norm(tair_cldm* h, const Fwd& f, const bf16* const* x, const int* ldx, int HW, int C,
                    double* const* st, const int* off, float eps, int silu, bf16* const* y, const int* ldy,
                    int y_split = 0, const Out8* o8 = nullptr) {
  bool fused = true;
  for (int i = 0; i < f.n; ++i) fused = fused && st[i];
  if (!fused) {
    TRY(run_gn(h, f, x, ldx, HW, C, eps, off));
    return run_gn_apply(h, f, x, ldx, HW, C, silu, y, ldy, y_split, o8);
  }
  GnArgs g[2];
  for (int i = 0; i < f.n; ++i) {
    g[i] = GnArgs{x[i], ldx[i], V(h, off[i]), V(h, off[i] + C), nullptr, nullptr, nullptr, y[i], ldy[i],
                  st[i], (int)h->gst_rs, eps};
    g[i].x_lo = gn_hi_only() ? 0 : lo_of(h, x[i]);  // a residual-stream input is read as hi + lo
    g[i].y_split = y_split;
    set_out8(h, g[i], f, i, o8, C);
  }
  return launch(h, 2, 0, f.s, [&] {
    return groupnorm_apply_grouped(g, f.n, f.B, HW, C, silu, f.s, h->cfg.groups);
  }, "gn_apply_fused HW=" + std::to_string(HW) + " C=" + std::to_string(C), gn_alg_bytes(g, f.n, f.B, HW, C),
     "gn_apply");
}

// GroupNorm on load: the consumer GEMM normalises its activation operand itself from the
// producer statistics, so the GroupNorm apply pass (and its launch) disappears.  Measured slower than the
// separate apply pass so far (profiles/r04_gn*_b*.log), hence opt-in: TAIR_GN_FUSE=1 fuses the inputs held
// as one bf16 plane (ResBlock conv2 on conv1's output), TAIR_GN_TRUNK=1 also the residual-stream inputs
// (hi + lo planes: ResBlock conv1), which the fused load reads as the hi plane alone.  Only halo-tile convs
// take it (gemm_gn_ok): proj_in and the skip ResBlocks' conv2 always keep the apply.
bool gn_fuse_on() {
  static const bool on = [] { const char* e = getenv("TAIR_GN_FUSE"); return e && atoi(e) != 0; }();
  return on;
}
bool gn_fuse_trunk() {
  static const bool on = [] { const char* e = getenv("TAIR_GN_TRUNK"); return e && atoi(e) != 0; }();
  return on && gn_fuse_on();
}
void set_gn_load(tair_cldm* h, GemmArgs& a, const double* st, int off, int C, float eps, int silu, int hw) {
  a.gn_st = st;
  a.gn_rs = (int)h->gst_rs;
  a.gn_G = h->cfg.groups;
  a.gn_eps = eps;
  a.gn_gamma = V(h, off);
  a.gn_beta = V(h, off + C);
  a.gn_silu = silu;
  a.rows_per_b = hw;
}
// every lane's GEMM has a GroupNorm-on-load plan (else the caller runs the separate apply)
bool gn_load_ok(tair_cldm* h, const GemmArgs* a, int n) {
  if (h->dry) return true;
  for (int i = 0; i < n; ++i)
    if (!a[i].gn_st || !gemm_gn_ok(a[i])) return false;
  return true;
}
void clear_gn_load(GemmArgs& a) {
  a.gn_st = nullptr;
  a.gn_gamma = a.gn_beta = nullptr;
}

// ResBlock._forward (unet.py:203-223) per lane: x[i] -> out[i] (out may alias x only when cin == cout).
// xst[i]: producer statistics of x[i] (or null); otg[i]: statistics targets of out[i].
hipError_t resblock(tair_cldm* h, const Fwd& f, const ResW* const* r, const bf16* const* x, const int* ldx,
                    double* const* xst, bf16* const* out, const int* ldo, const Tg* otg, int lvl) {
  const int Hh = h->lev_h[lvl], Ww = h->lev_w[lvl], HW = Hh * Ww;
  const int cin = r[0]->cin, cout = r[0]->cout;
  const int n = f.n;
  int off[2], ldc[2] = {cin, cin}, ldh[2] = {cout, cout};
  bf16 *T[2], *H1[2];
  double* s1[2] = {nullptr, nullptr};
  for (int i = 0; i < n; ++i) {
    off[i] = r[i]->gn1;
    T[i] = f.l[i].w->T;
    H1[i] = f.l[i].w->H1;
    s1[i] = new_stat(h);
  }
  // fp8 (configs[4]): the convs on e4m3 GroupNorm outputs (a skip K-extension stays bf16)
  const bool f8 = r[0]->c1.p8 != nullptr, f8b = r[0]->c2.p8 != nullptr;
  Out8 o1, o2;
  for (int i = 0; i < n; ++i) {
    if (f8) o1.w8[i] = &r[i]->c1;
    if (f8b) o2.w8[i] = &r[i]->c2;
  }
  GemmArgs a[2];
  bool fuse = !f8 && gn_fuse_trunk();
  for (int i = 0; i < n; ++i) fuse = fuse && xst[i];
  for (int i = 0; i < n && fuse; ++i) {
    a[i] = conv(A_CONV3, x[i], ldx[i], cin, f.B, Hh, Ww, Hh, Ww, r[i]->c1);
    set_gn_load(h, a[i], xst[i], off[i], cin, 1e-5f, 1, HW);
  }
  fuse = fuse && gn_load_ok(h, a, n);
  if (!fuse) TRY(run_norm(h, f, x, ldx, HW, cin, xst, off, 1e-5f, 1, T, ldc, 0, f8 ? &o1 : nullptr));
  for (int i = 0; i < n; ++i) {
    if (!fuse)
      a[i] = f8 ? conv8(f, i, cin, Hh, Ww, r[i]->c1) : conv(A_CONV3, T[i], cin, cin, f.B, Hh, Ww, Hh, Ww, r[i]->c1);
    a[i].bias = V(h, r[i]->b1);
    a[i].emb = f.l[i].tab + r[i]->emb_off;
    a[i].ld_emb = f.l[i].tab_ld;
    a[i].emb_row = f.emb_row;
    a[i].out = H1[i];
    a[i].ldo = cout;
    a[i].st[0] = stat_tgt(h, s1[i], cout, 0, HW);
  }
  TRY(run_gemm(h, a, f, f8 ? 9.0 * cin / r[0]->c1.ld8 : 1.0));
  for (int i = 0; i < n; ++i) off[i] = r[i]->gn2;
  const bf16* cH1[2] = {H1[0], n > 1 ? H1[1] : nullptr};
  // (a skip ResBlock's conv2 carries the 1x1 skip conv as a K-extension: never a halo plan, so GroupNorm on
  // load would re-plan it onto the tile kernels, measured slower -- it keeps the separate apply)
  fuse = !f8b && gn_fuse_on() && !r[0]->skip;
  for (int i = 0; i < n; ++i) fuse = fuse && s1[i];
  for (int i = 0; i < n; ++i) {
    if (fuse) {  // conv2 reads conv1's output and normalises it on load
      a[i] = conv(A_CONV3, H1[i], cout, cout, f.B, Hh, Ww, Hh, Ww, r[i]->c2);
      set_gn_load(h, a[i], s1[i], off[i], cout, 1e-5f, 1, HW);
    }
  }
  fuse = fuse && gn_load_ok(h, a, n);
  if (!fuse) TRY(run_norm(h, f, cH1, ldh, HW, cout, s1, off, 1e-5f, 1, T, ldh, 0, f8b ? &o2 : nullptr));
  for (int i = 0; i < n; ++i) {
    if (!fuse)
      a[i] = f8b ? conv8(f, i, cout, Hh, Ww, r[i]->c2) : conv(A_CONV3, T[i], cout, cout, f.B, Hh, Ww, Hh, Ww, r[i]->c2);
    a[i].bias = V(h, r[i]->b2);
    if (r[i]->skip) {  // 1x1 skip conv at fp32-accurate weights: x . W_hi + x . W_lo
      a[i].X = x[i];
      a[i].ldx = ldx[i];
      a[i].Kx = 2 * cin;
      a[i].x_wrap = cin;
    } else {
      a[i].res = x[i];
      a[i].ld_res = ldx[i];
      a[i].res_lo = lo_of(h, x[i]);
    }
    a[i].out = out[i];
    a[i].ldo = ldo[i];
    a[i].out_lo = lo_of(h, out[i]);
    set_tg(a[i], otg[i]);
  }
  return run_gemm(h, a, f, f8b ? 9.0 * cout / r[0]->c2.ld8 : 1.0);
}

// SpatialTransformer.forward (attention.py:334-353) + BasicTransformerBlock (:265-274), in place on x[i]
hipError_t transformer(tair_cldm* h, const Fwd& f, const STW* const* st, bf16* const* x, const int* ldx,
                       double* const* xst, const Tg* otg, int lvl) {
  const int HW = h->lev_h[lvl] * h->lev_w[lvl];
  const int C = st[0]->C, heads = st[0]->heads;
  const int M = f.B * HW;
  const int n = f.n;
  const float scale = 1.f / std::sqrt((float)h->cfg.head_channels);
  int off[2], ldC[2] = {C, C};
  bf16 *T[2], *X0[2];
  const bf16 *cT[2], *cX0[2];
  for (int i = 0; i < n; ++i) {
    off[i] = st[i]->gn;
    T[i] = f.l[i].w->T;
    X0[i] = f.l[i].w->X0;
    cT[i] = T[i];
    cX0[i] = X0[i];
  }
  const bf16* cx[2] = {x[0], n > 1 ? x[1] : nullptr};
  // fp8 (configs[4]): proj_in on the GroupNorm's e4m3 output, the three LayerNorm-fed linears on an e4m3
  // LayerNorm output; kf = logical / padded K
  const bool f8 = st[0]->qkv.p8 != nullptr;
  const bool f8in = st[0]->pin.p8 != nullptr;
  Out8 o8;
  for (int i = 0; i < n && f8in; ++i) o8.w8[i] = &st[i]->pin;
  GemmArgs a[2];
  // (proj_in keeps the separate GroupNorm apply: the product plans GroupNorm on load into halo convs only)
  TRY(run_norm(h, f, cx, ldx, HW, C, xst, off, 1e-6f, 0, T, ldC, 0, f8in ? &o8 : nullptr));
  const double kf = f8 ? (double)C / st[0]->qkv.ld8 : 1.0;
  // bf16: LayerNorms folded into their consumers when every lane has the folded
  // weights, statistics slots are free and the producers' plans can emit row statistics
  double* ls[3][2] = {};
  bool fold = !f8;
  for (int i = 0; i < n; ++i) fold = fold && st[i]->fold;
  if (fold) {
    GemmArgs pa = dense(X0[0], C, M, st[0]->pin);
    pa.tile_sem = f.l[0].w->gemm_tickets;
    fold = gemm_rowstats_ok(pa);
  }
  for (int j = 0; j < 3 && fold; ++j)
    for (int i = 0; i < n && fold; ++i) fold = (ls[j][i] = new_lnstat(h, M)) != nullptr;
  // the weights of a folded transformer hold W diag(gamma) (finalize): running it unfolded would apply gamma twice
  // (round 5's TAIR_SK_WIDE drift: a wide proj_in plan turned the fold off here, v rel-L2 2.5e-3 -> 6.4e-3)
  if (!f8 && !fold && !h->dry)
    for (int i = 0; i < n; ++i)
      if (st[i]->fold) {
        set_error("transformer: LayerNorm folded into the weights but no row-statistics plan / slot for M=%d C=%d", M, C);
        return hipErrorInvalidValue;
      }
  for (int i = 0; i < n; ++i) {
    a[i] = f8in ? dense8gn(f, i, M, st[i]->pin) : dense(T[i], C, M, st[i]->pin);
    a[i].bias = V(h, st[i]->pinb);
    a[i].out = X0[i];
    a[i].ldo = C;
    if (fold) a[i].rst = ls[0][i];
  }
  TRY(run_gemm(h, a, f, f8in ? (double)C / st[0]->pin.ld8 : 1.0));
  // self-attention
  auto ln_lin = [&](int ln_off_sel, const Weight STW::*wsel) -> hipError_t {
    for (int i = 0; i < n; ++i) off[i] = ln_off_sel == 1 ? st[i]->ln1 : ln_off_sel == 2 ? st[i]->ln2 : st[i]->ln3;
    if (fold) {  // raw X0 against W diag(gamma); mean / rstd / beta in the epilogue
      for (int i = 0; i < n; ++i) {
        const STW& w = *st[i];
        a[i] = dense(X0[i], C, M, w.*wsel);
        a[i].lnst = ls[ln_off_sel - 1][i];
        a[i].lncs = V(h, ln_off_sel == 1 ? w.cs_qkv : ln_off_sel == 2 ? w.cs_q2 : w.cs_ff1);
        a[i].bias = V(h, ln_off_sel == 1 ? w.fb_qkv : ln_off_sel == 2 ? w.fb_q2 : w.fb_ff1);
        a[i].ln_c = (float)C;
        a[i].ln_eps = 1e-5f;
      }
      return hipSuccess;
    }
    if (f8) {
      TRY(run_ln8(h, f, cX0, M, C, off));
      for (int i = 0; i < n; ++i) a[i] = dense8(f, i, M, st[i]->*wsel);
    } else {
      TRY(run_ln(h, f, cX0, M, C, off, T));
      for (int i = 0; i < n; ++i) a[i] = dense(T[i], C, M, st[i]->*wsel);
    }
    return hipSuccess;
  };
  TRY(ln_lin(1, &STW::qkv));
  for (int i = 0; i < n; ++i) {
    a[i].out = f.l[i].w->QKV;
    a[i].ldo = 3 * C;
  }
  TRY(run_gemm(h, a, f, kf));
  {
    AttnArgs g[2];
    for (int i = 0; i < n; ++i) {
      const tair_cldm::Scratch& w = *f.l[i].w;
      g[i] = AttnArgs{w.QKV, 3 * C, w.QKV + C, 3 * C, w.QKV + 2 * C, 3 * C, w.A, C, HW,
                      w.partial, w.partial_cap * sizeof(float), w.attn_tickets, ATTN_TICKETS};
    }
    const double fl = 4.0 * n * f.B * HW * (double)HW * C;
    const double qkvo = 4.0 * n * f.B * HW * C * 2;  // q, k, v, o: [B][S][C] bf16 each
    TRY(launch(h, 1, fl, f.s, [&] { return attention_grouped(g, n, f.B, heads, HW, HW, scale, f.s); },
               "attn self S=" + std::to_string(HW) + " heads=" + std::to_string(heads) + " B=" + std::to_string(f.B),
               qkvo, "attn"));
  }
  for (int i = 0; i < n; ++i) {
    a[i] = dense(f.l[i].w->A, C, M, st[i]->o1);
    a[i].bias = V(h, st[i]->o1b);
    a[i].res = X0[i];
    a[i].ld_res = C;
    a[i].out = X0[i];
    a[i].ldo = C;
    if (fold) a[i].rst = ls[1][i];
  }
  TRY(run_gemm(h, a, f));
  // cross-attention on the cached K/V of c_txt
  TRY(ln_lin(2, &STW::q2));
  for (int i = 0; i < n; ++i) {
    a[i].out = f.l[i].w->QKV;
    a[i].ldo = C;
  }
  TRY(run_gemm(h, a, f, kf));
  {
    const int L = h->cfg.context_len;
    AttnArgs g[2];
    for (int i = 0; i < n; ++i) {
      const tair_cldm::Scratch& w = *f.l[i].w;
      g[i] = AttnArgs{w.QKV, C, st[i]->kvcache, 2 * C, st[i]->kvcache + C, 2 * C, w.A, C, f.ctx_bstride,
                      w.partial, w.partial_cap * sizeof(float), w.attn_tickets, ATTN_TICKETS};
    }
    const double fl = 4.0 * n * f.B * HW * (double)L * C;
    // q, o: [B][S][C]; the cached K / V of the context: [L][C] each per prompt (shared over the batch when
    // ctx_bstride is 0)
    const double kv = 2.0 * L * C * 2 * (f.ctx_bstride ? f.B : 1);
    const double qo = 2.0 * f.B * HW * C * 2;
    TRY(launch(h, 1, fl, f.s, [&] { return attention_grouped(g, n, f.B, heads, HW, L, scale, f.s); },
               "attn cross S=" + std::to_string(HW) + " heads=" + std::to_string(heads) + " B=" + std::to_string(f.B),
               n * (kv + qo), "attn"));
  }
  for (int i = 0; i < n; ++i) {
    a[i] = dense(f.l[i].w->A, C, M, st[i]->o2);
    a[i].bias = V(h, st[i]->o2b);
    a[i].res = X0[i];
    a[i].ld_res = C;
    a[i].out = X0[i];
    a[i].ldo = C;
    if (fold) a[i].rst = ls[2][i];
  }
  TRY(run_gemm(h, a, f));
  // GEGLU feed-forward
  TRY(ln_lin(3, &STW::ff1));
  for (int i = 0; i < n; ++i) {  // ff1 rows interleaved at load: the epilogue emits x * gelu(gate)
    if (!fold) a[i].bias = V(h, st[i]->ff1b);  // (folded: bias + W beta, set by ln_lin)
    a[i].act = 2;
    a[i].out = f.l[i].w->F;
    a[i].ldo = 4 * C;
  }
  TRY(run_gemm(h, a, f, kf));
  for (int i = 0; i < n; ++i) {
    a[i] = dense(f.l[i].w->F, 4 * C, M, st[i]->ff2);
    a[i].bias = V(h, st[i]->ff2b);
    a[i].res = X0[i];
    a[i].ld_res = C;
    a[i].out = X0[i];
    a[i].ldo = C;
  }
  TRY(run_gemm(h, a, f));
  // proj_out + residual (in place on x)
  for (int i = 0; i < n; ++i) {
    a[i] = dense(X0[i], C, M, st[i]->pout);
    a[i].bias = V(h, st[i]->poutb);
    a[i].res = x[i];
    a[i].ld_res = ldx[i];
    a[i].res_lo = lo_of(h, x[i]);
    a[i].out = x[i];
    a[i].ldo = ldx[i];
    a[i].out_lo = lo_of(h, x[i]);
    set_tg(a[i], otg[i]);
  }
  return run_gemm(h, a, f);
}

Fwd make_fwd(tair_cldm* h, hipStream_t s, int B, const int* emb_row, int ctx_bstride, bool control) {
  Fwd f{};
  f.s = s;
  f.B = B;
  f.emb_row = emb_row;
  f.ctx_bstride = ctx_bstride;
  f.n = control ? 2 : 1;
  f.l[0] = Lane{&h->ws[0], h->tab_u, h->unet.emb_total, 0};
  f.l[1] = Lane{&h->ws[1], h->tab_c, h->cn.emb_total, 1};
  return f;
}
Fwd lane_fwd(const Fwd& f, int i) {  // one lane alone (non-grouped launches)
  Fwd g = f;
  g.n = 1;
  g.l[0] = f.l[i];
  return g;
}
Fwd main_fwd(tair_cldm* h, hipStream_t s, int B) { return make_fwd(h, s, B, h->rows_iota, 0, false); }

// cross-attention K/V caches for every SpatialTransformer of a net (attention.py:78-81 hoisted:
// they depend only on c_txt)
hipError_t kv_caches(tair_cldm* h, Net& net, int ctx_rows, hipStream_t s) {
  const Fwd f = main_fwd(h, s, 1);
  auto one = [&](STW& st) -> hipError_t {
    GemmArgs a = dense(h->ctx_bf, h->cfg.context_dim, ctx_rows, st.kv2);
    a.out = st.kvcache;
    a.ldo = 2 * st.C;
    return run_gemm1(h, a, f);
  };
  for (auto& b : net.enc)
    if (b.has_st) TRY(one(b.st));
  TRY(one(net.midst));
  for (auto& d : net.dec)
    if (d.has_st) TRY(one(d.st));
  return hipSuccess;
}

// time_embed MLP + all emb_layers for `rows` timesteps (util.py:128-148, unet.py:475-480,
// 166-172): tab[row][emb_off + n] = Linear(SiLU(time_embed(sinusoid(t_row))))
hipError_t time_tables(tair_cldm* h, Net& net, const int64_t* t, int rows, float* tab, hipStream_t s) {
  const int mc = h->cfg.model_channels;
  const Fwd f = main_fwd(h, s, 1);
  TRY(launch(h, 4, 0, s, [&] { return timestep_sinusoid(t, rows, mc, h->sinus, s); }));
  TRY(launch(h, 4, 0, s, [&] { return f32_to_bf16(h->sinus, rows * mc, h->temb_a, s); }));
  GemmArgs a = dense(h->temb_a, mc, rows, net.te0);
  a.bias = V(h, net.te0b);
  a.act = 1;
  a.out = h->temb_b;
  a.ldo = h->time_dim;
  TRY(run_gemm1(h, a, f));
  a = dense(h->temb_b, h->time_dim, rows, net.te2);
  a.bias = V(h, net.te2b);
  a.act = 1;  // emb is only consumed as SiLU(emb) by every emb_layers (unet.py:166-172)
  a.out = h->temb_a;
  a.ldo = h->time_dim;
  TRY(run_gemm1(h, a, f));
  a = dense(h->temb_a, h->time_dim, rows, net.emb);
  a.bias = V(h, net.embb);
  a.out = tab;
  a.ldo = net.emb_total;
  a.out_f32 = 1;
  return run_gemm1(h, a, f);
}

tair_cldm::Cat& cat_of(tair_cldm* h, int j) { return h->cat[j]; }

// Encoder + middle of the networks on f's lanes (UNet and/or ControlNet, controlnet.py:323-337).
// With both on one Fwd they run in lockstep as grouped launches.  UNet block i writes the right
// half of concat buffer 11-i, ControlNet block i its own cn_out[i]; middles: UNet -> cat0 left half,
// ControlNet -> cn_mid.  GroupNorm statistics: every block output that a GroupNorm consumes next
// gets a slot; dec_st[j] are the slots of the decoder's concat inputs, fed from here only when no
// control residual will be added to the skip (skip_stats) -- otherwise the zero convs feed them.
hipError_t enc_mid(tair_cldm* h, const Fwd& f, double* const* dec_st, bool skip_stats) {
  const int nenc = (int)h->unet.enc.size();  // 12
  const int lastlvl = h->nlev - 1;
  const int n = f.n;
  auto netp = [&](int k) -> Net& { return f.l[k].net == 0 ? h->unet : h->cn; };
  double* cur[2] = {nullptr, nullptr};  // statistics of the current block input
  for (int i = 0; i < nenc; ++i) {
    const EncBlock* b[2];
    bf16* out[2];
    int ldo[2];
    const bf16* in[2] = {nullptr, nullptr};
    int ldi[2] = {0, 0};
    Tg tg[2];                           // targets of the block's final output
    double* nxt[2] = {nullptr, nullptr};
    const bool next_gn = (i + 1 == nenc) || h->unet.enc[i + 1].kind == BK_RES;  // mid1 or a ResBlock
    for (int k = 0; k < n; ++k) {
      b[k] = &netp(k).enc[i];
      const int lvl = b[k]->level;
      const int HWl = h->lev_h[lvl] * h->lev_w[lvl];
      const int Cb = b[k]->kind == BK_RES ? b[k]->res.cout : b[k]->conv.cout;
      if (next_gn) nxt[k] = new_stat(h);
      add_tgt(tg[k], stat_tgt(h, nxt[k], Cb, 0, HWl));
      if (f.l[k].net == 0) {
        tair_cldm::Cat& dst = cat_of(h, nenc - 1 - i);
        out[k] = dst.p + dst.ch;
        ldo[k] = dst.ch + dst.cs;
        if (skip_stats) add_tgt(tg[k], stat_tgt(h, dec_st[nenc - 1 - i], dst.ch + dst.cs, dst.ch, HWl));
        if (i > 0) {
          tair_cldm::Cat& src = cat_of(h, nenc - i);
          in[k] = src.p + src.ch;
          ldi[k] = src.ch + src.cs;
        }
      } else {
        out[k] = h->cn_out[i];
        ldo[k] = Cb;
        if (i > 0) {
          const EncBlock& pb = h->cn.enc[i - 1];
          in[k] = h->cn_out[i - 1];
          ldi[k] = pb.kind == BK_RES ? pb.res.cout : pb.conv.cout;
        }
      }
    }
    const int lvl = b[0]->level;
    if (b[0]->kind == BK_CONVIN) {  // 4- vs 8-channel inputs: different FLOP counts, one launch per network
      for (int k = 0; k < n; ++k) {
        const bool cn = f.l[k].net == 1;
        // (hi, lo, hi) planes of 4 / 8 input channels, zero-padded to one 64-channel chunk (build_conv3 pad64)
        GemmArgs a = conv(A_CONV3, cn ? h->in_c : h->in_u, CONVIN_LD, CONVIN_LD, f.B, h->lev_h[0], h->lev_w[0],
                          h->lev_h[0], h->lev_w[0], b[k]->conv.w);
        a.flop_k = 9 * (cn ? h->cfg.in_channels + h->cfg.hint_channels : h->cfg.in_channels);
        a.bias = V(h, b[k]->conv.b);
        a.out = out[k];
        a.ldo = ldo[k];
        a.out_lo = lo_of(h, out[k]);
        set_tg(a, tg[k]);
        TRY(run_gemm1(h, a, lane_fwd(f, k)));
      }
    } else if (b[0]->kind == BK_DOWN) {
      GemmArgs a[2];
      for (int k = 0; k < n; ++k) {
        a[k] = conv(A_CONV3_S2, in[k], ldi[k], b[k]->conv.cin, f.B, h->lev_h[lvl - 1], h->lev_w[lvl - 1],
                    h->lev_h[lvl], h->lev_w[lvl], b[k]->conv.w);
        a[k].bias = V(h, b[k]->conv.b);
        a[k].out = out[k];
        a[k].ldo = ldo[k];
        a[k].out_lo = lo_of(h, out[k]);
        set_tg(a[k], tg[k]);
      }
      TRY(run_gemm(h, a, f));
    } else {
      const ResW* r[2] = {&b[0]->res, n > 1 ? &b[1]->res : nullptr};
      if (b[0]->has_st) {
        const int HWl = h->lev_h[lvl] * h->lev_w[lvl];
        double* sst[2] = {nullptr, nullptr};
        Tg rtg[2];
        for (int k = 0; k < n; ++k) {
          sst[k] = new_stat(h);
          add_tgt(rtg[k], stat_tgt(h, sst[k], r[k]->cout, 0, HWl));
        }
        TRY(resblock(h, f, r, in, ldi, cur, out, ldo, rtg, lvl));
        const STW* st[2] = {&b[0]->st, n > 1 ? &b[1]->st : nullptr};
        TRY(transformer(h, f, st, out, ldo, sst, tg, lvl));
      } else {
        TRY(resblock(h, f, r, in, ldi, cur, out, ldo, tg, lvl));
      }
    }
    cur[0] = nxt[0];
    cur[1] = nxt[1];
  }
  tair_cldm::Cat& c0 = cat_of(h, 0);
  const int ld0 = c0.ch + c0.cs;
  const int C = h->unet.mid1.cout;
  const int HWm = h->lev_h[lastlvl] * h->lev_w[lastlvl];
  const ResW* m1[2];
  const ResW* m2[2];
  const STW* ms[2];
  const bf16* in[2];
  int ldi[2], ldr[2] = {C, C}, ldo[2];
  bf16 *R[2], *out[2];
  const bf16* cR[2];
  double *sR[2] = {nullptr, nullptr}, *sR2[2] = {nullptr, nullptr};
  Tg tR[2], tR2[2], tout[2];
  for (int k = 0; k < n; ++k) {
    Net& net = netp(k);
    m1[k] = &net.mid1;
    m2[k] = &net.mid2;
    ms[k] = &net.midst;
    const bool u = f.l[k].net == 0;
    in[k] = u ? c0.p + c0.ch : h->cn_out[nenc - 1];
    ldi[k] = u ? ld0 : C;
    R[k] = f.l[k].w->R;
    cR[k] = R[k];
    out[k] = u ? c0.p : h->cn_mid;
    ldo[k] = u ? ld0 : C;
    sR[k] = new_stat(h);
    sR2[k] = new_stat(h);
    add_tgt(tR[k], stat_tgt(h, sR[k], C, 0, HWm));
    add_tgt(tR2[k], stat_tgt(h, sR2[k], C, 0, HWm));
    if (u && skip_stats) add_tgt(tout[k], stat_tgt(h, dec_st[0], ld0, 0, HWm));
  }
  TRY(resblock(h, f, m1, in, ldi, cur, R, ldr, tR, lastlvl));
  TRY(transformer(h, f, ms, R, ldr, sR, tR2, lastlvl));
  return resblock(h, f, m2, cR, ldr, sR2, out, ldo, tout, lastlvl);
}

// The ControlNet + UNet body on prepared inputs (in_u, in_c, kv caches, emb tables): encoder +
// middle of both networks, the zero convs, then the UNet decoder alone, in three stages (body_begin,
// enc_mid, body_dec).  The ControlNet encoder runs on a forked stream beside the UNet's (the step graph and
// eager forwards); the dry-run FLOP count groups both networks' layers per launch on one stream.  Measured
// alternatives (profiles/r06_step_schedule_ab.txt): grouped launches on one stream, and the
// stages captured as separate single-stream graphs (the runtime's packet-batched launch path: host 0.1 instead
// of 4.4 ms per B = 1 step) with the encoders fully or partly overlapped -- all slower on the GPU.
struct BodyState {
  double* dec_st[16] = {};
  double* out_st = nullptr;
};

hipError_t body_begin(tair_cldm* h, const Fwd& f, BodyState& bs) {
  const int ndec = (int)h->unet.dec.size();
  // statistics slots of this forward: zeroed once, before either network starts
  h->gst_next = 0;
  if (h->gn_fused && !h->dry)
    TRY(zero_bytes(h->gst, (size_t)h->gst_slots * STAT_REPL * h->gst_rs * sizeof(double), f.s));
  h->lst_next = 0;
  if (h->lst && !h->dry) TRY(zero_bytes(h->lst, 2 * (size_t)f.B * h->ln_slot_rows / h->cfg.max_batch * sizeof(double) +
                                                     16 * 256 * sizeof(double), f.s));
  for (int j = 0; j < ndec; ++j) bs.dec_st[j] = new_stat(h);
  bs.out_st = new_stat(h);
  return hipSuccess;
}

// zero convs: 0 all before the decoder on f.s, 1 on the side stream cstream in the decoder's consumption order
// (event per skip)
hipError_t body_dec(tair_cldm* h, const Fwd& f, bool control, const float* scales, BodyState& bs, int zc_mode);

hipError_t body(tair_cldm* h, const Fwd& f, bool control, const float* scales) {
  const Fwd fu = lane_fwd(f, 0);
  BodyState bs;
  TRY(body_begin(h, f, bs));
  const bool fork = control && !h->dry;
  if (fork) {
    Fwd fc = lane_fwd(f, 1);
    fc.s = h->cstream;
    TRY(hipEventRecord(h->ev_fork, f.s));
    TRY(hipStreamWaitEvent(fc.s, h->ev_fork, 0));
    TRY(enc_mid(h, fc, bs.dec_st, !control));
    TRY(hipEventRecord(h->ev_join, fc.s));
    TRY(enc_mid(h, fu, bs.dec_st, !control));
    TRY(hipStreamWaitEvent(f.s, h->ev_join, 0));
  } else {
    TRY(enc_mid(h, control ? f : fu, bs.dec_st, !control));
  }
  return body_dec(h, f, control, scales, bs, control && !h->dry ? 1 : 0);
}

hipError_t body_dec(tair_cldm* h, const Fwd& f, bool control, const float* scales, BodyState& bs, int zc_mode) {
  const int nenc = (int)h->unet.enc.size();  // 12
  const int ndec = (int)h->unet.dec.size();
  const int lastlvl = h->nlev - 1;
  const Fwd fu = lane_fwd(f, 0);
  double* const* dec_st = bs.dec_st;
  double* out_st = bs.out_st;
  // ---- the zero convs accumulate scale*(W h + b) in place into the skip slots.  They run on a side
  // stream in the decoder's consumption order (middle first, then encoder block 11, 10, ...), and
  // decoder block j waits only for the zero conv of its own skip (block 11-j): the 13 launches
  // overlap the decoder instead of preceding it.  Each also produces the GroupNorm statistics of
  // the skip half (or, for the middle, the left half) of the decoder's concat input.
  const bool zc_side = control && zc_mode == 1;
  Fwd fz = lane_fwd(f, 1);  // ControlNet scratch: idle now, and disjoint from the decoder's
  if (zc_side) {
    fz.s = h->cstream;
    TRY(hipEventRecord(h->ev_fork, f.s));
    TRY(hipStreamWaitEvent(fz.s, h->ev_fork, 0));
  }
  // zero conv of ControlNet output i (i = nenc: middle_block_out) into the decoder's skip slot
  auto zero_conv = [&](int i) -> hipError_t {
    if (i == nenc) {
      const int C = h->cn.mid1.cout;
      tair_cldm::Cat& c0 = cat_of(h, 0);
      const int HWm = h->lev_h[lastlvl] * h->lev_w[lastlvl];
      GemmArgs z = dense(h->cn_mid, C, f.B * HWm, h->cn.mid_out.w);
      z.bias = V(h, h->cn.mid_out.b);
      z.alpha = scales ? scales[nenc] : 1.f;
      z.scale_bias = 1;
      z.res = c0.p;
      z.ld_res = c0.ch + c0.cs;
      z.res_lo = lo_of(h, c0.p);
      z.out = c0.p;
      z.ldo = c0.ch + c0.cs;
      z.out_lo = z.res_lo;
      z.st[0] = stat_tgt(h, dec_st[0], c0.ch + c0.cs, 0, HWm);
      return run_gemm1(h, z, fz);
    }
    const EncBlock& b = h->cn.enc[i];
    const int lvl = b.level;
    const int HWl = h->lev_h[lvl] * h->lev_w[lvl];
    const int Cb = (b.kind == BK_RES) ? b.res.cout : b.conv.cout;
    tair_cldm::Cat& dst = cat_of(h, nenc - 1 - i);
    GemmArgs z = dense(h->cn_out[i], Cb, f.B * HWl, b.zero.w);
    z.bias = V(h, b.zero.b);
    z.alpha = scales ? scales[i] : 1.f;
    z.scale_bias = 1;
    z.res = dst.p + dst.ch;
    z.ld_res = dst.ch + dst.cs;
    z.res_lo = lo_of(h, dst.p);
    z.out = dst.p + dst.ch;
    z.ldo = dst.ch + dst.cs;
    z.out_lo = z.res_lo;
    z.st[0] = stat_tgt(h, dec_st[nenc - 1 - i], dst.ch + dst.cs, dst.ch, HWl);
    return run_gemm1(h, z, fz);
  };
  if (control) {
    TRY(zero_conv(nenc));  // ordered before ev_zc[nenc - 1] on the side stream
    for (int i = nenc - 1; i >= 0; --i) {
      TRY(zero_conv(i));
      if (zc_side) TRY(hipEventRecord(h->ev_zc[i], fz.s));
    }
  }
  // ---- UNet decoder
  for (int j = 0; j < ndec; ++j) {
    const DecBlock& d = h->unet.dec[j];
    tair_cldm::Cat& src = cat_of(h, j);
    if (zc_side) TRY(hipStreamWaitEvent(f.s, h->ev_zc[nenc - 1 - j], 0));
    const int lvl = d.level;
    const int HWl = h->lev_h[lvl] * h->lev_w[lvl];
    bf16* out;
    int ldo;
    Tg fin;  // statistics targets of the block's final output
    if (j + 1 < ndec) {
      tair_cldm::Cat& nxt = cat_of(h, j + 1);
      out = nxt.p;
      ldo = nxt.ch + nxt.cs;
      const int HWn = h->lev_h[nxt.level] * h->lev_w[nxt.level];
      add_tgt(fin, stat_tgt(h, dec_st[j + 1], nxt.ch + nxt.cs, 0, HWn));
    } else {
      out = h->Dout;
      ldo = d.ch_out;
      add_tgt(fin, stat_tgt(h, out_st, d.ch_out, 0, h->lev_h[0] * h->lev_w[0]));
    }
    bf16* rdst = d.has_up ? fu.l[0].w->R : out;
    const int rld = d.has_up ? d.res.cout : ldo;
    const ResW* r[1] = {&d.res};
    const bf16* in[1] = {src.p};
    const int ldi[1] = {src.ch + src.cs};
    double* xst[1] = {dec_st[j]};
    Tg rtg[1];
    double* sst[1] = {nullptr};
    if (d.has_st) {
      sst[0] = new_stat(h);
      add_tgt(rtg[0], stat_tgt(h, sst[0], d.res.cout, 0, HWl));
    } else if (!d.has_up) {
      rtg[0] = fin;
    }
    TRY(resblock(h, fu, r, in, ldi, xst, &rdst, &rld, rtg, lvl));
    if (d.has_st) {
      const STW* st[1] = {&d.st};
      Tg stg[1];
      if (!d.has_up) stg[0] = fin;
      TRY(transformer(h, fu, st, &rdst, &rld, sst, stg, lvl));
    }
    if (d.has_up) {
      GemmArgs a = conv(A_CONV3_UP, fu.l[0].w->R, d.res.cout, d.res.cout, f.B, h->lev_h[lvl], h->lev_w[lvl],
                        h->lev_h[lvl - 1], h->lev_w[lvl - 1], d.up.w);
      a.bias = V(h, d.up.b);
      a.out = out;
      a.ldo = ldo;
      a.out_lo = lo_of(h, out);
      set_tg(a, fin);
      TRY(run_gemm1(h, a, fu));
    }
  }
  // ---- out: GN + SiLU + conv 320 -> 4 (fp32 v)
  {
    const int HW = h->lev_h[0] * h->lev_w[0];
    const int C = h->cfg.model_channels;
    const bf16* x[1] = {h->Dout};
    const int ld[1] = {C};
    const int off[1] = {h->unet.out_gn};
    bf16* T[1] = {fu.l[0].w->T};
    double* xs[1] = {out_st};
    const int ld3[1] = {3 * C};
    // GN + SiLU written as (hi, lo, hi) planes and the 320 -> 4 conv over them: v at fp32 accuracy
    // (the last layer's bf16 rounding alone was ~1.7e-3 of v's error)
    TRY(run_norm(h, fu, x, ld, HW, C, xs, off, 1e-5f, 1, T, ld3, 1));
    GemmArgs a = conv(A_CONV3, fu.l[0].w->T, 3 * C, 3 * C, f.B, h->lev_h[0], h->lev_w[0], h->lev_h[0], h->lev_w[0],
                      h->unet.out_conv.w);
    a.kplanes = 3;
    a.bias = V(h, h->unet.out_conv.b);
    a.out = h->v_out;
    a.ldo = h->cfg.out_channels;
    a.out_f32 = 1;
    TRY(run_gemm1(h, a, fu));
  }
  return hipSuccess;
}

hipError_t export_feats(tair_cldm* h, int B, float* const feats[4], hipStream_t s) {
  if (!feats) return hipSuccess;
  const int idxs[4] = {2, 5, 8, 11};
  const int ndec = (int)h->unet.dec.size();
  for (int k = 0; k < 4; ++k) {
    if (!feats[k]) continue;
    const int j = idxs[k];
    if (j >= ndec) continue;
    const DecBlock& d = h->unet.dec[j];
    const bf16* src;
    int ld, lvl;
    if (j + 1 < ndec) {
      tair_cldm::Cat& nxt = cat_of(h, j + 1);
      src = nxt.p;
      ld = nxt.ch + nxt.cs;
      lvl = nxt.level;
    } else {
      src = h->Dout;
      ld = d.ch_out;
      lvl = 0;
    }
    const int HW = h->lev_h[lvl] * h->lev_w[lvl];
    TRY(launch(h, 4, 0, s, [&] { return nhwc_bf16_to_nchw_f32(src, ld, B, d.ch_out, HW, feats[k], s); }));
  }
  return hipSuccess;
}

// NCHW fp32 [B, C, HW] -> NHWC bf16 (hi, lo, hi) planes: y[p][c_off + c], [plane + c_off + c], [2 plane + ...]
__global__ void nchw_to_split_kernel(const float* x, int B, int C, int HW, bf16* y, int ldy, int c_off, int plane) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)B * C * HW) return;
  const long b = i / ((long)C * HW);
  const long rem = i - b * C * HW;
  const int p = (int)(rem % HW), c = (int)(rem / HW);
  const float v = x[i];
  const bf16 hi = (bf16)v, lo = (bf16)(v - (float)hi);
  bf16* o = y + (size_t)(b * HW + p) * ldy + c_off + c;
  o[0] = hi;
  o[plane] = lo;
  o[2 * plane] = hi;
}
hipError_t nchw_split(const float* x, int B, int C, int HW, bf16* y, int ldy, int c_off, int plane, hipStream_t s) {
  const long n = (long)B * C * HW;
  hipLaunchKernelGGL(nchw_to_split_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, B, C, HW, y, ldy, c_off, plane);
  return hipGetLastError();
}

// conv_in inputs as (hi, lo, hi) bf16 planes in 64-channel rows: in_u [M][CONVIN_LD] (channels plane * ci + c),
// in_c [M][CONVIN_LD] (planes of [x, hint]: plane * (ci + hc) + c); the pad channels stay zero
hipError_t prepare_inputs(tair_cldm* h, int B, const float* x, const float* c_img, hipStream_t s) {
  const int HW = h->lev_h[0] * h->lev_w[0];
  const int ci = h->cfg.in_channels, hc = h->cfg.hint_channels;
  TRY(launch(h, 4, 0, s, [&] { return nchw_split(x, B, ci, HW, h->in_u, CONVIN_LD, 0, ci, s); }));
  if (c_img) {
    TRY(launch(h, 4, 0, s, [&] { return nchw_split(x, B, ci, HW, h->in_c, CONVIN_LD, 0, ci + hc, s); }));
    TRY(launch(h, 4, 0, s, [&] { return nchw_split(c_img, B, hc, HW, h->in_c, CONVIN_LD, ci, ci + hc, s); }));
  }
  return hipSuccess;
}

hipError_t prepare_ctx(tair_cldm* h, const float* c_txt, int cb, hipStream_t s) {
  const int rows = cb * h->cfg.context_len;
  TRY(launch(h, 4, 0, s, [&] { return f32_to_bf16(c_txt, rows * h->cfg.context_dim, h->ctx_bf, s); }));
  TRY(kv_caches(h, h->unet, rows, s));
  TRY(kv_caches(h, h->cn, rows, s));
  return hipSuccess;
}

}  // namespace

// ==========================================================================================
// C ABI
// ==========================================================================================
extern "C" {

const char* tair_last_error(void) { return tair::g_err; }
const char* tair_version(void) { return "tair_amd 0.1 (gfx950)"; }

int tair_cldm_default_cfg(tair_cldm_cfg* c) {
  if (!c) return TAIR_ERR_ARG;
  memset(c, 0, sizeof(*c));
  c->model_channels = 320;
  c->num_levels = 4;
  c->channel_mult[0] = 1;
  c->channel_mult[1] = 2;
  c->channel_mult[2] = 4;
  c->channel_mult[3] = 4;
  c->num_res_blocks = 2;
  c->num_attention_ds = 3;
  c->attention_ds[0] = 4;
  c->attention_ds[1] = 2;
  c->attention_ds[2] = 1;
  c->head_channels = 64;
  c->context_dim = 1024;
  c->context_len = 77;
  c->in_channels = 4;
  c->hint_channels = 4;
  c->out_channels = 4;
  c->groups = 32;
  c->max_batch = 1;
  c->latent_h = 64;
  c->latent_w = 64;
  c->compute_dtype = TAIR_DTYPE_BF16;
  return TAIR_OK;
}

static hipError_t create_events(hipEvent_t* ev, int n) {
  for (int i = 0; i < n; ++i) TRY(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  return hipSuccess;
}

static int fail_hip(hipError_t e) {
  if (tair::g_err[0] == 0) tair::set_error("HIP error: %s", hipGetErrorString(e));
  return TAIR_ERR_HIP;
}

int tair_cldm_create(const tair_cldm_cfg* cfg, tair_cldm** out) {
  tair::g_err[0] = 0;
  if (!cfg || !out) {
    set_error("create: null argument");
    return TAIR_ERR_ARG;
  }
  const int mc = cfg->model_channels;
  if (mc % 64 || cfg->num_levels < 1 || cfg->num_levels > 8 || cfg->max_batch < 1 || cfg->head_channels != 64 ||
      cfg->groups < 1 || cfg->context_dim % 64 || cfg->latent_h % (1 << (cfg->num_levels - 1)) ||
      cfg->latent_w % (1 << (cfg->num_levels - 1))) {
    set_error("create: unsupported configuration (model_channels %% 64, head_channels == 64, latent divisible)");
    return TAIR_ERR_ARG;
  }
  if (cfg->compute_dtype != TAIR_DTYPE_BF16 && cfg->compute_dtype != TAIR_DTYPE_FP8) {
    set_error("create: compute_dtype %d (TAIR_DTYPE_BF16 or TAIR_DTYPE_FP8)", cfg->compute_dtype);
    return TAIR_ERR_ARG;
  }
  auto h = new tair_cldm();
  h->cfg = *cfg;
  h->nlev = cfg->num_levels;
  {
    const char* lf = getenv("TAIR_LN_FOLD");
    h->ln_fold = cfg->compute_dtype != TAIR_DTYPE_FP8 && !(lf && atoi(lf) == 0);
  }
  h->time_dim = 4 * mc;
  for (int l = 0; l < h->nlev; ++l) {
    h->lev_ch.push_back(mc * cfg->channel_mult[l]);
    h->lev_h.push_back(cfg->latent_h >> l);
    h->lev_w.push_back(cfg->latent_w >> l);
  }
  // ---- networks
  build_time(h, h->unet, "unet");
  build_encoder(h, h->unet, "unet", cfg->in_channels, false);
  build_decoder(h, h->unet, "unet");
  finish_emb(h, h->unet, "unet", true);
  build_time(h, h->cn, "controlnet");
  build_encoder(h, h->cn, "controlnet", cfg->in_channels + cfg->hint_channels, true);
  finish_emb(h, h->cn, "controlnet", false);
  // ---- workspace (sized for max_batch)
  const size_t B = cfg->max_batch;
  size_t t_el = 0, h1_el = 0, x0_el = 0, g_el = 0, cn_el = 0, r_el = 0;
  int cmax = 0;
  auto upd = [](size_t& v, size_t x) { v = x > v ? x : v; };
  size_t t8_bytes = 0, t8_rows = 0;
  auto res_sz = [&](const ResW& r, int lvl) {
    const size_t hw = (size_t)h->lev_h[lvl] * h->lev_w[lvl];
    if (r.c1.p8 || r.c2.p8) upd(t8_bytes, hw * std::max(r.cin, r.cout));  // e4m3 conv inputs [pixel][C] bytes
    upd(t_el, hw * r.cin);
    upd(t_el, hw * r.cout);
    upd(h1_el, hw * r.cout);
    cmax = std::max(cmax, std::max(r.cin, r.cout));
  };
  auto st_sz = [&](const STW& w, int lvl) {
    const size_t hw = (size_t)h->lev_h[lvl] * h->lev_w[lvl];
    upd(t8_bytes, hw * round_up(w.C, 128));
    upd(t8_rows, hw);
    upd(t_el, hw * w.C);
    upd(x0_el, hw * w.C);
    upd(g_el, hw * w.C);
  };
  for (auto* net : {&h->unet, &h->cn}) {
    for (auto& b : net->enc) {
      if (b.kind == BK_RES) res_sz(b.res, b.level);
      if (b.has_st) st_sz(b.st, b.level);
      if (net == &h->cn) {
        const int C = b.kind == BK_RES ? b.res.cout : b.conv.cout;
        upd(cn_el, (size_t)h->lev_h[b.level] * h->lev_w[b.level] * C);
      }
    }
    res_sz(net->mid1, h->nlev - 1);
    st_sz(net->midst, h->nlev - 1);
    upd(r_el, (size_t)h->lev_h[h->nlev - 1] * h->lev_w[h->nlev - 1] * net->mid1.cout);
    for (auto& d : net->dec) {
      res_sz(d.res, d.level);
      if (d.has_st) st_sz(d.st, d.level);
      if (d.has_up) upd(r_el, (size_t)h->lev_h[d.level] * h->lev_w[d.level] * d.res.cout);
    }
  }
  upd(t_el, (size_t)h->lev_h[0] * h->lev_w[0] * mc);
  const size_t M0 = (size_t)h->lev_h[0] * h->lev_w[0];
  for (int k = 0; k < 2; ++k) {
    tair_cldm::Scratch& w = h->ws[k];
    w.T = (bf16*)dmalloc(h, B * t_el * 2);
    w.H1 = (bf16*)dmalloc(h, B * h1_el * 2);
    w.X0 = (bf16*)dmalloc(h, B * x0_el * 2);
    w.QKV = (bf16*)dmalloc(h, B * x0_el * 3 * 2);
    w.A = (bf16*)dmalloc(h, B * x0_el * 2);
    w.G = (bf16*)dmalloc(h, B * g_el * 8 * 2);
    w.F = (bf16*)dmalloc(h, B * g_el * 4 * 2);
    w.R = trunk_alloc(h, B * r_el);
    w.ss = (float*)dmalloc(h, B * std::max(cmax, 8 * mc) * 2 * 4);
    w.gnws = (float*)dmalloc(h, B * cfg->groups * 64 * 2 * 4);
    // split-K GEMM partials / attention KV-split partials: 8 M floats serve the B = 1 plans; batched
    // tiles split the 64^2-level GEMMs (M = B*4096, N <= 640) up to 4 ways
    w.partial_cap = std::min(std::max((size_t)8 << 20, (size_t)4 * B * M0 * 2 * mc), (size_t)1 << 30);
    w.partial = (float*)dmalloc(h, w.partial_cap * 4);
    w.gn_tickets = (int*)dmalloc(h, (size_t)B * cfg->groups * sizeof(int));
    w.gemm_tickets = (int*)dmalloc(h, (size_t)GEMM_TICKETS * sizeof(int));
    static const bool attn_ink = [] { const char* e = getenv("TAIR_ATTN_INK"); return e && atoi(e) != 0; }();
    w.attn_tickets = attn_ink ? (int*)dmalloc(h, (size_t)ATTN_TICKETS * sizeof(int)) : nullptr;
    if (cfg->compute_dtype == TAIR_DTYPE_FP8) {
      w.T8 = (uint8_t*)dmalloc(h, B * t8_bytes);
      w.ts8 = (float*)dmalloc(h, B * t8_rows * sizeof(float));
    }
  }
  // GroupNorm statistics slots (producer epilogues -> apply pass); needs batch-uniform 64-row tiles
  // and groups of >= 4 channels (every GroupNorm'd tensor has >= model_channels channels)
  {
    bool ok = (mc / cfg->groups) >= 4 && cfg->groups <= 64 && (mc % cfg->groups) == 0;
    for (int l = 0; l < h->nlev; ++l) ok = ok && (h->lev_h[l] * h->lev_w[l]) % 64 == 0;
    h->gn_fused = ok;
    if (const char* ab = getenv("TAIR_ABLATE")) h->ablate = atoi(ab);

    gemm_set_skip_reduce((h->ablate >> 8) & 1);
    if (h->gn_fused) {
      h->gst_slots = 256;
      h->gst_rs = B * cfg->groups * 2;
      h->gst = (double*)dmalloc(h, (size_t)h->gst_slots * STAT_REPL * h->gst_rs * sizeof(double));
    }
    if (h->ln_fold && h->ln_slot_rows) h->lst = (double*)dmalloc(h, lst_doubles(h) * sizeof(double));
  }
  h->Dout = trunk_alloc(h, B * M0 * mc);
  for (auto& b : h->cn.enc) {
    const int C = b.kind == BK_RES ? b.res.cout : b.conv.cout;
    h->cn_out.push_back(trunk_alloc(h, B * (size_t)h->lev_h[b.level] * h->lev_w[b.level] * C));
  }
  h->cn_mid = trunk_alloc(h, B * (size_t)h->lev_h[h->nlev - 1] * h->lev_w[h->nlev - 1] * h->cn.mid2.cout);
  // conv_in inputs as (hi, lo, hi) planes of the fp32 latent / hint
  if (3 * (cfg->in_channels + cfg->hint_channels) > CONVIN_LD) {
    set_error("create: %d input + %d hint channels exceed the %d-channel conv_in row", cfg->in_channels,
              cfg->hint_channels, CONVIN_LD / 3);
    tair_cldm_destroy(h);
    return TAIR_ERR_ARG;
  }
  h->in_u = (bf16*)dmalloc(h, B * M0 * CONVIN_LD * 2);  // (dmalloc zero-fills: the pad channels stay zero)
  h->in_c = (bf16*)dmalloc(h, B * M0 * CONVIN_LD * 2);
  h->ctx_bf = (bf16*)dmalloc(h, B * cfg->context_len * cfg->context_dim * 2);
  h->v_out = (float*)dmalloc(h, B * M0 * cfg->out_channels * 4);
  // concat buffers of the decoder (one per output block)
  {
    std::vector<int> enc_ch, enc_lvl;
    for (auto& b : h->unet.enc) {
      enc_ch.push_back(b.kind == BK_RES ? b.res.cout : b.conv.cout);
      enc_lvl.push_back(b.level);
    }
    int ch = h->unet.mid2.cout;
    for (size_t j = 0; j < h->unet.dec.size(); ++j) {
      const int ei = (int)enc_ch.size() - 1 - (int)j;
      tair_cldm::Cat c;
      c.ch = ch;
      c.cs = enc_ch[ei];
      c.level = enc_lvl[ei];
      const size_t hw = (size_t)h->lev_h[c.level] * h->lev_w[c.level];
      c.p = trunk_alloc(h, B * hw * (c.ch + c.cs));
      h->cat.push_back(c);
      ch = h->unet.dec[j].ch_out;
    }
  }
  h->tab_rows = std::max((int)B, 1000);
  h->tab_u = (float*)dmalloc(h, (size_t)h->tab_rows * h->unet.emb_total * 4);
  h->tab_c = (float*)dmalloc(h, (size_t)h->tab_rows * h->cn.emb_total * 4);
  h->sinus = (float*)dmalloc(h, (size_t)h->tab_rows * mc * 4);
  h->temb_a = (bf16*)dmalloc(h, (size_t)h->tab_rows * h->time_dim * 2);
  h->temb_b = (bf16*)dmalloc(h, (size_t)h->tab_rows * h->time_dim * 2);
  h->t_dev = (int64_t*)dmalloc(h, (size_t)h->tab_rows * 8);
  h->rows_iota = (int*)dmalloc(h, B * 4);
  h->rows_step = (int*)dmalloc(h, B * 4);
  h->counter = (int*)dmalloc(h, 16);
  h->xs = (float*)dmalloc(h, B * M0 * cfg->in_channels * 4);
  if (!cfg->manifest_only) {
    std::vector<int> iota(B);
    for (size_t i = 0; i < B; ++i) iota[i] = (int)i;
    if (hipMemcpy(h->rows_iota, iota.data(), B * 4, hipMemcpyHostToDevice) != hipSuccess) h->allocs.push_back(nullptr);
  }
  for (void* p : h->allocs)
    if (!p) {
      set_error("create: hipMalloc failed");
      tair_cldm_destroy(h);
      return TAIR_ERR_HIP;
    }
  for (int i = 0; i < 13; ++i) h->s_scales[i] = 1.f;
  if (!cfg->manifest_only &&
      (gemm_init() != hipSuccess || hipStreamCreateWithFlags(&h->gstream, hipStreamNonBlocking) != hipSuccess ||
       hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking) != hipSuccess ||
       hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) != hipSuccess ||
       hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess ||
       create_events(h->ev_zc, 16) != hipSuccess ||
       hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming) != hipSuccess ||
       hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming) != hipSuccess)) {
    tair_cldm_destroy(h);
    return TAIR_ERR_HIP;
  }
  live_add(h);
  *out = h;
  return TAIR_OK;
}

int tair_cldm_destroy(tair_cldm* h) {
  if (!h) return TAIR_OK;
  live_remove(h);
  drop_step_graphs(h);
  if (h->gstream) hipStreamDestroy(h->gstream);
  if (h->cstream) hipStreamDestroy(h->cstream);
  if (h->ev_fork) hipEventDestroy(h->ev_fork);
  if (h->ev_join) hipEventDestroy(h->ev_join);
  for (auto& e : h->ev_zc)
    if (e) hipEventDestroy(e);
  if (h->ev_in) hipEventDestroy(h->ev_in);
  if (h->ev_out) hipEventDestroy(h->ev_out);
  for (auto e : h->ev_pool) hipEventDestroy(e);
  if (!h->cfg.manifest_only)
    for (void* p : h->allocs)
      if (p) hipFree(p);
  if (h->arena) hipFree(h->arena);
  if (h->sched_tabs) hipFree(h->sched_tabs);
  if (h->noise) hipFree(h->noise);
  if (h->sched_t_dev) hipFree(h->sched_t_dev);
  delete h;
  return TAIR_OK;
}

int tair_cldm_param_count(const tair_cldm* h, int* n) {
  if (!h || !n) return TAIR_ERR_ARG;
  *n = (int)h->params.size();
  return TAIR_OK;
}

int tair_cldm_param_info(const tair_cldm* h, int i, const char** key, int64_t shape[4], int* ndim) {
  if (!h || i < 0 || i >= (int)h->params.size()) return TAIR_ERR_ARG;
  const ParamDst* p = h->params[i].get();
  if (key) *key = p->key.c_str();
  if (shape)
    for (int d = 0; d < 4; ++d) shape[d] = p->shape[d];
  if (ndim) *ndim = p->ndim;
  return TAIR_OK;
}

int tair_cldm_load_param(tair_cldm* h, const char* key, const void* src, int src_dtype, const int64_t* shape,
                         int ndim) {
  tair::g_err[0] = 0;
  if (!h || !key || !src || !shape) {
    set_error("load_param: null argument");
    return TAIR_ERR_ARG;
  }
  auto it = h->by_key.find(key);
  if (it == h->by_key.end()) {
    set_error("load_param: unknown key '%s'", key);
    return TAIR_ERR_KEY;
  }
  ParamDst* p = it->second;
  if (h->cfg.manifest_only) {
    set_error("load_param: handle was created manifest_only");
    return TAIR_ERR_STATE;
  }
  if (ndim != p->ndim) {
    set_error("load_param: '%s' ndim %d != %d", key, ndim, p->ndim);
    return TAIR_ERR_ARG;
  }
  size_t n = 1;
  for (int d = 0; d < ndim; ++d) {
    if (shape[d] != p->shape[d]) {
      set_error("load_param: '%s' dim %d is %lld, expected %lld", key, d, (long long)shape[d],
                (long long)p->shape[d]);
      return TAIR_ERR_ARG;
    }
    n *= (size_t)shape[d];
  }
  if (src_dtype != TAIR_DTYPE_F32 && src_dtype != TAIR_DTYPE_BF16) {
    set_error("load_param: unsupported dtype %d", src_dtype);
    return TAIR_ERR_ARG;
  }
  auto val = [&](size_t i) -> float {
    return src_dtype == TAIR_DTYPE_F32 ? ((const float*)src)[i] : bf_bits2f(((const uint16_t*)src)[i]);
  };
  if (p->kind == PK_VEC) {
    p->vec_src.resize(n);
    for (size_t i = 0; i < n; ++i) p->vec_src[i] = val(i);
    p->loaded = true;
    p->dirty = true;
    h->finalized = false;
    return TAIR_OK;
  }
  p->dirty = true;
  if (p->keep_src) {  // a LayerNorm-folded linear: finalize packs W diag(gamma) from these fp32 rows
    p->w_src.resize(n);
    for (size_t i = 0; i < n; ++i) p->w_src[i] = val(i);
  }
  // weights: pack rows into bf16 [rows][width] then one strided copy into the packed buffer
  const int rows = (int)p->shape[0];
  int width;
  std::vector<uint16_t> packed;
  auto lo_bits = [](float v, uint16_t hi) { return f2bf_bits(v - bf_bits2f(hi)); };
  if (p->kind == PK_CONV3) {
    const int cin = (int)p->shape[1];
    const int planes = p->split == 3 ? 3 : 1;  // split 3: input channel plane q*cin + c holds (hi, hi, lo)[q]
    const int kc = planes * cin;
    const int kcp = std::max(kc, p->cpad);  // zero-padded input channels (packed resize zero-fills them)
    width = 9 * kcp;
    packed.resize((size_t)rows * width);
    // K order of the GEMM's conv modes (kernels.h AMode): channel-chunk-major for a (planed, padded) channel
    // count % 64 == 0, tap-major for the small-channel A_CONV3_SMALLC layout
    const bool chunked = kcp % 64 == 0;
    for (int co = 0; co < rows; ++co)
      for (int cq = 0; cq < kc; ++cq)
        for (int tap = 0; tap < 9; ++tap) {
          const int q = cq / cin, c = cq - q * cin;
          const size_t k = chunked ? (size_t)((cq / 64) * 9 + tap) * 64 + (cq % 64) : (size_t)tap * kc + cq;
          const float v = val(((size_t)co * cin + c) * 9 + tap);
          const uint16_t hi = f2bf_bits(v);
          packed[(size_t)co * width + k] = q < 2 ? hi : lo_bits(v, hi);
        }
  } else if (p->split == 2) {  // [out, in(, 1, 1)] -> columns [W_hi | W_lo]
    const int cin = (int)(n / rows);
    width = 2 * cin;
    packed.resize((size_t)rows * width);
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cin; ++c) {
        const float v = val((size_t)r * cin + c);
        const uint16_t hi = f2bf_bits(v);
        packed[(size_t)r * width + c] = hi;
        packed[(size_t)r * width + cin + c] = lo_bits(v, hi);
      }
  } else {
    width = (int)(n / rows);  // [out, in] or [out, in, 1, 1]
    packed.resize(n);
    for (size_t i = 0; i < n; ++i) packed[i] = f2bf_bits(val(i));
  }
  if (p->geglu_half > 0) {
    std::vector<uint16_t> perm(packed.size());
    for (int r = 0; r < rows; ++r)
      std::memcpy(&perm[(size_t)geglu_row(r, p->geglu_half) * width], &packed[(size_t)r * width], (size_t)width * 2);
    packed.swap(perm);
  }
  Weight* w = p->w;
  if (p->row_off + rows > w->rows || p->col_off + width > w->ldw) {
    set_error("load_param: '%s' does not fit its packed buffer", key);
    return TAIR_ERR_STATE;
  }
  hipError_t e = hipMemcpy2D(w->p + (size_t)p->row_off * w->ldw + p->col_off, (size_t)w->ldw * 2, packed.data(),
                             (size_t)width * 2, (size_t)width * 2, rows, hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail_hip(e);
  p->loaded = true;
  return TAIR_OK;
}

// LayerNorm folding of one transformer (bf16 path): norm{1,2,3} -> attn1 q|k|v, attn2 q, GEGLU proj.
// W'[n][k] = W[n][k] gamma[k] (bf16, from the fp32 rows kept at load), bias'[n] = bias[n] + sum_k
// W[n][k] beta[k] (fp64 sum), colsum[n] = sum_k bf16(W'[n][k]) (the epilogue's mean correction uses
// the same rounded weights the GEMM multiplies).  The fp32 rows are released once folded; a transformer
// whose norms change must have its weights loaded again.
int fold_st(tair_cldm* h, STW& st, std::vector<float>& ar) {
  if (!st.fold) return TAIR_OK;
  const int C = st.C;
  struct Item { const char* w; const char* ln; Weight* dst; int row_off, fb, cs, bias, geglu; };
  const Item items[5] = {
      {".attn1.to_q.weight", ".norm1", &st.qkv, 0, st.fb_qkv, st.cs_qkv, -1, 0},
      {".attn1.to_k.weight", ".norm1", &st.qkv, C, st.fb_qkv, st.cs_qkv, -1, 0},
      {".attn1.to_v.weight", ".norm1", &st.qkv, 2 * C, st.fb_qkv, st.cs_qkv, -1, 0},
      {".attn2.to_q.weight", ".norm2", &st.q2, 0, st.fb_q2, st.cs_q2, -1, 0},
      {".ff.net.0.proj.weight", ".norm3", &st.ff1, 0, st.fb_ff1, st.cs_ff1, st.ff1b, 4 * C},
  };
  for (const Item& it : items) {
    ParamDst* pw = h->by_key[st.tb + it.w];
    ParamDst* pg = h->by_key[st.tb + it.ln + ".weight"];
    ParamDst* pb = h->by_key[st.tb + it.ln + ".bias"];
    const bool ffb = it.bias >= 0;
    ParamDst* pfb = ffb ? h->by_key[st.tb + ".ff.net.0.proj.bias"] : nullptr;
    const int rows = (int)pw->shape[0];
    if (!pw->dirty && !pg->dirty && !pb->dirty && !(pfb && pfb->dirty)) {
      // folded and unchanged: the folded bias and column sums have no backing parameter, so carry them
      // over from the last finalized arena (ar starts from the PK_VEC parameters only)
      for (int r = 0; r < rows; ++r) {
        const int pr = it.geglu ? geglu_row(r, it.geglu) : it.row_off + r;
        ar[it.fb + pr] = h->arena_host[it.fb + pr];
        ar[it.cs + pr] = h->arena_host[it.cs + pr];
      }
      continue;
    }
    if (pw->w_src.empty()) {
      set_error("finalize: '%s' changed after '%s' was folded; load '%s' again", (st.tb + it.ln).c_str(),
                pw->key.c_str(), pw->key.c_str());
      return TAIR_ERR_STATE;
    }
    const float* g = pg->vec_src.data();
    const float* be = pb->vec_src.data();
    std::vector<uint16_t> packed((size_t)rows * C);
    std::vector<int> prow(rows);
    for (int r = 0; r < rows; ++r) {
      const int pr = it.geglu ? geglu_row(r, it.geglu) : it.row_off + r;
      prow[r] = pr;
      const float* wr = pw->w_src.data() + (size_t)r * C;
      double fb = 0.0, cs = 0.0;
      for (int k = 0; k < C; ++k) {
        const uint16_t q = f2bf_bits(wr[k] * g[k]);
        packed[(size_t)r * C + k] = q;
        cs += bf_bits2f(q);
        fb += (double)wr[k] * be[k];
      }
      ar[it.fb + pr] = (float)(fb + (ffb ? ar[it.bias + pr] : 0.0));
      ar[it.cs + pr] = (float)cs;
    }
    Weight* w = it.dst;
    if (it.geglu) {  // GEGLU rows interleave into a permutation of [0, rows): reorder, then one copy
      std::vector<uint16_t> perm(packed.size());
      for (int r = 0; r < rows; ++r)
        std::memcpy(&perm[(size_t)prow[r] * C], &packed[(size_t)r * C], (size_t)C * 2);
      packed.swap(perm);
    }
    hipError_t e = hipMemcpy2D(w->p + (size_t)(it.geglu ? 0 : it.row_off) * w->ldw, (size_t)w->ldw * 2, packed.data(),
                               (size_t)C * 2, (size_t)C * 2, rows, hipMemcpyHostToDevice);
    if (e != hipSuccess) return fail_hip(e);
    std::vector<float>().swap(pw->w_src);
  }
  return TAIR_OK;
}

int tair_cldm_finalize(tair_cldm* h) {
  tair::g_err[0] = 0;
  if (!h) return TAIR_ERR_ARG;
  if (h->cfg.manifest_only) {
    set_error("finalize: handle was created manifest_only");
    return TAIR_ERR_STATE;
  }
  std::vector<float> ar(h->arena_host.size(), 0.f);
  for (auto& up : h->params) {
    ParamDst* p = up.get();
    if (!p->loaded) {
      set_error("finalize: parameter '%s' was never loaded", p->key.c_str());
      return TAIR_ERR_STATE;
    }
    if (p->kind == PK_VEC)
      for (size_t i = 0; i < p->vec_src.size(); ++i)
        ar[p->vec_off + (p->geglu_half > 0 ? geglu_row((int)i, p->geglu_half) : (int)i)] += p->vec_src[i];
  }
  for (Net* net : {&h->unet, &h->cn}) {
    int rc = TAIR_OK;
    for (auto& b : net->enc)
      if (rc == TAIR_OK && b.has_st) rc = fold_st(h, b.st, ar);
    if (rc == TAIR_OK) rc = fold_st(h, net->midst, ar);
    for (auto& d : net->dec)
      if (rc == TAIR_OK && d.has_st) rc = fold_st(h, d.st, ar);
    if (rc != TAIR_OK) return rc;
  }
  // GroupNorm-fed fp8 consumers: static per-channel activation scales from the GroupNorm's gamma / beta
  std::vector<Weight*> gn8;
  for (Net* net : {&h->unet, &h->cn}) {
    auto res = [&](ResW& r) {
      if (r.c1.f8_gn >= 0) gn8.push_back(&r.c1);
      if (r.c2.f8_gn >= 0) gn8.push_back(&r.c2);
    };
    auto stw = [&](STW& st) {
      if (st.pin.f8_gn >= 0) gn8.push_back(&st.pin);
    };
    for (auto& b : net->enc) {
      if (b.kind == BK_RES) res(b.res);
      if (b.has_st) stw(b.st);
    }
    res(net->mid1);
    res(net->mid2);
    stw(net->midst);
    for (auto& d : net->dec) {
      res(d.res);
      if (d.has_st) stw(d.st);
    }
  }
  auto act_scale = [&](const Weight& w, int c) {  // a_c: power of two >= (|gamma| R + |beta|) / 448
    const float bound = std::fabs(ar[w.f8_gn + c]) * GN_F8_RANGE + std::fabs(ar[w.f8_gn + w.f8_cin + c]);
    if (!(bound > 0.f)) return 1.f;
    int ex;
    const float m = std::frexp(bound / 448.f, &ex);
    return std::ldexp(1.f, m == 0.5f ? ex - 1 : ex);
  };
  for (Weight* w : gn8)
    for (int c = 0; c < w->f8_cin; ++c) ar[w->inv8 + c] = 1.f / act_scale(*w, c);
  for (auto& up : h->params) up->dirty = false;
  if (!h->arena) {
    if (hipMalloc(&h->arena, ar.size() * 4) != hipSuccess) {
      set_error("finalize: hipMalloc failed");
      return TAIR_ERR_HIP;
    }
  }
  hipError_t e = hipMemcpy(h->arena, ar.data(), ar.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail_hip(e);
  h->arena_host = ar;  // the folded slots a later partial re-finalize carries over
  // fp8 twins: per-output-channel e4m3 from the packed bf16 weights (same row order, GEGLU interleave)
  auto quant = [&](Weight& w) -> hipError_t {  // (the LayerNorm-fed linears: per-token activation scales)
    return w.p8 ? quant_rows_fp8(w.p, w.rows, w.K, w.ldw, w.p8, w.ld8, w.s8, nullptr) : hipSuccess;
  };
  auto quant_st = [&](STW& st) -> hipError_t {
    TRY(quant(st.qkv));
    TRY(quant(st.q2));
    return quant(st.ff1);
  };
  for (Net* net : {&h->unet, &h->cn}) {
    for (auto& b : net->enc)
      if (b.has_st && (e = quant_st(b.st)) != hipSuccess) return fail_hip(e);
    if ((e = quant_st(net->midst)) != hipSuccess) return fail_hip(e);
    for (auto& d : net->dec)
      if (d.has_st && (e = quant_st(d.st)) != hipSuccess) return fail_hip(e);
  }
  if (!gn8.empty()) {  // fold a_c into the weights (per K column: the conv's channel-chunk-major order)
    size_t kmax = 0;
    for (Weight* w : gn8) kmax = std::max(kmax, (size_t)w->K);
    float* ak = nullptr;
    if ((e = hipMalloc(&ak, kmax * sizeof(float))) != hipSuccess) return fail_hip(e);
    std::vector<float> hk(kmax);
    for (Weight* w : gn8) {
      for (int k = 0; k < w->K; ++k) {
        const int c = w->f8_conv ? (k / 64 / 9) * 64 + k % 64 : k;
        hk[k] = act_scale(*w, c);
      }
      if ((e = hipMemcpy(ak, hk.data(), (size_t)w->K * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess ||
          (e = quant_rows_fp8_ex(w->p, w->rows, w->K, w->Kx, w->ldw, ak, w->p8, w->ldb8, w->ld8, w->s8, nullptr)) !=
              hipSuccess ||
          (e = hipDeviceSynchronize()) != hipSuccess) {
        hipFree(ak);
        return fail_hip(e);
      }
    }
    hipFree(ak);
  }
  if ((e = hipDeviceSynchronize()) != hipSuccess) return fail_hip(e);
  h->finalized = true;
  return TAIR_OK;
}

static int check_ready(tair_cldm* h) {
  if (!h) {
    set_error("null handle");
    return TAIR_ERR_ARG;
  }
  if (!h->cfg.manifest_only && !live(h)) {
    set_error("stale or foreign handle %p (destroyed, or never created)", (void*)h);
    return TAIR_ERR_STATE;
  }
  if (h->cfg.manifest_only) {
    set_error("handle was created manifest_only");
    return TAIR_ERR_STATE;
  }
  if (!h->finalized) {
    set_error("weights not finalized (call tair_cldm_finalize after loading every parameter)");
    return TAIR_ERR_STATE;
  }
  return TAIR_OK;
}

int tair_cldm_forward(tair_cldm* h, const tair_cldm_io* io, tair_stream_t stream) {
  tair::g_err[0] = 0;
  int rc = check_ready(h);
  if (rc) return rc;
  if (!io || !io->x || !io->t || !io->c_txt || !io->out || io->batch < 1 || io->batch > h->cfg.max_batch ||
      (io->c_txt_batch != 1 && io->c_txt_batch != io->batch)) {
    set_error("forward: bad io (batch %d, max %d, c_txt_batch %d)", io ? io->batch : -1, h->cfg.max_batch,
              io ? io->c_txt_batch : -1);
    return TAIR_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int B = io->batch;
  const bool control = io->c_img != nullptr;
  const Fwd f = make_fwd(h, s, B, h->rows_iota, io->c_txt_batch == 1 ? 0 : h->cfg.context_len, control);
  hipError_t e;
  auto run = [&]() -> hipError_t {
    TRY(launch(h, 4, 0, s, [&] { return hipMemcpyAsync(h->t_dev, io->t, B * 8, hipMemcpyDeviceToDevice, s); }));
    TRY(time_tables(h, h->unet, h->t_dev, B, h->tab_u, s));
    if (control) TRY(time_tables(h, h->cn, h->t_dev, B, h->tab_c, s));
    TRY(prepare_ctx(h, io->c_txt, io->c_txt_batch, s));
    TRY(prepare_inputs(h, B, io->x, io->c_img, s));
    TRY(body(h, f, control, io->control_scales));
    const int HW = h->lev_h[0] * h->lev_w[0];
    TRY(launch(h, 4, 0, s, [&] { return nhwc_f32_to_nchw_f32(h->v_out, B, h->cfg.out_channels, HW, io->out, s); }));
    TRY(export_feats(h, B, io->feats, s));
    return hipSuccess;
  };
  e = run();
  if (e != hipSuccess) return fail_hip(e);
  return TAIR_OK;
}

int tair_sampler_set_schedule(tair_cldm* h, int n_steps, const int64_t* model_t, const float* tables) {
  tair::g_err[0] = 0;
  if (!h || n_steps < 1 || n_steps > h->tab_rows || !model_t || !tables) {
    set_error("set_schedule: bad arguments");
    return TAIR_ERR_ARG;
  }
  std::vector<float> tabs_in(tables, tables + (size_t)5 * n_steps);
  if (h->n_steps == n_steps && h->sched_t == std::vector<int64_t>(model_t, model_t + n_steps) &&
      h->sched_tabs_host == tabs_in)
    return TAIR_OK;  // unchanged schedule: keep the captured step graph
  h->n_steps = n_steps;
  h->sched_t.assign(model_t, model_t + n_steps);
  h->sched_tabs_host = tabs_in;
  // Buffers are allocated once at capacity (tab_rows steps) so that their addresses -- baked into a
  // captured step graph -- never change; the graph is still invalidated (the step count it reads
  // from the device counter changes, and so may the batch).
  const size_t M0 = (size_t)h->lev_h[0] * h->lev_w[0];
  if (!h->sched_tabs && hipMalloc(&h->sched_tabs, (size_t)5 * h->tab_rows * 4) != hipSuccess) return TAIR_ERR_HIP;
  if (n_steps > h->noise_cap_steps) {  // grow only (the graph is rebuilt below anyway)
    if (h->noise) hipFree(h->noise);
    h->noise = nullptr;
    h->noise_cap_steps = 0;
    if (hipMalloc(&h->noise, (size_t)n_steps * h->cfg.max_batch * M0 * h->cfg.in_channels * 4) != hipSuccess) {
      set_error("set_schedule: cannot allocate the noise buffer");
      return TAIR_ERR_HIP;
    }
    h->noise_cap_steps = n_steps;
  }
  if (!h->sched_t_dev && hipMalloc(&h->sched_t_dev, (size_t)h->tab_rows * 8) != hipSuccess) return TAIR_ERR_HIP;
  if (hipMemcpy(h->sched_tabs, tables, (size_t)5 * n_steps * 4, hipMemcpyHostToDevice) != hipSuccess)
    return TAIR_ERR_HIP;
  if (hipMemcpy(h->sched_t_dev, model_t, (size_t)n_steps * 8, hipMemcpyHostToDevice) != hipSuccess)
    return TAIR_ERR_HIP;
  drop_step_graphs(h);
  h->graph_batch = -1;
  return TAIR_OK;
}

namespace {
__global__ void set_rows_kernel(const int* counter, int* rows, int B) {
  const int i = threadIdx.x;
  if (i < B) rows[i] = counter[0];
}
__global__ void advance_kernel(int* counter) {
  if (threadIdx.x == 0) counter[0] += 1;
}
__global__ void init_counter_kernel(int* counter, int n) {
  if (threadIdx.x == 0) {
    counter[0] = 0;
    counter[1] = n;
  }
}
// sampler update (spaced_sampler.py:141-189) fused with re-emitting the NHWC model inputs as (hi, lo, hi)
// bf16 planes of the fp32 latent (in_u: rows of CONVIN_LD channels, planes C apart; in_c: planes ldc apart
// with the latent at channels 0..C-1 of each plane)
__global__ void step_update_kernel(float* xs, const float* v, const float* noise, const float* tabs,
                                   const int* counter, int n, int C, bf16* in_u, bf16* in_c, int ldc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int it = counter[0], ns = counter[1];
  const int t = ns - 1 - it;
  const float sa = tabs[t], s1a = tabs[ns + t], c1 = tabs[2 * ns + t], c2 = tabs[3 * ns + t], var = tabs[4 * ns + t];
  const float xv = xs[i];
  const float x0 = sa * xv - s1a * v[i];
  const float mean = c1 * x0 + c2 * xv;
  const float xn = (t != 0) ? mean + sqrtf(var) * noise[(size_t)it * n + i] : mean;
  xs[i] = xn;
  const int row = i / C, c = i - row * C;
  const bf16 hi = (bf16)xn, lo = (bf16)(xn - (float)hi);
  bf16* u = in_u + (size_t)row * CONVIN_LD + c;
  u[0] = hi;
  u[C] = lo;
  u[2 * C] = hi;
  if (in_c) {
    bf16* q = in_c + (size_t)row * CONVIN_LD + c;
    q[0] = hi;
    q[ldc] = lo;
    q[2 * ldc] = hi;
  }
}
// NCHW [B,C,HW] fp32 -> NHWC [B*HW, C] fp32
__global__ void nchw2nhwc_f32_kernel(const float* x, int B, int C, int HW, float* y) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)B * C * HW) return;
  const long b = i / ((long)C * HW);
  const long rem = i - b * C * HW;
  const int p = (int)(rem % HW), c = (int)(rem / HW);
  y[(size_t)(b * HW + p) * C + c] = x[i];
}
}  // namespace

int tair_sampler_prepare(tair_cldm* h, const tair_sampler_io* io, tair_stream_t stream) {
  tair::g_err[0] = 0;
  int rc = check_ready(h);
  if (rc) return rc;
  if (!h->n_steps) {
    set_error("sampler_prepare: call tair_sampler_set_schedule first");
    return TAIR_ERR_STATE;
  }
  if (!io || !io->x_T || !io->noise || !io->c_txt || io->batch < 1 || io->batch > h->cfg.max_batch ||
      (io->c_txt_batch != 1 && io->c_txt_batch != io->batch)) {
    set_error("sampler_prepare: bad io");
    return TAIR_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int B = io->batch;
  const int HW = h->lev_h[0] * h->lev_w[0];
  const int C = h->cfg.in_channels;
  h->s_batch = B;
  h->s_ctx_bstride = io->c_txt_batch == 1 ? 0 : h->cfg.context_len;
  h->s_control = io->c_img != nullptr;
  for (int i = 0; i < 13; ++i) h->s_scales[i] = io->control_scales ? io->control_scales[i] : 1.f;
  auto run = [&]() -> hipError_t {
    // time-embedding tables for every step of the schedule: one batched GEMM chain per net
    TRY(time_tables(h, h->unet, h->sched_t_dev, h->n_steps, h->tab_u, s));
    if (h->s_control) TRY(time_tables(h, h->cn, h->sched_t_dev, h->n_steps, h->tab_c, s));
    TRY(prepare_ctx(h, io->c_txt, io->c_txt_batch, s));
    TRY(prepare_inputs(h, B, io->x_T, io->c_img, s));
    const long n = (long)B * C * HW;
    hipLaunchKernelGGL(nchw2nhwc_f32_kernel, dim3((n + 255) / 256), dim3(256), 0, s, io->x_T, B, C, HW, h->xs);
    TRY(hipGetLastError());
    for (int i = 0; i < h->n_steps; ++i)
      hipLaunchKernelGGL(nchw2nhwc_f32_kernel, dim3((n + 255) / 256), dim3(256), 0, s, io->noise + (size_t)i * n, B,
                         C, HW, h->noise + (size_t)i * n);
    TRY(hipGetLastError());
    hipLaunchKernelGGL(init_counter_kernel, dim3(1), dim3(64), 0, s, h->counter, h->n_steps);
    return hipGetLastError();
  };
  hipError_t e = run();
  if (e != hipSuccess) return fail_hip(e);
  return TAIR_OK;
}

int tair_sampler_set_context(tair_cldm* h, const float* c_txt, int c_txt_batch, tair_stream_t stream) {
  tair::g_err[0] = 0;
  int rc = check_ready(h);
  if (rc) return rc;
  if (!c_txt || (c_txt_batch != 1 && c_txt_batch != h->s_batch)) {
    set_error("set_context: bad arguments");
    return TAIR_ERR_ARG;
  }
  if ((c_txt_batch == 1 ? 0 : h->cfg.context_len) != h->s_ctx_bstride) {
    set_error("set_context: context batch layout changed since prepare");
    return TAIR_ERR_ARG;
  }
  hipError_t e = prepare_ctx(h, c_txt, c_txt_batch, (hipStream_t)stream);
  if (e != hipSuccess) return fail_hip(e);
  return TAIR_OK;
}

static hipError_t sampler_one_step(tair_cldm* h, hipStream_t s) {
  const int B = h->s_batch;
  const int HW = h->lev_h[0] * h->lev_w[0];
  const int C = h->cfg.in_channels;
  hipLaunchKernelGGL(set_rows_kernel, dim3(1), dim3(std::max(64, ((B + 63) / 64) * 64)), 0, s, h->counter,
                     h->rows_step, B);
  TRY(hipGetLastError());
  const Fwd f = make_fwd(h, s, B, h->rows_step, h->s_ctx_bstride, h->s_control);
  TRY(body(h, f, h->s_control, h->s_scales));
  const int n = B * HW * C;
  TRY(launch(h, 4, 0, s, [&] {
    hipLaunchKernelGGL(step_update_kernel, dim3((n + 255) / 256), dim3(256), 0, s, h->xs, h->v_out, h->noise,
                       h->sched_tabs, h->counter, n, C, h->in_u, h->s_control ? h->in_c : (bf16*)nullptr,
                       C + h->cfg.hint_channels);
    return hipGetLastError();
  }));
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, s, h->counter);
  return hipGetLastError();
}

static void drop_step_graphs(tair_cldm* h) {
  if (h->gexec) hipGraphExecDestroy(h->gexec);
  if (h->graph) hipGraphDestroy(h->graph);
  h->gexec = nullptr;
  h->graph = nullptr;
}

int tair_sampler_run(tair_cldm* h, int n_steps, int use_graph, tair_stream_t stream) {
  tair::g_err[0] = 0;
  int rc = check_ready(h);
  if (rc) return rc;
  if (!h->s_batch) {
    set_error("sampler_run: call tair_sampler_prepare first");
    return TAIR_ERR_STATE;
  }
  hipStream_t cs = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  if (use_graph && !h->prof && !h->dry) {
    hipStream_t s = h->gstream;
    e = hipEventRecord(h->ev_in, cs);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, h->ev_in, 0);
    if (e != hipSuccess) return fail_hip(e);
    // the captured step bakes in the batch, whether the ControlNet branch runs, the context batch
    // stride and the control scales (GEMM alpha): any change since the capture needs a new graph
    const bool same = h->gexec != nullptr && h->graph_batch == h->s_batch && h->graph_control == h->s_control &&
                      h->graph_ctx_bstride == h->s_ctx_bstride &&
                      std::memcmp(h->graph_scales, h->s_scales, sizeof(h->s_scales)) == 0;
    if (!same) drop_step_graphs(h);
    if (!same) {
      e = hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
      if (e != hipSuccess) return fail_hip(e);
      hipError_t ce = sampler_one_step(h, s);
      hipGraph_t g = nullptr;
      e = hipStreamEndCapture(s, &g);
      if (ce != hipSuccess) {
        if (g) hipGraphDestroy(g);
        return fail_hip(ce);
      }
      if (e != hipSuccess) return fail_hip(e);
      h->graph = g;
      e = hipGraphInstantiate(&h->gexec, g, nullptr, nullptr, 0);
      if (e != hipSuccess) return fail_hip(e);
      h->graph_batch = h->s_batch;
      h->graph_control = h->s_control;
      h->graph_ctx_bstride = h->s_ctx_bstride;
      std::memcpy(h->graph_scales, h->s_scales, sizeof(h->s_scales));
    }
    for (int i = 0; i < n_steps; ++i) {
      e = hipGraphLaunch(h->gexec, s);
      if (e != hipSuccess) return fail_hip(e);
    }
    e = hipEventRecord(h->ev_out, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(cs, h->ev_out, 0);
    if (e != hipSuccess) return fail_hip(e);
    return TAIR_OK;
  }
  hipStream_t s = cs;
  for (int i = 0; i < n_steps; ++i) {
    e = sampler_one_step(h, s);
    if (e != hipSuccess) return fail_hip(e);
  }
  return TAIR_OK;
}

int tair_sampler_get_x(tair_cldm* h, float* x_out, float* feats[4], tair_stream_t stream) {
  tair::g_err[0] = 0;
  if (!h || !x_out || !h->s_batch) {
    set_error("get_x: bad state");
    return TAIR_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int HW = h->lev_h[0] * h->lev_w[0];
  hipError_t e = nhwc_f32_to_nchw_f32(h->xs, h->s_batch, h->cfg.in_channels, HW, x_out, s);
  if (e != hipSuccess) return fail_hip(e);
  if (feats) {
    e = export_feats(h, h->s_batch, feats, s);
    if (e != hipSuccess) return fail_hip(e);
  }
  return TAIR_OK;
}

int tair_sampler_get_v(tair_cldm* h, float* v_out, tair_stream_t stream) {
  tair::g_err[0] = 0;
  if (!h || !v_out || !h->s_batch) {
    set_error("get_v: bad state");
    return TAIR_ERR_ARG;
  }
  const int HW = h->lev_h[0] * h->lev_w[0];
  hipError_t e = nhwc_f32_to_nchw_f32(h->v_out, h->s_batch, h->cfg.out_channels, HW, v_out, (hipStream_t)stream);
  if (e != hipSuccess) return fail_hip(e);
  return TAIR_OK;
}

int tair_profile_enable(tair_cldm* h, int enable) {
  if (!h) return TAIR_ERR_ARG;
  h->prof = enable != 0;
  h->prof_recs.clear();
  h->ev_used = 0;
  return TAIR_OK;
}

int tair_profile_read(tair_cldm* h, int cls, double* total_ms, int* launches, double* flops) {
  if (!h) return TAIR_ERR_ARG;
  double tot = 0, fl = 0;
  int n = 0;
  for (auto& r : h->prof_recs) {
    if (r.cls != cls) continue;
    if (hipEventSynchronize(r.b) != hipSuccess) return TAIR_ERR_HIP;
    float ms = 0;
    if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) return TAIR_ERR_HIP;
    tot += ms;
    fl += r.flops;
    ++n;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = n;
  if (flops) *flops = fl;
  return TAIR_OK;
}

int tair_profile_dump(tair_cldm* h, const char* path) {
  if (!h || !path) return TAIR_ERR_ARG;
  FILE* f = fopen(path, "w");
  if (!f) {
    set_error("profile_dump: cannot open %s", path);
    return TAIR_ERR_ARG;
  }
  fprintf(f, "idx,class,us,gflops,tflops_per_s,alg_mb,key,tag\n");
  int i = 0;
  for (auto& r : h->prof_recs) {
    if (hipEventSynchronize(r.b) != hipSuccess) {
      fclose(f);
      return TAIR_ERR_HIP;
    }
    float ms = 0;
    hipEventElapsedTime(&ms, r.a, r.b);
    fprintf(f, "%d,%d,%.2f,%.4f,%.2f,%.4f,%s,%s\n", i++, r.cls, ms * 1000.0, r.flops / 1e9,
            ms > 0 ? r.flops / (ms / 1000.0) / 1e12 : 0.0, r.alg / 1e6, r.key.empty() ? "other" : r.key.c_str(),
            r.tag.c_str());
  }
  fclose(f);
  return TAIR_OK;
}

int tair_cldm_flops(const tair_cldm* hc, int batch, double* flops) {
  tair_cldm* h = const_cast<tair_cldm*>(hc);
  if (!h || !flops || batch < 1) return TAIR_ERR_ARG;
  h->dry = true;
  h->dry_flops = 0;
  const Fwd f = make_fwd(h, nullptr, batch, nullptr, 0, true);
  hipError_t e = body(h, f, true, nullptr);
  h->dry = false;
  if (e != hipSuccess) return TAIR_ERR_HIP;
  *flops = h->dry_flops;
  return TAIR_OK;
}

}  // extern "C"
