// Host engine of libmmt_hip.so: parameter layout, workspace plan and the forward / backward
// launch sequence of the multimodal transformer training step, behind the C-ABI of include/mmt.h.
//
// Reference structure restated (model.py): per layer, per modality i
//   x1 = x0 + proj(MHA(LN1 x0))           MHA heads: q/k/v = Linear(C,hs/2)+tanh+Linear(hs/2,hs)
//   x2 = x1 + FFN(LN2 x1)                 FFN = Linear(C,4C)+ReLU+Linear(4C,C)
//   x3 = x2 + proj(CA(LNc x2, [x2_j]))    only for cross modalities; one softmax per KV stream, summed
// post: logits = Linear(V/2,V)(tanh(Linear(C,V/2)(LNf x))), loss = mean CE.
// All modalities' identical-shape ops run as ONE grouped launch (blockIdx.z = modality).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mmt.h"
#include "mmt_common.h"
#include "mmt_kernels.h"

namespace {

constexpr int MAXM = MMT_MAX_MODALITIES;

inline int64_t rup(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
inline int r8(int x) { return (int)rup(x < 1 ? 1 : x, 8); }

struct Mat {
  int64_t off = -1;  // fp32 offset of the [rows, cols] weight in the flat param buffer
  int rows = 0, cols = 0;
  int64_t pk = 0;    // bf16 element offset in the packed-weight region
  int ld = 0;        // packed leading dimension (multiple of 8)
  // MX-fp8 copy (precision fp8): byte offsets of the e4m3fn rows and E8M0 exponents in the fp8
  // pack region, row strides in bytes; pk8 < 0: no fp8 copy
  int64_t pk8 = -1, ps8 = -1;
  int ld8 = 0, lds8 = 0;
};

struct TensorInfo {
  std::string name;
  int64_t off;
  int nd;
  int64_t shape[2];
  int kind;
};

struct LM {  // parameters of one (layer, modality)
  int64_t ln1w, ln1b, ln2w, ln2b;
  Mat W1; int64_t b1; int64_t w2;
  Mat P0; int64_t bp0; Mat P2; int64_t bp2;
  Mat F0; int64_t bf0; Mat F2; int64_t bf2;
  bool cross = false;  // cross-attention active (cross flag and M > 1)
  int64_t lncw = -1, lncb = -1;
  Mat Wq; Mat Wkv[MAXM]; Mat C0; int64_t bc0 = -1; Mat C2; int64_t bc2 = -1;
};

struct PostM {
  int64_t lnw, lnb;
  Mat H0; int64_t b0; Mat H2; int64_t b2;
  int64_t tok;
};

struct ActLM {  // byte offsets of one (layer, modality)'s saved activations in the workspace
  size_t a, mean1, rstd1, h1, qkv, o, lse, p1, x1, c, mean2, rstd2, f, x2, x2h;
  size_t d, meanc, rstdc, qc, kv[MAXM], oc, ocj[MAXM], lsej[MAXM], pc, x3;
  size_t dm, dmj[MAXM];  // attention dropout keep bits (SA; CA per KV stream), dropout > 0 only
  // MX-fp8 copies of the fp8 GEMMs' A operands (precision fp8): LN1 / LN2 / LNc outputs and the
  // FFN hidden, e4m3fn bytes + E8M0 exponents
  size_t a8 = 0, as8 = 0, c8 = 0, cs8 = 0, f8 = 0, fs8 = 0, d8 = 0, ds8 = 0;
  size_t fm = 0;  // ReLU bits of the FFN hidden [R][4C / 8] (the ffn2 data gradient's ReLU')
};

struct Plan {
  int B = -1;
  size_t total = 0;
  size_t pack = 0;
  size_t slab = 0, slab_bytes = 0;  // split-K slabs of the weight-gradient GEMMs
  size_t flag = 0;                  // int32 non-finite-loss bitmask (bit i: modality i)
  size_t pack8 = 0;                 // MX-fp8 weight copies (precision fp8)
  std::vector<ActLM> act;  // [L*M]
  size_t xemb[MAXM];
  size_t lnf16[MAXM], meanf[MAXM], rstdf[MAXM], hh[MAXM], dlog[MAXM];
  // backward scratch, per modality. The data gradients a side-stream weight-gradient GEMM reads
  // (gbig, gq, gh1, gp, gpc, dkv) have two copies, one per backward-stage parity, so the main
  // stream may run a whole stage ahead of the side stream (mmt_backward joins once, at its end)
  size_t dres[MAXM], dln[MAXM], gdo[MAXM], gqkv[MAXM];
  size_t gbig[2][MAXM], gq[2][MAXM], gh1[2][MAXM], gp[2][MAXM], gpc[2][MAXM];
  // bf16 residual-gradient copies, rotated over 8 buffers (one per LayerNorm-backward / copy launch,
  // three per layer stage): a side-stream weight-gradient GEMM up to one stage behind still reads
  // its copy when the main stream writes the next ones
  size_t dres16[8][MAXM];
  size_t dvec[MAXM][MAXM];
  size_t dkv[2][MAXM][MAXM];
  size_t celoss[MAXM];  // float [512]: the cross-entropy blocks' loss shares (summed in block order)
  const void* gh1_pad_ws = nullptr;  // the workspace whose gh1 pad columns (written by no kernel) are zeroed
  size_t eperm[MAXM];  // int [R]: the rows in token order for the token-table gradient (mmt_launch_emb_sort)
  // KV-cache decode (generate): compact [B, *] rows of ONE new position per sequence
  struct Dec {
    size_t x0, a16, mean, rstd, h1, qkv, o16, p1, f, x2h, d16, qc, oc, pc, lnf16, hh;
    size_t kv[MAXM];
  } dec[MAXM];
  std::vector<size_t> dec_x;  // [L*M][3]: fp32 residual stream x1, x2, x3 of the new rows
};

}  // namespace

// the FFN's ReLU' as bits written by ffn0 (16x fewer bytes than the bf16 hidden the ffn2 data
// gradient reads back). MMT_RELU_BITS=1 or mmt_set_relu_bits(1) before mmt_create turns it on (latched
// per context: the bit rows are allocated only then); off by default: on the final round-5 build the
// bf16 aux measured faster (same box, profiles/r5am_relu_bits_final_ab.txt: C1 8.502 -> 8.477 ms,
// target 19.770 -> 19.505 ms), where the first version had been 0.1-0.7 % faster than the aux
static int g_relu_bits = [] {
  const char* e = getenv("MMT_RELU_BITS");
  return e ? atoi(e) : 0;
}();
extern "C" int mmt_set_relu_bits(int on) {
  const int old = g_relu_bits;
  g_relu_bits = on;
  return old;
}
// the FFN backward's dropout-masked bf16 residual-gradient copy (+ FFN output-bias gradient) in the
// epilogue of the last cross-attention K/V dX launch into that gradient (1, default, env
// MMT_DROP_COPY_FUSE) or a separate drop_copy pass (0)
static int g_drop_copy_fuse = [] {
  const char* e = getenv("MMT_DROP_COPY_FUSE");
  return e ? atoi(e) : 1;
}();
extern "C" int mmt_set_drop_copy_fuse(int on) {
  const int old = g_drop_copy_fuse;
  g_drop_copy_fuse = on;
  return old;
}

// hs 32: the Q/K/V stage-2 backward in the one-pass attention backward's epilogue (1, default, env
// MMT_ATTN_QKV2) or the separate qkv2 backward over the bf16 dQ / dK / dV (0); read at every step
static int g_attn_qkv2 = [] {
  const char* e = getenv("MMT_ATTN_QKV2");
  return e ? atoi(e) : 1;
}();
extern "C" int mmt_set_attn_qkv2(int on) {
  const int old = g_attn_qkv2;
  g_attn_qkv2 = on;
  return old;
}

struct mmt_ctx {
  mmt_config cfg;
  int M, C, H, L, T, hs, hh;
  int V[MAXM];
  bool any_cross = false;
  int ncross = 0;
  std::vector<TensorInfo> tensors;
  std::vector<LM> lm;  // [L*M]
  PostM post[MAXM];
  int64_t pos_off = 0;
  int64_t nparams = 0, nactive = 0;
  int64_t emb_begin = 0, emb_end = 0, post_begin = 0, post_end = 0;
  std::vector<int64_t> layer_begin, layer_end;
  // weight packing
  std::vector<PackSeg> segs;
  std::vector<int> tasks;
  // MX-fp8 weight copies (precision fp8): quantisation segments and the fp8 pack region size
  std::vector<MxSeg> mxsegs;
  int64_t pack8_bytes = 0;
  int mx_units = 0;
  MxSeg* d_mxsegs = nullptr;
  int tables_device = -1;
  bool fp8 = false;
  bool relu_bits = false;  // g_relu_bits at mmt_create
  // token-table gradient: the rows' sort runs at backward stage 0 on the side stream (it reads only the
  // forward's token ids); emb_ev marks its end for the embedding stage
  hipEvent_t emb_ev = nullptr;
  bool emb_sorted = false;
  int64_t pack_elems = 0;
  PackSeg* d_segs = nullptr;
  int* d_tasks = nullptr;
  // state
  Plan plan;
  int last_B = -1;
  bool fwd_ready = false;
  bool cache_ready = false;  // a forward filled the workspace's Q/K/V (decode may follow)
  bool last_training = false;
  uint64_t step_counter = 0;
  // dropout: seed of the next training forward (mmt_set_dropout_seed) and of the last one
  uint64_t next_seed = 0;
  bool next_seed_set = false;
  uint64_t fwd_seed = 0;
  bool fwd_drop = false;
  const int64_t* last_idx[MAXM] = {};  // forward token ids, read by the embedding backward stage
  std::string err;
  // live kernel timing (mmt_probe_set): launch-label patterns and the HIP event pairs recorded
  // around every matching launch, with that launch's algorithmic flops / HBM bytes
  struct ProbeEv {
    hipEvent_t a, b;
    int pat;
    double flops, bytes;
  };
  std::vector<std::string> probe_pats;
  bool probe_on = true;
  std::vector<ProbeEv> probe_events;  // recorded launches (events taken from probe_pool in order)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> probe_pool;  // created by mmt_probe_set, not in the timed loop
  int ldv[MAXM], ldvh[MAXM];
  // backward side stream: the weight-gradient GEMMs (nothing in the data-gradient chain reads
  // them) run there, overlapping the latency-bound data-gradient kernels; joined at stage ends
  hipStream_t side = nullptr;
  int side_device = -1;
  bool side_off = false;  // mmt_set_side_stream(ctx, 0): this context runs everything on the caller's stream
  bool side_off_req = false;  // the requested setting, latched into side_off by the next mmt_forward (a
                              // forward and its backward always see one setting: work forked to the side
                              // stream is always joined)
  // mmt_backward (all stages in one call): no join per stage; the side stream's work of stage t is
  // recorded in stage_ev[t & 1] and the main stream waits for it only at the start of stage t + 2,
  // the first stage that rewrites that parity's scratch (Plan). mmt_backward_stage called alone (the
  // data-parallel path: each stage's gradient range must be final for its all-reduce) joins per stage.
  bool defer_join = false;
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  std::vector<hipEvent_t> evpool;
  size_t evnext = 0;
  int d16 = 0;  // rotation index of the current dres16 copy (reset at backward stage 0)
};

namespace {

thread_local std::string g_create_err;

int fail(mmt_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(ctx, expr)                                                                             \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess) return fail(ctx, MMT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// -------------------------------------------------------------------------------------------
// parameter layout
// -------------------------------------------------------------------------------------------
struct Builder {
  mmt_ctx* c;
  int64_t cur = 0;
  int64_t alloc(int64_t n) {
    const int64_t o = cur;
    cur += rup(n > 0 ? n : 0, 16);
    return o;
  }
  void tensor(const std::string& name, int64_t off, int nd, int64_t s0, int64_t s1, int kind) {
    TensorInfo t;
    t.name = name; t.off = off; t.nd = nd; t.shape[0] = s0; t.shape[1] = s1; t.kind = kind;
    c->tensors.push_back(t);
  }
  Mat mat(const std::string& name, int rows, int cols, bool emit = true) {
    Mat m;
    m.rows = rows; m.cols = cols;
    m.off = alloc((int64_t)rows * cols);
    m.ld = r8(cols);
    if (emit) tensor(name, m.off, 2, rows, cols, 0);
    return m;
  }
  int64_t vec(const std::string& name, int n, int kind) {
    const int64_t o = alloc(n);
    tensor(name, o, 1, n, 0, kind);
    return o;
  }
};

void build_cross_params(Builder& b, LM& x, const std::string& p, int C, int H, int hs, int nkv) {
  x.lncw = -1;
  x.Wq = b.mat("", H * hs, C, false);
  for (int h = 0; h < H; ++h)
    b.tensor(p + "heads." + std::to_string(h) + ".query.weight", x.Wq.off + (int64_t)h * hs * C, 2, hs, C, 0);
  for (int j = 0; j < nkv; ++j) {
    x.Wkv[j] = b.mat("", H * 2 * hs, C, false);
    for (int h = 0; h < H; ++h)
      b.tensor(p + "heads." + std::to_string(h) + ".kv_projections." + std::to_string(j) + ".weight",
               x.Wkv[j].off + (int64_t)h * 2 * hs * C, 2, 2 * hs, C, 0);
  }
  x.C0 = b.mat(p + "proj.0.weight", C / 2, hs * H);
  x.bc0 = b.vec(p + "proj.0.bias", C / 2, 1);
  x.C2 = b.mat(p + "proj.2.weight", C, C / 2);
  x.bc2 = b.vec(p + "proj.2.bias", C, 1);
}

void build_layout(mmt_ctx* c) {
  Builder b{c};
  const int C = c->C, H = c->H, hs = c->hs, hh = c->hh, M = c->M, L = c->L;
  c->emb_begin = b.cur;
  for (int i = 0; i < M; ++i) {
    c->post[i].tok = b.alloc((int64_t)c->V[i] * C);
    b.tensor("pre_block.token_embedding_tables." + std::to_string(i) + ".weight", c->post[i].tok, 2, c->V[i], C, 0);
  }
  c->pos_off = b.alloc((int64_t)c->T * C);
  b.tensor("pre_block.position_embedding_table.weight", c->pos_off, 2, c->T, C, 0);
  c->emb_end = b.cur;
  c->lm.resize((size_t)L * M);
  const char* kinds[3] = {"key", "query", "value"};
  for (int l = 0; l < L; ++l) {
    c->layer_begin.push_back(b.cur);
    const std::string bl = "blocks." + std::to_string(l) + ".";
    for (int i = 0; i < M; ++i) {
      LM& x = c->lm[(size_t)l * M + i];
      const std::string p = bl + "sa_layers." + std::to_string(i) + ".";
      x.W1 = b.mat("", 3 * H * hh, C, false);
      x.b1 = b.alloc(3 * H * hh);
      x.w2 = b.alloc((int64_t)3 * H * hs * hh);
      for (int k = 0; k < 3; ++k)
        for (int h = 0; h < H; ++h) {
          const std::string hp = p + "heads." + std::to_string(h) + "." + kinds[k] + ".";
          const int blk = k * H + h;
          b.tensor(hp + "0.weight", x.W1.off + (int64_t)blk * hh * C, 2, hh, C, 0);
          b.tensor(hp + "0.bias", x.b1 + (int64_t)blk * hh, 1, hh, 0, 1);
          b.tensor(hp + "2.weight", x.w2 + (int64_t)blk * hs * hh, 2, hs, hh, 0);
        }
      x.P0 = b.mat(p + "proj.0.weight", C / 2, hs * H);
      x.bp0 = b.vec(p + "proj.0.bias", C / 2, 1);
      x.P2 = b.mat(p + "proj.2.weight", C, C / 2);
      x.bp2 = b.vec(p + "proj.2.bias", C, 1);
    }
    for (int i = 0; i < M; ++i) {
      LM& x = c->lm[(size_t)l * M + i];
      const std::string p = bl + "ffwd_layers." + std::to_string(i) + ".net.";
      x.F0 = b.mat(p + "0.weight", 4 * C, C);
      x.bf0 = b.vec(p + "0.bias", 4 * C, 1);
      x.F2 = b.mat(p + "2.weight", C, 4 * C);
      x.bf2 = b.vec(p + "2.bias", C, 1);
    }
    for (int i = 0; i < M; ++i) {
      LM& x = c->lm[(size_t)l * M + i];
      x.ln1w = b.vec(bl + "ln1_layers." + std::to_string(i) + ".weight", C, 2);
      x.ln1b = b.vec(bl + "ln1_layers." + std::to_string(i) + ".bias", C, 3);
      x.ln2w = b.vec(bl + "ln2_layers." + std::to_string(i) + ".weight", C, 2);
      x.ln2b = b.vec(bl + "ln2_layers." + std::to_string(i) + ".bias", C, 3);
    }
    for (int i = 0; i < M; ++i) {
      LM& x = c->lm[(size_t)l * M + i];
      if (!(c->cfg.cross_attention[i] && M > 1)) continue;
      x.cross = true;
      const std::string p = bl + "cross_attention_layers." + std::to_string(i) + ".";
      build_cross_params(b, x, p, C, H, hs, M - 1);
      x.lncw = b.vec(bl + "ln_cross_layers." + std::to_string(i) + ".weight", C, 2);
      x.lncb = b.vec(bl + "ln_cross_layers." + std::to_string(i) + ".bias", C, 3);
    }
    c->layer_end.push_back(b.cur);
  }
  c->post_begin = b.cur;
  for (int i = 0; i < M; ++i) {
    c->post[i].lnw = b.vec("post_block.fin_norm_layers." + std::to_string(i) + ".weight", C, 2);
    c->post[i].lnb = b.vec("post_block.fin_norm_layers." + std::to_string(i) + ".bias", C, 3);
  }
  for (int i = 0; i < M; ++i) {
    const std::string p = "post_block.soft_score_layers." + std::to_string(i) + ".";
    const int V = c->V[i], V2 = V / 2;
    c->post[i].H0 = b.mat(p + "0.weight", V2, C);
    c->post[i].b0 = b.vec(p + "0.bias", V2, 1);
    c->post[i].H2 = b.mat(p + "2.weight", V, V2);
    c->post[i].b2 = b.vec(p + "2.bias", V, 1);
  }
  c->post_end = b.cur;
  c->nactive = b.cur;
  // parameters that never receive a gradient: a CrossAttention built with zero KV modalities (M == 1,
  // model.py:198-200, 238). torch's AdamW skips them (no decay): they live past the active prefix.
  for (int l = 0; l < L; ++l)
    for (int i = 0; i < M; ++i) {
      if (!(c->cfg.cross_attention[i] && M == 1)) continue;
      LM dummy;
      const std::string bl = "blocks." + std::to_string(l) + ".";
      build_cross_params(b, dummy, bl + "cross_attention_layers." + std::to_string(i) + ".", C, H, hs, 0);
      b.vec(bl + "ln_cross_layers." + std::to_string(i) + ".weight", C, 2);
      b.vec(bl + "ln_cross_layers." + std::to_string(i) + ".bias", C, 3);
    }
  c->nparams = b.cur;

  // packed bf16 weights: every GEMM weight matrix with a padded leading dimension
  int64_t pk = 0;
  auto add = [&](Mat& m) {
    if (m.off < 0 || m.rows == 0) return;
    m.pk = pk;
    pk += rup((int64_t)m.rows * m.ld, 64);
    PackSeg s;
    s.src_off = m.off; s.dst_off = m.pk; s.rows = m.rows; s.cols = m.cols; s.dld = m.ld; s.pad_ = 0;
    const int si = (int)c->segs.size();
    c->segs.push_back(s);
    for (int r0 = 0; r0 < m.rows; r0 += 32) { c->tasks.push_back(si); c->tasks.push_back(r0); }
  };
  for (auto& x : c->lm) {
    add(x.W1); add(x.P0); add(x.P2); add(x.F0); add(x.F2);
    if (x.cross) {
      add(x.Wq);
      for (int j = 0; j < M - 1; ++j) add(x.Wkv[j]);
      add(x.C0); add(x.C2);
    }
  }
  for (int i = 0; i < M; ++i) { add(c->post[i].H0); add(c->post[i].H2); }
  c->pack_elems = pk;
  if (c->fp8) {
    // MX-fp8 copies of the weights of the fp8 forward GEMMs (Q/K/V stage 1, FFN, cross query)
    int64_t b8 = 0;
    auto add8 = [&](Mat& m) {
      if (m.off < 0 || m.rows == 0) return;
      m.ld8 = (int)rup(m.cols, 16);
      m.lds8 = (int)rup((m.cols + 31) / 32, 4);
      m.pk8 = b8;
      b8 += rup((int64_t)m.rows * m.ld8, 256);
      m.ps8 = b8;
      b8 += rup((int64_t)m.rows * m.lds8, 256);
      MxSeg sg{};
      sg.src = m.off; sg.dst = m.pk8; sg.sdst = m.ps8; sg.rows = m.rows; sg.cols = m.cols; sg.ld_src = m.cols;
      sg.ld8 = m.ld8; sg.lds8 = m.lds8;
      c->mxsegs.push_back(sg);
      c->mx_units = std::max(c->mx_units, m.rows * m.lds8);
    };
    for (auto& x : c->lm) {
      add8(x.W1); add8(x.F0); add8(x.F2);
      if (x.cross) add8(x.Wq);
    }
    c->pack8_bytes = b8;
  }
  for (int i = 0; i < M; ++i) {
    c->ldv[i] = r8(c->V[i]);
    c->ldvh[i] = r8(c->V[i] / 2);
  }
}

// -------------------------------------------------------------------------------------------
// workspace plan for batch B
// -------------------------------------------------------------------------------------------
// the non-finite-loss flag words sit right after the packed weights, at the same offset for every
// batch size, so querying them never replaces the plan of a pending backward / decode
size_t flag_offset(const mmt_ctx* c) { return (size_t)rup(c->pack_elems * 2, 256); }

// -------------------------------------------------------------------------------------------
// workspace plan for batch B (continued)
// -------------------------------------------------------------------------------------------
void make_plan(mmt_ctx* c, int B) {
  Plan& p = c->plan;
  p = Plan();
  p.B = B;
  size_t cur = 0;
  auto A = [&](size_t bytes) { const size_t o = cur; cur += (size_t)rup((int64_t)bytes, 256); return o; };
  const int64_t R = (int64_t)B * c->T;
  const int C = c->C, M = c->M, H = c->H;
  const size_t f4 = 4, b2 = 2;
  const int ldh1 = r8(3 * H * c->hh), ldp = r8(C / 2);
  const size_t bhT = (size_t)B * H * c->T;
  const size_t mbytes = c->cfg.dropout > 0.f ? (size_t)mmt_attn_mask_dwords(B, H, c->T) * 4 : 0;
  p.pack = A((size_t)c->pack_elems * b2);
  p.flag = A(256);  // == flag_offset(c): fixed for every batch size (mmt_loss_flag_offset)
  p.pack8 = c->fp8 ? A((size_t)c->pack8_bytes) : 0;
  p.act.resize((size_t)c->L * M);
  for (int i = 0; i < M; ++i) p.xemb[i] = A(R * C * f4);
  for (int l = 0; l < c->L; ++l)
    for (int i = 0; i < M; ++i) {
      ActLM& a = p.act[(size_t)l * M + i];
      const LM& x = c->lm[(size_t)l * M + i];
      a.a = A(R * C * b2); a.mean1 = A(R * f4); a.rstd1 = A(R * f4);
      a.h1 = A(R * ldh1 * b2); a.qkv = A(R * 3 * C * b2); a.o = A(R * C * b2); a.lse = A(bhT * f4);
      a.p1 = A(R * ldp * b2); a.x1 = A(R * C * f4);
      a.c = A(R * C * b2); a.mean2 = A(R * f4); a.rstd2 = A(R * f4);
      a.f = A(R * 4 * C * b2); a.x2 = A(R * C * f4);
      a.fm = c->relu_bits ? A(R * (4 * C / 8)) : 0;
      a.x2h = c->any_cross ? A(R * C * b2) : 0;
      a.dm = mbytes ? A(mbytes) : 0;
      if (c->fp8) {
        const int ldsC = (int)rup(C / 32, 4), ldsF = (int)rup(4 * C / 32, 4);
        a.a8 = A(R * C); a.c8 = A(R * C); a.f8 = A(R * 4 * C);
        if (x.cross) a.d8 = A(R * C);
        a.as8 = A(R * ldsC); a.cs8 = A(R * ldsC); a.fs8 = A(R * ldsF);
        if (x.cross) a.ds8 = A(R * ldsC);
      }
      if (x.cross) {
        a.d = A(R * C * b2); a.meanc = A(R * f4); a.rstdc = A(R * f4); a.qc = A(R * C * b2);
        for (int j = 0; j < M - 1; ++j) {
          a.kv[j] = A(R * 2 * C * b2);
          a.ocj[j] = A(R * C * b2);
          a.lsej[j] = A(bhT * f4);
          a.dmj[j] = mbytes ? A(mbytes) : 0;
        }
        a.oc = A(R * C * b2); a.pc = A(R * ldp * b2); a.x3 = A(R * C * f4);
      }
    }
  int maxvh = 8, maxv = 8;
  for (int i = 0; i < M; ++i) { maxvh = std::max(maxvh, c->ldvh[i]); maxv = std::max(maxv, c->ldv[i]); }
  for (int i = 0; i < M; ++i) {
    p.lnf16[i] = A(R * C * b2); p.meanf[i] = A(R * f4); p.rstdf[i] = A(R * f4);
    p.hh[i] = A(R * c->ldvh[i] * b2); p.dlog[i] = A(R * c->ldv[i] * b2);
  }
  for (int i = 0; i < M; ++i) {
    p.dres[i] = A(R * C * f4); p.dln[i] = A(R * C * f4);
    p.eperm[i] = A(R * 4);
    p.celoss[i] = A(512 * 4);
    for (int k = 0; k < 8; ++k) p.dres16[k][i] = A(R * C * b2);
    p.gdo[i] = A(R * C * b2); p.gqkv[i] = A(R * 3 * C * b2);
    for (int k = 0; k < 2; ++k) {
      p.gbig[k][i] = A(R * std::max(4 * C, maxvh) * b2);
      p.gq[k][i] = A(R * C * b2);
      p.gh1[k][i] = A(R * ldh1 * b2); p.gp[k][i] = A(R * ldp * b2);
      p.gpc[k][i] = (c->any_cross && c->cfg.cross_attention[i]) ? A(R * ldp * b2) : p.gp[k][i];
      if (c->any_cross && c->cfg.cross_attention[i])
        for (int j = 0; j < M - 1; ++j) p.dkv[k][i][j] = A(R * 2 * C * b2);
    }
    for (int j = 0; j < M; ++j) p.dvec[i][j] = A(bhT * f4);
  }
  // weight-gradient split-K slabs: room for 16 splits of the largest grouped dW launch
  {
    int64_t mx = 0, heads = 0;
    mx = std::max<int64_t>(mx, (int64_t)M * 4 * C * C);                  // FFN (either matrix)
    mx = std::max<int64_t>(mx, (int64_t)M * r8(3 * H * c->hh) * C);      // Q/K/V stage 1
    mx = std::max<int64_t>(mx, (int64_t)MMT_MAX_GROUP * 2 * C * C);      // cross-attention KV
    for (int i = 0; i < M; ++i) heads += (int64_t)c->V[i] * (c->V[i] / 2 + 4) + (int64_t)(c->V[i] / 2 + 4) * C;
    mx = std::max<int64_t>(mx, heads);
    p.slab_bytes = (size_t)mx * 16 * f4;
    p.slab = A(p.slab_bytes);
  }
  // decode scratch (tiny: B rows)
  p.dec_x.resize((size_t)c->L * M * 3);
  for (int i = 0; i < M; ++i) {
    Plan::Dec& d = p.dec[i];
    d.x0 = A(B * C * f4); d.a16 = A(B * C * b2); d.mean = A(B * f4); d.rstd = A(B * f4);
    d.h1 = A(B * ldh1 * b2); d.qkv = A(B * 3 * C * b2); d.o16 = A(B * C * b2); d.p1 = A(B * ldp * b2);
    d.f = A(B * 4 * C * b2); d.x2h = A(B * C * b2); d.d16 = A(B * C * b2); d.qc = A(B * C * b2);
    d.oc = A(B * C * b2); d.pc = A(B * ldp * b2); d.lnf16 = A(B * C * b2); d.hh = A(B * c->ldvh[i] * b2);
    for (int j = 0; j < M - 1; ++j) d.kv[j] = A(B * 2 * C * b2);
  }
  for (auto& o : p.dec_x) o = A(B * C * f4);
  p.total = cur;
}

template <class T>
inline T* at(void* ws, size_t off) { return reinterpret_cast<T*>(reinterpret_cast<char*>(ws) + off); }

// grouped-GEMM helpers ------------------------------------------------------------------------
GemmProblem gp_fwd(const bf16_t* X, int ldx, const bf16_t* Wpk, const Mat& W, int R) {
  GemmProblem g{};
  g.A = X; g.lda = ldx; g.B = Wpk + W.pk; g.ldb = W.ld;
  g.M = R; g.N = W.rows; g.K = W.cols; g.alpha = 1.f;
  return g;
}
// dX = dY W : dY [R, W.rows] (ld ldy), result [R, W.cols]
GemmProblem gp_dx(const bf16_t* dY, int ldy, const bf16_t* Wpk, const Mat& W, int R) {
  GemmProblem g{};
  g.A = dY; g.lda = ldy; g.B = Wpk + W.pk; g.ldb = W.ld;
  g.M = R; g.N = W.cols; g.K = W.rows; g.alpha = 1.f;
  return g;
}
// dW += dY^T X : out [W.rows, W.cols] fp32 in the grad buffer
GemmProblem gp_dw(const bf16_t* dY, int ldy, const bf16_t* X, int ldx, float* grads, const Mat& W, int R) {
  GemmProblem g{};
  g.A = dY; g.lda = ldy; g.B = X; g.ldb = ldx;
  g.M = W.rows; g.N = W.cols; g.K = R; g.o32 = grads + W.off; g.ldc = W.cols; g.alpha = 1.f;
  return g;
}

// live-probe pattern match: "label" exact, "*suffix" (e.g. "*_dw": every weight-gradient GEMM),
// "prefix*"; returns the index of the first matching pattern or -1
int probe_match_one(const mmt_ctx* c, const char* what) {
  const size_t n = std::strlen(what);
  for (size_t i = 0; i < c->probe_pats.size(); ++i) {
    const std::string& p = c->probe_pats[i];
    if (p.empty()) continue;
    if (p[0] == '*') {
      const size_t k = p.size() - 1;
      if (n >= k && std::strcmp(what + n - k, p.c_str() + 1) == 0) return (int)i;
    } else if (p.back() == '*') {
      if (std::strncmp(what, p.c_str(), p.size() - 1) == 0) return (int)i;
    } else if (p == what) {
      return (int)i;
    }
  }
  return -1;
}
// a merged launch is labelled "a+b+...": it matches when any part does
int probe_match(const mmt_ctx* c, const char* what) {
  std::string w(what);
  size_t b = 0;
  while (true) {
    const size_t e = w.find('+', b);
    const int r = probe_match_one(c, w.substr(b, e == std::string::npos ? std::string::npos : e - b).c_str());
    if (r >= 0 || e == std::string::npos) return r;
    b = e + 1;
  }
}

// algorithmic cost of one grouped GEMM launch: 2MNK flops; every operand read once and every
// output written once (bf16 activations / packed bf16 weights, fp32 bias / residual / outputs)
void gemm_cost(const GemmBatch& b, int epi, double* fl, double* by) {
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    const double M = P.M, N = P.N, K = P.K;
    *fl += 2.0 * M * N * K;
    double x = (M * K + N * K) * 2.0;
    if (P.bias) x += N * 4.0;
    const bool f32_out = epi == EPI_BIAS_RESID_F32 || epi == EPI_STORE_F32 || epi == EPI_ACC_F32;
    x += M * N * (f32_out ? 4.0 : 2.0);
    if (epi == EPI_BIAS_RESID_F32) x += M * N * 4.0 + (P.o16 ? M * N * 2.0 : 0.0);
    if (epi == EPI_ACC_F32) x += M * N * 4.0;
    // tanh' / ReLU' operand: the bf16 hidden rows, or one bit per element (ReLU' bits, mask8)
    if (epi == EPI_DTANH_BF16 || epi == EPI_DRELU_BF16) x += (epi == EPI_DRELU_BF16 && P.mask8) ? M * N / 8.0 : M * N * 2.0;
    // ReLU' bits written by the forward (EPI_BIAS_RELU_BF16 with mask8)
    if (epi == EPI_BIAS_RELU_BF16 && P.mask8) x += M * N / 8.0;
    // MX-fp8 copy of the output (the next fp8 GEMM's A operand): e4m3fn bytes + one E8M0 byte per 32
    if (P.o8) x += M * N * (1.0 + 1.0 / 32.0);
    // fused LayerNorm backward: LN input and the accumulated gradient read, that gradient (+ its bf16
    // copy) written, row statistics read
    if (epi == EPI_LN_BWD_F32) x += M * N * 8.0 + (P.o16 ? M * N * 2.0 : 0.0) + M * 8.0;
    *by += x;
  }
}

// weight gradient dW[M,N] += dY[K,M]^T X[K,N]: both operands read once, the fp32 gradient written once
void wgrad_cost(const GemmBatch& b, double* fl, double* by) {
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    const double M = P.M, N = P.N, K = P.K;
    *fl += 2.0 * M * N * K;
    *by += (M * K + N * K) * 2.0 + M * N * 4.0;
  }
}

// causal attention, causal-useful count (a = 1/2): per (batch, head, KV stream)
// forward 2 T^2 hs (QK^T and PV over the T(T+1)/2 kept scores), backward 2.5x that (S, dP, dV,
// dQ, dK). Bytes: Q, K, V, O (+ per-stream outputs of a multi-stream problem), log-sum-exp and
// dropout keep bits read / written once; backward adds dO, the row dot products and dQ, dK, dV.
void attn_cost(const AttnBatch& ab, int B, int T, int H, int hs, bool bwd, bool drop, double* fl, double* by) {
  const double C = (double)H * hs, rows = (double)B * T, bhT = (double)B * H * T;
  const double mask = drop ? (double)mmt_attn_mask_dwords(B, H, T) * 4.0 : 0.0;
  for (int g = 0; g < ab.count; ++g) {
    const double ns = ab.p[g].nstreams;
    const double f = 2.0 * (double)B * H * ns * (double)T * T * hs;
    *fl += bwd ? 2.5 * f : f;
    double x = rows * C * 2.0 * (2.0 + 2.0 * ns) + ns * (bhT * 4.0 + mask);  // q, o, k_j, v_j, lse_j, bits
    if (ns > 1) x += ns * rows * C * 2.0;                                      // per-stream outputs o_j
    if (bwd) x += rows * C * 2.0 * (2.0 + 2.0 * ns) + ns * bhT * 4.0;         // dO, dQ, dK_j, dV_j, dvec_j
    if (bwd && ab.p[g].q2_w2) {
      // the stage-2 backward in the epilogue: dQ / dK / dV not written; h1 read, dh1 written (3 H x hs/2
      // columns each), W2 read and dW2 written (algorithmic: once; the kernel adds per workgroup through L2);
      // flops: dh1 = dX W2 and dW2 = dX^T h1
      const double hh = hs / 2;
      x += -rows * C * 2.0 * 3.0 + 2.0 * rows * 3.0 * H * hh * 2.0 + 3.0 * H * hs * hh * 4.0 * 2.0;
      *fl += 2.0 * 2.0 * rows * 3.0 * C * hh;
    }
    *by += x;
  }
}

// MX-fp8 forward linear: A = e4m3fn activations [R, K] (lda bytes) + exponents, B = the weight's
// MX-fp8 copy in the fp8 pack region
GemmProblem gp_f8(const uint8_t* X8, int ldx, const uint8_t* Xs, int ldxs, const uint8_t* w8, const Mat& W, int R) {
  GemmProblem g{};
  g.A = reinterpret_cast<const bf16_t*>(X8); g.lda = ldx; g.sa = Xs; g.lds_a = ldxs;
  g.B = reinterpret_cast<const bf16_t*>(w8 + W.pk8); g.ldb = W.ld8; g.sb = w8 + W.ps8; g.lds_b = W.lds8;
  g.M = R; g.N = W.rows; g.K = W.cols; g.alpha = 1.f;
  return g;
}

// dropout sites (model.py:69 SA probabilities, :91 SA projection, :151 CA probabilities,
// :116 CA projection, :171 FFN output); one hash key per (seed, layer, modality, site)
enum DropSite { DS_SA_PROB = 0, DS_SA_PROJ = 1, DS_FFN = 2, DS_CA_PROB = 3, DS_CA_PROJ = 4 };

struct Runner {
  mmt_ctx* c;
  hipStream_t s;
  void* ws;
  const float* params;
  const bf16_t* wpk;
  int B, R;
  int rc = MMT_OK;
  bool drop = false;  // dropout active for this forward / its backward
  uint64_t seed = 0;

  // element kept iff mmt_keep(mmt_hash(key, row, col >> 1), col, thr) ; kept values scaled by 1 / (1 - p)
  template <class Pm>
  void set_drop(Pm& p, int l, int i, int site) const {
    if (!drop) { p.drop_key = 0; p.drop_thr = 0; p.drop_scale = 1.f; return; }
    const double pr = c->cfg.dropout;
    p.drop_key = mmt_hash((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)((l * MAXM + i) * 8 + site));
    p.drop_thr = (uint32_t)std::min(65535.0, std::max(1.0, std::floor(pr * 65536.0)));  // 16-bit halves (mmt_keep)
    p.drop_scale = (float)(1.0 / (1.0 - pr));
  }

  bool ok(hipError_t e, const char* what) {
    if (e != hipSuccess && rc == MMT_OK) rc = fail(c, MMT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return e == hipSuccess;
  }
  // live kernel timing (mmt_probe_set): HIP events around every launch whose label matches one of
  // the probe patterns, recorded on the stream the launch goes to (the side stream for weight
  // gradients), each tagged with the launch's algorithmic flops and bytes
  int probe_begin(const char* what, hipStream_t st) {
    if (!c->probe_on || c->probe_pats.empty()) return -1;
    const int pat = probe_match(c, what);
    if (pat < 0) return -1;
    if (c->probe_events.size() >= c->probe_pool.size()) return -1;  // pool exhausted: stop recording
    mmt_ctx::ProbeEv e{};
    e.a = c->probe_pool[c->probe_events.size()].first;
    e.b = c->probe_pool[c->probe_events.size()].second;
    e.pat = pat;
    hipEventRecord(e.a, st);
    c->probe_events.push_back(e);
    return (int)c->probe_events.size() - 1;
  }
  void probe_end(int id, hipStream_t st, double flops, double bytes) {
    if (id < 0) return;
    mmt_ctx::ProbeEv& e = c->probe_events[id];
    e.flops = flops;
    e.bytes = bytes;
    hipEventRecord(e.b, st);
  }
  // MX-fp8 forward GEMM (precision fp8): A / B e4m3fn + E8M0 (mmt_launch_gemm_f8)
  void gemm8(const GemmBatch& b, int epi, const char* what) {
    if (rc != MMT_OK) return;
    const int id = probe_begin(what, s);
    if (gemm_hint) {
      GemmBatch h = b;
      h.tile_hint = gemm_hint;
      ok(mmt_launch_gemm_f8(h, epi, s), what);
    } else {
      ok(mmt_launch_gemm_f8(b, epi, s), what);
    }
    if (id >= 0) {
      double fl = 0, by = 0;
      gemm_cost(b, epi, &fl, &by);
      // 1-byte operands plus one E8M0 exponent byte per 32 K elements of every row of A and B
      for (int g = 0; g < b.count; ++g) by -= ((double)b.p[g].M + b.p[g].N) * b.p[g].K * (1.0 - 1.0 / 32.0);
      probe_end(id, s, fl, by);
    }
  }
  // backward-data GEMM dy = A B (EPI_STORE_F32 into lb's dy) followed by the LayerNorm backward lb
  // (model.py:189-190, 210, 330 under autograd): ONE launch with the LayerNorm fused into the GEMM's
  // epilogue when every problem's rows fit one tile (C == 256 or 512; MMT_LN_FUSE=0 disables), else
  // the two passes. The fused launch never materialises dy (the fp32 round trip of the two-pass form)
  void gemm_ln_bwd(const GemmBatch& dx, const LnBatch& lb, int R, int C, const char* gname, const char* lname) {
    if (rc != MMT_OK) return;
    static const bool fuse = [] {
      const char* e = getenv("MMT_LN_FUSE");
      return e ? atoi(e) != 0 : true;
    }();
    if (fuse && lb.count == dx.count) {
      GemmBatch f = dx;
      for (int g = 0; g < f.count; ++g) {
        GemmProblem& P = f.p[g];
        const LnProblem& Lp = lb.p[g];
        P.o32 = Lp.dx; P.ldc = C;
        P.resid = Lp.x; P.ldres = C;
        P.ln_gamma = Lp.gamma; P.ln_mean = Lp.mean; P.ln_rstd = Lp.rstd;
        P.ln_dgamma = Lp.dgamma; P.ln_dbeta = Lp.dbeta;
        P.o16 = Lp.dx16; P.ldo16 = C; P.dbias = Lp.dsum;
        P.drop_key = Lp.drop_key; P.drop_thr = Lp.drop_thr; P.drop_scale = Lp.drop_scale;
        P.bias = nullptr; P.aux = nullptr; P.split_stride = 0;
      }
      if (mmt_gemm_ln_bwd_ok(f)) {
        const int id = probe_begin(gname, s);
        ok(mmt_launch_gemm_ln_bwd(f, s), gname);
        if (id >= 0) {
          double fl = 0, by = 0;
          gemm_cost(f, EPI_LN_BWD_F32, &fl, &by);
          probe_end(id, s, fl, by);
        }
        return;
      }
    }
    gemm(dx, true, false, EPI_STORE_F32, 1, gname);
    ok(mmt_launch_ln_bwd(lb, R, C, s), lname);
  }
  // the attention out-projection Linear(C, C/2) -> tanh -> Linear(C/2, C) + dropout + residual as one fused
  // launch (mmt_launch_mlp2: h stays in LDS between the products); false (nothing launched) when the
  // shape is outside the fused kernel or MMT_MLP2=0, and the caller runs the two GEMMs
  // bwd: the backward-data pair (mmt_launch_mlp2_bwd: dh = (dY W2) tanh', dx = dh W0)
  bool mlp2(const GemmProblem* g1s, const GemmProblem* g2s, int n, const char* what, bool bwd = false) {
    // forward fused by default: C1 8.80 -> 8.70 ms/step (standalone 45.9 -> 43.0 us at C1, 119.6 -> 112.8 us
    // at the target). The backward pair: fused at C = 256 only by default (MMT_MLP2_BWD: 2 = that, 1 =
    // every width, 0 = never). Standalone the fused backward measured 33.5 / 80.6 us against 29.3 / 61.6 us
    // for the pair (C1 / target, tools/mlp2_bench.py; one block per CU at 136 KiB of LDS with both B
    // operands read transposed cannot hide what the two 2-3 blocks-per-CU GEMMs overlap, profiles/r5h_*),
    // but in the C1 step beside the side stream it wins: 7.975 / 7.982 -> 7.949 / 7.960 ms (round 6,
    // profiles/r6x_c1_env_ab.txt); at C = 512 it stays two GEMMs
    static const bool on = [] {
      const char* e = getenv("MMT_MLP2");
      return e ? atoi(e) != 0 : true;
    }();
    static const int bwd_mode = [] {
      const char* e = getenv("MMT_MLP2_BWD");
      return e ? atoi(e) : 2;
    }();
    const bool on_bwd = bwd_mode == 1 || (bwd_mode == 2 && n >= 1 && g1s[0].N == 128);
    if (rc != MMT_OK || !on || (bwd && !on_bwd) || n < 1) return false;
    Mlp2Batch chunk[(MMT_MAX_GROUP + MMT_MLP2_GROUP - 1) / MMT_MLP2_GROUP] = {};
    const int nch = (n + MMT_MLP2_GROUP - 1) / MMT_MLP2_GROUP;
    for (int i = 0; i < n; ++i) {
      Mlp2Batch& b = chunk[i / MMT_MLP2_GROUP];
      b.g1[b.count] = g1s[i];
      b.g2[b.count] = g2s[i];
      ++b.count;
    }
    for (int k = 0; k < nch; ++k)
      if (!(bwd ? mmt_mlp2_bwd_ok(chunk[k]) : mmt_mlp2_ok(chunk[k]))) return false;
    const int id = probe_begin(what, s);
    for (int k = 0; k < nch; ++k) ok(bwd ? mmt_launch_mlp2_bwd(chunk[k], s) : mmt_launch_mlp2(chunk[k], s), what);
    if (id >= 0) {
      double fl = 0, by = 0;
      GemmBatch g1{}, g2{};
      g1.count = g2.count = n;
      for (int g = 0; g < n; ++g) { g1.p[g] = g1s[g]; g2.p[g] = g2s[g]; }
      gemm_cost(g1, bwd ? EPI_DTANH_BF16 : EPI_BIAS_TANH_BF16, &fl, &by);
      gemm_cost(g2, bwd ? EPI_STORE_BF16 : EPI_BIAS_RESID_F32, &fl, &by);
      for (int g = 0; g < n; ++g) by -= (double)g2s[g].M * g2s[g].K * 2.0;  // h / dh is not read back
      probe_end(id, s, fl, by);
    }
    return true;
  }
  // forward residual GEMM with the next LayerNorm's forward fused (mmt_launch_gemm_resid_ln)
  bool gemm_resid_ln(const GemmBatch& b, const char* what) {
    if (rc != MMT_OK || !mmt_gemm_resid_ln_ok(b)) return false;
    const int id = probe_begin(what, s);
    ok(mmt_launch_gemm_resid_ln(b, s), what);
    if (id >= 0) {
      double fl = 0, by = 0;
      gemm_cost(b, EPI_BIAS_RESID_F32, &fl, &by);
      for (int g = 0; g < b.count; ++g)
        if (b.p[g].lnf_y) by += (double)b.p[g].M * b.p[g].N * 2.0 + b.p[g].M * 8.0;
      probe_end(id, s, fl, by);
    }
    return true;
  }
  // GemmBatch::tile_hint for the main-stream GEMMs launched while it is set (run_forward: beside the
  // side stream's keep-bit launches)
  int gemm_hint = 0;
  void gemm(const GemmBatch& b, bool akc, bool bkc, int epi, int splits, const char* what) {
    if (rc != MMT_OK) return;
    const int id = probe_begin(what, s);
    if (gemm_hint) {
      GemmBatch h = b;
      h.tile_hint = gemm_hint;
      ok(mmt_launch_gemm(h, akc, bkc, epi, splits, s), what);
    } else {
      ok(mmt_launch_gemm(b, akc, bkc, epi, splits, s), what);
    }
    if (id >= 0) {
      double fl = 0, by = 0;
      gemm_cost(b, epi, &fl, &by);
      probe_end(id, s, fl, by);
    }
  }
  // fork the side stream off the main one (everything enqueued on `s` so far happens first)
  hipStream_t side_stream() const { return c->side_off ? nullptr : c->side; }
  hipStream_t side() {
    if (!side_stream()) return s;
    hipEvent_t e = c->evpool[c->evnext++ % c->evpool.size()];
    ok(hipEventRecord(e, s), "event record");
    ok(hipStreamWaitEvent(c->side, e, 0), "stream wait");
    return c->side;
  }
  // the main stream waits for everything enqueued on the side stream
  void join() {
    flush(true);
    if (!side_stream()) return;
    hipEvent_t e = c->evpool[c->evnext++ % c->evpool.size()];
    ok(hipEventRecord(e, c->side), "event record");
    ok(hipStreamWaitEvent(s, e, 0), "stream wait");
  }
  // weight-gradient GEMMs go to the side stream in batches: dwgemm() queues one, flush() forks the
  // side stream once (after everything its queued GEMMs read is enqueued on the main stream) and
  // launches them. Every fork / join is a barrier packet costing ~10 us of main-stream idle, so
  // the stage code flushes a few times per layer instead of forking per GEMM.
  std::vector<std::pair<GemmBatch, const char*>> pend;
  // hold: the stage's intermediate flushes keep their launches queued for the stage-end flush (one fork
  // per stage instead of one per flush point; each fork's event record costs the main stream a gap)
  bool hold = false;
  void flush(bool force = false) {
    if (hold && !force && rc == MMT_OK) return;
    if (pend.empty() || rc != MMT_OK) { pend.clear(); return; }
    hipStream_t ss = side_stream() ? side() : s;
    // merge consecutive queued weight-gradient batches of the same tile kind into one launch (up
    // to MMT_MAX_GROUP problems): more tiles per launch -> fewer K splits -> fewer partial bytes
    std::vector<std::pair<GemmBatch, std::string>> merged;
    for (auto& q : pend) {
      if (!merged.empty()) {
        GemmBatch& m = merged.back().first;
        if (m.count + q.first.count <= MMT_MAX_GROUP && mmt_gemm_wgrad_big(m) == mmt_gemm_wgrad_big(q.first)) {
          for (int g = 0; g < q.first.count; ++g) m.p[m.count++] = q.first.p[g];
          merged.back().second += std::string("+") + q.second;
          continue;
        }
      }
      merged.emplace_back(q.first, q.second);
    }
    for (auto& q : merged) wgrad(q.first, q.second.c_str(), ss);
    pend.clear();
  }
  void wgrad(const GemmBatch& b, const char* what, hipStream_t st) {
    const int id = probe_begin(what, st);
    ok(mmt_launch_gemm_wgrad(b, W<float>(c->plan.slab), (int64_t)c->plan.slab_bytes, st), what);
    if (id >= 0) {
      double fl = 0, by = 0;
      wgrad_cost(b, &fl, &by);
      probe_end(id, st, fl, by);
    }
  }
  // weight-gradient GEMMs share one split-K slab region: they run in launch order on ONE stream
  // (the side stream when there is one), so no two of them ever write the slabs at once (a
  // probed launch no longer jumps to the main stream: ADVICE r1)
  void dwgemm(const GemmBatch& b, const char* what, int hint = 0) {
    if (rc != MMT_OK) return;
    pend.emplace_back(b, what);  // launched (merged) at the next flush(), on the side stream if any
    pend.back().first.tile_hint = hint;
    // hs 64 (the two-pass attention backward beside them): 96 blocks per launch leave it more CUs. Same box,
    // two passes: C3 142.6-142.9 -> 141.0-141.2 ms (its attention backward 1244 -> 1038 us live), target
    // 19.36-19.40 -> 19.28-19.31, C4 equal; at hs 32 (C1) 96 measured equal to 128 on one box, +0.2 % on
    // another (profiles/r6ak_wgrad_blocks_ab.txt, r6al_wgrad96_ab.txt). MMT_WGRAD_BLOCKS overrides both
    pend.back().first.dw_blocks = c->hs >= 64 ? 96 : 0;
  }
  void attn(const AttnBatch& ab, bool bwd, float scale, const char* what) {
    if (rc != MMT_OK) return;
    const int id = probe_begin(what, s);
    if (bwd) ok(mmt_launch_attn_bwd(ab, B, c->T, c->H, c->hs, scale, s), what);
    else ok(mmt_launch_attn_fwd(ab, B, c->T, c->H, c->hs, scale, s), what);
    if (id >= 0) {
      double fl = 0, by = 0;
      attn_cost(ab, B, c->T, c->H, c->hs, bwd, drop, &fl, &by);
      probe_end(id, s, fl, by);
    }
  }
  template <class T> T* W(size_t off) { return at<T>(ws, off); }
  const float* P(int64_t off) { return params + off; }
};

// -------------------------------------------------------------------------------------------
// forward
// -------------------------------------------------------------------------------------------
int run_forward(mmt_ctx* c, Runner& r, const int64_t* const* idx, const int64_t* const* tgt, float* const* logits,
                float* losses) {
  const int M = c->M, C = c->C, H = c->H, hs = c->hs, R = r.R, B = r.B, T = c->T;
  const int ldh1 = r8(3 * H * c->hh), ldp = r8(C / 2);
  const float scale = 1.0f / std::sqrt((float)hs);
  Plan& p = c->plan;
  bf16_t* wpk = r.W<bf16_t>(p.pack);
  r.wpk = wpk;
  // keep bits of layer ll's self- and cross-attention dropout, one side-stream launch each (the
  // mask kernel reads nothing the main stream writes: a fork orders it after the previous step)
  hipStream_t ss = r.s;
  // MMT_MASK_AHEAD=1: layer l + 1's keep bits are made while layer l computes (one fork and one join per
  // layer) instead of all later layers' while layer 0 computes. The masks then overlap each layer's attention
  // forward instead of layer 0's GEMMs (C3 attention forward 394 -> 955 us live). Default: from 12 layers on,
  // where the later layers' pile beside layer 0 grows past what one layer's GEMMs hide: C4 (24 layers) 312.4 ->
  // 308.6 ms, C3 (12) 141.1 -> 140.5-140.9, target (6) 19.07 -> 19.04, C1 (6) 7.87 -> 7.90
  // (profiles/r6ab_mask_ab.txt, r6ae_c4_mask_ab.txt); MMT_MASK_AHEAD=0 / 1 forces it
  static const int mask_ahead_env = [] {
    const char* e = getenv("MMT_MASK_AHEAD");
    return e ? atoi(e) : -1;
  }();
  // (2: layer l + 1's bits forked after layer l's self-attention forward, so they overlap that layer's
  // GEMMs, which take the tile hint until the next join, rather than its attention)
  const int ahead_mode = mask_ahead_env >= 0 ? mask_ahead_env : (c->L >= 12 ? 1 : 0);
  const bool mask_ahead = ahead_mode != 0;
  static const int mask_t2 = [] {
    const char* e = getenv("MMT_MASK_T2");
    return e ? atoi(e) : 1;
  }();
  auto gen_masks = [&](int ll) {
    if (ll <= 1 || mask_ahead) ss = r.side();  // layer 0: one fork; layers 1..L-1: one fork for all
    const LM* xl = &c->lm[(size_t)ll * M];
    const ActLM* al = &p.act[(size_t)ll * M];
    AttnBatch mb{}; mb.count = M;
    for (int i = 0; i < M; ++i) {
      r.set_drop(mb.p[i], ll, i, DS_SA_PROB);
      mb.p[i].nstreams = 1; mb.p[i].dmask[0] = r.W<uint32_t>(al[i].dm);
    }
    r.ok(mmt_launch_attn_mask(mb, B, T, H, ss), "attn_mask");
    if (!c->any_cross) return;
    AttnBatch mc{}; mc.count = 0;
    for (int i = 0; i < M; ++i) {
      if (!xl[i].cross) continue;
      AttnProblem& q = mc.p[mc.count++];
      r.set_drop(q, ll, i, DS_CA_PROB);
      q.nstreams = M - 1;
      for (int j = 0; j < M - 1; ++j) q.dmask[j] = r.W<uint32_t>(al[i].dmj[j]);
    }
    if (mc.count) r.ok(mmt_launch_attn_mask(mc, B, T, H, ss), "ca_attn_mask");
  };
  if (!r.ok(mmt_launch_pack(c->d_segs, (int)c->segs.size(), (int64_t)c->tasks.size() / 2, c->d_tasks, r.params, wpk,
                            r.s), "pack"))
    return r.rc;
  const bool f8 = c->fp8;
  uint8_t* w8 = f8 ? r.W<uint8_t>(p.pack8) : nullptr;
  const int ldsC = (int)rup(C / 32, 4), ldsF = (int)rup(4 * C / 32, 4);
  if (f8) {
    r.ok(mmt_launch_mx_quant(c->d_mxsegs, (int)c->mxsegs.size(), c->mx_units, r.params, w8, r.s), "mx_quant");
    if ((C / 32) % 4) {  // exponent bytes past C/32 of a row: finite (127) for the K-step that straddles C
      for (int l = 0; l < c->L; ++l)
        for (int i = 0; i < M; ++i) {
          const ActLM& a = p.act[(size_t)l * M + i];
          r.ok(hipMemsetAsync(r.W<uint8_t>(a.as8), 127, (size_t)R * ldsC, r.s), "memset exps");
          r.ok(hipMemsetAsync(r.W<uint8_t>(a.cs8), 127, (size_t)R * ldsC, r.s), "memset exps");
          if (c->lm[(size_t)l * M + i].cross) r.ok(hipMemsetAsync(r.W<uint8_t>(a.ds8), 127, (size_t)R * ldsC, r.s), "memset exps");
        }
    }
  }
  auto ln8 = [&](LnProblem& q, size_t y8, size_t s8) {
    if (!f8) return;
    q.y8 = r.W<uint8_t>(y8); q.s8 = r.W<uint8_t>(s8); q.ld8 = C; q.lds8 = ldsC;
  };
  {
    EmbBatch eb{};
    eb.count = M;
    for (int i = 0; i < M; ++i) {
      eb.p[i].idx = idx[i]; eb.p[i].tok = r.P(c->post[i].tok); eb.p[i].pos = r.P(c->pos_off);
      eb.p[i].x = r.W<float>(p.xemb[i]); eb.p[i].V = c->V[i];
    }
    r.ok(mmt_launch_embed_fwd(eb, B, T, C, r.s), "embed_fwd");
  }
  std::vector<const float*> xin(M);
  for (int i = 0; i < M; ++i) xin[i] = r.W<float>(p.xemb[i]);
  // LayerNorm forwards already done by the previous residual GEMM's epilogue (lnf_fused: the post
  // block's); fused only in bf16 at C == 256 (whole rows per 256x256 tile), MMT_LN_FUSE=0 or
  // MMT_LN_FUSE_FWD=0 disables
  static const int ln_fuse = [] {
    const char* e = getenv("MMT_LN_FUSE");
    const char* f = getenv("MMT_LN_FUSE_FWD");
    return (e ? atoi(e) != 0 : true) ? (f ? atoi(f) : 1) : 0;
  }();
  // C = 512 (128 x 512 tile) only with MMT_LN_FUSE_FWD=2: measured slower on the 2-stage ring
  // (target 20.09 -> 20.43 ms, profiles/r3u_ab.txt)
  const bool fuse_fwd = ln_fuse && !f8 && (C == 256 || (C == 512 && ln_fuse == 2));
  std::vector<char> ln1_done(M, 0), lnf_done(M, 0);
  for (int l = 0; l < c->L && r.rc == MMT_OK; ++l) {
    const LM* x = &c->lm[(size_t)l * M];
    const ActLM* a = &p.act[(size_t)l * M];
    // attention dropout keep bits: layer 0's made on the side stream while the first LayerNorm and
    // Q/K/V GEMMs run, all later layers' while layer 0 computes (two forks, two joins per forward)
    if (r.drop && l == 0) gen_masks(0);
    LnBatch lb{}; lb.count = 0;
    for (int i = 0; i < M; ++i) {
      if (ln1_done[i]) continue;
      LnProblem& q = lb.p[lb.count++];
      q.x = xin[i]; q.gamma = r.P(x[i].ln1w); q.beta = r.P(x[i].ln1b);
      q.y = r.W<bf16_t>(a[i].a); q.mean = r.W<float>(a[i].mean1); q.rstd = r.W<float>(a[i].rstd1);
      ln8(q, a[i].a8, a[i].as8);
    }
    if (lb.count) r.ok(mmt_launch_ln_fwd(lb, R, C, r.s), "ln1_fwd");
    std::fill(ln1_done.begin(), ln1_done.end(), 0);
    lb.count = M;
    GemmBatch g{}; g.count = M;
    // per-head stage 2 (model.py:39, 44, 49) fused into the stage-1 GEMM's epilogue at hs 32 / 64
    // (qkv2_fused), else its own launch; MMT_QKV2_FUSE=0 keeps the separate kernel
    static const bool qkv2_fuse = [] {
      const char* e = getenv("MMT_QKV2_FUSE");
      return e ? atoi(e) != 0 : true;
    }();
    for (int i = 0; i < M; ++i) {
      g.p[i] = f8 ? gp_f8(r.W<uint8_t>(a[i].a8), C, r.W<uint8_t>(a[i].as8), ldsC, w8, x[i].W1, R)
                  : gp_fwd(r.W<bf16_t>(a[i].a), C, wpk, x[i].W1, R);
      g.p[i].bias = r.P(x[i].b1); g.p[i].o16 = r.W<bf16_t>(a[i].h1); g.p[i].ldo16 = ldh1;
    }
    // (the 128 x 128 bf16 tile only: not on the fp8 kernel, not where the GEMM takes the 256 x 256 tile)
    const bool fuse_qkv2 = qkv2_fuse && (c->hh == 16 || c->hh == 32) && !f8 && !mmt_gemm_wgrad_big(g);
    for (int i = 0; i < M; ++i) {
      if (fuse_qkv2) {
        g.p[i].qkv2_w2 = r.P(x[i].w2); g.p[i].qkv2_out = r.W<bf16_t>(a[i].qkv);
        g.p[i].qkv2_ld = 3 * C; g.p[i].qkv2_hh = c->hh;
      }
    }
    if (f8) r.gemm8(g, EPI_BIAS_TANH_BF16, "qkv1");
    else r.gemm(g, true, true, EPI_BIAS_TANH_BF16, 1, "qkv1");
    for (int i = 0; i < M; ++i) g.p[i].qkv2_out = nullptr;  // g is reused by the next GEMMs
    if (!fuse_qkv2) {
      Qkv2Batch qb{}; qb.count = M;
      for (int i = 0; i < M; ++i) {
        qb.p[i].h1 = r.W<bf16_t>(a[i].h1); qb.p[i].w2 = r.P(x[i].w2); qb.p[i].out = r.W<bf16_t>(a[i].qkv);
      }
      r.ok(mmt_launch_qkv2_fwd(qb, R, 3 * H, hs, ldh1, 3 * C, r.s), "qkv2_fwd");
    }
    AttnBatch ab{}; ab.count = M;
    for (int i = 0; i < M; ++i) {
      AttnProblem& q = ab.p[i];
      bf16_t* qkv = r.W<bf16_t>(a[i].qkv);
      q.q = qkv + C; q.q_ld = 3 * C; q.k[0] = qkv; q.v[0] = qkv + 2 * C; q.kv_ld = 3 * C; q.kv_hstride = hs;
      q.o = r.W<bf16_t>(a[i].o); q.o_ld = C; q.lse[0] = r.W<float>(a[i].lse); q.nstreams = 1;
      r.set_drop(q, l, i, DS_SA_PROB);
      if (r.drop) q.dmask[0] = r.W<uint32_t>(a[i].dm);
    }
    if (r.drop && (l <= 1 || mask_ahead)) {
      r.join();  // this layer's keep bits (SA and CA) are in (layer 1: every later layer's too)
      r.gemm_hint = 0;
      if (mask_ahead) {
        if (ahead_mode == 1 && l + 1 < c->L) gen_masks(l + 1);
      } else if (l == 0) {
        for (int ll = 1; ll < c->L; ++ll) gen_masks(ll);
        // until layer 1's join the later layers' keep bits fill the CUs the side stream can reach: a
        // ping-pong GEMM block needs a CU with none of them on it (all its VGPRs and 128 KiB of LDS), the
        // 128 x 256 tile fits beside them (MMT_MASK_T2=0: the ping-pong kernel throughout)
        if (mask_t2) r.gemm_hint = 1;
      }
    }
    r.attn(ab, false, scale, "attn_fwd");
    if (r.drop && ahead_mode == 2 && l + 1 < c->L) {
      gen_masks(l + 1);
      if (mask_t2) r.gemm_hint = 1;
    }
    // ln2 in the fused out-projection's epilogue (MMT_LN2_FUSE=0: the separate ln_fwd pass; fp8 keeps
    // it, the pass also writes the MX-fp8 copy)
    static const bool ln2_env = [] {
      const char* e = getenv("MMT_LN2_FUSE");
      return e ? atoi(e) != 0 : true;
    }();
    const bool ln2_fuse = ln2_env && !f8;
    bool ln2_done = false;
    {
      // out-projection: Linear(C, C/2) -> tanh -> Linear(C/2, C) -> dropout -> + residual (model.py:82-92,
      // 224), fused into one launch where the shape allows (C = 256 / 512), else two GEMMs
      GemmProblem pg1[MAXM], pg2[MAXM];
      for (int i = 0; i < M; ++i) {
        GemmProblem& g1 = pg1[i];
        g1 = gp_fwd(r.W<bf16_t>(a[i].o), C, wpk, x[i].P0, R);
        g1.bias = r.P(x[i].bp0); g1.o16 = r.W<bf16_t>(a[i].p1); g1.ldo16 = ldp;
        GemmProblem& g2 = pg2[i];
        g2 = gp_fwd(r.W<bf16_t>(a[i].p1), ldp, wpk, x[i].P2, R);
        g2.bias = r.P(x[i].bp2); g2.resid = xin[i]; g2.ldres = C;
        g2.o32 = r.W<float>(a[i].x1); g2.ldc = C;
        r.set_drop(g2, l, i, DS_SA_PROJ);
        if (ln2_fuse) {  // the fused launch owns whole rows: ln2 runs in its epilogue (no MX-fp8 copy)
          g2.lnf_gamma = r.P(x[i].ln2w); g2.lnf_beta = r.P(x[i].ln2b); g2.lnf_y = r.W<bf16_t>(a[i].c);
          g2.lnf_mean = r.W<float>(a[i].mean2); g2.lnf_rstd = r.W<float>(a[i].rstd2);
        }
      }
      const bool fused = r.mlp2(pg1, pg2, M, "proj");  // (nothing launched when it returns false)
      ln2_done = fused && ln2_fuse;
      if (!fused) {
        for (int i = 0; i < M; ++i) g.p[i] = pg1[i];
        r.gemm(g, true, true, EPI_BIAS_TANH_BF16, 1, "proj0");
        for (int i = 0; i < M; ++i) { g.p[i] = pg2[i]; g.p[i].lnf_y = nullptr; }
        r.gemm(g, true, true, EPI_BIAS_RESID_F32, 1, "proj2");
      }
    }
    if (!ln2_done) {
      for (int i = 0; i < M; ++i) {
        lb.p[i].x = r.W<float>(a[i].x1); lb.p[i].gamma = r.P(x[i].ln2w); lb.p[i].beta = r.P(x[i].ln2b);
        lb.p[i].y = r.W<bf16_t>(a[i].c); lb.p[i].mean = r.W<float>(a[i].mean2); lb.p[i].rstd = r.W<float>(a[i].rstd2);
        ln8(lb.p[i], a[i].c8, a[i].cs8);
      }
      r.ok(mmt_launch_ln_fwd(lb, R, C, r.s), "ln2_fwd");
    }
    for (int i = 0; i < M; ++i) {
      g.p[i] = f8 ? gp_f8(r.W<uint8_t>(a[i].c8), C, r.W<uint8_t>(a[i].cs8), ldsC, w8, x[i].F0, R)
                  : gp_fwd(r.W<bf16_t>(a[i].c), C, wpk, x[i].F0, R);
      g.p[i].bias = r.P(x[i].bf0); g.p[i].o16 = r.W<bf16_t>(a[i].f); g.p[i].ldo16 = 4 * C;
      if (r.c->relu_bits) { g.p[i].mask8 = r.W<uint8_t>(a[i].fm); g.p[i].ldm8 = 4 * C / 8; }
      if (f8) { g.p[i].o8 = r.W<uint8_t>(a[i].f8); g.p[i].ld8 = 4 * C; g.p[i].s8 = r.W<uint8_t>(a[i].fs8); g.p[i].lds8 = ldsF; }
    }
    if (f8) r.gemm8(g, EPI_BIAS_RELU_BF16, "ffn0");
    else r.gemm(g, true, true, EPI_BIAS_RELU_BF16, 1, "ffn0");
    for (int i = 0; i < M; ++i) g.p[i].mask8 = nullptr;  // g is reused
    for (int i = 0; i < M; ++i) {
      g.p[i] = f8 ? gp_f8(r.W<uint8_t>(a[i].f8), 4 * C, r.W<uint8_t>(a[i].fs8), ldsF, w8, x[i].F2, R)
                  : gp_fwd(r.W<bf16_t>(a[i].f), 4 * C, wpk, x[i].F2, R);
      g.p[i].bias = r.P(x[i].bf2); g.p[i].resid = r.W<float>(a[i].x1); g.p[i].ldres = C;
      g.p[i].o32 = r.W<float>(a[i].x2); g.p[i].ldc = C;
      if (c->any_cross) { g.p[i].o16 = r.W<bf16_t>(a[i].x2h); g.p[i].ldo16 = C; }
      r.set_drop(g.p[i], l, i, DS_FFN);
    }
    bool lnc_done = false;
    if (fuse_fwd) {
      // the LayerNorm that reads each problem's x2 next: lnc (cross-attention query side), else the
      // next layer's ln1, else (last layer) the post block's
      for (int i = 0; i < M; ++i) {
        GemmProblem& q = g.p[i];
        if (c->any_cross && x[i].cross) {
          q.lnf_gamma = r.P(x[i].lncw); q.lnf_beta = r.P(x[i].lncb); q.lnf_y = r.W<bf16_t>(a[i].d);
          q.lnf_mean = r.W<float>(a[i].meanc); q.lnf_rstd = r.W<float>(a[i].rstdc);
        } else if (l + 1 < c->L) {
          const LM& xn = c->lm[(size_t)(l + 1) * M + i];
          const ActLM& an = p.act[(size_t)(l + 1) * M + i];
          q.lnf_gamma = r.P(xn.ln1w); q.lnf_beta = r.P(xn.ln1b); q.lnf_y = r.W<bf16_t>(an.a);
          q.lnf_mean = r.W<float>(an.mean1); q.lnf_rstd = r.W<float>(an.rstd1);
        } else {
          q.lnf_gamma = r.P(c->post[i].lnw); q.lnf_beta = r.P(c->post[i].lnb); q.lnf_y = r.W<bf16_t>(p.lnf16[i]);
          q.lnf_mean = r.W<float>(p.meanf[i]); q.lnf_rstd = r.W<float>(p.rstdf[i]);
        }
      }
      if (r.gemm_resid_ln(g, "ffn2")) {
        for (int i = 0; i < M; ++i) {
          if (c->any_cross && x[i].cross) lnc_done = true;
          else if (l + 1 < c->L) ln1_done[i] = 1;
          else lnf_done[i] = 1;
        }
      } else {
        for (int i = 0; i < M; ++i) g.p[i].lnf_y = nullptr;
        r.gemm(g, true, true, EPI_BIAS_RESID_F32, 1, "ffn2");
      }
    } else if (f8) {
      r.gemm8(g, EPI_BIAS_RESID_F32, "ffn2");
    } else {
      r.gemm(g, true, true, EPI_BIAS_RESID_F32, 1, "ffn2");
    }
    for (int i = 0; i < M; ++i) g.p[i].lnf_y = nullptr;  // g is reused: no stale LayerNorm outputs
    std::vector<const float*> xout(M);
    for (int i = 0; i < M; ++i) xout[i] = r.W<float>(a[i].x2);
    if (c->any_cross) {
      std::vector<int> cx;
      for (int i = 0; i < M; ++i) if (x[i].cross) cx.push_back(i);
      LnBatch lc{}; lc.count = (int)cx.size();
      GemmBatch gq{}; gq.count = (int)cx.size();
      for (size_t u = 0; u < cx.size(); ++u) {
        const int i = cx[u];
        lc.p[u].x = r.W<float>(a[i].x2); lc.p[u].gamma = r.P(x[i].lncw); lc.p[u].beta = r.P(x[i].lncb);
        lc.p[u].y = r.W<bf16_t>(a[i].d); lc.p[u].mean = r.W<float>(a[i].meanc); lc.p[u].rstd = r.W<float>(a[i].rstdc);
        ln8(lc.p[u], a[i].d8, a[i].ds8);
        gq.p[u] = f8 ? gp_f8(r.W<uint8_t>(a[i].d8), C, r.W<uint8_t>(a[i].ds8), ldsC, w8, x[i].Wq, R)
                     : gp_fwd(r.W<bf16_t>(a[i].d), C, wpk, x[i].Wq, R);
        gq.p[u].o16 = r.W<bf16_t>(a[i].qc); gq.p[u].ldo16 = C;
      }
      if (!lnc_done) r.ok(mmt_launch_ln_fwd(lc, R, C, r.s), "lnc_fwd");
      if (f8) r.gemm8(gq, EPI_STORE_BF16, "ca_q");
      else r.gemm(gq, true, true, EPI_STORE_BF16, 1, "ca_q");
      // KV projections of the other modalities' post-FFN states, grouped up to 8 per launch
      GemmBatch gk{}; gk.count = 0;
      for (int i : cx) {
        int jj = 0;
        for (int j = 0; j < M; ++j) {
          if (j == i) continue;
          gk.p[gk.count] = gp_fwd(r.W<bf16_t>(a[j].x2h), C, wpk, x[i].Wkv[jj], R);
          gk.p[gk.count].o16 = r.W<bf16_t>(a[i].kv[jj]); gk.p[gk.count].ldo16 = 2 * C;
          ++gk.count; ++jj;
          if (gk.count == MMT_MAX_GROUP) { r.gemm(gk, true, true, EPI_STORE_BF16, 1, "ca_kv"); gk.count = 0; }
        }
      }
      if (gk.count) r.gemm(gk, true, true, EPI_STORE_BF16, 1, "ca_kv");
      AttnBatch cb{}; cb.count = (int)cx.size();
      for (size_t u = 0; u < cx.size(); ++u) {
        const int i = cx[u];
        AttnProblem& q = cb.p[u];
        q.q = r.W<bf16_t>(a[i].qc); q.q_ld = C;
        for (int j = 0; j < M - 1; ++j) {
          bf16_t* kv = r.W<bf16_t>(a[i].kv[j]);
          q.k[j] = kv; q.v[j] = kv + hs; q.oj[j] = r.W<bf16_t>(a[i].ocj[j]); q.lse[j] = r.W<float>(a[i].lsej[j]);
        }
        q.kv_ld = 2 * C; q.kv_hstride = 2 * hs; q.o = r.W<bf16_t>(a[i].oc); q.o_ld = C; q.nstreams = M - 1;
        r.set_drop(q, l, i, DS_CA_PROB);
        if (r.drop)
          for (int j = 0; j < M - 1; ++j) q.dmask[j] = r.W<uint32_t>(a[i].dmj[j]);
      }
      r.attn(cb, false, scale, "ca_attn_fwd");
      GemmBatch g0{}; g0.count = (int)cx.size();
      GemmBatch g2{}; g2.count = (int)cx.size();
      for (size_t u = 0; u < cx.size(); ++u) {
        const int i = cx[u];
        g0.p[u] = gp_fwd(r.W<bf16_t>(a[i].oc), C, wpk, x[i].C0, R);
        g0.p[u].bias = r.P(x[i].bc0); g0.p[u].o16 = r.W<bf16_t>(a[i].pc); g0.p[u].ldo16 = ldp;
        g2.p[u] = gp_fwd(r.W<bf16_t>(a[i].pc), ldp, wpk, x[i].C2, R);
        g2.p[u].bias = r.P(x[i].bc2); g2.p[u].resid = r.W<float>(a[i].x2); g2.p[u].ldres = C;
        g2.p[u].o32 = r.W<float>(a[i].x3); g2.p[u].ldc = C;
        r.set_drop(g2.p[u], l, i, DS_CA_PROJ);
        xout[i] = r.W<float>(a[i].x3);
      }
      if (!r.mlp2(g0.p, g2.p, g0.count, "ca_proj")) {
        r.gemm(g0, true, true, EPI_BIAS_TANH_BF16, 1, "ca_proj0");
        r.gemm(g2, true, true, EPI_BIAS_RESID_F32, 1, "ca_proj2");
      }
    }
    xin = xout;
  }
  if (r.rc != MMT_OK) return r.rc;
  // post block + CE
  LnBatch lf{}; lf.count = 0;
  GemmBatch h0{}; h0.count = M;
  GemmBatch h2{}; h2.count = M;
  for (int i = 0; i < M; ++i) {
    if (!lnf_done[i]) {
      LnProblem& q = lf.p[lf.count++];
      q.x = xin[i]; q.gamma = r.P(c->post[i].lnw); q.beta = r.P(c->post[i].lnb);
      q.y = r.W<bf16_t>(p.lnf16[i]); q.mean = r.W<float>(p.meanf[i]); q.rstd = r.W<float>(p.rstdf[i]);
    }
    h0.p[i] = gp_fwd(r.W<bf16_t>(p.lnf16[i]), C, wpk, c->post[i].H0, R);
    h0.p[i].bias = r.P(c->post[i].b0); h0.p[i].o16 = r.W<bf16_t>(p.hh[i]); h0.p[i].ldo16 = c->ldvh[i];
    h2.p[i] = gp_fwd(r.W<bf16_t>(p.hh[i]), c->ldvh[i], wpk, c->post[i].H2, R);
    h2.p[i].bias = r.P(c->post[i].b2); h2.p[i].o32 = logits[i]; h2.p[i].ldc = c->V[i];
  }
  if (tgt) {  // the loss accumulators and this forward's flag word, zeroed by the LN launch
    lf.zero_f = losses; lf.nzero_f = M;
    lf.zero_i = r.W<int>(p.flag); lf.nzero_i = 1;
  }
  if (lf.count) {
    r.ok(mmt_launch_ln_fwd(lf, R, C, r.s), "lnf_fwd");
  } else if (tgt) {  // every post-block LayerNorm was fused: zero the accumulators here
    r.ok(hipMemsetAsync(losses, 0, sizeof(float) * M, r.s), "memset losses");
    r.ok(hipMemsetAsync(r.W<int>(p.flag), 0, sizeof(int), r.s), "memset flag");
  }
  r.gemm(h0, true, true, EPI_BIAS_TANH_BF16, 1, "head0");
  r.gemm(h2, true, true, EPI_STORE_F32, 1, "head2");
  if (tgt && r.rc == MMT_OK) {
    CeBatch cb{}; cb.count = M;
    for (int i = 0; i < M; ++i) {
      cb.p[i].logits = logits[i]; cb.p[i].tgt = tgt[i]; cb.p[i].dlogits = r.W<bf16_t>(p.dlog[i]);
      cb.p[i].loss = losses + i; cb.p[i].V = c->V[i]; cb.p[i].ld_d = c->ldv[i];
      cb.p[i].flag = r.W<int>(p.flag); cb.p[i].bit = 1 << i;
      cb.p[i].part = r.W<float>(p.celoss[i]);
    }
    r.ok(mmt_launch_ce_fwd(cb, R, r.s), "ce_fwd");
  }
  return r.rc;
}

// -------------------------------------------------------------------------------------------
// KV-cache decode (generate, reference model.py:404-446): the forward of ONE new position t per
// sequence, every layer and modality, on compact [B, *] rows. The self- and cross-attention keys /
// values of positions < t are the ones the prefill forward (mmt_forward, same workspace) left in
// its saved Q/K/V and cross-K/V buffers (row b*T + s); this step appends row t to them and runs
// the decode attention over 0..t. Eval semantics (no dropout). The packed bf16 weights are the
// ones the prefill forward made.
// -------------------------------------------------------------------------------------------
int run_decode(mmt_ctx* c, Runner& r, int t, const int64_t* const* idx, float* const* logits) {
  const int M = c->M, C = c->C, H = c->H, hs = c->hs, B = r.B, T = c->T;
  const int R = B;  // compact rows
  const int ldh1 = r8(3 * H * c->hh), ldp = r8(C / 2);
  const float scale = 1.0f / std::sqrt((float)hs);
  Plan& p = c->plan;
  const bf16_t* wpk = r.W<bf16_t>(p.pack);
  r.wpk = wpk;
  auto scatter_rows = [&](bf16_t* cache, int ld, const bf16_t* rows, const char* what) {
    // compact row b -> cache row b*T + t
    r.ok(hipMemcpy2DAsync(cache + (size_t)t * ld, (size_t)T * ld * 2, rows, (size_t)ld * 2, (size_t)ld * 2, B,
                          hipMemcpyDeviceToDevice, r.s), what);
  };
  {
    EmbBatch eb{};
    eb.count = M;
    for (int i = 0; i < M; ++i) {
      eb.p[i].idx = idx[i]; eb.p[i].tok = r.P(c->post[i].tok); eb.p[i].pos = r.P(c->pos_off) + (int64_t)t * C;
      eb.p[i].x = r.W<float>(p.dec[i].x0); eb.p[i].V = c->V[i];
    }
    r.ok(mmt_launch_embed_fwd(eb, B, 1, C, r.s), "dec_embed");
  }
  std::vector<const float*> xin(M);
  for (int i = 0; i < M; ++i) xin[i] = r.W<float>(p.dec[i].x0);
  for (int l = 0; l < c->L && r.rc == MMT_OK; ++l) {
    const LM* x = &c->lm[(size_t)l * M];
    const ActLM* a = &p.act[(size_t)l * M];
    auto X = [&](int i, int k) { return r.W<float>(p.dec_x[((size_t)l * M + i) * 3 + k]); };
    LnBatch lb{}; lb.count = M;
    for (int i = 0; i < M; ++i) {
      const Plan::Dec& d = p.dec[i];
      lb.p[i].x = xin[i]; lb.p[i].gamma = r.P(x[i].ln1w); lb.p[i].beta = r.P(x[i].ln1b);
      lb.p[i].y = r.W<bf16_t>(d.a16); lb.p[i].mean = r.W<float>(d.mean); lb.p[i].rstd = r.W<float>(d.rstd);
    }
    r.ok(mmt_launch_ln_fwd(lb, R, C, r.s), "dec_ln1");
    GemmBatch g{}; g.count = M;
    for (int i = 0; i < M; ++i) {
      g.p[i] = gp_fwd(r.W<bf16_t>(p.dec[i].a16), C, wpk, x[i].W1, R);
      g.p[i].bias = r.P(x[i].b1); g.p[i].o16 = r.W<bf16_t>(p.dec[i].h1); g.p[i].ldo16 = ldh1;
    }
    r.gemm(g, true, true, EPI_BIAS_TANH_BF16, 1, "dec_qkv1");
    Qkv2Batch qb{}; qb.count = M;
    for (int i = 0; i < M; ++i) {
      qb.p[i].h1 = r.W<bf16_t>(p.dec[i].h1); qb.p[i].w2 = r.P(x[i].w2); qb.p[i].out = r.W<bf16_t>(p.dec[i].qkv);
    }
    r.ok(mmt_launch_qkv2_fwd(qb, R, 3 * H, hs, ldh1, 3 * C, r.s), "dec_qkv2");
    DecodeAttnBatch ab{}; ab.count = M;
    for (int i = 0; i < M; ++i) {
      bf16_t* cache = r.W<bf16_t>(a[i].qkv);
      scatter_rows(cache, 3 * C, r.W<bf16_t>(p.dec[i].qkv), "dec_kv_append");
      DecodeAttnProblem& q = ab.p[i];
      q.q = r.W<bf16_t>(p.dec[i].qkv) + C; q.q_ld = 3 * C;
      q.k[0] = cache; q.v[0] = cache + 2 * C; q.kv_ld = 3 * C; q.kv_hstride = hs;
      q.o = r.W<bf16_t>(p.dec[i].o16); q.o_ld = C; q.nstreams = 1;
    }
    r.ok(mmt_launch_attn_decode(ab, B, t, T, H, hs, scale, r.s), "dec_attn");
    for (int i = 0; i < M; ++i) {
      g.p[i] = gp_fwd(r.W<bf16_t>(p.dec[i].o16), C, wpk, x[i].P0, R);
      g.p[i].bias = r.P(x[i].bp0); g.p[i].o16 = r.W<bf16_t>(p.dec[i].p1); g.p[i].ldo16 = ldp;
    }
    r.gemm(g, true, true, EPI_BIAS_TANH_BF16, 1, "dec_proj0");
    for (int i = 0; i < M; ++i) {
      g.p[i] = gp_fwd(r.W<bf16_t>(p.dec[i].p1), ldp, wpk, x[i].P2, R);
      g.p[i].bias = r.P(x[i].bp2); g.p[i].resid = xin[i]; g.p[i].ldres = C;
      g.p[i].o32 = X(i, 0); g.p[i].ldc = C;
    }
    r.gemm(g, true, true, EPI_BIAS_RESID_F32, 1, "dec_proj2");
    for (int i = 0; i < M; ++i) {
      const Plan::Dec& d = p.dec[i];
      lb.p[i].x = X(i, 0); lb.p[i].gamma = r.P(x[i].ln2w); lb.p[i].beta = r.P(x[i].ln2b);
      lb.p[i].y = r.W<bf16_t>(d.a16); lb.p[i].mean = r.W<float>(d.mean); lb.p[i].rstd = r.W<float>(d.rstd);
    }
    r.ok(mmt_launch_ln_fwd(lb, R, C, r.s), "dec_ln2");
    for (int i = 0; i < M; ++i) {
      g.p[i] = gp_fwd(r.W<bf16_t>(p.dec[i].a16), C, wpk, x[i].F0, R);
      g.p[i].bias = r.P(x[i].bf0); g.p[i].o16 = r.W<bf16_t>(p.dec[i].f); g.p[i].ldo16 = 4 * C;
    }
    r.gemm(g, true, true, EPI_BIAS_RELU_BF16, 1, "dec_ffn0");
    for (int i = 0; i < M; ++i) {
      g.p[i] = gp_fwd(r.W<bf16_t>(p.dec[i].f), 4 * C, wpk, x[i].F2, R);
      g.p[i].bias = r.P(x[i].bf2); g.p[i].resid = X(i, 0); g.p[i].ldres = C;
      g.p[i].o32 = X(i, 1); g.p[i].ldc = C;
      if (c->any_cross) { g.p[i].o16 = r.W<bf16_t>(p.dec[i].x2h); g.p[i].ldo16 = C; }
    }
    r.gemm(g, true, true, EPI_BIAS_RESID_F32, 1, "dec_ffn2");
    std::vector<const float*> xout(M);
    for (int i = 0; i < M; ++i) xout[i] = X(i, 1);
    if (c->any_cross) {
      std::vector<int> cx;
      for (int i = 0; i < M; ++i) if (x[i].cross) cx.push_back(i);
      LnBatch lc{}; lc.count = (int)cx.size();
      GemmBatch gq{}; gq.count = (int)cx.size();
      for (size_t u = 0; u < cx.size(); ++u) {
        const int i = cx[u];
        const Plan::Dec& d = p.dec[i];
        lc.p[u].x = X(i, 1); lc.p[u].gamma = r.P(x[i].lncw); lc.p[u].beta = r.P(x[i].lncb);
        lc.p[u].y = r.W<bf16_t>(d.d16); lc.p[u].mean = r.W<float>(d.mean); lc.p[u].rstd = r.W<float>(d.rstd);
        gq.p[u] = gp_fwd(r.W<bf16_t>(d.d16), C, wpk, x[i].Wq, R);
        gq.p[u].o16 = r.W<bf16_t>(d.qc); gq.p[u].ldo16 = C;
      }
      r.ok(mmt_launch_ln_fwd(lc, R, C, r.s), "dec_lnc");
      r.gemm(gq, true, true, EPI_STORE_BF16, 1, "dec_ca_q");
      GemmBatch gk{}; gk.count = 0;
      for (int i : cx) {
        int jj = 0;
        for (int j = 0; j < M; ++j) {
          if (j == i) continue;
          gk.p[gk.count] = gp_fwd(r.W<bf16_t>(p.dec[j].x2h), C, wpk, x[i].Wkv[jj], R);
          gk.p[gk.count].o16 = r.W<bf16_t>(p.dec[i].kv[jj]); gk.p[gk.count].ldo16 = 2 * C;
          ++gk.count; ++jj;
          if (gk.count == MMT_MAX_GROUP) { r.gemm(gk, true, true, EPI_STORE_BF16, 1, "dec_ca_kv"); gk.count = 0; }
        }
      }
      if (gk.count) r.gemm(gk, true, true, EPI_STORE_BF16, 1, "dec_ca_kv");
      DecodeAttnBatch cb{}; cb.count = (int)cx.size();
      for (size_t u = 0; u < cx.size(); ++u) {
        const int i = cx[u];
        DecodeAttnProblem& q = cb.p[u];
        q.q = r.W<bf16_t>(p.dec[i].qc); q.q_ld = C;
        for (int j = 0; j < M - 1; ++j) {
          bf16_t* kv = r.W<bf16_t>(a[i].kv[j]);
          scatter_rows(kv, 2 * C, r.W<bf16_t>(p.dec[i].kv[j]), "dec_cakv_append");
          q.k[j] = kv; q.v[j] = kv + hs;
        }
        q.kv_ld = 2 * C; q.kv_hstride = 2 * hs; q.o = r.W<bf16_t>(p.dec[i].oc); q.o_ld = C; q.nstreams = M - 1;
      }
      r.ok(mmt_launch_attn_decode(cb, B, t, T, H, hs, scale, r.s), "dec_ca_attn");
      GemmBatch g0{}; g0.count = (int)cx.size();
      GemmBatch g2{}; g2.count = (int)cx.size();
      for (size_t u = 0; u < cx.size(); ++u) {
        const int i = cx[u];
        g0.p[u] = gp_fwd(r.W<bf16_t>(p.dec[i].oc), C, wpk, x[i].C0, R);
        g0.p[u].bias = r.P(x[i].bc0); g0.p[u].o16 = r.W<bf16_t>(p.dec[i].pc); g0.p[u].ldo16 = ldp;
        g2.p[u] = gp_fwd(r.W<bf16_t>(p.dec[i].pc), ldp, wpk, x[i].C2, R);
        g2.p[u].bias = r.P(x[i].bc2); g2.p[u].resid = X(i, 1); g2.p[u].ldres = C;
        g2.p[u].o32 = X(i, 2); g2.p[u].ldc = C;
        xout[i] = X(i, 2);
      }
      r.gemm(g0, true, true, EPI_BIAS_TANH_BF16, 1, "dec_ca_proj0");
      r.gemm(g2, true, true, EPI_BIAS_RESID_F32, 1, "dec_ca_proj2");
    }
    xin = xout;
  }
  if (r.rc != MMT_OK) return r.rc;
  LnBatch lf{}; lf.count = M;
  GemmBatch h0{}; h0.count = M;
  GemmBatch h2{}; h2.count = M;
  for (int i = 0; i < M; ++i) {
    const Plan::Dec& d = p.dec[i];
    lf.p[i].x = xin[i]; lf.p[i].gamma = r.P(c->post[i].lnw); lf.p[i].beta = r.P(c->post[i].lnb);
    lf.p[i].y = r.W<bf16_t>(d.lnf16); lf.p[i].mean = r.W<float>(d.mean); lf.p[i].rstd = r.W<float>(d.rstd);
    h0.p[i] = gp_fwd(r.W<bf16_t>(d.lnf16), C, wpk, c->post[i].H0, R);
    h0.p[i].bias = r.P(c->post[i].b0); h0.p[i].o16 = r.W<bf16_t>(d.hh); h0.p[i].ldo16 = c->ldvh[i];
    h2.p[i] = gp_fwd(r.W<bf16_t>(d.hh), c->ldvh[i], wpk, c->post[i].H2, R);
    h2.p[i].bias = r.P(c->post[i].b2); h2.p[i].o32 = logits[i]; h2.p[i].ldc = c->V[i];
  }
  r.ok(mmt_launch_ln_fwd(lf, R, C, r.s), "dec_lnf");
  r.gemm(h0, true, true, EPI_BIAS_TANH_BF16, 1, "dec_head0");
  r.gemm(h2, true, true, EPI_STORE_F32, 1, "dec_head2");
  return r.rc;
}

// -------------------------------------------------------------------------------------------
// backward stages: 0 = post block, 1..L = layers L-1..0, L+1 = embeddings
// -------------------------------------------------------------------------------------------
void colsum_add(Runner& r, ColsumBatch& cb, int u, const bf16_t* x, int ld, float* out, int N, const float* aptr,
                float alpha) {
  cb.p[u].x = x; cb.p[u].ld = ld; cb.p[u].out = out; cb.p[u].N = N; cb.p[u].alpha_ptr = aptr; cb.p[u].alpha = alpha;
}

// The bf16 residual-gradient copy dres16 written by a LayerNorm backward feeds the dropped
// branch that precedes it (layer lprev): its CA projection (cross modalities of a model with
// cross-attention), else its FFN. The copy carries that branch's dropout mask and its column
// sums are that branch's output-bias gradient. Modalities whose copy is rebuilt later (non-cross
// modalities of a cross model) and lprev < 0 (embeddings) get no copy.
// current dres16 copy (the last one written), and the next one in the rotation (for a writer)
inline bf16_t* d16_cur(mmt_ctx* c, Runner& r, int i) { return r.W<bf16_t>(c->plan.dres16[c->d16 & 7][i]); }
inline void d16_advance(mmt_ctx* c) { ++c->d16; }

void set_dres16_consumer(mmt_ctx* c, Runner& r, LnProblem& lp, int i, int lprev, float* grads) {
  lp.dx16 = nullptr; lp.dsum = nullptr;
  lp.drop_key = 0; lp.drop_thr = 0; lp.drop_scale = 1.f;
  if (lprev < 0) return;
  const LM& x = c->lm[(size_t)lprev * c->M + i];
  if (c->any_cross) {
    if (!x.cross) return;
    r.set_drop(lp, lprev, i, DS_CA_PROJ);
    lp.dsum = grads + x.bc2;
  } else {
    r.set_drop(lp, lprev, i, DS_FFN);
    lp.dsum = grads + x.bf2;
  }
  lp.dx16 = d16_cur(c, r, i);  // the caller advanced the rotation for this launch
}

int run_backward_stage(mmt_ctx* c, Runner& r, int stage, const float* loss_grads, float* grads) {
  const int M = c->M, C = c->C, H = c->H, hs = c->hs, R = r.R, B = r.B, T = c->T, L = c->L;
  const int ldh1 = r8(3 * H * c->hh), ldp = r8(C / 2);
  const float scale = 1.0f / std::sqrt((float)hs);
  Plan& p = c->plan;
  const bf16_t* wpk = r.W<bf16_t>(p.pack);
  const int par = stage & 1;  // copy of the side-stream-read scratch this stage writes (Plan)
  if (stage == 0) {
    c->d16 = 0;
    HIPCHK(c, hipMemsetAsync(grads, 0, sizeof(float) * c->nactive, r.s));  // the active prefix only
    // the token-table gradient's row sort (stable: a fixed summation order) needs only the forward's
    // token ids: it runs now on the side stream, off the critical path (27.6 us serial at C1 as the
    // embedding stage's first launch in round 5)
    c->emb_sorted = false;
    {
      EmbBatch eb{}; eb.count = M;
      for (int i = 0; i < M; ++i) {
        eb.p[i].idx = c->last_idx[i]; eb.p[i].V = c->V[i]; eb.p[i].perm = r.W<int>(p.eperm[i]);
      }
      if (mmt_emb_sort_ok(eb, R, C)) {
        if (!c->emb_ev) HIPCHK(c, hipEventCreateWithFlags(&c->emb_ev, hipEventDisableTiming));
        const hipStream_t ss = r.side_stream() ? r.side() : r.s;
        if (r.ok(mmt_launch_emb_sort(eb, R, ss), "emb_sort") && r.ok(hipEventRecord(c->emb_ev, ss), "event record"))
          c->emb_sorted = true;
      }
    }
    const float invR = 1.0f / (float)R;
    GemmBatch dw{}; dw.count = M;
    GemmBatch dx{}; dx.count = M;
    ColsumBatch cs{}; cs.count = M;
    for (int i = 0; i < M; ++i) {
      const PostM& q = c->post[i];
      const bf16_t* dl = r.W<bf16_t>(p.dlog[i]);
      dw.p[i] = gp_dw(dl, c->ldv[i], r.W<bf16_t>(p.hh[i]), c->ldvh[i], grads, q.H2, R);
      dw.p[i].alpha_ptr = loss_grads + i; dw.p[i].alpha = invR;
      colsum_add(r, cs, i, dl, c->ldv[i], grads + q.b2, c->V[i], loss_grads + i, invR);
      dx.p[i] = gp_dx(dl, c->ldv[i], wpk, q.H2, R);
      dx.p[i].alpha_ptr = loss_grads + i; dx.p[i].alpha = invR;
      dx.p[i].aux = r.W<bf16_t>(p.hh[i]); dx.p[i].ldaux = c->ldvh[i];
      dx.p[i].o16 = r.W<bf16_t>(p.gbig[par][i]); dx.p[i].ldo16 = c->ldvh[i];
    }
    r.dwgemm(dw, "head2_dw");
    r.ok(mmt_launch_colsum(cs, R, r.s), "head2_db");
    for (int i = 0; i < M; ++i) dx.p[i].dbias = grads + c->post[i].b0;  // head0 bias grad fused
    r.gemm(dx, true, false, EPI_DTANH_BF16, 1, "head2_dx");
    for (int i = 0; i < M; ++i) {
      const PostM& q = c->post[i];
      const bf16_t* g = r.W<bf16_t>(p.gbig[par][i]);
      dw.p[i] = gp_dw(g, c->ldvh[i], r.W<bf16_t>(p.lnf16[i]), C, grads, q.H0, R);
      dx.p[i] = gp_dx(g, c->ldvh[i], wpk, q.H0, R);
      dx.p[i].o32 = r.W<float>(p.dln[i]); dx.p[i].ldc = C;
    }
    r.dwgemm(dw, "head0_dw");
    r.flush();
    LnBatch lb{}; lb.count = M;
    d16_advance(c);
    std::vector<const float*> xfin(M);
    for (int i = 0; i < M; ++i) {
      const ActLM& a = p.act[(size_t)(L - 1) * M + i];
      xfin[i] = (L == 0) ? r.W<float>(p.xemb[i]) : (c->lm[(size_t)(L - 1) * M + i].cross ? r.W<float>(a.x3) : r.W<float>(a.x2));
      r.ok(hipMemsetAsync(r.W<float>(p.dres[i]), 0, sizeof(float) * (size_t)R * C, r.s), "memset dres");
      lb.p[i].x = xfin[i]; lb.p[i].gamma = r.P(c->post[i].lnw); lb.p[i].mean = r.W<float>(p.meanf[i]);
      lb.p[i].rstd = r.W<float>(p.rstdf[i]); lb.p[i].dy = r.W<float>(p.dln[i]); lb.p[i].dx = r.W<float>(p.dres[i]);
      set_dres16_consumer(c, r, lb.p[i], i, L - 1, grads);
      lb.p[i].dgamma = grads + c->post[i].lnw; lb.p[i].dbeta = grads + c->post[i].lnb;
    }
    r.gemm_ln_bwd(dx, lb, R, C, "head0_dx", "lnf_bwd");
    return r.rc;
  }
  // layer stage
  const int l = L - stage;
  const LM* x = &c->lm[(size_t)l * M];
  const ActLM* a = &p.act[(size_t)l * M];
  std::vector<const float*> xin(M);
  for (int i = 0; i < M; ++i) {
    if (l == 0) xin[i] = r.W<float>(p.xemb[i]);
    else {
      const ActLM& pa = p.act[(size_t)(l - 1) * M + i];
      xin[i] = c->lm[(size_t)(l - 1) * M + i].cross ? r.W<float>(pa.x3) : r.W<float>(pa.x2);
    }
  }
  if (c->any_cross) {
    // MMT_DROP_COPY_FUSE=0 / mmt_set_drop_copy_fuse(0): the separate drop_copy pass for every modality
    const bool fuse_copy = g_drop_copy_fuse != 0;
    std::vector<int> cx;
    for (int i = 0; i < M; ++i) if (x[i].cross) cx.push_back(i);
    const int nc = (int)cx.size();
    GemmBatch dw{}; dw.count = nc;
    GemmBatch dx{}; dx.count = nc;
    for (int u = 0; u < nc; ++u) {
      const int i = cx[u];
      // dres16[i] already carries this projection's dropout mask; its bias grad came with it
      const bf16_t* g = d16_cur(c, r, i);
      dw.p[u] = gp_dw(g, C, r.W<bf16_t>(a[i].pc), ldp, grads, x[i].C2, R);
      dx.p[u] = gp_dx(g, C, wpk, x[i].C2, R);
      dx.p[u].aux = r.W<bf16_t>(a[i].pc); dx.p[u].ldaux = ldp; dx.p[u].o16 = r.W<bf16_t>(p.gpc[par][i]); dx.p[u].ldo16 = ldp;
      dx.p[u].dbias = grads + x[i].bc0;
    }
    r.dwgemm(dw, "ca_proj2_dw");
    GemmProblem pdx0[MAXM];
    for (int u = 0; u < nc; ++u) {
      const int i = cx[u];
      pdx0[u] = gp_dx(r.W<bf16_t>(p.gpc[par][i]), ldp, wpk, x[i].C0, R);
      pdx0[u].o16 = r.W<bf16_t>(p.gdo[i]); pdx0[u].ldo16 = C;
    }
    const bool fused = r.mlp2(dx.p, pdx0, nc, "ca_proj_dx", true);
    if (!fused) r.gemm(dx, true, false, EPI_DTANH_BF16, 1, "ca_proj2_dx");
    for (int u = 0; u < nc; ++u) {
      const int i = cx[u];
      const bf16_t* g = r.W<bf16_t>(p.gpc[par][i]);
      dw.p[u] = gp_dw(g, ldp, r.W<bf16_t>(a[i].oc), C, grads, x[i].C0, R);
      dx.p[u] = pdx0[u];
    }
    r.dwgemm(dw, "ca_proj0_dw");
    if (!fused) r.gemm(dx, true, false, EPI_STORE_BF16, 1, "ca_proj0_dx");
    r.flush();
    AttnBatch ab{}; ab.count = nc;
    for (int u = 0; u < nc; ++u) {
      const int i = cx[u];
      AttnProblem& q = ab.p[u];
      q.q = r.W<bf16_t>(a[i].qc); q.q_ld = C;
      for (int j = 0; j < M - 1; ++j) {
        bf16_t* kv = r.W<bf16_t>(a[i].kv[j]);
        q.k[j] = kv; q.v[j] = kv + hs; q.oj[j] = r.W<bf16_t>(a[i].ocj[j]); q.lse[j] = r.W<float>(a[i].lsej[j]);
        q.dvec[j] = r.W<float>(p.dvec[i][j]);
        bf16_t* dkv = r.W<bf16_t>(p.dkv[par][i][j]);
        q.dk[j] = dkv; q.dv[j] = dkv + hs;
      }
      q.kv_ld = 2 * C; q.kv_hstride = 2 * hs; q.o = r.W<bf16_t>(a[i].oc); q.o_ld = C; q.nstreams = M - 1;
      q.dout = r.W<bf16_t>(p.gdo[i]); q.dout_ld = C; q.dq = r.W<bf16_t>(p.gq[par][i]); q.dq_ld = C;
      // fp32 rows for the one-pass hs-32 backward's dQ sum over the KV streams: dln is free here (the
      // cross-query dX GEMM after the attention writes it)
      q.dq32 = r.W<float>(p.dln[i]); q.dq32_ld = C;
      q.dkv_ld = 2 * C; q.dkv_hstride = 2 * hs;
      r.set_drop(q, l, i, DS_CA_PROB);
      if (r.drop)
        for (int j = 0; j < M - 1; ++j) q.dmask[j] = r.W<uint32_t>(a[i].dmj[j]);
    }
    r.attn(ab, true, scale, "ca_attn_bwd");
    for (int u = 0; u < nc; ++u) {
      const int i = cx[u];
      const bf16_t* g = r.W<bf16_t>(p.gq[par][i]);
      dw.p[u] = gp_dw(g, C, r.W<bf16_t>(a[i].d), C, grads, x[i].Wq, R);
      dx.p[u] = gp_dx(g, C, wpk, x[i].Wq, R);
      dx.p[u].o32 = r.W<float>(p.dln[i]); dx.p[u].ldc = C;
    }
    r.dwgemm(dw, "ca_q_dw");
    LnBatch lc{}; lc.count = nc;
    for (int u = 0; u < nc; ++u) {
      const int i = cx[u];
      lc.p[u].x = r.W<float>(a[i].x2); lc.p[u].gamma = r.P(x[i].lncw); lc.p[u].mean = r.W<float>(a[i].meanc);
      lc.p[u].rstd = r.W<float>(a[i].rstdc); lc.p[u].dy = r.W<float>(p.dln[i]); lc.p[u].dx = r.W<float>(p.dres[i]);
      lc.p[u].dgamma = grads + x[i].lncw; lc.p[u].dbeta = grads + x[i].lncb;
    }
    r.gemm_ln_bwd(dx, lc, R, C, "ca_q_dx", "lnc_bwd");
    // KV projections: dWkv += dkv^T x2_j ; dres[j] += dkv Wkv (one launch per query modality:
    // different query modalities accumulate into the same dres[j]). The LAST query modality that
    // accumulates into dres[j] also writes its bf16 copy for the FFN backward in that epilogue (FFN
    // dropout mask, FFN output-bias gradient as column sums): a separate drop_copy pass re-read the
    // fp32 rows (6 x 38 us per step at the target). Only a modality no launch accumulates into (one
    // cross modality: its own dres) keeps the copy pass.
    d16_advance(c);
    std::vector<int> last_writer(M, -1);
    for (int i : cx)
      for (int j = 0; j < M; ++j)
        if (j != i) last_writer[j] = i;
    // the fused copy is only right if no later launch of this stage accumulates into dres[j] (the FFN
    // backward reads the copy): launches run in cx order and last_writer[j] is the last i of cx that
    // writes dres[j]; copied[j] checks that invariant as the launches are built
    std::vector<char> copied(M, 0);
    for (int i : cx) {
      GemmBatch kw{}; kw.count = 0;
      GemmBatch kx{}; kx.count = 0;
      int jj = 0;
      for (int j = 0; j < M; ++j) {
        if (j == i) continue;
        if (copied[j]) return fail(c, MMT_ERR_STATE, "cross K/V dX: dres written after its fused bf16 copy");
        const bf16_t* g = r.W<bf16_t>(p.dkv[par][i][jj]);
        kw.p[kw.count++] = gp_dw(g, 2 * C, r.W<bf16_t>(a[j].x2h), C, grads, x[i].Wkv[jj], R);
        GemmProblem d = gp_dx(g, 2 * C, wpk, x[i].Wkv[jj], R);
        d.o32 = r.W<float>(p.dres[j]); d.ldc = C;
        if (last_writer[j] == i && fuse_copy) {
          copied[j] = 1;
          d.o16 = d16_cur(c, r, j); d.ldo16 = C; d.dbias = grads + x[j].bf2;
          r.set_drop(d, l, j, DS_FFN);
        }
        kx.p[kx.count++] = d;
        ++jj;
        if (kw.count == MMT_MAX_GROUP) {
          r.dwgemm(kw, "ca_kv_dw"); r.gemm(kx, true, false, EPI_ACC_F32, 1, "ca_kv_dx");
          kw.count = 0; kx.count = 0;
        }
      }
      if (kw.count) { r.dwgemm(kw, "ca_kv_dw"); r.gemm(kx, true, false, EPI_ACC_F32, 1, "ca_kv_dx"); }
    }
    r.flush();
    // bf16 copy for the FFN backward of the modalities no fused epilogue covered
    DropCopyBatch db{}; db.count = 0;
    for (int i = 0; i < M; ++i) {
      if (fuse_copy && last_writer[i] >= 0) continue;
      DropCopyProblem& q = db.p[db.count++];
      q.src = r.W<float>(p.dres[i]); q.dst = d16_cur(c, r, i); q.dsum = grads + x[i].bf2;
      r.set_drop(q, l, i, DS_FFN);
    }
    if (db.count) r.ok(mmt_launch_drop_copy(db, R, C, r.s), "dres16");
  }
  if (r.rc != MMT_OK) return r.rc;
  // FFN
  GemmBatch dw{}; dw.count = M;
  GemmBatch dx{}; dx.count = M;
  LnBatch lb{}; lb.count = M;
  for (int i = 0; i < M; ++i) {
    // dres16[i] carries the FFN dropout mask; the FFN output-bias grad was summed with it
    const bf16_t* g = d16_cur(c, r, i);
    dw.p[i] = gp_dw(g, C, r.W<bf16_t>(a[i].f), 4 * C, grads, x[i].F2, R);
    dx.p[i] = gp_dx(g, C, wpk, x[i].F2, R);
    dx.p[i].aux = r.W<bf16_t>(a[i].f); dx.p[i].ldaux = 4 * C; dx.p[i].o16 = r.W<bf16_t>(p.gbig[par][i]); dx.p[i].ldo16 = 4 * C;
    dx.p[i].dbias = grads + x[i].bf0;
    if (r.c->relu_bits) { dx.p[i].mask8 = r.W<uint8_t>(a[i].fm); dx.p[i].ldm8 = 4 * C / 8; }  // ReLU' from bits
  }
  // MMT_DW_ATTN_SMALL=1: the FFN weight gradients (the side-stream launches still running when the
  // self-attention backward starts) on the 128 x 128 tile, whose 64 KiB of LDS leave room on their CUs for
  // one of the attention backward's 80 KiB workgroups
  static const int dw_attn_small = [] {
    const char* e = getenv("MMT_DW_ATTN_SMALL");
    return e ? atoi(e) : 0;
  }();
  const int ffn_dw_hint = dw_attn_small ? 2 : 0;
  r.dwgemm(dw, "ffn2_dw", ffn_dw_hint);
  r.gemm(dx, true, false, EPI_DRELU_BF16, 1, "ffn2_dx");
  for (int i = 0; i < M; ++i) {
    const bf16_t* g = r.W<bf16_t>(p.gbig[par][i]);
    dw.p[i] = gp_dw(g, 4 * C, r.W<bf16_t>(a[i].c), C, grads, x[i].F0, R);
    dx.p[i] = gp_dx(g, 4 * C, wpk, x[i].F0, R);
    dx.p[i].o32 = r.W<float>(p.dln[i]); dx.p[i].ldc = C;
  }
  r.dwgemm(dw, "ffn0_dw", ffn_dw_hint);
  r.flush();
  d16_advance(c);
  for (int i = 0; i < M; ++i) {
    lb.p[i].x = r.W<float>(a[i].x1); lb.p[i].gamma = r.P(x[i].ln2w); lb.p[i].mean = r.W<float>(a[i].mean2);
    lb.p[i].rstd = r.W<float>(a[i].rstd2); lb.p[i].dy = r.W<float>(p.dln[i]); lb.p[i].dx = r.W<float>(p.dres[i]);
    lb.p[i].dx16 = d16_cur(c, r, i); lb.p[i].dgamma = grads + x[i].ln2w; lb.p[i].dbeta = grads + x[i].ln2b;
    r.set_drop(lb.p[i], l, i, DS_SA_PROJ);  // the copy feeds the SA projection backward
    lb.p[i].dsum = grads + x[i].bp2;
  }
  r.gemm_ln_bwd(dx, lb, R, C, "ffn0_dx", "ln2_bwd");
  // SA output projection
  for (int i = 0; i < M; ++i) {
    const bf16_t* g = d16_cur(c, r, i);
    dw.p[i] = gp_dw(g, C, r.W<bf16_t>(a[i].p1), ldp, grads, x[i].P2, R);
    dx.p[i] = gp_dx(g, C, wpk, x[i].P2, R);
    dx.p[i].aux = r.W<bf16_t>(a[i].p1); dx.p[i].ldaux = ldp; dx.p[i].o16 = r.W<bf16_t>(p.gp[par][i]); dx.p[i].ldo16 = ldp;
    dx.p[i].dbias = grads + x[i].bp0;
  }
  r.dwgemm(dw, "proj2_dw");
  {
    // both data-gradient products in one launch where the fused kernel takes the shape (C = 256 / 512)
    GemmProblem pdx0[MAXM];
    for (int i = 0; i < M; ++i) {
      const bf16_t* g = r.W<bf16_t>(p.gp[par][i]);
      pdx0[i] = gp_dx(g, ldp, wpk, x[i].P0, R);
      pdx0[i].o16 = r.W<bf16_t>(p.gdo[i]); pdx0[i].ldo16 = C;
    }
    const bool fused = r.mlp2(dx.p, pdx0, M, "proj_dx", true);
    if (!fused) r.gemm(dx, true, false, EPI_DTANH_BF16, 1, "proj2_dx");
    for (int i = 0; i < M; ++i) {
      const bf16_t* g = r.W<bf16_t>(p.gp[par][i]);
      dw.p[i] = gp_dw(g, ldp, r.W<bf16_t>(a[i].o), C, grads, x[i].P0, R);
      dx.p[i] = pdx0[i];
    }
    r.dwgemm(dw, "proj0_dw");
    if (!fused) r.gemm(dx, true, false, EPI_STORE_BF16, 1, "proj0_dx");
  }
  r.flush();
  AttnBatch ab{}; ab.count = M;
  for (int i = 0; i < M; ++i) {
    AttnProblem& q = ab.p[i];
    bf16_t* qkv = r.W<bf16_t>(a[i].qkv);
    bf16_t* gq = r.W<bf16_t>(p.gqkv[i]);
    q.q = qkv + C; q.q_ld = 3 * C; q.k[0] = qkv; q.v[0] = qkv + 2 * C; q.kv_ld = 3 * C; q.kv_hstride = hs;
    q.o = r.W<bf16_t>(a[i].o); q.o_ld = C; q.lse[0] = r.W<float>(a[i].lse); q.nstreams = 1;
    q.dout = r.W<bf16_t>(p.gdo[i]); q.dout_ld = C; q.dvec[0] = r.W<float>(p.dvec[i][0]);
    q.dq = gq + C; q.dq_ld = 3 * C; q.dk[0] = gq; q.dv[0] = gq + 2 * C; q.dkv_ld = 3 * C; q.dkv_hstride = hs;
    r.set_drop(q, l, i, DS_SA_PROB);
    if (r.drop) q.dmask[0] = r.W<uint32_t>(a[i].dm);
  }
  // hs 32: the Q/K/V stage-2 backward runs in the attention kernel's epilogue (dQ / dK / dV stay on chip:
  // dh1, dW2, db1 leave it), so the separate qkv2 backward and its gqkv round trip go
  const bool q2 = g_attn_qkv2 && mmt_attn_bwd_fuses_qkv2(ab, T, hs);
  if (q2)
    for (int i = 0; i < M; ++i) {
      AttnProblem& q = ab.p[i];
      q.q2_h1 = r.W<bf16_t>(a[i].h1); q.q2_dh1 = r.W<bf16_t>(p.gh1[par][i]); q.q2_ld = ldh1;
      q.q2_w2 = r.P(x[i].w2); q.q2_dw2 = grads + x[i].w2; q.q2_db1 = grads + x[i].b1;
    }
  Qkv2Batch qb{}; qb.count = M;
  for (int i = 0; i < M; ++i) {
    qb.p[i].h1 = r.W<bf16_t>(a[i].h1); qb.p[i].w2 = r.P(x[i].w2); qb.p[i].dout = r.W<bf16_t>(p.gqkv[i]);
    qb.p[i].dh1 = r.W<bf16_t>(p.gh1[par][i]); qb.p[i].dw2 = grads + x[i].w2;
    qb.p[i].db1 = grads + x[i].b1;  // stage-1 bias gradient: column sums of dh1, fused
  }
  // dh1 rows are padded to ldh1 (a multiple of 8) and the qkv2 backward writes only the 3 H hh columns;
  // the stage-1 dX GEMM reads K in 8-column chunks against zero weight-pack pad rows, so the pad must be
  // finite: zeroed once per workspace (no kernel writes it). Garbage there made the gradient NaN at
  // shapes with 3 H hh % 8 != 0 (hs 8 / 24 with odd head counts; round 6)
  if (p.gh1_pad_ws != r.ws && ldh1 > 3 * H * c->hh) {
    const size_t cols = 3 * (size_t)H * c->hh;
    for (int k = 0; k < 2; ++k)
      for (int i = 0; i < M; ++i)
        r.ok(hipMemset2DAsync(r.W<bf16_t>(p.gh1[k][i]) + cols, (size_t)ldh1 * 2, 0, ((size_t)ldh1 - cols) * 2, (size_t)R, r.s),
             "gh1 pad");
    p.gh1_pad_ws = r.ws;
  }
  r.attn(ab, true, scale, "attn_bwd");
  if (!q2) r.ok(mmt_launch_qkv2_bwd(qb, R, 3 * H, hs, ldh1, 3 * C, r.s), "qkv2_bwd");
  for (int i = 0; i < M; ++i) {
    const bf16_t* g = r.W<bf16_t>(p.gh1[par][i]);
    dw.p[i] = gp_dw(g, ldh1, r.W<bf16_t>(a[i].a), C, grads, x[i].W1, R);
    dx.p[i] = gp_dx(g, ldh1, wpk, x[i].W1, R);
    dx.p[i].o32 = r.W<float>(p.dln[i]); dx.p[i].ldc = C;
  }
  r.dwgemm(dw, "qkv1_dw");
  r.flush();
  d16_advance(c);
  for (int i = 0; i < M; ++i) {
    lb.p[i].x = xin[i]; lb.p[i].gamma = r.P(x[i].ln1w); lb.p[i].mean = r.W<float>(a[i].mean1);
    lb.p[i].rstd = r.W<float>(a[i].rstd1); lb.p[i].dy = r.W<float>(p.dln[i]); lb.p[i].dx = r.W<float>(p.dres[i]);
    lb.p[i].dgamma = grads + x[i].ln1w; lb.p[i].dbeta = grads + x[i].ln1b;
    set_dres16_consumer(c, r, lb.p[i], i, l - 1, grads);
  }
  r.gemm_ln_bwd(dx, lb, R, C, "qkv1_dx", "ln1_bwd");
  return r.rc;
}

int check_cfg(const mmt_config* cfg, std::string& msg) {
  if (!cfg) { msg = "null config"; return MMT_ERR_INVALID; }
  const int M = cfg->num_modalities;
  if (M < 1 || M > MAXM) { msg = "num_modalities must be 1..8"; return MMT_ERR_INVALID; }
  if (cfg->n_embd <= 0 || cfg->n_head <= 0 || cfg->n_layer < 0 || cfg->block_size <= 0) {
    msg = "n_embd, n_head, block_size must be positive and n_layer >= 0"; return MMT_ERR_INVALID;
  }
  if (cfg->n_embd % cfg->n_head) { msg = "n_embd must be divisible by n_head"; return MMT_ERR_UNSUPPORTED; }
  const int hs = cfg->n_embd / cfg->n_head;
  if (!(hs == 8 || hs == 16 || hs == 24 || hs == 32 || hs == 48 || hs == 64)) {
    msg = "head size n_embd/n_head must be one of 8,16,24,32,48,64 (got " + std::to_string(hs) + ")";
    return MMT_ERR_UNSUPPORTED;
  }
  if (cfg->n_embd % 8 || cfg->n_embd > 1024) { msg = "n_embd must be a multiple of 8 and <= 1024"; return MMT_ERR_UNSUPPORTED; }
  for (int i = 0; i < M; ++i)
    if (cfg->vocab_sizes[i] < 1) { msg = "vocab sizes must be >= 1"; return MMT_ERR_INVALID; }
  if (cfg->dropout < 0.f || cfg->dropout >= 1.f) { msg = "dropout must be in [0, 1)"; return MMT_ERR_INVALID; }
  if (cfg->precision != 0 && cfg->precision != 1) { msg = "precision must be 0 (bf16) or 1 (fp8)"; return MMT_ERR_INVALID; }
  if (cfg->precision == 1 && cfg->n_embd % 32) {
    msg = "precision fp8 needs n_embd % 32 == 0 (MX blocks of 32 along every fp8 GEMM's K)"; return MMT_ERR_UNSUPPORTED;
  }
  return MMT_OK;
}

int ensure_device_tables(mmt_ctx* c) {
  // the pack tables live on the device of the caller's current stream (rebuilt when the
  // model moves to another device)
  int dev = -1;
  HIPCHK(c, hipGetDevice(&dev));
  if (c->d_segs && c->tables_device == dev) return MMT_OK;
  if (c->d_segs) { (void)hipFree(c->d_segs); c->d_segs = nullptr; }
  if (c->d_tasks) { (void)hipFree(c->d_tasks); c->d_tasks = nullptr; }
  if (c->d_mxsegs) { (void)hipFree(c->d_mxsegs); c->d_mxsegs = nullptr; }
  if (c->segs.empty()) return MMT_OK;
  HIPCHK(c, hipMalloc(&c->d_segs, sizeof(PackSeg) * c->segs.size()));
  HIPCHK(c, hipMalloc(&c->d_tasks, sizeof(int) * c->tasks.size()));
  HIPCHK(c, hipMemcpy(c->d_segs, c->segs.data(), sizeof(PackSeg) * c->segs.size(), hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_tasks, c->tasks.data(), sizeof(int) * c->tasks.size(), hipMemcpyHostToDevice));
  if (!c->mxsegs.empty()) {
    HIPCHK(c, hipMalloc(&c->d_mxsegs, sizeof(MxSeg) * c->mxsegs.size()));
    HIPCHK(c, hipMemcpy(c->d_mxsegs, c->mxsegs.data(), sizeof(MxSeg) * c->mxsegs.size(), hipMemcpyHostToDevice));
  }
  c->tables_device = dev;
  return MMT_OK;
}

// the side stream (weight-gradient GEMMs in the backward, dropout keep bits in the forward), made
// lazily on the caller's current device; MMT_SIDE_STREAM=0 runs everything on the caller's stream
void ensure_side(mmt_ctx* c) {
  static const bool use_side = [] {
    const char* e = getenv("MMT_SIDE_STREAM");
    return !e || atoi(e) != 0;
  }();
  int dev = -1;
  if (!use_side || hipGetDevice(&dev) != hipSuccess || (c->side && c->side_device == dev)) return;
  if (c->side) (void)hipStreamDestroy(c->side);
  for (auto& e : c->evpool) (void)hipEventDestroy(e);  // events of the previous device
  c->evpool.clear();
  c->side = nullptr;
  // MMT_SIDE_PRIORITY (optional): HIP stream priority of the side stream (lower = higher priority,
  // clamped to the device's range); unset = default priority
  static const char* prio_env = getenv("MMT_SIDE_PRIORITY");
  // (a CU-masked side stream measured far slower -- it cannot be created non-blocking, so it
  // serialises against the caller's stream: profiles/r3q_side_cumask_ab.txt; removed in round 4)
  hipError_t ce;
  if (prio_env) {
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    const int pr = std::max(greatest, std::min(least, atoi(prio_env)));
    ce = hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, pr);
  } else {
    ce = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  }
  if (ce != hipSuccess) c->side = nullptr;
  c->side_device = dev;
  while (c->side && c->evpool.size() < 64) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) break;
    c->evpool.push_back(e);
  }
  for (auto& e : c->stage_ev) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
    if (c->side && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
  }
  if ((c->evpool.empty() || !c->stage_ev[0] || !c->stage_ev[1]) && c->side) {
    (void)hipStreamDestroy(c->side);
    c->side = nullptr;
  }
}

}  // namespace

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

const char* mmt_version(void) { return "mmt_hip 0.1 gfx950"; }
const char* mmt_create_error(void) { return g_create_err.c_str(); }

mmt_ctx* mmt_create(const mmt_config* cfg) {
  std::string msg;
  if (check_cfg(cfg, msg) != MMT_OK) { g_create_err = msg; return nullptr; }
  mmt_ctx* c = new (std::nothrow) mmt_ctx();
  if (!c) { g_create_err = "out of memory"; return nullptr; }
  c->cfg = *cfg;
  c->M = cfg->num_modalities; c->C = cfg->n_embd; c->H = cfg->n_head; c->L = cfg->n_layer; c->T = cfg->block_size;
  c->hs = c->C / c->H; c->hh = c->hs / 2;
  for (int i = 0; i < c->M; ++i) {
    c->V[i] = cfg->vocab_sizes[i];
    if (cfg->cross_attention[i] && c->M > 1) { c->any_cross = true; ++c->ncross; }
  }
  if (c->M - 1 > MMT_MAX_STREAMS) { g_create_err = "too many KV streams"; delete c; return nullptr; }
  c->fp8 = cfg->precision == 1;
  c->relu_bits = g_relu_bits != 0;
  build_layout(c);
  return c;
}

void mmt_destroy(mmt_ctx* c) {
  if (!c) return;
  if (c->d_segs) (void)hipFree(c->d_segs);
  if (c->d_tasks) (void)hipFree(c->d_tasks);
  if (c->d_mxsegs) (void)hipFree(c->d_mxsegs);
  for (auto& e : c->probe_pool) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
  for (auto& e : c->evpool) (void)hipEventDestroy(e);
  for (auto& e : c->stage_ev) if (e) (void)hipEventDestroy(e);
  if (c->emb_ev) (void)hipEventDestroy(c->emb_ev);
  if (c->side) (void)hipStreamDestroy(c->side);
  delete c;
}

const char* mmt_last_error(const mmt_ctx* c) { return c ? c->err.c_str() : "null context"; }
int64_t mmt_param_count(const mmt_ctx* c) { return c ? c->nparams : 0; }
int64_t mmt_param_active_count(const mmt_ctx* c) { return c ? c->nactive : 0; }
int32_t mmt_tensor_count(const mmt_ctx* c) { return c ? (int32_t)c->tensors.size() : 0; }

int mmt_tensor_info(const mmt_ctx* c, int32_t i, char* name, int32_t cap, int64_t* off, int32_t* nd, int64_t* shape,
                    int32_t* kind) {
  if (!c || i < 0 || i >= (int32_t)c->tensors.size()) return MMT_ERR_INVALID;
  const TensorInfo& t = c->tensors[i];
  if (name && cap > 0) {
    std::strncpy(name, t.name.c_str(), cap - 1);
    name[cap - 1] = 0;
  }
  if (off) *off = t.off;
  if (nd) *nd = t.nd;
  if (shape) { shape[0] = t.shape[0]; shape[1] = t.shape[1]; }
  if (kind) *kind = t.kind;
  return MMT_OK;
}

int64_t mmt_loss_flag_offset(mmt_ctx* c, int32_t batch) {
  if (!c || batch < 1) return -1;
  return (int64_t)flag_offset(c);  // batch-independent: the current plan is left alone
}

int64_t mmt_workspace_bytes(mmt_ctx* c, int32_t batch) {
  if (!c || batch < 1) return -1;
  make_plan(c, batch);
  c->last_B = batch;
  c->fwd_ready = false;
  c->cache_ready = false;
  return (int64_t)c->plan.total;
}

int mmt_forward(mmt_ctx* c, void* stream, int32_t batch, const int64_t* const* idx, const int64_t* const* tgt,
                const float* params, float* const* logits, float* losses, void* workspace, int32_t training) {
  if (!c) return MMT_ERR_INVALID;
  if (batch < 1 || !idx || !params || !logits || !workspace) return fail(c, MMT_ERR_INVALID, "mmt_forward: null argument");
  if (c->plan.B != batch) make_plan(c, batch);
  int rc = ensure_device_tables(c);
  if (rc) return rc;
  c->side_off = c->side_off_req;
  Runner r{c, (hipStream_t)stream, workspace, params, nullptr, batch, batch * c->T};
  // dropout (training mode only, as nn.Dropout): one seed per training forward, reused by its backward
  r.drop = training && c->cfg.dropout > 0.f;
  if (r.drop) {
    if (c->next_seed_set) r.seed = c->next_seed;
    else r.seed = ((uint64_t)mmt_hash((uint32_t)c->cfg.seed, (uint32_t)(c->cfg.seed >> 32), (uint32_t)c->step_counter) << 32) |
                  mmt_hash((uint32_t)(c->cfg.seed >> 32), (uint32_t)c->cfg.seed, (uint32_t)(c->step_counter >> 32) ^ 0xA5A5A5A5u);
    c->next_seed_set = false;
    ++c->step_counter;
  }
  if (r.drop) ensure_side(c);
  c->fwd_drop = r.drop;
  c->fwd_seed = r.seed;
  c->fwd_ready = false;
  for (int i = 0; i < c->M; ++i) c->last_idx[i] = idx[i];
  rc = run_forward(c, r, idx, tgt, logits, losses);
  if (rc == MMT_OK && tgt) c->fwd_ready = true;
  c->cache_ready = rc == MMT_OK;  // the saved Q/K/V of this forward serve mmt_decode_step
  c->last_training = training != 0;
  return rc;
}

int mmt_decode_step(mmt_ctx* c, void* stream, int32_t batch, int32_t pos, const int64_t* const* idx,
                    const float* params, float* const* logits, void* workspace) {
  if (!c) return MMT_ERR_INVALID;
  if (!idx || !params || !logits || !workspace) return fail(c, MMT_ERR_INVALID, "mmt_decode_step: null argument");
  if (c->plan.B != batch || !c->cache_ready)
    return fail(c, MMT_ERR_STATE, "mmt_decode_step: run mmt_forward (prefill) on this batch and workspace first");
  if (c->fwd_drop)
    return fail(c, MMT_ERR_STATE, "mmt_decode_step: the prefill forward sampled dropout (training mode); decode "
                                  "has eval semantics: run the prefill with training = 0");
  if (c->fp8)
    return fail(c, MMT_ERR_STATE, "mmt_decode_step: precision fp8 prefills with MX-fp8 GEMMs the bf16 decode "
                                  "would not reproduce: re-run mmt_forward per token");
  if (pos < 1 || pos >= c->T) return fail(c, MMT_ERR_INVALID, "mmt_decode_step: position outside 1..block_size-1");
  Runner r{c, (hipStream_t)stream, workspace, params, nullptr, batch, batch};
  return run_decode(c, r, pos, idx, logits);
}

int32_t mmt_backward_stage_count(const mmt_ctx* c) { return c ? c->L + 2 : 0; }

int mmt_backward_stage_range(const mmt_ctx* c, int32_t stage, int64_t* begin, int64_t* end) {
  if (!c || stage < 0 || stage > c->L + 1) return MMT_ERR_INVALID;
  int64_t b, e;
  if (stage == 0) { b = c->post_begin; e = c->post_end; }
  else if (stage == c->L + 1) { b = c->emb_begin; e = c->emb_end; }
  else { const int l = c->L - stage; b = c->layer_begin[l]; e = c->layer_end[l]; }
  if (begin) *begin = b;
  if (end) *end = e;
  return MMT_OK;
}

}  // extern "C"

extern "C" {

int mmt_backward_stage(mmt_ctx* c, void* stream, int32_t stage, const float* loss_grads, const float* params,
                       float* grads, void* workspace) {
  if (!c) return MMT_ERR_INVALID;
  if (!c->fwd_ready) return fail(c, MMT_ERR_STATE, "mmt_backward: no forward with targets to differentiate");
  if (stage < 0 || stage > c->L + 1) return fail(c, MMT_ERR_INVALID, "bad backward stage");
  ensure_side(c);
  Runner r{c, (hipStream_t)stream, workspace, params, nullptr, c->plan.B, c->plan.B * c->T};
  r.drop = c->fwd_drop;
  r.seed = c->fwd_seed;
  if (stage == c->L + 1) {
    EmbBatch eb{}; eb.count = c->M;
    for (int i = 0; i < c->M; ++i) {
      eb.p[i].idx = c->last_idx[i]; eb.p[i].dx = r.W<float>(c->plan.dres[i]);
      eb.p[i].dtok = grads + c->post[i].tok; eb.p[i].dpos = grads + c->pos_off; eb.p[i].V = c->V[i];
      eb.p[i].part = r.W<float>(c->plan.dln[i]);  // R x C fp32, free once the layers are done
      if (c->emb_sorted) eb.p[i].perm = r.W<int>(c->plan.eperm[i]);  // sorted at stage 0
    }
    if (c->emb_sorted) r.ok(hipStreamWaitEvent(r.s, c->emb_ev, 0), "stream wait");
    c->emb_sorted = false;
    r.ok(mmt_launch_embed_bwd(eb, r.B, c->T, c->C, r.s), "embed_bwd");
    return r.rc;
  }
  const bool defer = c->defer_join && r.side_stream();
  if (defer && stage >= 2)  // the side stream's work of stage - 2 read this stage's scratch copies
    r.ok(hipStreamWaitEvent(r.s, c->stage_ev[stage & 1], 0), "stream wait");
  // MMT_FLUSH_HOLD=1: one side-stream fork per stage (every stage but the last layer's, whose weight
  // gradients would otherwise only start after its data-gradient chain, at the end of the step)
  static const int flush_hold = [] {
    const char* e = getenv("MMT_FLUSH_HOLD");
    return e ? atoi(e) : 0;
  }();
  r.hold = defer && flush_hold && stage < c->L;
  const int rc = run_backward_stage(c, r, stage, loss_grads, grads);
  r.hold = false;
  if (defer) {
    r.flush(true);
    r.ok(hipEventRecord(c->stage_ev[stage & 1], c->side), "event record");
  } else {
    r.join();  // the stage's gradient range is complete on the caller's stream (DP all-reduce order)
  }
  return rc ? rc : r.rc;
}

int mmt_backward(mmt_ctx* c, void* stream, const float* loss_grads, const float* params, float* grads,
                 void* workspace) {
  if (!c) return MMT_ERR_INVALID;
  // one join at the end instead of one per stage (mmt_ctx::defer_join); the embedding stage is the
  // last and runs on the caller's stream only, so the join closes over every weight gradient
  c->defer_join = true;
  int rc = MMT_OK;
  for (int s = 0; s < c->L + 2 && rc == MMT_OK; ++s) rc = mmt_backward_stage(c, stream, s, loss_grads, params, grads, workspace);
  c->defer_join = false;
  // the join also on the error path: no weight-gradient GEMM (or its split-K slab) of this backward is
  // left running on the side stream once control is back with the caller
  Runner r{c, (hipStream_t)stream, workspace, params, nullptr, c->plan.B, c->plan.B * c->T};
  r.join();
  return rc ? rc : r.rc;
}

int mmt_adamw_step(mmt_ctx* c, void* stream, float* params, const float* grads, float* m, float* v, int64_t n,
                   int64_t step, float lr, float b1, float b2, float eps, float wd) {
  if (step < 1 || !params || !grads || !m || !v) return fail(c, MMT_ERR_INVALID, "mmt_adamw_step: bad argument");
  const double bc1 = 1.0 - std::pow((double)b1, (double)step);
  const double bc2 = 1.0 - std::pow((double)b2, (double)step);
  const hipError_t e = mmt_launch_adamw(params, grads, m, v, n, lr, b1, b2, eps, wd, (float)bc1,
                                        (float)std::sqrt(bc2), (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, MMT_ERR_HIP, std::string("adamw: ") + hipGetErrorString(e));
  return MMT_OK;
}

int mmt_eval_direction(mmt_ctx* c, void* stream, int32_t batch, int32_t T, int32_t V, const float* logits,
                       const int64_t* xb, const int64_t* yb, const double* vocab, int32_t is_percent,
                       int32_t* wins_losses, double* certainty_sum) {
  const hipError_t e = mmt_launch_eval_direction(logits, xb, yb, vocab, batch, T, V, is_percent, wins_losses,
                                                 certainty_sum, (hipStream_t)stream);
  if (e != hipSuccess) return fail(c, MMT_ERR_HIP, std::string("eval_direction: ") + hipGetErrorString(e));
  return MMT_OK;
}

}  // extern "C"


// seed of the dropout masks of the next training forward (and its backward); without a call the
// engine derives one from mmt_config.seed and a per-context counter
extern "C" int mmt_set_dropout_seed(mmt_ctx* c, uint64_t seed) {
  if (!c) return MMT_ERR_INVALID;
  c->next_seed = seed;
  c->next_seed_set = true;
  return MMT_OK;
}

// live per-kernel timing: HIP events around every launch whose label matches one of the
// comma-separated patterns of `label` (e.g. "*_dw,attn_fwd,attn_bwd,ffn0"), recorded on the stream
// the launch runs on, so bench.py can price kernels inside the timed region.
// serial mode for measurement (bench.py's serial roofline leg): 0 = everything of this context on the
// caller's stream, 1 = the side stream again. Latched: the next mmt_forward applies it, so a call between
// a forward and its backward (or between backward stages) never strands forked side-stream work
extern "C" int mmt_set_side_stream(mmt_ctx* c, int32_t on) {
  if (!c) return MMT_ERR_INVALID;
  c->side_off_req = on == 0;
  return MMT_OK;
}

extern "C" int mmt_probe_set(mmt_ctx* c, const char* label) {
  if (!c) return MMT_ERR_INVALID;
  c->probe_events.clear();
  c->probe_pats.clear();
  if (label) {
    std::string cur;
    for (const char* q = label;; ++q) {
      if (*q == ',' || *q == 0) {
        if (!cur.empty()) c->probe_pats.push_back(cur);
        cur.clear();
        if (!*q) break;
      } else if (*q != ' ') {
        cur += *q;
      }
    }
  }
  // event pairs for the recorded launches, made here (event creation is a host call of tens of
  // microseconds: inside the timed loop it starved the GPU); recording stops when they run out
  static const size_t pool = [] {
    const char* e = getenv("MMT_PROBE_EVENTS");
    return (size_t)(e ? atoi(e) : 4096);
  }();
  while (!c->probe_pats.empty() && c->probe_pool.size() < pool) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess) break;
    if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); break; }
    c->probe_pool.push_back({a, b});
  }
  return MMT_OK;
}

extern "C" int mmt_probe_enable(mmt_ctx* c, int32_t on) {
  if (!c) return MMT_ERR_INVALID;
  c->probe_on = on != 0;
  return MMT_OK;
}

extern "C" int32_t mmt_probe_count(const mmt_ctx* c) { return c ? (int32_t)c->probe_pats.size() : 0; }

extern "C" int mmt_probe_read_at(mmt_ctx* c, int32_t pat, double* total_ms, int64_t* launches, double* flops,
                                 double* bytes) {
  if (!c) return MMT_ERR_INVALID;
  double tot = 0.0, fl = 0.0, by = 0.0;
  int64_t n = 0;
  for (auto& e : c->probe_events) {
    if (pat >= 0 && e.pat != pat) continue;
    float ms = 0.f;
    if (hipEventSynchronize(e.b) != hipSuccess) return fail(c, MMT_ERR_HIP, "probe event sync");
    if (hipEventElapsedTime(&ms, e.a, e.b) != hipSuccess) return fail(c, MMT_ERR_HIP, "probe elapsed");
    tot += ms;
    fl += e.flops;
    by += e.bytes;
    ++n;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = n;
  if (flops) *flops = fl;
  if (bytes) *bytes = by;
  return MMT_OK;
}

extern "C" int mmt_probe_read(mmt_ctx* c, double* total_ms, int64_t* launches) {
  return mmt_probe_read_at(c, -1, total_ms, launches, nullptr, nullptr);
}
