// Single-problem C-ABI wrappers over the kernel launchers (include/mmt.h, mmt_op_*), used by the
// kernel-level parity tests. Same kernels the engine launches, one group member.
#include <hip/hip_runtime.h>

#include "mmt.h"
#include "mmt_kernels.h"

static int st(hipError_t e) { return e == hipSuccess ? MMT_OK : MMT_ERR_HIP; }

extern "C" {

int mmt_op_gemm(void* stream, int32_t a_kc, int32_t b_kc, int32_t epi, int32_t splits, int32_t M, int32_t N,
                int32_t K, const void* A, int32_t lda, const void* B, int32_t ldb, const float* bias, const void* aux,
                int32_t ldaux, const float* resid, int32_t ldres, float* o32, int32_t ldc, void* o16, int32_t ldo16,
                float alpha) {
  if (epi < 0 || epi >= EPI_COUNT || M < 0 || N < 0 || K < 0) return MMT_ERR_INVALID;
  if ((lda & 7) || (ldb & 7)) return MMT_ERR_INVALID;  // 16-byte operand staging
  GemmBatch b{};
  b.count = 1;
  GemmProblem& p = b.p[0];
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb; p.bias = bias;
  p.aux = (const bf16_t*)aux; p.ldaux = ldaux; p.resid = resid; p.ldres = ldres; p.o32 = o32; p.ldc = ldc;
  p.o16 = (bf16_t*)o16; p.ldo16 = ldo16; p.alpha = alpha; p.M = M; p.N = N; p.K = K;
  const hipError_t e = mmt_launch_gemm(b, a_kc != 0, b_kc != 0, epi, splits, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return MMT_ERR_UNSUPPORTED;
  return st(e);
}

int mmt_op_gemm_qkv(void* stream, int32_t M, int32_t N, int32_t K, const void* A, int32_t lda, const void* B,
                    int32_t ldb, const float* bias, void* h1, int32_t ldh1, const float* w2, int32_t hh, void* out,
                    int32_t ld_out) {
  if (M < 0 || N < 0 || K < 0 || !out || !w2) return MMT_ERR_INVALID;
  GemmBatch b{};
  b.count = 1;
  GemmProblem& p = b.p[0];
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb; p.bias = bias;
  p.o16 = (bf16_t*)h1; p.ldo16 = ldh1; p.alpha = 1.f; p.M = M; p.N = N; p.K = K;
  p.qkv2_w2 = w2; p.qkv2_out = (bf16_t*)out; p.qkv2_ld = ld_out; p.qkv2_hh = hh;
  const hipError_t e = mmt_launch_gemm(b, true, true, EPI_BIAS_TANH_BF16, 1, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return MMT_ERR_UNSUPPORTED;
  return st(e);
}

int mmt_op_gemm_wgrad(void* stream, int32_t M, int32_t N, int32_t K, const void* A, int32_t lda, const void* B,
                      int32_t ldb, float* out, int32_t ldc, float alpha, void* slab, int64_t slab_bytes) {
  if (M < 0 || N < 0 || K < 0 || (lda & 7) || (ldb & 7) || !out) return MMT_ERR_INVALID;
  GemmBatch b{};
  b.count = 1;
  GemmProblem& p = b.p[0];
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb;
  p.o32 = out; p.ldc = ldc; p.alpha = alpha; p.M = M; p.N = N; p.K = K;
  const hipError_t e = mmt_launch_gemm_wgrad(b, (float*)slab, slab ? slab_bytes : 0, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return MMT_ERR_UNSUPPORTED;
  return st(e);
}

int mmt_op_mlp2(void* stream, int32_t M, int32_t C, const void* x, int32_t ldx, const void* w0, int32_t ldw0,
                const float* b0, const void* w2, int32_t ldw2, const float* b2, void* h, int32_t ldh, const float* resid,
                float* out, void* out16, uint32_t drop_key, uint32_t drop_thr, float drop_scale, const float* lnf_gamma,
                const float* lnf_beta, void* lnf_y, float* lnf_mean, float* lnf_rstd) {
  if (M < 1 || C < 2) return MMT_ERR_INVALID;
  Mlp2Batch b{};
  b.count = 1;
  GemmProblem& p1 = b.g1[0];
  p1.A = (const bf16_t*)x; p1.lda = ldx; p1.B = (const bf16_t*)w0; p1.ldb = ldw0; p1.bias = b0;
  p1.o16 = (bf16_t*)h; p1.ldo16 = ldh; p1.alpha = 1.f; p1.M = M; p1.N = C / 2; p1.K = C;
  GemmProblem& p2 = b.g2[0];
  p2.A = (const bf16_t*)h; p2.lda = ldh; p2.B = (const bf16_t*)w2; p2.ldb = ldw2; p2.bias = b2;
  p2.resid = resid; p2.ldres = C; p2.o32 = out; p2.ldc = C; p2.o16 = (bf16_t*)out16; p2.ldo16 = C;
  p2.alpha = 1.f; p2.M = M; p2.N = C; p2.K = C / 2;
  p2.drop_key = drop_key; p2.drop_thr = drop_thr; p2.drop_scale = drop_scale;
  p2.lnf_gamma = lnf_gamma; p2.lnf_beta = lnf_beta; p2.lnf_y = (bf16_t*)lnf_y; p2.lnf_mean = lnf_mean;
  p2.lnf_rstd = lnf_rstd;
  if (!mmt_mlp2_ok(b)) return MMT_ERR_UNSUPPORTED;
  return st(mmt_launch_mlp2(b, (hipStream_t)stream));
}

int mmt_op_mlp2_bwd(void* stream, int32_t M, int32_t C, const void* dy, int32_t lddy, const void* w2, int32_t ldw2,
                    const void* h, int32_t ldh, float alpha, const void* w0, int32_t ldw0, void* dh, int32_t lddh,
                    float* db0, void* dx) {
  if (M < 1 || C < 2) return MMT_ERR_INVALID;
  Mlp2Batch b{};
  b.count = 1;
  GemmProblem& p1 = b.g1[0];
  p1.A = (const bf16_t*)dy; p1.lda = lddy; p1.B = (const bf16_t*)w2; p1.ldb = ldw2; p1.aux = (const bf16_t*)h;
  p1.ldaux = ldh; p1.o16 = (bf16_t*)dh; p1.ldo16 = lddh; p1.dbias = db0; p1.alpha = alpha; p1.M = M; p1.N = C / 2;
  p1.K = C;
  GemmProblem& p2 = b.g2[0];
  p2.A = (const bf16_t*)dh; p2.lda = lddh; p2.B = (const bf16_t*)w0; p2.ldb = ldw0; p2.o16 = (bf16_t*)dx; p2.ldo16 = C;
  p2.alpha = 1.f; p2.M = M; p2.N = C; p2.K = C / 2;
  if (!mmt_mlp2_bwd_ok(b)) return MMT_ERR_UNSUPPORTED;
  return st(mmt_launch_mlp2_bwd(b, (hipStream_t)stream));
}

int mmt_op_layernorm_fwd(void* stream, int32_t R, int32_t C, const float* x, const float* gamma, const float* beta,
                         void* y16, float* mean, float* rstd) {
  LnBatch b{};
  b.count = 1;
  b.p[0].x = x; b.p[0].gamma = gamma; b.p[0].beta = beta; b.p[0].y = (bf16_t*)y16; b.p[0].mean = mean; b.p[0].rstd = rstd;
  return st(mmt_launch_ln_fwd(b, R, C, (hipStream_t)stream));
}

int mmt_op_layernorm_bwd(void* stream, int32_t R, int32_t C, const float* x, const float* gamma, const float* mean,
                         const float* rstd, const float* dy, float* dx, void* dx16, float* dgamma, float* dbeta) {
  LnBatch b{};
  b.count = 1;
  LnProblem& p = b.p[0];
  p.x = x; p.gamma = gamma; p.mean = (float*)mean; p.rstd = (float*)rstd; p.dy = dy; p.dx = dx; p.dx16 = (bf16_t*)dx16;
  p.dgamma = dgamma; p.dbeta = dbeta;
  return st(mmt_launch_ln_bwd(b, R, C, (hipStream_t)stream));
}

int mmt_op_gemm_ln_bwd(void* stream, int32_t M, int32_t N, int32_t K, const void* A, int32_t lda, const void* B,
                       int32_t ldb, float alpha, const float* x, const float* gamma, const float* mean,
                       const float* rstd, float* dx, void* dx16, float* dgamma, float* dbeta, float* dsum,
                       uint32_t drop_key, uint32_t drop_thr, float drop_scale) {
  if (M < 0 || N < 0 || K < 0) return MMT_ERR_INVALID;
  GemmBatch b{};
  b.count = 1;
  GemmProblem& p = b.p[0];
  p.A = (const bf16_t*)A; p.lda = lda; p.B = (const bf16_t*)B; p.ldb = ldb; p.alpha = alpha; p.M = M; p.N = N; p.K = K;
  p.resid = x; p.ldres = N; p.o32 = dx; p.ldc = N; p.o16 = (bf16_t*)dx16; p.ldo16 = N; p.dbias = dsum;
  p.ln_gamma = gamma; p.ln_mean = mean; p.ln_rstd = rstd; p.ln_dgamma = dgamma; p.ln_dbeta = dbeta;
  p.drop_key = drop_key; p.drop_thr = drop_thr; p.drop_scale = drop_scale;
  if (!mmt_gemm_ln_bwd_ok(b)) return MMT_ERR_UNSUPPORTED;
  return st(mmt_launch_gemm_ln_bwd(b, (hipStream_t)stream));
}

static void fill_attn(AttnProblem& p, int nstreams, const void* q, int q_ld, const void* const* k, const void* const* v,
                      int kv_ld, int kv_hstride) {
  p.q = (const bf16_t*)q; p.q_ld = q_ld; p.kv_ld = kv_ld; p.kv_hstride = kv_hstride; p.nstreams = nstreams;
  for (int j = 0; j < nstreams; ++j) { p.k[j] = (const bf16_t*)k[j]; p.v[j] = (const bf16_t*)v[j]; }
}

int mmt_op_attention_fwd(void* stream, int32_t B, int32_t T, int32_t H, int32_t hs, int32_t nstreams, const void* q,
                         int32_t q_ld, const void* const* k, const void* const* v, int32_t kv_ld, int32_t kv_hstride,
                         void* o, int32_t o_ld, void* const* oj, float* const* lse) {
  if (nstreams < 1 || nstreams > MMT_MAX_STREAMS) return MMT_ERR_INVALID;
  AttnBatch b{};
  b.count = 1;
  AttnProblem& p = b.p[0];
  fill_attn(p, nstreams, q, q_ld, k, v, kv_ld, kv_hstride);
  p.o = (bf16_t*)o; p.o_ld = o_ld;
  for (int j = 0; j < nstreams; ++j) {
    p.oj[j] = oj ? (bf16_t*)oj[j] : nullptr;
    p.lse[j] = lse[j];
  }
  const float scale = 1.0f / __builtin_sqrtf((float)hs);
  const hipError_t e = mmt_launch_attn_fwd(b, B, T, H, hs, scale, (hipStream_t)stream);
  return e == hipErrorInvalidValue ? MMT_ERR_UNSUPPORTED : st(e);
}

int mmt_op_attention_bwd_ws(void* stream, int32_t B, int32_t T, int32_t H, int32_t hs, int32_t nstreams,
                            const void* q, int32_t q_ld, const void* const* k, const void* const* v, int32_t kv_ld,
                            int32_t kv_hstride, const void* o, int32_t o_ld, const void* const* oj,
                            const float* const* lse, const void* dout, int32_t dout_ld, float* const* dvec, void* dq,
                            int32_t dq_ld, void* const* dk, void* const* dv, int32_t dkv_ld, int32_t dkv_hstride,
                            float* dq32, int32_t dq32_ld);
int mmt_op_attention_bwd(void* stream, int32_t B, int32_t T, int32_t H, int32_t hs, int32_t nstreams, const void* q,
                         int32_t q_ld, const void* const* k, const void* const* v, int32_t kv_ld, int32_t kv_hstride,
                         const void* o, int32_t o_ld, const void* const* oj, const float* const* lse, const void* dout,
                         int32_t dout_ld, float* const* dvec, void* dq, int32_t dq_ld, void* const* dk, void* const* dv,
                         int32_t dkv_ld, int32_t dkv_hstride) {
  return mmt_op_attention_bwd_ws(stream, B, T, H, hs, nstreams, q, q_ld, k, v, kv_ld, kv_hstride, o, o_ld, oj, lse, dout,
                                 dout_ld, dvec, dq, dq_ld, dk, dv, dkv_ld, dkv_hstride, nullptr, 0);
}

int mmt_op_attention_bwd_ws(void* stream, int32_t B, int32_t T, int32_t H, int32_t hs, int32_t nstreams,
                            const void* q, int32_t q_ld, const void* const* k, const void* const* v, int32_t kv_ld,
                            int32_t kv_hstride, const void* o, int32_t o_ld, const void* const* oj,
                            const float* const* lse, const void* dout, int32_t dout_ld, float* const* dvec, void* dq,
                            int32_t dq_ld, void* const* dk, void* const* dv, int32_t dkv_ld, int32_t dkv_hstride,
                            float* dq32, int32_t dq32_ld) {
  if (nstreams < 1 || nstreams > MMT_MAX_STREAMS) return MMT_ERR_INVALID;
  AttnBatch b{};
  b.count = 1;
  AttnProblem& p = b.p[0];
  fill_attn(p, nstreams, q, q_ld, k, v, kv_ld, kv_hstride);
  p.o = (bf16_t*)o; p.o_ld = o_ld;
  for (int j = 0; j < nstreams; ++j) {
    p.oj[j] = oj ? (bf16_t*)oj[j] : nullptr;
    p.lse[j] = (float*)lse[j];
    p.dvec[j] = dvec[j];
    p.dk[j] = (bf16_t*)dk[j];
    p.dv[j] = (bf16_t*)dv[j];
  }
  p.dout = (const bf16_t*)dout; p.dout_ld = dout_ld; p.dq = (bf16_t*)dq; p.dq_ld = dq_ld;
  p.dkv_ld = dkv_ld; p.dkv_hstride = dkv_hstride;
  p.dq32 = dq32; p.dq32_ld = dq32_ld;
  const float scale = 1.0f / __builtin_sqrtf((float)hs);
  const hipError_t e = mmt_launch_attn_bwd(b, B, T, H, hs, scale, (hipStream_t)stream);
  return e == hipErrorInvalidValue ? MMT_ERR_UNSUPPORTED : st(e);
}

int mmt_op_qkv2_fwd(void* stream, int32_t R, int32_t nblk, int32_t hs, const void* h1, int32_t ld_h1, const float* w2,
                    void* out, int32_t ld_out) {
  Qkv2Batch b{};
  b.count = 1;
  b.p[0].h1 = (const bf16_t*)h1; b.p[0].w2 = w2; b.p[0].out = (bf16_t*)out;
  const hipError_t e = mmt_launch_qkv2_fwd(b, R, nblk, hs, ld_h1, ld_out, (hipStream_t)stream);
  return e == hipErrorInvalidValue ? MMT_ERR_UNSUPPORTED : st(e);
}

int mmt_op_qkv2_bwd(void* stream, int32_t R, int32_t nblk, int32_t hs, const void* h1, int32_t ld_h1, const float* w2,
                    const void* dout, int32_t ld_out, void* dh1, float* dw2) {
  Qkv2Batch b{};
  b.count = 1;
  b.p[0].h1 = (const bf16_t*)h1; b.p[0].w2 = w2; b.p[0].dout = (const bf16_t*)dout; b.p[0].dh1 = (bf16_t*)dh1;
  b.p[0].dw2 = dw2;
  const hipError_t e = mmt_launch_qkv2_bwd(b, R, nblk, hs, ld_h1, ld_out, (hipStream_t)stream);
  return e == hipErrorInvalidValue ? MMT_ERR_UNSUPPORTED : st(e);
}

int mmt_op_colsum(void* stream, int32_t R, int32_t N, const void* x, int32_t ld, float* out, float alpha) {
  ColsumBatch b{};
  b.count = 1;
  b.p[0].x = (const bf16_t*)x; b.p[0].ld = ld; b.p[0].out = out; b.p[0].N = N; b.p[0].alpha = alpha;
  return st(mmt_launch_colsum(b, R, (hipStream_t)stream));
}

int mmt_op_cross_entropy(void* stream, int32_t R, int32_t V, const float* logits, const int64_t* tgt, void* dlogits,
                         int32_t ld_d, float* loss) {
  CeBatch b{};
  b.count = 1;
  b.p[0].logits = logits; b.p[0].tgt = tgt; b.p[0].dlogits = (bf16_t*)dlogits; b.p[0].loss = loss; b.p[0].V = V;
  b.p[0].ld_d = ld_d;
  return st(mmt_launch_ce_fwd(b, R, (hipStream_t)stream));
}

int mmt_op_embedding_fwd(void* stream, int32_t B, int32_t T, int32_t C, int32_t V, const int64_t* idx, const float* tok,
                         const float* pos, float* x) {
  EmbBatch b{};
  b.count = 1;
  b.p[0].idx = idx; b.p[0].tok = tok; b.p[0].pos = pos; b.p[0].x = x; b.p[0].V = V;
  return st(mmt_launch_embed_fwd(b, B, T, C, (hipStream_t)stream));
}

int mmt_op_embedding_bwd(void* stream, int32_t B, int32_t T, int32_t C, int32_t V, const int64_t* idx, const float* dx,
                         float* dtok, float* dpos) {
  EmbBatch b{};
  b.count = 1;
  b.p[0].idx = idx; b.p[0].dx = dx; b.p[0].dtok = dtok; b.p[0].dpos = dpos; b.p[0].V = V;
  return st(mmt_launch_embed_bwd(b, B, T, C, (hipStream_t)stream));
}

int mmt_op_embedding_bwd_ws(void* stream, int32_t B, int32_t T, int32_t C, int32_t V, const int64_t* idx,
                            const float* dx, float* dtok, float* dpos, float* scratch) {
  EmbBatch b{};
  b.count = 1;
  b.p[0].idx = idx; b.p[0].dx = dx; b.p[0].dtok = dtok; b.p[0].dpos = dpos; b.p[0].V = V; b.p[0].part = scratch;
  return st(mmt_launch_embed_bwd(b, B, T, C, (hipStream_t)stream));
}

}  // extern "C"

// ---- MX-fp8 (C4's fp8 path) -------------------------------------------------------------------
int mmt_op_mx_quant(void* stream, int32_t rows, int32_t cols, const float* src, int32_t ld_src, void* dst8,
                    int32_t ld8, void* s8, int32_t lds8) {
  if (rows < 0 || cols < 0 || (cols & 31) || (ld_src & 3) || (ld8 & 15) || lds8 * 32 < cols || !src || !dst8 || !s8)
    return MMT_ERR_INVALID;
  // one "base" for source and destinations: offsets relative to the source / destination pointers
  MxSeg S{};
  S.src = 0; S.dst = 0; S.sdst = (const uint8_t*)s8 - (const uint8_t*)dst8;
  S.rows = rows; S.cols = cols; S.ld_src = ld_src; S.ld8 = ld8; S.lds8 = lds8;
  return st(mmt_launch_mx_quant1(S, src, (uint8_t*)dst8, (hipStream_t)stream));
}

int mmt_op_gemm_f8(void* stream, int32_t epi, int32_t M, int32_t N, int32_t K, const void* A8, int32_t lda,
                   const void* sa, int32_t lds_a, const void* B8, int32_t ldb, const void* sb, int32_t lds_b,
                   const float* bias, const float* resid, int32_t ldres, float* o32, int32_t ldc, void* o16,
                   int32_t ldo16, void* o8, int32_t ld8, void* s8, int32_t lds8) {
  GemmBatch b{};
  b.count = 1;
  GemmProblem& p = b.p[0];
  p.A = (const bf16_t*)A8; p.lda = lda; p.B = (const bf16_t*)B8; p.ldb = ldb;
  p.sa = (const uint8_t*)sa; p.lds_a = lds_a; p.sb = (const uint8_t*)sb; p.lds_b = lds_b;
  p.bias = bias; p.resid = resid; p.ldres = ldres; p.o32 = o32; p.ldc = ldc; p.o16 = (bf16_t*)o16; p.ldo16 = ldo16;
  p.o8 = (uint8_t*)o8; p.ld8 = ld8; p.s8 = (uint8_t*)s8; p.lds8 = lds8;
  p.M = M; p.N = N; p.K = K; p.alpha = 1.f;
  const hipError_t e = mmt_launch_gemm_f8(b, epi, (hipStream_t)stream);
  if (e == hipErrorInvalidValue) return MMT_ERR_UNSUPPORTED;
  return st(e);
}

int mmt_op_layernorm_fwd_f8(void* stream, int32_t R, int32_t C, const float* x, const float* gamma, const float* beta,
                            void* y16, float* mean, float* rstd, void* y8, int32_t ld8, void* s8, int32_t lds8) {
  if (C & 31) return MMT_ERR_UNSUPPORTED;
  LnBatch b{};
  b.count = 1;
  LnProblem& p = b.p[0];
  p.x = x; p.gamma = gamma; p.beta = beta; p.y = (bf16_t*)y16; p.mean = mean; p.rstd = rstd;
  p.y8 = (uint8_t*)y8; p.ld8 = ld8; p.s8 = (uint8_t*)s8; p.lds8 = lds8;
  return st(mmt_launch_ln_fwd(b, R, C, (hipStream_t)stream));
}
