/* mmt.h — C-ABI of libmmt_hip.so, the MI355X-native (gfx950) training hot path of the
 * multimodal transformer of tsnuk/trade-AId-multimodal-transformer.
 *
 * The reference exposes no C / FFI boundary on this path: its boundary is the
 * Python module API that main.py imports. Each entry point below replaces one piece of that
 * Python surface; the Python host layer (trade-aid-multimodal-transformer_amd/model.py,
 * mmt_optim.py, training_utils.py) binds them through ctypes exactly as INTEGRATION.md shows.
 *
 *   mmt_create / mmt_destroy      <- MultimodalTransformer.__init__ (reference model.py:358-370):
 *                                    dims from config_utils (model.py:25-27), cross flags from
 *                                    all_modality_params[i][8] (model.py:196)
 *   mmt_tensor_count/_info        <- MultimodalTransformer.state_dict() key set and shapes
 *                                    (reference main.py:470, 635) over one flat fp32 buffer
 *   mmt_forward                   <- MultimodalTransformer.forward(idx_list, targets_list)
 *                                    (model.py:380-402): logits per modality + mean CE losses
 *   mmt_backward[_stage]          <- total_loss.backward() of main.py:646-649 (autograd over
 *                                    model.py), gradients into a flat fp32 buffer
 *   mmt_adamw_step                <- torch.optim.AdamW(m.parameters(), lr).step() (main.py:464, 650)
 *   mmt_decode_step               <- one token of MultimodalTransformer.generate (model.py:404-446),
 *                                    with a KV cache instead of the reference's full re-forward
 *   mmt_eval_direction            <- the per-sample loop of calculate_evaluation_metrics
 *                                    (training_utils.py:259-304)
 *   mmt_op_*                      primitive kernels, exported for kernel-level parity tests.
 *
 * Conventions: every pointer is a device pointer unless stated; memory is owned by the caller
 * (PyTorch allocates parameters, gradients, moments, logits and the workspace); the library
 * never frees caller memory. All work is asynchronous on the caller's HIP stream (`stream` is a
 * hipStream_t passed as void*). Every function returns 0 (MMT_OK) or a negative mmt_status;
 * no C++ exception crosses the ABI; mmt_last_error() describes the last failure.
 */
#ifndef MMT_H_
#define MMT_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMT_MAX_MODALITIES 8

enum mmt_status {
  MMT_OK = 0,
  MMT_ERR_INVALID = -1,     /* bad argument / shape */
  MMT_ERR_UNSUPPORTED = -2, /* configuration outside what the kernels implement */
  MMT_ERR_HIP = -3,         /* a HIP runtime call or launch failed */
  MMT_ERR_STATE = -4        /* call order violated (e.g. backward without matching forward) */
};

typedef struct mmt_config {
  int32_t num_modalities;                       /* M, 1..8 */
  int32_t n_embd;                               /* C */
  int32_t n_head;                               /* H, head size C/H in {8,16,24,32,48,64} */
  int32_t n_layer;                              /* L */
  int32_t block_size;                           /* T (max sequence length, positional table rows) */
  int32_t vocab_sizes[MMT_MAX_MODALITIES];      /* V_i >= 1 */
  int32_t cross_attention[MMT_MAX_MODALITIES];  /* all_modality_params[i][8] */
  float dropout;                                /* nn.Dropout p (model.py:57,87,107,134,171) */
  uint64_t seed;                                /* dropout RNG seed */
  int32_t precision;                            /* 0: bf16 MFMA; 1: MX-fp8 forward GEMMs (C4;
                                                   Q/K/V stage 1, FFN, cross-attention query;
                                                   needs n_embd % 32 == 0) */
} mmt_config;

typedef struct mmt_ctx mmt_ctx;

/* lifecycle */
mmt_ctx* mmt_create(const mmt_config* cfg); /* NULL on failure, see mmt_create_error() */
const char* mmt_create_error(void);
void mmt_destroy(mmt_ctx* ctx);
const char* mmt_last_error(const mmt_ctx* ctx);
const char* mmt_version(void);

/* parameter layout: one flat fp32 buffer; each reference state_dict tensor is a contiguous slice */
int64_t mmt_param_count(const mmt_ctx* ctx);        /* elements of the flat buffer */
int64_t mmt_param_active_count(const mmt_ctx* ctx); /* prefix that receives gradients */
int32_t mmt_tensor_count(const mmt_ctx* ctx);
int mmt_tensor_info(const mmt_ctx* ctx, int32_t i, char* name, int32_t name_cap, int64_t* offset, int32_t* ndim,
                    int64_t* shape /* [2] */, int32_t* kind /* 0 weight(N(0,.02)) 1 bias(0) 2 ln weight(1) 3 ln bias(0) */);

/* workspace (saved activations + packed bf16 weights + backward scratch) for a batch size */
int64_t mmt_workspace_bytes(mmt_ctx* ctx, int32_t batch);

/* forward: idx[i], tgt[i] int64 [batch, T] (tgt may be NULL: no loss); logits[i] fp32 [batch, T, V_i];
 * losses fp32 [M] (mean CE per modality, written only when tgt != NULL); training != 0 enables dropout */
int mmt_forward(mmt_ctx* ctx, void* stream, int32_t batch, const int64_t* const* idx, const int64_t* const* tgt,
                const float* params, float* const* logits, float* losses, void* workspace, int32_t training);

/* KV-cache decode step of generate (reference model.py:404-446, which re-runs the whole forward
 * per new token): the forward of ONE new position `pos` (1 <= pos < block_size) of every sequence
 * and modality. idx[i]: int64 [batch] tokens of modality i at position pos; logits[i]: fp32
 * [batch, V_i], the logits at position pos. Keys / values of positions < pos come from the last
 * mmt_forward on this workspace (the prefill: prompt right-padded to block_size) and the decode
 * steps since, which this step extends by position pos. Eval semantics (no dropout); the weights
 * are the ones packed by that prefill forward. MMT_ERR_STATE without a prefill, after a prefill
 * that sampled dropout (training != 0 with dropout > 0: its keys / values are not the eval ones),
 * and at precision fp8 (the prefill's MX-fp8 GEMMs would not match a bf16 decode). */
int mmt_decode_step(mmt_ctx* ctx, void* stream, int32_t batch, int32_t pos, const int64_t* const* idx,
                    const float* params, float* const* logits, void* workspace);

/* failure detection (the reference's guard is the NaN check on eval losses,
 * main.py:606): byte offset in the workspace of two int32 bitmasks (the same for every batch size;
 * the query never touches the workspace plan of a pending backward or decode). The
 * loss kernel sets bit i of both when modality i's mean CE is NaN or Inf; word 0 is cleared by
 * every mmt_forward with targets (the last forward's flags), word 1 only by the caller (sticky
 * since the caller last cleared it; zero it when the workspace is allocated). Read them when the
 * host syncs anyway; no kernel ever traps. */
int64_t mmt_loss_flag_offset(mmt_ctx* ctx, int32_t batch);

/* dropout (model.py:57/69, 87/91, 107/116, 134/151, 171; nn.Dropout(p) in training mode only):
 * masks are a counter hash of (seed, layer, modality, site, row, column) regenerated in the
 * backward, so nothing is stored. Sets the seed of the NEXT training forward (and its backward);
 * without a call the engine derives one from mmt_config.seed and a per-context counter. */
int mmt_set_dropout_seed(mmt_ctx* ctx, uint64_t seed);

/* backward of sum_i loss_grads[i] * loss_i through the last mmt_forward (same workspace/params).
 * grads: fp32 flat buffer of the active prefix (mmt_param_active_count elements) — OVERWRITTEN
 * (zeroed then accumulated); the never-used tail past it has no gradient (reference: .grad None). */
int mmt_backward(mmt_ctx* ctx, void* stream, const float* loss_grads, const float* params, float* grads,
                 void* workspace);
/* the same, split into stages (post-block, layer L-1 .. layer 0, embeddings) so a caller can
 * all-reduce each finished gradient range while the next stage computes (DP overlap). */
int32_t mmt_backward_stage_count(const mmt_ctx* ctx);
int mmt_backward_stage_range(const mmt_ctx* ctx, int32_t stage, int64_t* begin, int64_t* end);
int mmt_backward_stage(mmt_ctx* ctx, void* stream, int32_t stage, const float* loss_grads, const float* params,
                       float* grads, void* workspace);

/* fused AdamW over n elements (torch.optim.AdamW semantics, decoupled decay, bias correction) */
int mmt_adamw_step(mmt_ctx* ctx, void* stream, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                   int64_t n, int64_t step, float lr, float beta1, float beta2, float eps, float weight_decay);

/* directional metric for one numeric modality: logits fp32 [batch, T, V]; xb/yb int64 [batch, T];
 * vocab fp64 [V]; accumulates wins_losses[0..1] (int32) and certainty_sum (fp64) on device */
int mmt_eval_direction(mmt_ctx* ctx, void* stream, int32_t batch, int32_t T, int32_t V, const float* logits,
                       const int64_t* xb, const int64_t* yb, const double* vocab, int32_t is_percent,
                       int32_t* wins_losses, double* certainty_sum);

/* live kernel timing (no reference counterpart: the reference has no profiler):
 * HIP events around every engine launch whose label matches one of the comma-separated
 * patterns of `label` — an exact label ("ffn0", "attn_fwd", "attn_bwd", "qkv1_dw", ...), "*suffix"
 * ("*_dw": every weight-gradient GEMM) or "prefix*" — recorded on the stream that launch runs on
 * (the side stream for weight gradients). NULL or "" disables. Each recorded launch carries its
 * algorithmic flops and HBM bytes (every operand read once, every output written once; attention
 * causal-useful). mmt_probe_read_at waits for the events of pattern `pattern` (-1: all) and
 * returns the summed device time, launch count, flops and bytes; mmt_probe_read = all patterns. */
int mmt_probe_set(mmt_ctx* ctx, const char* label);
int32_t mmt_probe_count(const mmt_ctx* ctx);
int mmt_probe_read(mmt_ctx* ctx, double* total_ms, int64_t* launches);
int mmt_probe_read_at(mmt_ctx* ctx, int32_t pattern, double* total_ms, int64_t* launches, double* flops,
                      double* bytes);
/* Pause (on = 0) / resume (on != 0) the probe's recording without clearing it: the bench samples
 * one step in eight, so the probe's event records stay out of the other steps. */
int mmt_probe_enable(mmt_ctx* ctx, int32_t on);
/* Serial mode for measurement: on = 0 runs every launch of this context on the caller's stream (no
 * side stream for the weight gradients and keep bits), on != 0 restores the default. Latched: the
 * next mmt_forward applies it (a forward and its backward always run under one setting). */
int mmt_set_side_stream(mmt_ctx* ctx, int32_t on);

/* ---- device-resident batcher: get_batch (training_utils.py:333-384) on HBM token streams ---- */
/* in-place random walk of one int32 training stream (data_utils.py:342-351 as reached through
 * training_utils.py:350-360): x += uniform{0,+-1..+-r} where r < x < V - r */
int mmt_batch_jitter(void* stream, int32_t* data, int64_t n, int32_t rand_size, int32_t vocab_size, uint64_t seed,
                     uint64_t counter);
/* batch start indices uniform over valid positions (generate_batch_starting_indices,
 * training_utils.py:33-181): cum_valid / file_start int64 [nfiles] describe the split */
int mmt_batch_indices(void* stream, int32_t batch, const int64_t* cum_valid, const int64_t* file_start, int32_t nfiles,
                      int32_t first_offset, uint64_t seed, uint64_t counter, int64_t* ix);
/* x[m] = data[m][ix : ix+T], y[m] = data[m][ix+1 : ix+T+1] (int64 [batch, T]); data/x/y are host
 * arrays of nmod device pointers */
int mmt_batch_gather(void* stream, int32_t nmod, const int32_t* const* data, const int64_t* ix, int32_t batch,
                     int32_t T, int64_t* const* x, int64_t* const* y);

/* ---- bit-exact device walk: get_batch's jitter (data_utils.py:342-351 through
 * training_utils.py:350-360) with the reference's own Python `random` stream (MT19937) ----
 * mt_state: device uint32[625] = CPython random.getstate()[1] (624 key words + index).
 * words: device buffer of mmt_exact_words_bytes(nwords) bytes; mmt_exact_gen fills it with the
 * generator's stream from mt_state (one workgroup; nwords >= the draws of one walk). mmt_exact_walk
 * walks data[r] (int32, n[r] elements) for every r with rand_size[r] != 0 (0 = None) in order,
 * each eligible element (r < x < V - r) taking the next accepted draw of random.choice, then moves
 * mt_state past the last word drawn. *status is set to 1 if the words ran out (never, at the
 * sizes mmt_exact_words_bytes is asked for by the Python batcher). scratch: see
 * mmt_exact_walk_scratch_bytes(max n[r], nwords). All asynchronous on `stream`. */
int64_t mmt_exact_words_bytes(int64_t nwords);
int64_t mmt_exact_walk_scratch_bytes(int64_t max_n, int64_t nwords);
int mmt_exact_gen(void* stream, const uint32_t* mt_state, uint32_t* words, int64_t nwords);
int mmt_exact_walk(void* stream, int32_t nmod, int32_t* const* data, const int64_t* n, const int32_t* rand_size,
                   const int32_t* vocab, uint32_t* mt_state, const uint32_t* words, int64_t nwords, void* scratch,
                   int64_t scratch_bytes, int32_t* status);
/* tuning knob: bit 0 / bit 1 = the slice-streamed hs-64 attention dK/dV / dQ pass, bit 2 = dK/dV at 3 waves
 * per SIMD, bit 3 = the slice-streamed hs-64 forward (default 15); returns the old value */
int mmt_attn_set_ring(int v);
/* tuning knob: attention dropout keep-bit tiles made per wave by attn_mask_kernel (1, 2, 4, 8 or 16; 0 = the env
 * MMT_MASK_G, default 16 at T >= 1024, else 8). The bits do not depend on it. Returns the old value */
int mmt_attn_set_mask_g(int g);
/* tuning knob: 1 = the big GEMM launches with K < 1024 (the d512 FFN / cross-attention K/V products) on a
 * 128 x 256 tile at two workgroups per CU instead of the 256 x 256 ping-pong kernel; 0 (default, env
 * MMT_GEMM_T2) = the ping-pong kernel. Returns the old value */
int mmt_gemm_set_t2(int v);

/* ---- primitive kernels (single problem), for kernel-level parity tests ------------------- */
/* GEMM pipeline variant (tuning knob, process-wide). 128x128 tile: bits 0-3 forward / backward-data,
 * bits 4-7 weight gradients: 0 = K-step 64 x 2 LDS stages, 1 = 32 x 2, 2 = 32 x 3, 3 = 32 x 4,
 * 4 = 64 x 3, 5 = 32 x 3 and 6 = 32 x 2 at 3+ blocks per CU (64-row epilogue passes). 256x256 tile:
 * bits 8-11 (0 = environment / default policy, 1 / 2 / 3 = BK 32 x 4 / x 3 / x 2); bit 16: the 256x256 tile
 * whatever K. Returns -1 for a field out of range. variant < 0: the default policy (128x128: 6 for
 * bf16-output epilogues without an aux operand, else 0; 256x256: 1 for the weight gradients, else
 * BK 64 x 2). */
int mmt_gemm_set_variant(int variant);
/* splits: split-K factor of EPI atomic_f32 launches (<= 0: automatic) */
int mmt_op_gemm(void* stream, int32_t a_kc, int32_t b_kc, int32_t epi, int32_t splits, int32_t M, int32_t N,
                int32_t K, const void* A, int32_t lda, const void* B, int32_t ldb, const float* bias,
                const void* aux, int32_t ldaux, const float* resid, int32_t ldres, float* o32, int32_t ldc,
                void* o16, int32_t ldo16, float alpha);
/* Q/K/V projection of the engine's forward (reference model.py:36-50, every head's key / query /
 * value MLP at once): h1[M, N] = bf16(tanh(A[M, K] B[N, K]^T + bias)) (stage 1, N = 3 H hh) and, fused
 * into the same GEMM's epilogue, stage 2 out[m, blk*2hh + o] = bf16(sum_i w2[blk][o][i] h1[m, blk*hh + i])
 * (w2 fp32 [N/hh][2hh][hh]). hh must be 16 or 32 and the GEMM must run on the 128 x 128 tile (not M,
 * N >= 256 with K >= 1024), else MMT_ERR_UNSUPPORTED (the engine then runs stage 2 as mmt_op_qkv2_fwd's
 * separate kernel); ld_out % 8 == 0, 16-B aligned out. */
int mmt_op_gemm_qkv(void* stream, int32_t M, int32_t N, int32_t K, const void* A, int32_t lda, const void* B,
                    int32_t ldb, const float* bias, void* h1, int32_t ldh1, const float* w2, int32_t hh, void* out,
                    int32_t ld_out);
/* weight gradient out[M, N] += alpha * A[K, M]^T B[K, N] (A, B bf16, MN-contiguous rows of K):
 * split-K into fp32 slabs in `slab` (device scratch of slab_bytes; NULL/0: one K pass) + a reduce
 * pass, the engine's path for every dW of the backward */
int mmt_op_gemm_wgrad(void* stream, int32_t M, int32_t N, int32_t K, const void* A, int32_t lda, const void* B,
                      int32_t ldb, float* out, int32_t ldc, float alpha, void* slab, int64_t slab_bytes);
/* attention out-projection as ONE fused launch (the engine's forward path at C = 256 / 512; replaces the
 * pair mmt_op_gemm(bias_tanh_bf16) + mmt_op_gemm(bias_resid_f32), reference model.py:82-92 / 102-117):
 *   h[M, C/2]  = bf16(tanh(x[M, C] W0[C/2, C]^T + b0))      (stored: the backward reads it)
 *   out[M, C]  = resid + keep(m, n) * (h W2[C, C/2]^T + b2)  (fp32; hash dropout of drop_key / drop_thr,
 *                kept values times drop_scale, 0: off), out16 (nullable) its bf16 copy;
 *   lnf_y (nullable) = bf16(LayerNorm(out) * lnf_gamma + lnf_beta), lnf_mean / lnf_rstd its row statistics
 * with h kept in LDS between the products. C must be 256 or 512 (else MMT_ERR_UNSUPPORTED); row strides
 * ldx, ldw0 (W0), ldw2 (W2), ldh (h); out / resid / out16 / lnf_y have stride C. */
int mmt_op_mlp2(void* stream, int32_t M, int32_t C, const void* x, int32_t ldx, const void* w0, int32_t ldw0,
                const float* b0, const void* w2, int32_t ldw2, const float* b2, void* h, int32_t ldh, const float* resid,
                float* out, void* out16, uint32_t drop_key, uint32_t drop_thr, float drop_scale, const float* lnf_gamma,
                const float* lnf_beta, void* lnf_y, float* lnf_mean, float* lnf_rstd);
/* its backward-data pair as ONE launch (the engine's backward path at C = 256 / 512; replaces
 * mmt_op_gemm(dtanh_bf16) + mmt_op_gemm(store_bf16)): dh[M, C/2] = bf16(alpha (dy[M, C] W2[C, C/2]) (1 - h^2))
 * with db0 (nullable) += its fp32 column sums, dx[M, C] = bf16(dh W0[C/2, C]); W2 / W0 are the forward
 * weights as stored ([C][C/2] / [C/2][C], row strides ldw2 / ldw0), h the forward's saved tanh output */
int mmt_op_mlp2_bwd(void* stream, int32_t M, int32_t C, const void* dy, int32_t lddy, const void* w2, int32_t ldw2,
                    const void* h, int32_t ldh, float alpha, const void* w0, int32_t ldw0, void* dh, int32_t lddh,
                    float* db0, void* dx);
int mmt_op_layernorm_fwd(void* stream, int32_t R, int32_t C, const float* x, const float* gamma, const float* beta,
                         void* y16, float* mean, float* rstd);
int mmt_op_layernorm_bwd(void* stream, int32_t R, int32_t C, const float* x, const float* gamma, const float* mean,
                         const float* rstd, const float* dy, float* dx, void* dx16, float* dgamma, float* dbeta);
/* backward-data GEMM with the LayerNorm backward of its rows fused (the engine's path when C == 256;
 * replaces the pair mmt_op_gemm(EPI store_f32) + mmt_op_layernorm_bwd, model.py:189-190 under
 * autograd): dy = alpha * A[M, K] B[K, N] (A K-contiguous, B MN-contiguous, bf16), never stored;
 * dx[M, N] += rstd * (g dy - mean(g dy) - xhat mean(g dy xhat)) with xhat = (x - mean) * rstd;
 * dx16 (nullable) = bf16(keep(m, n) * dx) with the hash mask of drop_key / drop_thr (0: no mask,
 * kept values times drop_scale) and dsum (nullable) += its column sums; dgamma += colsum(dy xhat),
 * dbeta += colsum(dy). N must be 256 or 512; row strides: A lda, B ldb, x / dx N, dx16 N.
 * MMT_ERR_UNSUPPORTED when the shape does not fit the fused kernel. */
int mmt_op_gemm_ln_bwd(void* stream, int32_t M, int32_t N, int32_t K, const void* A, int32_t lda, const void* B,
                       int32_t ldb, float alpha, const float* x, const float* gamma, const float* mean,
                       const float* rstd, float* dx, void* dx16, float* dgamma, float* dbeta, float* dsum,
                       uint32_t drop_key, uint32_t drop_thr, float drop_scale);
/* causal attention over nstreams KV streams; layouts as in the engine (row = b*T + t).
 * lse[j] (float [B*H*T] per stream, written by the forward, read by the backward) is in the LOG2
 * domain: lse = log2(sum_k 2^(log2(e) * scale * q.k)) = ln(sum_k e^(scale q.k)) / ln 2, with scale =
 * hs^-0.5 -- a natural-log LSE from another implementation must be divided by ln 2 first. */
int mmt_op_attention_fwd(void* stream, int32_t B, int32_t T, int32_t H, int32_t hs, int32_t nstreams,
                         const void* q, int32_t q_ld, const void* const* k, const void* const* v, int32_t kv_ld,
                         int32_t kv_hstride, void* o, int32_t o_ld, void* const* oj, float* const* lse);
int mmt_op_attention_bwd(void* stream, int32_t B, int32_t T, int32_t H, int32_t hs, int32_t nstreams,
                         const void* q, int32_t q_ld, const void* const* k, const void* const* v, int32_t kv_ld,
                         int32_t kv_hstride, const void* o, int32_t o_ld, const void* const* oj,
                         const float* const* lse, const void* dout, int32_t dout_ld, float* const* dvec, void* dq,
                         int32_t dq_ld, void* const* dk, void* const* dv, int32_t dkv_ld, int32_t dkv_hstride);
/* the same with a caller scratch of fp32 rows [B*T][>= H*hs] (dq32_ld % 4 == 0, 16-B aligned; contents
 * undefined afterwards): the one-pass hs-32 backward (T <= 256) sums dQ over several KV streams there,
 * so cross-attention takes it too (without scratch it takes the two-pass kernels) */
int mmt_op_attention_bwd_ws(void* stream, int32_t B, int32_t T, int32_t H, int32_t hs, int32_t nstreams,
                            const void* q, int32_t q_ld, const void* const* k, const void* const* v, int32_t kv_ld,
                            int32_t kv_hstride, const void* o, int32_t o_ld, const void* const* oj,
                            const float* const* lse, const void* dout, int32_t dout_ld, float* const* dvec, void* dq,
                            int32_t dq_ld, void* const* dk, void* const* dv, int32_t dkv_ld, int32_t dkv_hstride,
                            float* dq32, int32_t dq32_ld);
int mmt_op_qkv2_fwd(void* stream, int32_t R, int32_t nblk, int32_t hs, const void* h1, int32_t ld_h1,
                    const float* w2, void* out, int32_t ld_out);
int mmt_op_qkv2_bwd(void* stream, int32_t R, int32_t nblk, int32_t hs, const void* h1, int32_t ld_h1,
                    const float* w2, const void* dout, int32_t ld_out, void* dh1, float* dw2);
int mmt_op_colsum(void* stream, int32_t R, int32_t N, const void* x, int32_t ld, float* out, float alpha);
int mmt_op_cross_entropy(void* stream, int32_t R, int32_t V, const float* logits, const int64_t* tgt,
                         void* dlogits, int32_t ld_d, float* loss);
int mmt_op_embedding_fwd(void* stream, int32_t B, int32_t T, int32_t C, int32_t V, const int64_t* idx,
                         const float* tok, const float* pos, float* x);
int mmt_op_embedding_bwd(void* stream, int32_t B, int32_t T, int32_t C, int32_t V, const int64_t* idx,
                         const float* dx, float* dtok, float* dpos);
/* the same with a caller scratch of >= B*T*C floats (the engine passes a free backward buffer): each
 * row chunk's LDS-privatised token-table slabs are stored there and one reduce pass adds them into
 * dtok, so the rows split into short chunks without global atomics; dtok is accumulated (+=) */
int mmt_op_embedding_bwd_ws(void* stream, int32_t B, int32_t T, int32_t C, int32_t V, const int64_t* idx,
                            const float* dx, float* dtok, float* dpos, float* scratch);
// token-table gradient variant of the scratch path (mmt_op_embedding_bwd_ws, the engine's): 1 (default,
// env MMT_EMB_SORT) = counting sort of the rows by token + run sums (no LDS float atomics), 0 = the
// LDS-privatised slabs with per-chunk partial tables; returns the previous value (tests, A/B)
int mmt_emb_set_sort(int on);
// per-head Q/K/V stage-2 backward at hs 32 / 64 (mmt_op_qkv2_bwd, the engine's): bit 0 (hs 32) / bit 1
// (hs 64) set = each load instruction reads whole row slices and the tile is redistributed through
// LDS, clear = loads in the MFMA fragment layout; default 2 (env MMT_QKV2_COAL); returns the previous
// value (tests, A/B)
int mmt_qkv2_set_coal(int on);
// FFN ReLU' as bits (the ffn0 epilogue writes one bit per hidden element, the ffn2 data gradient reads
// them instead of the bf16 hidden rows): 1 = on, 0 = off (default, env MMT_RELU_BITS). Latched by
// mmt_create (the bit rows are part of that context's workspace); returns the previous value (tests, A/B)
int mmt_set_relu_bits(int on);
// the FFN backward's dropout-masked bf16 residual-gradient copy and FFN output-bias gradient: 1 (default,
// env MMT_DROP_COPY_FUSE) = in the epilogue of the last cross-attention K/V data-gradient GEMM that
// accumulates into that residual gradient, 0 = a separate pass; returns the previous value (tests, A/B)
int mmt_set_drop_copy_fuse(int on);
// hs 32 self-attention backward: 1 (default, env MMT_ATTN_QKV2) = the Q/K/V stage-2 backward (dh1 =
// (dX W2) * tanh', dW2, db1) in the one-pass attention backward's epilogue, dQ / dK / dV never written;
// 0 = the separate stage-2 backward over bf16 dQ / dK / dV. Read at every step; returns the previous value
int mmt_set_attn_qkv2(int on);
// rows per workgroup of the fused out-projection MLP forward at C = 256 (mmt_op_mlp2 and the engine's):
// 128 (8 waves, one workgroup per CU) or 64 (4 waves, three per CU); default 128 (env MMT_MLP2_BM);
// returns the previous value (tests, A/B)
int mmt_mlp2_set_bm(int bm);

/* ---- MX-fp8 primitives (C4's fp8 path; BASELINE configs[4]) --------------------------------
 * MX-fp8 = OCP e4m3fn bytes + one E8M0 exponent byte (bias 127) per 32 consecutive K elements of a
 * row: exponent e = the smallest with amax(block) / 2^e <= 448, value = fp8(x * 2^-e) (RNE). */
int mmt_op_mx_quant(void* stream, int32_t rows, int32_t cols, const float* src, int32_t ld_src, void* dst8,
                    int32_t ld8, void* s8, int32_t lds8);
/* Y = X W^T on MX-fp8 X [M][K] (lda bytes) / W [N][K] (ldb bytes) with exponents sa [M][lds_a],
 * sb [N][lds_b] (K % 32 == 0, lds % 4 == 0); epi as mmt_op_gemm's forward epilogues; o8 / s8
 * (nullable): an MX-fp8 copy of a bf16 output (N % 32 == 0) */
int mmt_op_gemm_f8(void* stream, int32_t epi, int32_t M, int32_t N, int32_t K, const void* A8, int32_t lda,
                   const void* sa, int32_t lds_a, const void* B8, int32_t ldb, const void* sb, int32_t lds_b,
                   const float* bias, const float* resid, int32_t ldres, float* o32, int32_t ldc, void* o16,
                   int32_t ldo16, void* o8, int32_t ld8, void* s8, int32_t lds8);
/* LayerNorm forward that also writes an MX-fp8 copy of its output (C % 32 == 0) */
int mmt_op_layernorm_fwd_f8(void* stream, int32_t R, int32_t C, const float* x, const float* gamma, const float* beta,
                            void* y16, float* mean, float* rstd, void* y8, int32_t ld8, void* s8, int32_t lds8);

#ifdef __cplusplus
}
#endif
#endif /* MMT_H_ */
