// Host-visible launcher declarations for the gfx950 kernels (internal to libmmt_hip.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef MMT_MAX_GROUP
#define MMT_MAX_GROUP 8
#endif
typedef uint16_t bf16_t;

// ------------------------------------------------------------------------------------------
// GEMM: C[M,N] (epi)= alpha * sum_k A(m,k) B(k,n), bf16 operands, fp32 MFMA accumulation.
//   A(m,k) = a_kc ? A[m*lda + k] : A[k*lda + m]
//   B(k,n) = b_kc ? B[n*ldb + k] : B[k*ldb + n]
// Forward linear   Y = X W^T : a_kc=1, b_kc=1
// Backward data   dX = dY W  : a_kc=1, b_kc=0
// Weight grad     dW = dY^T X: a_kc=0, b_kc=0 (split-K, atomic fp32 accumulate)
// ------------------------------------------------------------------------------------------
enum MmtEpi {
  EPI_STORE_BF16 = 0,   // o16 = alpha*acc (+bias)
  EPI_BIAS_TANH_BF16,   // o16 = tanh(alpha*acc + bias)
  EPI_BIAS_RELU_BF16,   // o16 = relu(alpha*acc + bias)
  EPI_BIAS_RESID_F32,   // o32 = resid + drop(alpha*acc + bias) ; o16 (optional) = bf16 copy
  EPI_STORE_F32,        // o32 = alpha*acc (+bias)
  EPI_DTANH_BF16,       // o16 = alpha*acc * (1 - aux^2)
  EPI_DRELU_BF16,       // o16 = aux > 0 ? alpha*acc : 0
  EPI_ACC_F32,          // o32 += alpha*acc
  EPI_ATOMIC_F32,       // atomicAdd(o32, alpha*acc)
  // LayerNorm backward of the rows this GEMM's dy = alpha*acc belongs to (the block's tile must
  // span every column: N == 256 on the 256x256 tile, N == 512 on 128x512; mmt_launch_gemm_ln_bwd):
  //   xhat = (resid - ln_mean) * ln_rstd ; o32 += ln_rstd * (g dy - mean(g dy) - xhat mean(g dy xhat))
  //   o16 (optional) = bf16 of the dropout-masked o32 (mask as EPI_BIAS_RESID_F32), dbias += its column
  //   sums; ln_dgamma += column sums of dy * xhat, ln_dbeta += column sums of dy  (ln_bwd_kernel fused)
  EPI_LN_BWD_F32,
  EPI_COUNT
};

struct GemmProblem {
  const bf16_t* A;
  const bf16_t* B;
  const float* bias;
  const bf16_t* aux;
  const float* resid;
  float* o32;
  bf16_t* o16;
  const float* alpha_ptr;  // optional device scalar multiplier
  float alpha;
  int M, N, K;
  int lda, ldb, ldc, ldaux, ldres, ldo16;
  // dropout of the branch output (EPI_BIAS_RESID_F32 only; drop_thr == 0: off):
  // element (m, n) kept iff mmt_keep(mmt_hash(drop_key, m, n >> 1), n, drop_thr) (16-bit threshold,
  // mmt_common.h), kept values scaled by drop_scale
  uint32_t drop_key, drop_thr;
  float drop_scale;
  // fused bias gradient (bf16-output epilogues, SWAP layouts): dbias[n] += sum_m out[m, n]
  float* dbias;
  // split-K slabs: split s writes o32 + s * split_stride (elements); 0 = one output
  int64_t split_stride;
  // MX-fp8 (mmt_launch_gemm_f8): A and B hold e4m3fn bytes (lda / ldb in bytes = elements) and
  // these their E8M0 block exponents, one byte per 32 K elements (row stride in bytes, % 4 == 0)
  const uint8_t* sa;
  const uint8_t* sb;
  int lds_a, lds_b;
  // optional MX-fp8 copy of a bf16-output epilogue (the next fp8 GEMM's A operand): e4m3fn bytes
  // [M][ld8] and block exponents [M][lds8] over 32 consecutive output columns
  uint8_t* o8;
  uint8_t* s8;
  int ld8, lds8;
  // EPI_LN_BWD_F32: the LayerNorm's weight, saved row statistics and parameter gradients (the LN
  // input rows are resid / ldres, the accumulated input gradient o32 / ldc)
  const float* ln_gamma;
  const float* ln_mean;
  const float* ln_rstd;
  float* ln_dgamma;
  float* ln_dbeta;
  // EPI_BIAS_RESID_F32 + the NEXT LayerNorm's forward on the stored rows (whole rows per block:
  // mmt_launch_gemm_resid_ln): lnf_y = bf16((o32 - mean) * rstd * lnf_gamma + lnf_beta) [M][N], and
  // the row statistics lnf_mean / lnf_rstd (as ln_fwd_kernel, eps 1e-5); null lnf_y: off
  const float* lnf_gamma;
  const float* lnf_beta;
  bf16_t* lnf_y;
  float* lnf_mean;
  float* lnf_rstd;
  // EPI_BIAS_TANH_BF16 (forward, a_kc = b_kc = 1) + the per-head Q/K/V stage 2 fused into the
  // epilogue (model.py:39, 44, 49): o16 = h1 = tanh(alpha acc + bias) as usual, and for each
  // qkv2_hh-wide column block blk of h1 (qkv2_hh = 16 or 32)
  //   qkv2_out[m, blk*2hh + o] = bf16(sum_i qkv2_w2[blk][o][i] * bf16(h1[m, blk*hh + i]))
  // (qkv2_w2 fp32 [nblk][2hh][hh], qkv2_ld % 8 == 0, 16-B aligned out); null qkv2_out: off
  const float* qkv2_w2;
  bf16_t* qkv2_out;
  int qkv2_ld, qkv2_hh;
  // ReLU masks as bits (round 5): EPI_BIAS_RELU_BF16 also writes mask8[m * ldm8 + n / 8] bit n % 8 =
  // (stored bf16 output > 0); EPI_DRELU_BF16 with mask8 set (aux null) reads those bits instead of
  // the bf16 aux rows (16x fewer bytes). SWAP epilogues only; null: off
  uint8_t* mask8;
  int ldm8;
};

struct GemmBatch {
  GemmProblem p[MMT_MAX_GROUP];
  int count;
  int xcd_plane;  // split-K launches: 1 = XCD-major remap of the whole (tile, split) plane
  int tile_hint;  // launch policy only: 1 = a big launch with K < 1024 takes the 128 x 256 two-per-CU tile,
                  // 2 = a weight gradient takes the 128 x 128 tile
  int dw_blocks;  // weight gradients: blocks per launch the split-K factor aims at (0: MMT_WGRAD_BLOCKS / 128)
  // diagnostic builds only (-DMMT_GEMM_STAMPS, tools/gemm_stamps.py): per-block s_memtime stamps
  unsigned long long* stamps;
};

hipError_t mmt_launch_gemm(const GemmBatch& b, bool a_kc, bool b_kc, int epi, int splits, hipStream_t s);
// backward-data GEMM dy = alpha * A B (A K-contiguous, B MN-contiguous) with the LayerNorm backward of
// its rows fused (EPI_LN_BWD_F32) on a tile spanning the row: every problem needs N == 256 (256x256
// tile) or N == 512 (128x512; all problems alike) and 16-B aligned rows. Returns hipErrorInvalidValue otherwise (the caller runs the two passes)
bool mmt_gemm_ln_bwd_ok(const GemmBatch& b);
// forward residual GEMM (EPI_BIAS_RESID_F32) with the next LayerNorm's forward fused on the problems
// whose lnf_y is set; every problem needs N == 256 (256x256 tile) or N == 512 (128x512; all alike),
// any K. hipErrorInvalidValue
// otherwise (the caller launches the LayerNorm itself)
bool mmt_gemm_resid_ln_ok(const GemmBatch& b);
hipError_t mmt_launch_gemm_resid_ln(const GemmBatch& b, hipStream_t s);
hipError_t mmt_launch_gemm_ln_bwd(const GemmBatch& b, hipStream_t s);
// weight gradients o32 += alpha * A^T B over K rows (both operands MN-contiguous): split-K into fp32
// slabs in `slab` (capacity slab_bytes) + one reduce pass; without room, one K pass accumulating
hipError_t mmt_launch_gemm_wgrad(const GemmBatch& b, float* slab, int64_t slab_bytes, hipStream_t s);

// Fused two-GEMM MLP (round 5; SURVEY K6 / K11: the attention out-projection Linear(C, C/2) -> tanh ->
// Linear(C/2, C) of model.py:82-92, 102-117): per problem
//   h   = tanh(A W0^T + b0)            (g1: A [M][K1] bf16, B = W0 [N1][K1] packed, bias b0, o16 = h out)
//   out = epilogue(h W2^T + b2)        (g2: B = W2 [N2][N1] packed, bias b2, EPI_BIAS_RESID_F32 fields:
//                                        resid, o32, optional o16 / dropout / next-LayerNorm lnf_*)
// with h resident in LDS between the two products (it is still stored to g1.o16 for the backward).
// N1 = 128 or 256, N2 = 2 N1, K1 = N2 (C = 256 or 512); hipErrorInvalidValue otherwise (the caller
// runs the two GEMMs).
// (at most MMT_MLP2_GROUP problems per launch: two GemmProblem arrays of 8 would pass the 4 KiB
// kernel-argument limit; the engine launches groups of up to 8 modalities in chunks)
#define MMT_MLP2_GROUP 4
struct Mlp2Batch {
  GemmProblem g1[MMT_MLP2_GROUP];
  GemmProblem g2[MMT_MLP2_GROUP];
  int count;
};
bool mmt_mlp2_ok(const Mlp2Batch& b);
hipError_t mmt_launch_mlp2(const Mlp2Batch& b, hipStream_t s);
// its backward-data pair in one launch: dh = alpha (dY W2) * (1 - h^2) (g1: A = dY [M][C], B = W2 [C][C/2]
// MN-contiguous, aux = h, o16 = dh, dbias += column sums of dh (nullable)), dx = dh W0 (g2: B = W0
// [C/2][C] MN-contiguous, o16 = dx); dh stays in LDS between the products and is stored for the W0
// weight gradient
bool mmt_mlp2_bwd_ok(const Mlp2Batch& b);
hipError_t mmt_launch_mlp2_bwd(const Mlp2Batch& b, hipStream_t s);
// forward linear Y = X W^T on MX-fp8 operands (A = X [M][K], B = W [N][K], both K-contiguous e4m3fn
// with E8M0 exponents per 32 K elements; K % 32 == 0) via v_mfma_scale_f32_32x32x64_f8f6f4, any
// of the bf16 GEMM's forward epilogues; fp32 accumulation
hipError_t mmt_launch_gemm_f8(const GemmBatch& b, int epi, hipStream_t s);
// whether a batch runs on the 256x256 tile (weight-gradient launches can only be merged when equal;
// the fused Q/K/V stage 2 needs the 128x128 tile)
bool mmt_gemm_wgrad_big(const GemmBatch& b);

// ------------------------------------------------------------------------------------------
// LayerNorm (eps = 1e-5, weight+bias). Row-major [R, C] fp32 in, bf16 out; saves mean/rstd.
// ------------------------------------------------------------------------------------------
struct LnProblem {
  const float* x;       // [R, C]
  const float* gamma;
  const float* beta;
  bf16_t* y;            // [R, C] (ld = C)
  float* mean;          // [R]
  float* rstd;          // [R]
  // optional MX-fp8 copy of y (an fp8 GEMM's A operand): e4m3fn [R][ld8], E8M0 [R][lds8] per 32
  // columns (C % 32 == 0)
  uint8_t* y8;
  uint8_t* s8;
  int ld8, lds8;
  // backward
  const float* dy;      // [R, C] fp32
  float* dx;            // [R, C] fp32, ACCUMULATED (dx += ...)
  bf16_t* dx16;         // optional bf16 copy of the accumulated dx
  float* dgamma;        // atomic accumulate
  float* dbeta;
  // dropout mask applied to the dx16 copy only (the gradient of the dropped branch that consumes
  // it): dx16[r, c] = keep(r, c) ? dx * drop_scale : 0 ; drop_thr == 0: plain copy
  uint32_t drop_key, drop_thr;
  float drop_scale;
  float* dsum;          // optional: dsum[c] += sum_r (masked) dx16 value (the consumer's bias gradient)
};
struct LnBatch {
  LnProblem p[MMT_MAX_GROUP];
  int count;
  // forward: optional words zeroed by the launch (the loss accumulators and this forward's
  // non-finite flag the cross-entropy kernel adds into next), instead of two memset launches
  float* zero_f; int nzero_f;
  int* zero_i; int nzero_i;
};
hipError_t mmt_launch_ln_fwd(const LnBatch& b, int R, int C, hipStream_t s);
hipError_t mmt_launch_ln_bwd(const LnBatch& b, int R, int C, hipStream_t s);

// ------------------------------------------------------------------------------------------
// Causal attention, one wave per 32-row tile, 32x32x16 bf16 MFMA, fp32 online softmax.
// Q rows (b*T+t) at q + row*q_ld + head*hs ; stream j K/V at k[j]/v[j] + row*kv_ld + head*kv_hstride.
// Output O (sum over streams of the per-stream normalised outputs) at o + row*o_ld + head*hs.
// ------------------------------------------------------------------------------------------
#define MMT_MAX_STREAMS 8
struct AttnProblem {
  const bf16_t* q; int q_ld;
  const bf16_t* k[MMT_MAX_STREAMS];
  const bf16_t* v[MMT_MAX_STREAMS];
  int kv_ld, kv_hstride;
  bf16_t* o; int o_ld;
  bf16_t* oj[MMT_MAX_STREAMS];   // per-stream normalised outputs (nullable when nstreams == 1)
  float* lse[MMT_MAX_STREAMS];   // [B*H*T] per stream, log2 domain: log2 sum_s 2^(log2e * scale * q.k_s)
  // backward
  const bf16_t* dout; int dout_ld;
  float* dvec[MMT_MAX_STREAMS];  // rowsum(dO * O_j) per stream [B*H*T]
  bf16_t* dq; int dq_ld;
  // optional fp32 scratch rows [B*T][>= H*hs] (dq32_ld % 4 == 0, 16-B aligned): the one-pass hs-32
  // backward sums dQ over several KV streams there (required for it when nstreams > 1)
  float* dq32; int dq32_ld;
  // optional (one KV stream, hs 32, the one-pass backward; set only when mmt_attn_bwd_fuses_qkv2 says so):
  // the per-head Q/K/V stage-2 backward (Qkv2Problem, model.py:36-50) fused into the attention backward's
  // epilogue, so dQ / dK / dV never leave the kernel: for kind k in {K, Q, V} (column blocks 0, C, 2C of
  // the interleaved layout) and blk = k * H + head, dh1[r][blk*16 + i] = (sum_o W2[blk][o][i] dX[r][o]) *
  // (1 - h1[r][blk*16 + i]^2), dW2[blk] += dX^T h1, db1[blk*16 + i] += sum_r dh1 (atomic). dq / dk / dv
  // are then not written.
  const bf16_t* q2_h1; bf16_t* q2_dh1; int q2_ld;
  const float* q2_w2; float* q2_dw2; float* q2_db1;
  bf16_t* dk[MMT_MAX_STREAMS];
  bf16_t* dv[MMT_MAX_STREAMS];
  int dkv_ld, dkv_hstride;
  int nstreams;
  // dropout on the normalised probabilities (drop_thr == 0: off): element (query t, key s) of
  // stream j, head slot bh = b*H + h, kept iff mmt_hash(mmt_hash(drop_key, j, MMT_STREAM_SALT),
  // bh*T + t, s >> 1) passes mmt_keep(., s, drop_thr); kept probabilities scaled by drop_scale
  uint32_t drop_key, drop_thr;
  float drop_scale;
  // keep bits of that mask (required when drop_thr != 0), made by mmt_launch_attn_mask and read by
  // the forward and both backward kernels. Per stream, per (bh, query tile qt, key tile kt <= qt)
  // tile index t = bh * ntri + qt*(qt+1)/2 + kt (ntri = nt*(nt+1)/2), two 128-B records of the
  // S^T tile's accumulator elements e (query qt*32 + r, key kt*32 + (e&3) + 8(e>>2) + 4u, lane
  // r + 32u): key-major words at dmask[j] + 32 t (dword 2e + u, bit r: the dK/dV pass, keys on
  // lanes) and lane words at dmask[j] + 32 (ntiles + t) (16 bits per lane, bit e: forward and dQ)
  uint32_t* dmask[MMT_MAX_STREAMS];
};
// tiles of one stream's mask, and its dwords (both records; see AttnProblem::dmask)
inline int64_t mmt_attn_mask_tiles(int B, int H, int T) {
  const int64_t nt = (T + 31) / 32;
  return (int64_t)B * H * (nt * (nt + 1) / 2);
}
inline int64_t mmt_attn_mask_dwords(int B, int H, int T) { return 2 * 32 * mmt_attn_mask_tiles(B, H, T); }
struct AttnBatch { AttnProblem p[MMT_MAX_GROUP]; int count; };
hipError_t mmt_launch_attn_fwd(const AttnBatch& b, int B, int T, int H, int hs, float scale, hipStream_t s);
hipError_t mmt_launch_attn_bwd(const AttnBatch& b, int B, int T, int H, int hs, float scale, hipStream_t s);
// true when mmt_launch_attn_bwd runs this batch on the one-pass hs-32 kernel with one KV stream, which
// can take the Q/K/V stage-2 backward in its epilogue (AttnProblem::q2_*)
bool mmt_attn_bwd_fuses_qkv2(const AttnBatch& b, int T, int hs);
// hs 64 dK/dV pass streaming the query slices through an LDS-DMA ring (mmt_attn2.hip)
// variant (the mmt_attn_set_ring bits): 4 = 3 waves per SIMD (default), else 2
hipError_t mmt_attn_bwd_dkdv_ring64(const AttnBatch& b, int B, int T, int H, float scale, bool drop, int variant,
                                    hipStream_t s);
// hs 64 dQ pass (and D_j) streaming the key slices through an LDS-DMA ring (mmt_attn2.hip)
hipError_t mmt_attn_bwd_dq_ring64(const AttnBatch& b, int B, int T, int H, float scale, bool drop, hipStream_t s);
hipError_t mmt_attn_fwd_ring64(const AttnBatch& b, int B, int T, int H, float scale, bool drop, hipStream_t s);
// hs 64, T <= 512, one KV stream: dQ, dK, dV in one pass, one workgroup per (batch, head) (mmt_attn2.hip)
hipError_t mmt_attn_bwd_fused64(const AttnBatch& b, int B, int T, int H, float scale, bool drop, hipStream_t s);
// fill dmask[j] (j < nstreams) of every problem with drop_thr != 0 from its counter hash
hipError_t mmt_launch_attn_mask(const AttnBatch& b, int B, int T, int H, hipStream_t s);

// KV-cache decode attention (generate): the query of position t of sequence b (compact row b)
// against cached keys / values of positions 0..t (rows b*T + s), per-stream softmax, outputs summed
struct DecodeAttnProblem {
  const bf16_t* q; int q_ld;                 // [B, *] compact
  const bf16_t* k[MMT_MAX_STREAMS];
  const bf16_t* v[MMT_MAX_STREAMS];          // cache [B*T, kv_ld]
  int kv_ld, kv_hstride;
  bf16_t* o; int o_ld;                       // [B, *] compact
  int nstreams;
};
struct DecodeAttnBatch { DecodeAttnProblem p[MMT_MAX_GROUP]; int count; };
hipError_t mmt_launch_attn_decode(const DecodeAttnBatch& b, int B, int t, int T, int H, int hs, float scale,
                                  hipStream_t s);

// ------------------------------------------------------------------------------------------
// Per-head Q/K/V stage 2: block-diagonal [hs/2 -> hs] maps (model.py:39,44,49), nblk = 3*H.
//   out[r, blk*hs + o] = sum_i W2[blk][o][i] * h1[r, blk*hs/2 + i]
// ------------------------------------------------------------------------------------------
struct Qkv2Problem {
  const bf16_t* h1;    // [R, nblk*hs/2] (ld = ld_h1)
  const float* w2;     // [nblk][hs][hs/2] fp32 master weights
  bf16_t* out;         // [R, nblk*hs] (ld = ld_out)
  // backward
  const bf16_t* dout;  // [R, nblk*hs]
  bf16_t* dh1;         // [R, nblk*hs/2] = (W2^T dout) * (1 - h1^2)
  float* dw2;          // atomic accumulate [nblk][hs][hs/2]
  float* db1;          // optional: atomic accumulate of the column sums of dh1 [nblk*hs/2] (the stage-1
                       // bias gradient, model.py:36-50), fused so no separate column-sum pass reads dh1
};
struct Qkv2Batch { Qkv2Problem p[MMT_MAX_GROUP]; int count; };
hipError_t mmt_launch_qkv2_fwd(const Qkv2Batch& b, int R, int nblk, int hs, int ld_h1, int ld_out, hipStream_t s);
hipError_t mmt_launch_qkv2_bwd(const Qkv2Batch& b, int R, int nblk, int hs, int ld_h1, int ld_out, hipStream_t s);

// ------------------------------------------------------------------------------------------
// Misc elementwise / reduction kernels
// ------------------------------------------------------------------------------------------
struct EmbProblem {
  const int64_t* idx;   // [B*T]
  const float* tok;     // [V, C]
  const float* pos;     // [T, C]
  float* x;             // [B*T, C]
  const float* dx;      // backward: [B*T, C]
  float* dtok;          // accumulated (+=)
  float* dpos;          // atomic
  // optional scratch of >= B*T*C floats: the token-table blocks store their LDS-privatised slabs
  // there as per-chunk partial tables and one reduce pass adds them into dtok (short row chunks,
  // no global atomics); nullptr: atomic flush
  float* part;
  // optional int [B*T]: the rows in token order (stable), written by mmt_launch_emb_sort; when every
  // problem has it, mmt_launch_embed_bwd takes the sorted path without sorting again
  int* perm;
  int V;
};
struct EmbBatch { EmbProblem p[MMT_MAX_GROUP]; int count; };
bool mmt_emb_sort_ok(const EmbBatch& b, int R, int C);
hipError_t mmt_launch_emb_sort(const EmbBatch& b, int R, hipStream_t s);
hipError_t mmt_launch_embed_fwd(const EmbBatch& b, int B, int T, int C, hipStream_t s);
hipError_t mmt_launch_embed_bwd(const EmbBatch& b, int B, int T, int C, hipStream_t s);

struct CeProblem {
  const float* logits;   // [R, V]
  const int64_t* tgt;    // [R]
  bf16_t* dlogits;       // [R, ld_d] = softmax - onehot (pad columns zeroed)
  float* loss;           // scalar, accumulate (+=) of the mean
  // nullable float [512]: each block stores its share there and one wave adds them to loss in block
  // order (run-to-run identical losses); null: one atomic per block (arrival order)
  float* part;
  int* flag;             // nullable: flag[0], flag[1] |= bit when this problem's loss is NaN / Inf (no trap)
  int V, ld_d, bit;
};
struct CeBatch { CeProblem p[MMT_MAX_GROUP]; int count; };
hipError_t mmt_launch_ce_fwd(const CeBatch& b, int R, hipStream_t s);

struct ColsumProblem {
  const bf16_t* x;       // [R, ld]
  float* out;            // [N] atomic accumulate alpha * sum_r x[r, n]
  const float* alpha_ptr;
  float alpha;
  int N, ld;
};
struct ColsumBatch { ColsumProblem p[MMT_MAX_GROUP]; int count; };
hipError_t mmt_launch_colsum(const ColsumBatch& b, int R, hipStream_t s);

// fp32 -> bf16 copy of a list of matrices (rows x cols, src ld = cols, dst ld = dld, pad zeroed).
// task_dev holds (segment, first row) pairs; each task (one block) packs 32 rows.
struct PackSeg { int64_t src_off; int64_t dst_off; int rows; int cols; int dld; int pad_; };
hipError_t mmt_launch_pack(const PackSeg* segs_dev, int nseg, int64_t ntasks, const int* task_dev, const float* src,
                           bf16_t* dst, hipStream_t s);
hipError_t mmt_launch_f32_to_bf16(const float* src, bf16_t* dst, int64_t n, hipStream_t s);

// MX-fp8 quantisation of fp32 matrices [rows][cols] (row stride ld_src, cols % 32 == 0): e4m3fn
// bytes [rows][ld8] and E8M0 exponents [rows][lds8] per 32 columns; exponent bytes past cols/32 up
// to lds8 are written as 127 (2^0) so a K-step that straddles the end reads finite scales
struct MxSeg {
  int64_t src;   // fp32 element offset of the matrix in `base`
  int64_t dst;   // byte offset of the e4m3fn matrix
  int64_t sdst;  // byte offset of the exponent matrix
  int rows, cols, ld_src, ld8, lds8;
};
hipError_t mmt_launch_mx_quant(const MxSeg* segs_dev, int nseg, int max_units, const float* base, uint8_t* dst,
                               hipStream_t s);
hipError_t mmt_launch_mx_quant1(const MxSeg& S, const float* base, uint8_t* dst, hipStream_t s);
// dst = bf16(mask * src) over row-major [R, C] (mask as in LnProblem), dsum[c] += column sums
struct DropCopyProblem {
  const float* src;
  bf16_t* dst;
  float* dsum;  // nullable
  uint32_t drop_key, drop_thr;
  float drop_scale;
};
struct DropCopyBatch { DropCopyProblem p[MMT_MAX_GROUP]; int count; };
hipError_t mmt_launch_drop_copy(const DropCopyBatch& b, int R, int C, hipStream_t s);

hipError_t mmt_launch_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                            float eps, float wd, float bc1, float bc2_sqrt, hipStream_t s);

hipError_t mmt_launch_eval_direction(const float* logits, const int64_t* xb, const int64_t* yb, const double* vocab,
                                     int B, int T, int V, int is_pct, int* wins_losses, double* certainty,
                                     hipStream_t s);
