// Device helpers shared by the GEMM kernels (mmt_gemm.hip: 128 x 128 / 256 x 256 / 128 x 512 rings and the
// MX-fp8 kernel; mmt_gemm8.hip: the 256 x 256 ping-pong kernel): tile geometry, buffer descriptors, LDS-DMA
// issue, counted waits and the fused SWAP epilogue.
#pragma once
#include "mmt_common.h"
#include "mmt_kernels.h"

#include <stdint.h>

// Block tile configurations: WM x WN waves, each wave TM x TN MFMA 32x32 sub-tiles.
template <int WM_, int WN_, int TM_, int TN_>
struct TileCfg {
  static constexpr int WM = WM_, WN = WN_, TM = TM_, TN = TN_;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
};
// 128 x 128, 4 waves of 64 x 64: short-K shapes (2 blocks per CU overlap one block's prologue
// and epilogue with the other's main loop)
using TileS = TileCfg<2, 2, 2, 2>;
// 256 x 256, 8 waves (2 x 4) of 128 x 64: 32 MFMAs per wave per 64-deep K-step, so the one
// stage in flight has ~2 k cycles of matrix work per SIMD to land behind (long-K shapes, weight
// gradients); 128 KiB ring -> 1 block per CU
using TileL = TileCfg<2, 4, 4, 2>;
// 128 x 512, 8 waves (1 x 8) of 128 x 64 (TileL's per-wave shape): whole 512-wide rows per block for
// the fused LayerNorm-backward epilogue at C = 512 (BK 32 x 2 stages = 80 KiB of ring)
using TileW = TileCfg<1, 8, 4, 2>;

typedef __attribute__((address_space(3))) void lds_void;

// swizzle of the 16-B chunk index of a K-contiguous image row (BK/8 chunks per row):
//   BK 64 (128-B rows): chunk ^ ((row>>1)&7) ; BK 32 (64-B rows): chunk ^ ((row>>2)&3)
template <int BK>
__device__ __forceinline__ int kc_swz(int chunk, int row) {
  return BK == 64 ? (chunk ^ ((row >> 1) & 7)) : (chunk ^ ((row >> 2) & 3));
}

// Buffer resource (V#) as four SGPR words: base, range in bytes, raw dword access.
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 make_rsrc(const void* base, int64_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int32_t)((a >> 32) & 0xffffu));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((int32_t)min(bytes, (int64_t)0x7ffffff0));
  r[3] = 0x00020000;
  return r;
}

// One 16-B-per-lane LDS-DMA: LDS[lds_addr + 16*lane .. +16) = buffer[voff .. +16) (0 if out of
// range). Issued as inline asm on purpose: the compiler's waitcnt pass cannot tell the ring stage
// a DMA targets from the stage the fragment reads use and would drain vmcnt(0) before every
// fragment read (no pipelining at all); the kernel counts its own DMAs (wait_vm) instead.
__device__ __forceinline__ void dma16(const i32x4& rsrc, uint32_t lds_addr, int voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(lds_addr), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

// Buffer offsets are 32-bit, so a descriptor never spans a whole operand (an activation passes 2 GiB
// at, e.g., the C4 FFN hidden with B >= 64 per GPU): the K-contiguous operand's descriptor starts at
// the tile's first row (op_rsrc<true>, once per tile), the MN-contiguous operand's at the K-step's
// first row (op_rsrc<false>, per K-step); the launcher refuses leading dimensions whose tile-local
// span could still reach 2^31 bytes (mmt_launch_gemm).
template <bool KC>
__device__ __forceinline__ i32x4 op_rsrc(const void* base, int ld, int rows_total, int K, int r0, int k0, int esz = 2) {
  const char* b = reinterpret_cast<const char*>(base);
  return KC ? make_rsrc(b + (int64_t)r0 * ld * esz, (int64_t)(rows_total - r0) * ld * esz)
            : make_rsrc(b + (int64_t)k0 * ld * esz, (int64_t)(K - k0) * ld * esz);
}

// issue this wave's LDS-DMA pieces (1 KiB each) of one operand tile for K-step k0.
// the tile (ROWS x BK bf16) has ROWS*BK/512 pieces, split over NW waves; lane L writes LDS bytes
// [i*1024 + 16L, +16). rsrc: op_rsrc<KC>(.., r0, k0) (offsets are relative to the tile's row r0 for
// a K-contiguous operand, to the K-step's row k0 for an MN-contiguous one)
template <int BK, bool KC, int ROWS, int NW>
__device__ __forceinline__ void issue_tile(const i32x4& rsrc, char* img, int ld, int rows_total, int K,
                                           int r0, int k0, int wave, int lane) {
  constexpr int PPW = ROWS * BK / 512 / NW;  // pieces per wave
  constexpr int CPR = BK / 8;                // chunks per K-contiguous row
  constexpr int CPK = ROWS / 8;              // chunks per k-row of an MN-contiguous image
  static_assert(PPW >= 1 && (KC || CPK >= 16), "tile geometry");
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    const int i = wave * PPW + u;
    int voff;
    if (KC) {
      const int row = (64 / CPR) * i + lane / CPR;
      const int chunk = kc_swz<BK>(lane % CPR, row);
      const int grow = r0 + row, gk = k0 + chunk * 8;
      voff = (grow < rows_total && gk < K) ? (row * ld + gk) * 2 : 0x7fffffff;
    } else {
      const int kr = (64 / CPK) * i + lane / CPK;
      const int chunk = (lane % CPK) ^ ((kr & 3) << 2);
      const int gk = k0 + kr, gcol = r0 + chunk * 8;
      voff = (gk < K && gcol < rows_total) ? (kr * ld + gcol) * 2 : 0x7fffffff;
    }
    dma16(rsrc, __builtin_amdgcn_readfirstlane(lds_u32(img + i * 1024)), voff);
  }
}

// fragment for "lane row = sb + (lane&31), k = 16*s + 8*(lane>>5) + j" from a staged image
template <int BK, bool KC, int ROWS>
__device__ __forceinline__ bf16x8 frag(const char* img, int sb, int s, int lane) {
  if (KC) {
    const int row = sb + (lane & 31);
    const int ch = kc_swz<BK>(2 * s + (lane >> 5), row);
    return *reinterpret_cast<const bf16x8*>(img + row * (BK * 2) + ch * 16);
  } else {
    const int g = lane >> 4, i = lane & 15;
    const int q = i >> 2, p = i & 3;
    const int col = sb + 16 * (g & 1) + 4 * p;
    const int kr = 16 * s + 8 * (g >> 1) + q;  // kr & 3 == q ; (kr + 4) & 3 == q
    const int ch = (col >> 3) ^ (q << 2);
    const int within = (col & 7) * 2;
    const s16x4 lo = lds_tr16(img + kr * (ROWS * 2) + ch * 16 + within);
    const s16x4 hi = lds_tr16(img + (kr + 4) * (ROWS * 2) + ch * 16 + within);
    return join4(lo, hi);
  }
}

// one output element; returns the value stored (the bias-gradient column sum adds it up)
// PRE: the activation (alpha, bias, tanh) was already applied to the accumulators (qkv2_fused)
template <int EPI, bool PRE = false>
__device__ __forceinline__ float epi_scalar(const GemmProblem& P, float* o32, float alpha, int m, int n, float v) {
  float r = PRE ? v : alpha * v;
  if (!PRE && (EPI == EPI_BIAS_TANH_BF16 || EPI == EPI_BIAS_RELU_BF16 || EPI == EPI_BIAS_RESID_F32 ||
               EPI == EPI_STORE_F32 || EPI == EPI_STORE_BF16)) {
    if (P.bias) r += P.bias[n];
  }
  if (!PRE && EPI == EPI_BIAS_TANH_BF16) r = fast_tanh(r);
  if (EPI == EPI_BIAS_RELU_BF16) r = fmaxf(r, 0.0f);
  if (EPI == EPI_DTANH_BF16) { const float t = bf2f(P.aux[(int64_t)m * P.ldaux + n]); r *= (1.0f - t * t); }
  if (EPI == EPI_DRELU_BF16) {
    const bool keep = P.mask8 ? ((P.mask8[(int64_t)m * P.ldm8 + (n >> 3)] >> (n & 7)) & 1) != 0
                              : bf2f(P.aux[(int64_t)m * P.ldaux + n]) > 0.0f;
    r = keep ? r : 0.0f;
  }
  if (EPI == EPI_BIAS_RESID_F32) {
    if (P.drop_thr)
      r = mmt_keep(mmt_hash(P.drop_key, (uint32_t)m, (uint32_t)n >> 1), (uint32_t)n, P.drop_thr) ? r * P.drop_scale : 0.0f;
    r += P.resid[(int64_t)m * P.ldres + n];
  }
  const int64_t o = (int64_t)m * P.ldc + n;
  if (EPI == EPI_ACC_F32) {
    // + optional dropout-masked bf16 copy of the accumulated value (o16: the engine's last writer of a
    // residual-gradient row block), whose column sums the caller adds to dbias
    const float acc = o32[o] + r;
    o32[o] = acc;
    if (!P.o16) return r;
    float c = acc;
    if (P.drop_thr)
      c = mmt_keep(mmt_hash(P.drop_key, (uint32_t)m, (uint32_t)n >> 1), (uint32_t)n, P.drop_thr) ? c * P.drop_scale : 0.0f;
    P.o16[(int64_t)m * P.ldo16 + n] = f2bf(c);
    return c;
  }
  if (EPI == EPI_ATOMIC_F32) { atomicAdd(o32 + o, r); return r; }
  if (EPI == EPI_BIAS_RESID_F32 || EPI == EPI_STORE_F32) {
    o32[o] = r;
    if (EPI == EPI_BIAS_RESID_F32 && P.o16) P.o16[(int64_t)m * P.ldo16 + n] = f2bf(r);
    return r;
  }
  P.o16[(int64_t)m * P.ldo16 + n] = f2bf(r);
  return r;
}

// bf16 outputs feed later GEMMs as K-contiguous operands: their pad columns [N, ldo16) are kept
// zero so a K-step that straddles N reads zeros there.
template <int EPI>
__device__ __forceinline__ void epi_pad(const GemmProblem& P, int m, int n) {
  constexpr bool bf16_out = EPI == EPI_STORE_BF16 || EPI == EPI_BIAS_TANH_BF16 || EPI == EPI_BIAS_RELU_BF16 ||
                            EPI == EPI_DTANH_BF16 || EPI == EPI_DRELU_BF16;
  if (bf16_out || ((EPI == EPI_BIAS_RESID_F32 || EPI == EPI_ACC_F32) && P.o16)) {
    if (n < P.ldo16) P.o16[(int64_t)m * P.ldo16 + n] = 0;
  }
}

__device__ __forceinline__ void wait_vm(int n) {
  // counted wait on this wave's outstanding LDS-DMA pieces (immediate operand: one case each; every
  // count up to 16 exact — the 128 x 512 tile issues 5 pieces per stage — and above it vmcnt(16),
  // which waits for more, never for less)
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
  }
}

// Fused epilogue of a SWAP tile (acc[i][j]: rows = n sub-tile i, cols = m sub-tile j), staged through
// LDS at `ct` in passes of EPI_ROWS rows, then run row-major: a thread owns 8 consecutive columns,
// so every global access is 16 B per lane (bf16 x 8, or 2 x f32x4) and GBN/8 lanes cover one row
// segment. 16-B stores halve the store instructions of the 8-B form (the epilogue of a short-K tile
// is store-issue bound). Starts with a barrier (the caller's LDS reads of `ct` must be done).
// Staging of a pass's accumulator rows into the fp32 tile ct [EPI_ROWS][GBN + 4] (row m - pass rows, col n):
// 32x32x16 layout (gemm_kernel): acc[i][j] = the wave's n sub-tile i x m sub-tile j, lane = m, regs = n
template <class TL, int EPI_ROWS>
__device__ __forceinline__ void stage_acc(f32x16 (&acc)[TL::TN][TL::TM], float* ct, int pass, int lane, int wave) {
  constexpr int CT = TL::BN + 4, TM = TL::TM, TN = TL::TN;
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int h = lane >> 5, r = lane & 31;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int mf = wm * TM * 32 + 32 * j;  // first row of this sub-tile in the block tile
      if (mf / EPI_ROWS != pass) continue;
      const int ml = mf - pass * EPI_ROWS + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = wn * TN * 32 + 32 * i + 8 * g + 4 * h;
        *reinterpret_cast<f32x4*>(ct + ml * CT + nl) =
            f32x4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
      }
    }
}
// 16x16x32 layout (gemm8_kernel, 256 x 256 tile, 8 waves 2 (m) x 4 (n) of 128 x 64): acc[nb][mb] = n block nb
// (16 columns) x m block mb (16 rows) of the wave; lane & 15 = m, regs = n 4 (lane >> 4) + e
template <class TL, int EPI_ROWS>
__device__ __forceinline__ void stage_acc(f32x4 (&acc)[4][8], float* ct, int pass, int lane, int wave) {
  constexpr int CT = TL::BN + 4;
  const int wr = wave >> 2, wc = wave & 3;
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int mf = wr * 128 + 16 * mb;
    if (mf / EPI_ROWS != pass) continue;
    const int ml = mf - pass * EPI_ROWS + (lane & 15);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      *reinterpret_cast<f32x4*>(ct + ml * CT + wc * 64 + 16 * nb + 4 * (lane >> 4)) = acc[nb][mb];
  }
}

template <class TL, int EPI, int EPI_ROWS, bool PRE = false, class ACC>
__device__ __forceinline__ void epilogue_swap(const GemmProblem& P, ACC& acc, char* lds,
                                              float* o32, float alpha, int m0, int n0, int tid, int lane, int wave) {
  constexpr int GBM = TL::BM, GBN = TL::BN, NW = TL::NW, NT = TL::NT, TM = TL::TM, TN = TL::TN;
  const int M = P.M, N = P.N;
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int h = lane >> 5, r = lane & 31;
  // Stage the fp32 tile through LDS (EPI_ROWS rows per pass), then run the epilogue row-major:
  // a thread owns 8 consecutive columns, so every global access is 16 B per lane (bf16 x 8, or
  // 2 x f32x4) and GBN/8 lanes cover one row segment. 16-B stores halve the store instructions
  // of the 8-B form (the epilogue of a short-K tile is store-issue bound).
  // acc[i][j]: rows = n (sub-tile i), cols = m (sub-tile j)
  constexpr int CT = GBN + 4;  // fp32 row stride of the staged tile (16-B aligned, de-conflicted)
  constexpr int TPR = GBN / 8;          // threads per row
  constexpr int RPI = NT / TPR;         // rows per iteration
  constexpr int IT = EPI_ROWS / RPI;    // iterations per pass
  float* ct = reinterpret_cast<float*>(lds);
  const int c8 = tid % TPR;   // 8-column group of this thread
  const int rsub = tid / TPR; // row within an iteration
  const int n = n0 + 8 * c8;
  constexpr bool HAS_AUX = EPI == EPI_DTANH_BF16 || EPI == EPI_DRELU_BF16;
  constexpr bool HAS_RES = EPI == EPI_BIAS_RESID_F32 || EPI == EPI_ACC_F32;
  constexpr bool HAS_BIAS = !PRE && (EPI == EPI_BIAS_TANH_BF16 || EPI == EPI_BIAS_RELU_BF16 ||
                                     EPI == EPI_BIAS_RESID_F32 || EPI == EPI_STORE_F32 || EPI == EPI_STORE_BF16);
  // fused bias gradient (bf16-output epilogues): column sums of the stored values
  constexpr bool CAN_DB = EPI == EPI_STORE_BF16 || EPI == EPI_DTANH_BF16 || EPI == EPI_DRELU_BF16;
  // MX-fp8 copy of a forward activation (P.o8; needs N % 32 == 0 and the vector path)
  constexpr bool MX_OUT = EPI == EPI_BIAS_RELU_BF16 || EPI == EPI_BIAS_TANH_BF16 || EPI == EPI_STORE_BF16;
  // fused LayerNorm backward (whole rows per block: N == GBN, checked by the launcher)
  constexpr bool LNB = EPI == EPI_LN_BWD_F32;
  // (EPI_ACC_F32 with a bf16 copy: the copy's column sums)
  const bool want_db = (CAN_DB || LNB || (EPI == EPI_ACC_F32 && P.o16 != nullptr)) && P.dbias != nullptr;
  float cg[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, cb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x4 gam0 = {0.f, 0.f, 0.f, 0.f}, gam1 = {0.f, 0.f, 0.f, 0.f};
  if (LNB && n + 8 <= N) {
    gam0 = *reinterpret_cast<const f32x4*>(P.ln_gamma + n);
    gam1 = *reinterpret_cast<const f32x4*>(P.ln_gamma + n + 4);
  }
  // the fused next-LayerNorm's weight and bias columns, once (loaded per row they were re-read after
  // every row's stores, which the compiler cannot move them past)
  constexpr bool LNF = EPI == EPI_BIAS_RESID_F32 && (GBN == 256 || GBN == 512);
  f32x4 lg0 = {0.f, 0.f, 0.f, 0.f}, lg1 = lg0, lb0 = lg0, lb1 = lg0;
  if (LNF && P.lnf_y && n + 8 <= N) {
    lg0 = *reinterpret_cast<const f32x4*>(P.lnf_gamma + n);
    lg1 = *reinterpret_cast<const f32x4*>(P.lnf_gamma + n + 4);
    lb0 = *reinterpret_cast<const f32x4*>(P.lnf_beta + n);
    lb1 = *reinterpret_cast<const f32x4*>(P.lnf_beta + n + 4);
  }
  // 16-B vector accesses need bf16 leading dimensions % 8 and fp32 ones % 4 (bias pointers are
  // 64-B aligned by the parameter layout)
  // the kernel-argument fields the row loops read, pinned as wave-uniform values: read through P,
  // hipcc re-loaded them (s_load + lgkmcnt wait) in every row iteration -- up to 40 scalar loads per
  // pass in the LayerNorm-backward and ReLU epilogues. Not for the residual / accumulate epilogues
  // (pinned, the residual + LayerNorm-forward one spilled 40 VGPRs and the accumulate one re-loaded
  // more) nor ReLU' (its bf16-aux form measured 101 -> 117 us standalone at C1 pinned)
  // (EA(f): the pinned copy, or P.f read as before)
  constexpr bool PIN = !(EPI == EPI_BIAS_RESID_F32 || EPI == EPI_ACC_F32 || EPI == EPI_DRELU_BF16);
  struct {
    const float* resid; int ldres, ldc; bf16_t* o16; int ldo16; const bf16_t* aux; int ldaux;
    uint32_t drop_key, drop_thr; float drop_scale; uint8_t* mask8; int ldm8;
    const float* ln_mean; const float* ln_rstd; bf16_t* lnf_y; float* lnf_mean; float* lnf_rstd;
    uint8_t* o8; uint8_t* s8; int ld8, lds8;
  } ea{};
  if constexpr (PIN) {
    ea.resid = sgpr_ptr(P.resid);
    ea.ldres = __builtin_amdgcn_readfirstlane(P.ldres);
    ea.ldc = __builtin_amdgcn_readfirstlane(P.ldc);
    ea.o16 = sgpr_ptr(P.o16);
    ea.ldo16 = __builtin_amdgcn_readfirstlane(P.ldo16);
    ea.aux = sgpr_ptr(P.aux);
    ea.ldaux = __builtin_amdgcn_readfirstlane(P.ldaux);
    ea.drop_key = sgpr_u32(P.drop_key);
    ea.drop_thr = sgpr_u32(P.drop_thr);
    ea.drop_scale = sgpr_f32(P.drop_scale);
    ea.mask8 = sgpr_ptr(P.mask8);
    ea.ldm8 = __builtin_amdgcn_readfirstlane(P.ldm8);
    ea.ln_mean = sgpr_ptr(P.ln_mean);
    ea.ln_rstd = sgpr_ptr(P.ln_rstd);
    ea.lnf_y = sgpr_ptr(P.lnf_y);
    ea.lnf_mean = sgpr_ptr(P.lnf_mean);
    ea.lnf_rstd = sgpr_ptr(P.lnf_rstd);
    ea.o8 = sgpr_ptr(P.o8);
    ea.s8 = sgpr_ptr(P.s8);
    ea.ld8 = __builtin_amdgcn_readfirstlane(P.ld8);
    ea.lds8 = __builtin_amdgcn_readfirstlane(P.lds8);
  }
#define EA(f) (PIN ? ea.f : P.f)
  const bool vec_ok = ((P.ldo16 | P.ldaux) & 7) == 0 && ((P.ldc | P.ldres) & 3) == 0;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x4 bias0 = {0.f, 0.f, 0.f, 0.f}, bias1 = {0.f, 0.f, 0.f, 0.f};
  if (HAS_BIAS && P.bias && n + 8 <= N) {
    bias0 = *reinterpret_cast<const f32x4*>(P.bias + n);
    bias1 = *reinterpret_cast<const f32x4*>(P.bias + n + 4);
  }
  // the aux operand (tanh' / ReLU' input) of pass p + 1 is loaded while pass p runs, the first pass's
  // before the first staging: its HBM latency was exposed once per pass (ffn2 dX at the target: the
  // epilogue alone 110-150 us of a 260 us launch). The pass barriers are raw s_barriers behind an LDS
  // wait: __syncthreads() would also drain those loads (and the previous pass's stores) at every pass.
  u32x4 auxn[IT];  // (EPI_DRELU_BF16 with mask8: word 0 holds the 8 ReLU bits of this thread's columns)
  const bool use_m8 = EPI == EPI_DRELU_BF16 && P.mask8 != nullptr;
  auto load_aux = [&](int pass_) {
    if (!(n + 8 <= N && vec_ok)) return;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int m = m0 + pass_ * EPI_ROWS + it * RPI + rsub;
      if (m < M) {
        if (use_m8) auxn[it][0] = EA(mask8)[(int64_t)m * EA(ldm8) + (n >> 3)];
        else auxn[it] = *reinterpret_cast<const u32x4*>(EA(aux) + (int64_t)m * EA(ldaux) + n);
      }
    }
  };
  if constexpr (HAS_AUX) load_aux(0);
  // EPI_LN_BWD_F32: the operands of the next row this thread handles (LN input, accumulated gradient,
  // row statistics) are loaded while it finishes the current one -- across pass boundaries too -- so
  // the 16 row iterations of a tile expose one load latency instead of one each
  struct LnRow { f32x4 x0, x1, d0, d1; float mu, rs; };
  LnRow lnp = {};
  auto ln_load = [&](int pass_, int it_) {
    const int m = m0 + pass_ * EPI_ROWS + it_ * RPI + rsub;
    if (m < M && n + 8 <= N) {
      const float* xp = EA(resid) + (int64_t)m * EA(ldres) + n;
      const float* dp = o32 + (int64_t)m * EA(ldc) + n;
      lnp.x0 = *reinterpret_cast<const f32x4*>(xp);
      lnp.x1 = *reinterpret_cast<const f32x4*>(xp + 4);
      lnp.d0 = *reinterpret_cast<const f32x4*>(dp);
      lnp.d1 = *reinterpret_cast<const f32x4*>(dp + 4);
      lnp.mu = EA(ln_mean)[m];
      lnp.rs = EA(ln_rstd)[m];
    }
  };
  if constexpr (LNB) ln_load(0, 0);
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 1
  for (int pass = 0; pass < GBM / EPI_ROWS; ++pass) {
    lds_barrier();  // stage-ring / previous pass reads done
    stage_acc<TL, EPI_ROWS>(acc, ct, pass, lane, wave);
    lds_barrier();
    const int mb = m0 + pass * EPI_ROWS;
    if constexpr (LNB) {
      // a row's GBN columns are TPR = 32 consecutive threads (one half wave): row sums by 5 xor
      // shuffles inside the half. One row's loads ahead (ln_load; all IT rows' loads up front spill
      // next to the accumulators still live for the later passes)
      const float invn = 1.0f / (float)N;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int ml = it * RPI + rsub;
        const int m = mb + ml;
        const LnRow cur = lnp;
        if (it + 1 < IT) ln_load(pass, it + 1);
        else if (pass + 1 < GBM / EPI_ROWS) ln_load(pass + 1, 0);
        if (m >= M) continue;  // a whole half wave (one row) at once: the shuffles stay inside it
        const f32x4 xv[1][2] = {{cur.x0, cur.x1}}, dv[1][2] = {{cur.d0, cur.d1}};
        const float mu[1] = {cur.mu}, rs[1] = {cur.rs};
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(ct + ml * CT + 8 * c8);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(ct + ml * CT + 8 * c8 + 4);
        float dy[8], xh[8], gd[8];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dy[e] = alpha * v0[e];
          dy[e + 4] = alpha * v1[e];
          xh[e] = (xv[0][0][e] - mu[0]) * rs[0];
          xh[e + 4] = (xv[0][1][e] - mu[0]) * rs[0];
          gd[e] = dy[e] * gam0[e];
          gd[e + 4] = dy[e + 4] * gam1[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1 += gd[e];
          s2 += gd[e] * xh[e];
          cg[e] += dy[e] * xh[e];
          cb[e] += dy[e];
        }
#pragma unroll
        for (int o = 1; o < TPR; o <<= 1) {
          s1 += __shfl_xor(s1, o, 64);
          s2 += __shfl_xor(s2, o, 64);
        }
        s1 *= invn;
        s2 *= invn;
        float r[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          r[e] = dv[0][0][e] + rs[0] * (gd[e] - s1 - xh[e] * s2);
          r[e + 4] = dv[0][1][e] + rs[0] * (gd[e + 4] - s1 - xh[e + 4] * s2);
        }
        float* op = o32 + (int64_t)m * EA(ldc) + n;
        *reinterpret_cast<f32x4*>(op) = f32x4{r[0], r[1], r[2], r[3]};
        *reinterpret_cast<f32x4*>(op + 4) = f32x4{r[4], r[5], r[6], r[7]};
        if (EA(o16)) {
          if (EA(drop_thr)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // n is even: one hash per column pair (as ln_bwd_kernel)
              const uint32_t hq = mmt_hash(EA(drop_key), (uint32_t)m, (uint32_t)(n >> 1) + q);
              r[2 * q] = mmt_keep(hq, 0, EA(drop_thr)) ? r[2 * q] * EA(drop_scale) : 0.0f;
              r[2 * q + 1] = mmt_keep(hq, 1, EA(drop_thr)) ? r[2 * q + 1] * EA(drop_scale) : 0.0f;
            }
          }
          *reinterpret_cast<u32x4*>(EA(o16) + (int64_t)m * EA(ldo16) + n) =
              u32x4{pack2bf(r[0], r[1]), pack2bf(r[2], r[3]), pack2bf(r[4], r[5]), pack2bf(r[6], r[7])};
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] += r[e];
        }
      }
    } else if (n + 8 <= N && vec_ok) {
      // issue every operand load of this thread's rows first (memory-level parallelism)
      u32x4 auxv[IT];
      f32x4 resv[IT][2];
      if constexpr (HAS_AUX) {
#pragma unroll
        for (int it = 0; it < IT; ++it) auxv[it] = auxn[it];
        if (pass + 1 < GBM / EPI_ROWS) load_aux(pass + 1);
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int m = mb + it * RPI + rsub;
        if (m < M) {
          const float* rp = EPI == EPI_BIAS_RESID_F32 ? EA(resid) + (int64_t)m * EA(ldres) + n
                                                      : o32 + (int64_t)m * EA(ldc) + n;
          if (HAS_RES) {
            resv[it][0] = *reinterpret_cast<const f32x4*>(rp);
            resv[it][1] = *reinterpret_cast<const f32x4*>(rp + 4);
          }
        }
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int ml = it * RPI + rsub;
        const int m = mb + ml;
        if (m >= M) continue;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(ct + ml * CT + 8 * c8);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(ct + ml * CT + 8 * c8 + 4);
        float r[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          r[e] = PRE ? v0[e] : alpha * v0[e] + bias0[e];
          r[e + 4] = PRE ? v1[e] : alpha * v1[e] + bias1[e];
        }
        if (!PRE && EPI == EPI_BIAS_TANH_BF16) {
#pragma unroll
          for (int e = 0; e < 8; ++e) r[e] = fast_tanh(r[e]);
        }
        if (EPI == EPI_BIAS_RELU_BF16) {
#pragma unroll
          for (int e = 0; e < 8; ++e) r[e] = fmaxf(r[e], 0.0f);
        }
        if (HAS_AUX) {
          if (EPI == EPI_DRELU_BF16 && use_m8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) r[e] = ((auxv[it][0] >> e) & 1u) ? r[e] : 0.0f;
          } else {
            const u32x4 a = auxv[it];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float t0 = bf2f(a[q] & 0xffff), t1 = bf2f(a[q] >> 16);
              if (EPI == EPI_DTANH_BF16) {
                r[2 * q] *= (1.0f - t0 * t0);
                r[2 * q + 1] *= (1.0f - t1 * t1);
              } else {
                r[2 * q] = t0 > 0.0f ? r[2 * q] : 0.0f;
                r[2 * q + 1] = t1 > 0.0f ? r[2 * q + 1] : 0.0f;
              }
            }
          }
        }
        if (EPI == EPI_BIAS_RESID_F32 && EA(drop_thr)) {  // dropout on the branch output, then residual add
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // n is even: one hash per column pair
            const uint32_t hq = mmt_hash(EA(drop_key), (uint32_t)m, (uint32_t)(n >> 1) + q);
            r[2 * q] = mmt_keep(hq, 0, EA(drop_thr)) ? r[2 * q] * EA(drop_scale) : 0.0f;
            r[2 * q + 1] = mmt_keep(hq, 1, EA(drop_thr)) ? r[2 * q + 1] * EA(drop_scale) : 0.0f;
          }
        }
        if (HAS_RES) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            r[e] += resv[it][0][e];
            r[e + 4] += resv[it][1][e];
          }
        }
        if (EPI == EPI_BIAS_RESID_F32 || EPI == EPI_STORE_F32 || EPI == EPI_ACC_F32) {
          float* op = o32 + (int64_t)m * EA(ldc) + n;
          *reinterpret_cast<f32x4*>(op) = f32x4{r[0], r[1], r[2], r[3]};
          *reinterpret_cast<f32x4*>(op + 4) = f32x4{r[4], r[5], r[6], r[7]};
          if (EPI == EPI_BIAS_RESID_F32 && EA(o16))
            *reinterpret_cast<u32x4*>(EA(o16) + (int64_t)m * EA(ldo16) + n) =
                u32x4{pack2bf(r[0], r[1]), pack2bf(r[2], r[3]), pack2bf(r[4], r[5]), pack2bf(r[6], r[7])};
          if (EPI == EPI_ACC_F32 && EA(o16)) {
            // the dropout-masked bf16 copy of the accumulated rows (the consuming branch's dY) and
            // its column sums (that branch's output-bias gradient), as drop_copy_kernel
            if (EA(drop_thr)) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {  // n is even: one hash per column pair
                const uint32_t hq = mmt_hash(EA(drop_key), (uint32_t)m, (uint32_t)(n >> 1) + q);
                r[2 * q] = mmt_keep(hq, 0, EA(drop_thr)) ? r[2 * q] * EA(drop_scale) : 0.0f;
                r[2 * q + 1] = mmt_keep(hq, 1, EA(drop_thr)) ? r[2 * q + 1] * EA(drop_scale) : 0.0f;
              }
            }
            *reinterpret_cast<u32x4*>(EA(o16) + (int64_t)m * EA(ldo16) + n) =
                u32x4{pack2bf(r[0], r[1]), pack2bf(r[2], r[3]), pack2bf(r[4], r[5]), pack2bf(r[6], r[7])};
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[e] += r[e];
          }
          if (EPI == EPI_BIAS_RESID_F32 && (GBN == 256 || GBN == 512) && EA(lnf_y)) {
            // the next LayerNorm on this row (whole rows per block: N == GBN, mmt_launch_gemm_resid_ln;
            // lnf_y is uniform per problem and m < M per half wave, so every lane of the row's half
            // wave takes the shuffles): mean, then the centred sum of squares (as ln_fwd_kernel)
            float sm = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sm += r[e];
#pragma unroll
            for (int o = 1; o < TPR; o <<= 1) sm += __shfl_xor(sm, o, 64);
            const float mean = sm * (1.0f / (float)GBN);
            float q = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) q += (r[e] - mean) * (r[e] - mean);
#pragma unroll
            for (int o = 1; o < TPR; o <<= 1) q += __shfl_xor(q, o, 64);
            const float rstd = rsqrtf(q * (1.0f / (float)GBN) + 1e-5f);
            const f32x4 g0 = lg0, g1 = lg1, b0 = lb0, b1 = lb1;
            float y[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              y[e] = (r[e] - mean) * rstd * g0[e] + b0[e];
              y[e + 4] = (r[e + 4] - mean) * rstd * g1[e] + b1[e];
            }
            *reinterpret_cast<u32x4*>(EA(lnf_y) + (int64_t)m * N + n) =
                u32x4{pack2bf(y[0], y[1]), pack2bf(y[2], y[3]), pack2bf(y[4], y[5]), pack2bf(y[6], y[7])};
            if (c8 == 0) { EA(lnf_mean)[m] = mean; EA(lnf_rstd)[m] = rstd; }
          }
        } else {
          const u32x4 packed = {pack2bf(r[0], r[1]), pack2bf(r[2], r[3]), pack2bf(r[4], r[5]), pack2bf(r[6], r[7])};
          *reinterpret_cast<u32x4*>(EA(o16) + (int64_t)m * EA(ldo16) + n) = packed;
          if (EPI == EPI_BIAS_RELU_BF16 && EA(mask8)) {  // bit e: the stored bf16 value is > 0
            uint32_t mb = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const uint32_t lo = packed[q] & 0xffffu, hi = packed[q] >> 16;
              mb |= (uint32_t)(lo != 0 && lo < 0x8000u) << (2 * q);
              mb |= (uint32_t)(hi != 0 && hi < 0x8000u) << (2 * q + 1);
            }
            // 8 consecutive threads (one row, 64 columns) join their bytes: one 8-byte store instead
            // of eight byte stores (byte stores cost ffn0 8 % at the target)
            const int g0 = n - 8 * (c8 & 7);  // first column of this thread's group
            if (g0 + 64 <= N && (EA(ldm8) & 7) == 0) {  // uniform across the group
              uint32_t wv = mb;
              wv |= (uint32_t)__shfl_down((int)wv, 1, 64) << 8;
              wv |= (uint32_t)__shfl_down((int)wv, 2, 64) << 16;
              const uint32_t w2 = (uint32_t)__shfl_down((int)wv, 4, 64);
              if ((c8 & 7) == 0) *reinterpret_cast<u32x2*>(EA(mask8) + (int64_t)m * EA(ldm8) + (g0 >> 3)) = u32x2{wv, w2};
            } else {
              EA(mask8)[(int64_t)m * EA(ldm8) + (n >> 3)] = (uint8_t)mb;
            }
          }
          if (MX_OUT && EA(o8)) {
            // MX-fp8 copy: the 32-column block of this row is 4 consecutive threads (c8 & ~3)
            float am = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf(r[e]));
            am = fmaxf(am, __shfl_xor(am, 1, 64));
            am = fmaxf(am, __shfl_xor(am, 2, 64));
            const int ex = mx_exp(am);
            const float inv = mx_inv(ex);
            *reinterpret_cast<u32x2*>(EA(o8) + (int64_t)m * EA(ld8) + n) =
                u32x2{pack4fp8(r[0] * inv, r[1] * inv, r[2] * inv, r[3] * inv),
                      pack4fp8(r[4] * inv, r[5] * inv, r[6] * inv, r[7] * inv)};
            if ((c8 & 3) == 0) EA(s8)[(int64_t)m * EA(lds8) + (n >> 5)] = (uint8_t)(ex + 127);
          }
          if (CAN_DB) {
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[e] += r[e];
          }
        }
      }
    } else if (n < N) {
      // edge columns (and unaligned leading dimensions): scalar epilogue + zero pad columns
      for (int it = 0; it < IT; ++it) {
        const int ml = it * RPI + rsub;
        const int m = mb + ml;
        if (m >= M) continue;
        uint32_t mb = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = ct[ml * CT + 8 * c8 + e];
          if (n + e < N) {
            const float o = epi_scalar<EPI, PRE>(P, o32, alpha, m, n + e, v);
            cs[e] += o;
            if (EPI == EPI_BIAS_RELU_BF16) mb |= (uint32_t)(bf2f(f2bf(o)) > 0.0f) << e;
          } else {
            epi_pad<EPI>(P, m, n + e);
          }
        }
        if (EPI == EPI_BIAS_RELU_BF16 && EA(mask8)) EA(mask8)[(int64_t)m * EA(ldm8) + (n >> 3)] = (uint8_t)mb;
      }
    }
  }
  // column sums: rows of a column group live in lanes l, l^TPR, ... of every wave: fold those, then
  // the waves via LDS (the staged tile is dead: every thread has read its own rows), one atomic per
  // column
#undef EA
  auto flush_colsums = [&](float (&v)[8], float* dst) {
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = TPR; o < 64; o <<= 1) v[e] += __shfl_xor(v[e], o, 64);
    __syncthreads();
    float* red = ct;  // [NW waves][GBN columns]
    if (lane < TPR) {
      *reinterpret_cast<f32x4*>(red + wave * GBN + 8 * c8) = f32x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<f32x4*>(red + wave * GBN + 8 * c8 + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
    __syncthreads();
    if (tid < GBN && n0 + tid < N) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) sum += red[w * GBN + tid];
      atomicAdd(dst + n0 + tid, sum);
    }
  };
  if (want_db) flush_colsums(cs, P.dbias);
  if constexpr (LNB) {
    flush_colsums(cg, P.ln_dgamma);
    flush_colsums(cb, P.ln_dbeta);
  }
}
