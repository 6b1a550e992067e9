// Fused two-GEMM MLP for gfx950 (round 5): the attention out-projection of
// MultiHeadAttention / CrossAttention (reference model.py:82-92, 102-117)
//   h   = tanh(x W0^T + b0)          Linear(C, C/2) -> tanh
//   out = resid + drop(h W2^T + b2)  Linear(C/2, C) -> dropout -> residual add (model.py:224, 240)
// as ONE launch per modality group. A workgroup owns 128 rows and every column of both products:
//  * stage 1 streams x and W0 through a 3-slot LDS-DMA ring (BK 32, the gemm_kernel ring), 8 waves of
//    64 rows x N1/4 hidden columns (v_mfma_f32_32x32x16_bf16, SWAP layout: hidden on accumulator rows);
//  * its epilogue (bias, tanh, bf16) writes h into an LDS-resident image [128 rows][N1] (16-B chunk XOR
//    row swizzle: conflict-free writes and fragment reads) while the first W2 slices already stream;
//  * stage 2 reads its row operand from that image and streams only W2 (2-slot ring), 8 waves of 64 rows x
//    N2/4 output columns, and finishes in the shared fused epilogue (epilogue_swap: bias, hash dropout,
//    fp32 residual add, optional bf16 copy and the next LayerNorm's forward on the owned rows);
//  * h leaves for the backward (tanh' and the W2 weight gradient read it) from the LDS image as row-major
//    16-B stores at the very end.
// Against the two GEMM launches this removes the h round trip through HBM (written and read back: 2 x R x N1
// x 2 B), one launch and one prologue / epilogue per row tile. C = 256 (N1 128) and C = 512 (N1 256).
#include "mmt_gemm_dev.h"

#include <type_traits>

namespace {

constexpr int MLP_BM = 128;
constexpr int MLP_BK = 32;
constexpr int cmax(int a, int b) { return a > b ? a : b; }

// BM_: rows per workgroup, 128 (8 waves) or 64 (4 waves: the forward's small-C form, see mmt_launch_mlp2)
template <int N1, int BM_ = MLP_BM>
struct MlpCfg {
  static constexpr int BM = BM_, NW = BM_ / 16;
  static constexpr int N2 = 2 * N1, K1 = N2;
  using T1 = TileCfg<BM_ / 64, 4, 2, N1 / 128>;  // stage 1: BM x N1, waves BM/64 (m) x 4 (n), 64 x N1/4 each
  using T2 = TileCfg<BM_ / 64, 4, 2, N2 / 128>;  // stage 2: BM x N2, 64 x N2/4 each
  static constexpr int S1_STAGE = (BM_ + N1) * MLP_BK * 2;  // x + W0 images per K-step
  static constexpr int S1_ST = 3;
  static constexpr int S2_STAGE = N2 * MLP_BK * 2;              // W2 image per K-step
  static constexpr int S2_ST = 2;
  // the forward's W2 ring: a third slot where it fits inside the stage-1 ring (C = 256), so two slices
  // stream ahead of the stage-2 MFMAs
  static constexpr int S2F_ST = 3 * S2_STAGE <= S1_ST * S1_STAGE ? 3 : 2;
  static constexpr int EPI_ROWS = 32;
  static constexpr int CTILE = EPI_ROWS * (N2 + 4) * 4;
  static constexpr int RING = cmax(cmax(S1_ST * S1_STAGE, S2_ST * S2_STAGE), CTILE);
  static constexpr int HPITCH = N1 * 2;  // h image row pitch (bytes)
  static constexpr int HBYTES = BM_ * HPITCH;
  static constexpr int LDS = RING + HBYTES;
};

// h image: row m, 16-B chunk c (8 hidden columns) at m * HPITCH + ((c ^ (m & 15)) * 16)
template <int HP>
__device__ __forceinline__ int h_off(int m, int chunk) {
  return m * HP + ((chunk ^ (m & 15)) << 4);
}

}  // namespace

template <int N1, int BM>
__global__ __launch_bounds__(BM * 4, 1) void mlp2_kernel(Mlp2Batch batch) {
  using CF = MlpCfg<N1, BM>;
  constexpr int NW = CF::NW;
  using T1 = typename CF::T1;
  using T2 = typename CF::T2;
  constexpr int N2 = CF::N2, BK = MLP_BK;
  constexpr int TN1 = T1::TN, TN2 = T2::TN, TM = 2;  // 32 x 32 sub-tiles per wave
  constexpr int IMG_X = BM * BK * 2, IMG_W0 = N1 * BK * 2;
  constexpr int PIECES1 = (BM + N1) * BK / 512 / NW;  // LDS-DMA pieces per wave per stage-1 K-step
  constexpr int PIECES2 = N2 * BK / 512 / NW;            // per stage-2 K-step
  __shared__ __attribute__((aligned(1024))) char lds[CF::LDS];
  char* himg = lds + CF::RING;

  const int prob = blockIdx.z;
  const GemmProblem& P1 = batch.g1[prob];
  const GemmProblem& P2 = batch.g2[prob];
  const int M = __builtin_amdgcn_readfirstlane(P1.M);
  const int ntiles = (M + BM - 1) / BM;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  if (tile >= ntiles) return;
  const int m0 = tile * BM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / 4, wn = wave % 4;
  const int h = lane >> 5, r = lane & 31;

  // ---------------- stage 1: acc1 = W0 x^T (hidden on rows, m on lanes) over K1 = C ----------------
  f32x16 acc1[TN1][TM];
#pragma unroll
  for (int i = 0; i < TN1; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc1[i][j][e] = 0.f;
  {
    const int K = CF::K1;
    const int lda = __builtin_amdgcn_readfirstlane(P1.lda), ldb = __builtin_amdgcn_readfirstlane(P1.ldb);
    const i32x4 ra = op_rsrc<true>(P1.A, lda, M, K, m0, 0);
    const i32x4 rb = op_rsrc<true>(P1.B, ldb, N1, K, 0, 0);
    constexpr int nk = CF::K1 / BK;
    constexpr int ST = CF::S1_ST;
    auto issue = [&](int slot, int t) {
      char* st = lds + slot * CF::S1_STAGE;
      issue_tile<BK, true, BM, NW>(ra, st, lda, M, K, m0, t * BK, wave, lane);
      issue_tile<BK, true, N1, NW>(rb, st + IMG_X, ldb, N1, K, 0, t * BK, wave, lane);
    };
#pragma unroll
    for (int t = 0; t < ST - 1; ++t) issue(t, t);
    auto step = [&](int t, auto UC) {
      constexpr int U = decltype(UC)::value;
      wait_vm(PIECES1 * min(ST - 2, nk - 1 - t));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + ST - 1 < nk) issue((U + ST - 1) % ST, t + ST - 1);
      const char* imgA = lds + U * CF::S1_STAGE;
      const char* imgB = imgA + IMG_X;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 fa[TM], fb[TN1];
#pragma unroll
        for (int j = 0; j < TM; ++j) fa[j] = frag<BK, true, BM>(imgA, wm * 64 + 32 * j, s, lane);
#pragma unroll
        for (int i = 0; i < TN1; ++i) fb[i] = frag<BK, true, N1>(imgB, wn * TN1 * 32 + 32 * i, s, lane);
#pragma unroll
        for (int i = 0; i < TN1; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc1[i][j] = mfma32(fb[i], fa[j], acc1[i][j]);
      }
    };
    static_assert(nk % ST == 2 || nk % ST == 1 || nk % ST == 0, "");
    int t = 0;
    for (; t + ST <= nk; t += ST) {
      step(t, std::integral_constant<int, 0>{});
      step(t + 1, std::integral_constant<int, 1>{});
      step(t + 2, std::integral_constant<int, 2>{});
    }
    if (t < nk) step(t, std::integral_constant<int, 0>{});
    if (t + 1 < nk) step(t + 1, std::integral_constant<int, 1>{});
  }

  // ---------------- stage 2 prologue: the first W2 slice streams while stage 1 finishes ----------------
  constexpr int K2 = N1;
  constexpr int nk2 = K2 / BK;
  const int ldw2 = __builtin_amdgcn_readfirstlane(P2.ldb);
  const i32x4 rw2 = op_rsrc<true>(P2.B, ldw2, N2, K2, 0, 0);
  auto issue2 = [&](int slot, int t) {
    issue_tile<BK, true, N2, NW>(rw2, lds + slot * CF::S2_STAGE, ldw2, N2, K2, 0, t * BK, wave, lane);
  };
  constexpr int S2F = CF::S2F_ST;
  // with the 3-slot ring the stage-1 bias is loaded before the W2 slices: loads issued after them would
  // make the first wait for the bias drain the slices too (vmcnt counts in issue order). The 2-slot ring
  // (C = 512) loads it in the epilogue as before (held across the barrier it measured 2-5 us slower)
  f32x4 bvs[TN1][4];
  if constexpr (S2F > 2) {
#pragma unroll
    for (int i = 0; i < TN1; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        bvs[i][g] = *reinterpret_cast<const f32x4*>(P1.bias + wn * TN1 * 32 + 32 * i + 8 * g + 4 * h);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave's last stage-1 fragment reads are done: the ring is free
#pragma unroll
  for (int t = 0; t < S2F - 1; ++t)
    if (t < nk2) issue2(t, t);

  // stage-1 epilogue: h = tanh(acc1 + b0) -> bf16 -> the LDS image (lane (r, h) of sub-tile (i, j) holds
  // rows m = wm 64 + 32 j + r, hidden n = wn TN1 32 + 32 i + 8 g + 4 h + e)
  {
#pragma unroll
    for (int i = 0; i < TN1; ++i) {
      const int nb = wn * TN1 * 32 + 32 * i;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 bv = S2F > 2 ? bvs[i][g] : *reinterpret_cast<const f32x4*>(P1.bias + nb + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int m = wm * 64 + 32 * j + r;
          const uint32_t lo = pack2bf(fast_tanh(acc1[i][j][4 * g] + bv[0]), fast_tanh(acc1[i][j][4 * g + 1] + bv[1]));
          const uint32_t hi = pack2bf(fast_tanh(acc1[i][j][4 * g + 2] + bv[2]), fast_tanh(acc1[i][j][4 * g + 3] + bv[3]));
          *reinterpret_cast<u32x2*>(himg + h_off<CF::HPITCH>(m, (nb >> 3) + g) + 8 * h) = u32x2{lo, hi};
        }
      }
    }
  }

  // ---------------- stage 2: acc2 = W2 h^T (output column on rows, m on lanes) over K2 = N1 ----------------
  f32x16 acc2[TN2][TM];
#pragma unroll
  for (int i = 0; i < TN2; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc2[i][j][e] = 0.f;
  {
    // (the h image is published by the first step's barrier)
    auto step2 = [&](int t, auto UC) {
      constexpr int U = decltype(UC)::value;
      wait_vm(PIECES2 * min(S2F - 2, nk2 - 1 - t));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // slice t landed for every wave; slice t - 1's reads are done
      if (t + S2F - 1 < nk2) issue2((U + S2F - 1) % S2F, t + S2F - 1);
      const char* imgW = lds + U * CF::S2_STAGE;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 fa[TM], fb[TN2];
        // h fragment: row m = wm 64 + 32 j + (lane & 31), hidden k = t BK + 16 s + 8 (lane >> 5) + 0..7
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int m = wm * 64 + 32 * j + r;
          fa[j] = *reinterpret_cast<const bf16x8*>(himg + h_off<CF::HPITCH>(m, (t * BK + 16 * s) / 8 + h));
        }
#pragma unroll
        for (int i = 0; i < TN2; ++i) fb[i] = frag<BK, true, N2>(imgW, wn * TN2 * 32 + 32 * i, s, lane);
#pragma unroll
        for (int i = 0; i < TN2; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc2[i][j] = mfma32(fb[i], fa[j], acc2[i][j]);
      }
    };
#pragma unroll
    for (int t = 0; t < nk2; t += S2F) {
      step2(t, std::integral_constant<int, 0>{});
      if (t + 1 < nk2) step2(t + 1, std::integral_constant<int, 1>{});
      if constexpr (S2F > 2) {
        if (t + 2 < nk2) step2(t + 2, std::integral_constant<int, (S2F > 2 ? 2 : 0)>{});
      }
    }
  }

  // ---------------- stage-2 epilogue (ring area; the h image is untouched) ----------------
  float alpha = P2.alpha;
  epilogue_swap<T2, EPI_BIAS_RESID_F32, CF::EPI_ROWS>(P2, acc2, lds, P2.o32, alpha, m0, 0, tid, lane, wave);

  // ---------------- h for the backward: LDS image -> row-major 16-B stores ----------------
  {
    constexpr int CPR = N1 / 8;  // chunks per row
    bf16_t* ho = P1.o16;
    const int ldo = P1.ldo16;
#pragma unroll
    for (int q = tid; q < BM * CPR; q += 64 * NW) {
      const int m = q / CPR, c = q % CPR;
      if (m0 + m < M)
        *reinterpret_cast<u32x4*>(ho + (int64_t)(m0 + m) * ldo + 8 * c) =
            *reinterpret_cast<const u32x4*>(himg + h_off<CF::HPITCH>(m, c));
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Backward of the same MLP (reference model.py:82-92 under autograd), the two data-gradient products in
// one launch:
//   dh = (dY W2) * (1 - h^2)    stage 1: dY [M][C] (the branch gradient, dropout mask applied) K-contiguous,
//                               W2 [C][C/2] MN-contiguous (transposed LDS reads), h the forward's saved
//                               tanh output (prefetched at kernel start), db0 += column sums of dh
//   dx = dh W0                  stage 2: dh from the LDS image, W0 [C/2][C] MN-contiguous
// dh also leaves for the W0 weight gradient (side stream). g1: A = dY, B = W2, aux = h, o16 = dh, dbias =
// db0 (nullable); g2: B = W0, o16 = dx.
// ---------------------------------------------------------------------------------------------
template <int N1>
__global__ __launch_bounds__(512, 1) void mlp2_bwd_kernel(Mlp2Batch batch) {
  using CF = MlpCfg<N1>;
  using T2 = typename CF::T2;
  constexpr int N2 = CF::N2, BK = MLP_BK;
  constexpr int TN1 = CF::T1::TN, TN2 = T2::TN, TM = 2;
  constexpr int IMG_X = MLP_BM * BK * 2;
  constexpr int PIECES1 = (MLP_BM + N1) * BK / 512 / 8;
  __shared__ __attribute__((aligned(1024))) char lds[CF::LDS];
  char* himg = lds + CF::RING;

  const int prob = blockIdx.z;
  const GemmProblem& P1 = batch.g1[prob];
  const GemmProblem& P2 = batch.g2[prob];
  const int M = __builtin_amdgcn_readfirstlane(P1.M);
  const int ntiles = (M + MLP_BM - 1) / MLP_BM;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  if (tile >= ntiles) return;
  const int m0 = tile * MLP_BM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / 4, wn = wave % 4;
  const int h = lane >> 5, r = lane & 31;

  // tanh' input: h[m][n] for this lane's accumulator elements (4 consecutive columns per (i, j, g)),
  // issued before the ring so its latency hides under stage 1
  u32x2 hv[TN1][TM][4];
  {
    const bf16_t* hp = P1.aux;
    const int ldh = P1.ldaux;
#pragma unroll
    for (int i = 0; i < TN1; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wm * 64 + 32 * j + r;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = wn * TN1 * 32 + 32 * i + 8 * g + 4 * h;
          hv[i][j][g] = m < M ? *reinterpret_cast<const u32x2*>(hp + (int64_t)m * ldh + n) : u32x2{0u, 0u};
        }
      }
#pragma unroll
    for (int i = 0; i < TN1; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) asm volatile("" : "+v"(hv[i][j][g]));  // consumed: its wait sits here
  }

  f32x16 acc1[TN1][TM];
#pragma unroll
  for (int i = 0; i < TN1; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc1[i][j][e] = 0.f;
  {
    const int K = CF::K1;
    const int lda = __builtin_amdgcn_readfirstlane(P1.lda), ldb = __builtin_amdgcn_readfirstlane(P1.ldb);
    const i32x4 ra = op_rsrc<true>(P1.A, lda, M, K, m0, 0);
    const bf16_t* const Bp = P1.B;
    constexpr int nk = CF::K1 / BK;
    constexpr int ST = CF::S1_ST;
    auto issue = [&](int slot, int t) {
      char* st = lds + slot * CF::S1_STAGE;
      issue_tile<BK, true, MLP_BM, 8>(ra, st, lda, M, K, m0, t * BK, wave, lane);
      issue_tile<BK, false, N1, 8>(op_rsrc<false>(Bp, ldb, N1, K, 0, t * BK), st + IMG_X, ldb, N1, K, 0, t * BK, wave, lane);
    };
#pragma unroll
    for (int t = 0; t < ST - 1; ++t) issue(t, t);
    auto step = [&](int t, auto UC) {
      constexpr int U = decltype(UC)::value;
      wait_vm(PIECES1 * min(ST - 2, nk - 1 - t));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + ST - 1 < nk) issue((U + ST - 1) % ST, t + ST - 1);
      const char* imgA = lds + U * CF::S1_STAGE;
      const char* imgB = imgA + IMG_X;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 fa[TM], fb[TN1];
#pragma unroll
        for (int j = 0; j < TM; ++j) fa[j] = frag<BK, true, MLP_BM>(imgA, wm * 64 + 32 * j, s, lane);
#pragma unroll
        for (int i = 0; i < TN1; ++i) fb[i] = frag<BK, false, N1>(imgB, wn * TN1 * 32 + 32 * i, s, lane);
#pragma unroll
        for (int i = 0; i < TN1; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc1[i][j] = mfma32(fb[i], fa[j], acc1[i][j]);
      }
    };
    int t = 0;
    for (; t + ST <= nk; t += ST) {
      step(t, std::integral_constant<int, 0>{});
      step(t + 1, std::integral_constant<int, 1>{});
      step(t + 2, std::integral_constant<int, 2>{});
    }
    if (t < nk) step(t, std::integral_constant<int, 0>{});
    if (t + 1 < nk) step(t + 1, std::integral_constant<int, 1>{});
  }

  constexpr int K2 = N1;
  constexpr int nk2 = K2 / BK;
  const int ldw0 = __builtin_amdgcn_readfirstlane(P2.ldb);
  const bf16_t* const W0p = P2.B;
  auto issue2 = [&](int slot, int t) {
    issue_tile<BK, false, N2, 8>(op_rsrc<false>(W0p, ldw0, N2, K2, 0, t * BK), lds + slot * CF::S2_STAGE, ldw0, N2, K2,
                                 0, t * BK, wave, lane);
  };
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the stage-1 ring is free
  issue2(0, 0);

  // stage-1 epilogue: dh = acc1 (1 - h^2) -> bf16 -> the LDS image; db0 column sums in fp32 (the two m
  // sub-tiles, then the 32 lanes of the half: xor shuffles; the two m-halves of the block through LDS
  // beyond the stage-2 ring, then one coalesced atomic per column per block: per-wave atomics onto the
  // same N1 addresses from every block serialised at the memory side)
  float* red = reinterpret_cast<float*>(lds + CF::S2_ST * CF::S2_STAGE);
  static_assert(CF::S2_ST * CF::S2_STAGE + 2 * N1 * 4 <= CF::RING, "column-sum area inside the ring");
  {
    float* db = P1.dbias;
    const float alpha = P1.alpha;
#pragma unroll
    for (int i = 0; i < TN1; ++i) {
      const int nb = wn * TN1 * 32 + 32 * i;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int ml = wm * 64 + 32 * j + r;
          float d[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t w = hv[i][j][g][e >> 1];
            const float t = bf2f((e & 1) ? (w >> 16) : (w & 0xffff));
            d[e] = m0 + ml < M ? alpha * acc1[i][j][4 * g + e] * (1.0f - t * t) : 0.f;
            cs[e] += d[e];
          }
          *reinterpret_cast<u32x2*>(himg + h_off<CF::HPITCH>(ml, (nb >> 3) + g) + 8 * h) =
              u32x2{pack2bf(d[0], d[1]), pack2bf(d[2], d[3])};
        }
        if (db) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) cs[e] += __shfl_xor(cs[e], o, 64);
          }
          if (r == 0) *reinterpret_cast<f32x4*>(red + wm * N1 + nb + 8 * g + 4 * h) = f32x4{cs[0], cs[1], cs[2], cs[3]};
        }
      }
    }
  }

  f32x16 acc2[TN2][TM];
#pragma unroll
  for (int i = 0; i < TN2; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc2[i][j][e] = 0.f;
  {
    auto step2 = [&](int t, auto UC) {
      constexpr int U = decltype(UC)::value;
      wait_vm(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + 1 < nk2) issue2(U ^ 1, t + 1);
      const char* imgW = lds + U * CF::S2_STAGE;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 fa[TM], fb[TN2];
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int m = wm * 64 + 32 * j + r;
          fa[j] = *reinterpret_cast<const bf16x8*>(himg + h_off<CF::HPITCH>(m, (t * BK + 16 * s) / 8 + h));
        }
#pragma unroll
        for (int i = 0; i < TN2; ++i) fb[i] = frag<BK, false, N2>(imgW, wn * TN2 * 32 + 32 * i, s, lane);
#pragma unroll
        for (int i = 0; i < TN2; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc2[i][j] = mfma32(fb[i], fa[j], acc2[i][j]);
      }
    };
#pragma unroll
    for (int t = 0; t < nk2; t += 2) {
      step2(t, std::integral_constant<int, 0>{});
      if (t + 1 < nk2) step2(t + 1, std::integral_constant<int, 1>{});
    }
  }

  if (P1.dbias && tid < N1) atomicAdd(P1.dbias + tid, red[tid] + red[N1 + tid]);  // (published by the stage-2 barriers)
  epilogue_swap<T2, EPI_STORE_BF16, CF::EPI_ROWS>(P2, acc2, lds, P2.o32, P2.alpha, m0, 0, tid, lane, wave);

  {
    constexpr int CPR = N1 / 8;
    bf16_t* ho = P1.o16;
    const int ldo = P1.ldo16;
#pragma unroll
    for (int q = tid; q < MLP_BM * CPR; q += 512) {
      const int m = q / CPR, c = q % CPR;
      if (m0 + m < M)
        *reinterpret_cast<u32x4*>(ho + (int64_t)(m0 + m) * ldo + 8 * c) =
            *reinterpret_cast<const u32x4*>(himg + h_off<CF::HPITCH>(m, c));
    }
  }
}

// a field the fused kernels do not implement must be unset: the engine then falls back to the two GEMMs
// instead of the fused launch silently dropping that output (MX-fp8 copies, ReLU bits, the fused Q/K/V
// stage 2, split-K, and per direction the epilogue operands the other direction's kernel reads)
static bool mlp2_unused_clear(const GemmProblem& p1, const GemmProblem& p2, bool bwd) {
  for (const GemmProblem* p : {&p1, &p2})
    if (p->o8 || p->s8 || p->mask8 || p->qkv2_out || p->split_stride || p->sa || p->sb || p->ln_dgamma ||
        p->ln_dbeta)
      return false;
  if (bwd) return !p1.resid && !p1.bias && !p2.bias && !p2.resid && !p2.dbias && !p2.aux && !p2.o32 &&
                  !p2.lnf_y && !p2.drop_thr;
  return !p1.aux && !p1.resid && !p1.dbias && !p1.o32 && !p2.aux && !p2.dbias && !p1.drop_thr;
}

bool mmt_mlp2_bwd_ok(const Mlp2Batch& b) {
  if (b.count <= 0 || b.count > MMT_MLP2_GROUP) return false;
  const int n1 = b.g1[0].N;
  if (n1 != 128 && n1 != 256) return false;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& p1 = b.g1[g];
    const GemmProblem& p2 = b.g2[g];
    if (p1.N != n1 || p1.K != 2 * n1 || p2.N != 2 * n1 || p2.K != n1 || p2.M != p1.M || p1.M < 1) return false;
    if (!p1.A || !p1.B || !p1.aux || !p1.o16 || !p2.B || !p2.o16) return false;
    if ((p1.lda & 7) || (p1.ldb & 7) || (p2.ldb & 7) || (p1.ldo16 & 7) || (p1.ldaux & 3) || (p2.ldo16 & 7) ||
        p1.lda < p1.K || p1.ldb < p1.N || p2.ldb < p2.N || p1.ldo16 < n1 || p1.ldaux < n1)
      return false;
    if (((uintptr_t)p1.A | (uintptr_t)p1.B | (uintptr_t)p2.B | (uintptr_t)p1.o16 | (uintptr_t)p2.o16) & 15) return false;
    if (((uintptr_t)p1.aux) & 7) return false;
    if (p2.alpha_ptr || p1.alpha_ptr || p2.alpha != 1.0f || p2.bias) return false;
    if (!mlp2_unused_clear(p1, p2, true)) return false;
    if ((int64_t)513 * std::max(p1.lda, std::max(p1.ldb, p2.ldb)) * 2 >= ((int64_t)1 << 31)) return false;
  }
  return true;
}

hipError_t mmt_launch_mlp2_bwd(const Mlp2Batch& b, hipStream_t s) {
  if (!mmt_mlp2_bwd_ok(b)) return hipErrorInvalidValue;
  int mt = 0;
  for (int g = 0; g < b.count; ++g) mt = std::max(mt, (b.g1[g].M + MLP_BM - 1) / MLP_BM);
  if (b.g1[0].N == 128) hipLaunchKernelGGL(mlp2_bwd_kernel<128>, dim3(mt, 1, b.count), dim3(512), 0, s, b);
  else hipLaunchKernelGGL(mlp2_bwd_kernel<256>, dim3(mt, 1, b.count), dim3(512), 0, s, b);
  return hipGetLastError();
}

bool mmt_mlp2_ok(const Mlp2Batch& b) {
  if (b.count <= 0 || b.count > MMT_MLP2_GROUP) return false;
  const int n1 = b.g1[0].N;
  if (n1 != 128 && n1 != 256) return false;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& p1 = b.g1[g];
    const GemmProblem& p2 = b.g2[g];
    if (p1.N != n1 || p1.K != 2 * n1 || p2.N != 2 * n1 || p2.K != n1 || p2.M != p1.M || p1.M < 1) return false;
    if (!p1.A || !p1.B || !p1.bias || !p1.o16 || !p2.B || !p2.bias || !p2.resid || !p2.o32) return false;
    if ((p1.lda & 7) || (p1.ldb & 7) || (p2.ldb & 7) || (p1.ldo16 & 7) || (p2.ldc & 3) || (p2.ldres & 3) ||
        (p2.o16 && (p2.ldo16 & 7)) || p1.lda < p1.K || p1.ldb < p1.K || p2.ldb < p2.K || p1.ldo16 < n1)
      return false;
    if (((uintptr_t)p1.A | (uintptr_t)p1.B | (uintptr_t)p2.B | (uintptr_t)p1.o16 | (uintptr_t)p2.o32 |
         (uintptr_t)p2.resid | (uintptr_t)p1.bias | (uintptr_t)p2.o16) & 15)  // 16-B epilogue stores / loads
      return false;
    if (!mlp2_unused_clear(p1, p2, false)) return false;
    if (p2.alpha_ptr || p1.alpha_ptr || p1.alpha != 1.0f) return false;
    if ((int64_t)513 * std::max(p1.lda, std::max(p1.ldb, p2.ldb)) * 2 >= ((int64_t)1 << 31)) return false;
    if (p2.lnf_y && (!p2.lnf_gamma || !p2.lnf_beta || !p2.lnf_mean || !p2.lnf_rstd ||
                     (((uintptr_t)p2.lnf_y | (uintptr_t)p2.lnf_gamma | (uintptr_t)p2.lnf_beta) & 15)))
      return false;
  }
  return true;
}

// rows per forward workgroup at C = 256 (N1 128): 128 (8 waves, 80 KiB LDS, 163 VGPRs: one workgroup per
// CU) or 64 (4 waves, 52 KiB: three per CU, so one's epilogue stores overlap the others' MFMAs);
// MMT_MLP2_BM, or mmt_mlp2_set_bm() for in-process A/B
static int g_mlp2_bm = [] {
  const char* e = getenv("MMT_MLP2_BM");
  return e ? atoi(e) : 128;
}();
extern "C" int mmt_mlp2_set_bm(int bm) {
  const int old = g_mlp2_bm;
  g_mlp2_bm = bm;
  return old;
}

hipError_t mmt_launch_mlp2(const Mlp2Batch& b, hipStream_t s) {
  if (!mmt_mlp2_ok(b)) return hipErrorInvalidValue;
  const int bm = (b.g1[0].N == 128 && g_mlp2_bm == 64) ? 64 : 128;
  int mt = 0;
  for (int g = 0; g < b.count; ++g) mt = std::max(mt, (b.g1[g].M + bm - 1) / bm);
  if (b.g1[0].N == 128) {
    if (bm == 64) hipLaunchKernelGGL((mlp2_kernel<128, 64>), dim3(mt, 1, b.count), dim3(256), 0, s, b);
    else hipLaunchKernelGGL((mlp2_kernel<128, 128>), dim3(mt, 1, b.count), dim3(512), 0, s, b);
  } else {
    hipLaunchKernelGGL((mlp2_kernel<256, 128>), dim3(mt, 1, b.count), dim3(512), 0, s, b);
  }
  return hipGetLastError();
}
