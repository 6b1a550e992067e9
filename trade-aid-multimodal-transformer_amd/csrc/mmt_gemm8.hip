// 256 x 256 ping-pong bf16 GEMM for gfx950 (round 5; launched by mmt_gemm.hip's launch_t).
#include "mmt_gemm_dev.h"

#include <type_traits>

// ---------------------------------------------------------------------------------------------
// 256 x 256 ping-pong GEMM (round 5): 512 threads = two groups of 4 waves, each wave a 128 (m) x 64 (n)
// output of v_mfma_f32_16x16x32_bf16 accumulators (acc[4 n blocks][8 m blocks] f32x4, SWAP layout:
// lane & 15 = m, registers = n). A K-tile (BK 64) is consumed in four PHASES, one quadrant (64 m x 32 n x
// K 64 = 16 MFMAs per wave) each; a phase is a LOAD segment (that quadrant's fragment reads + one
// half-tile of the next K-tile's LDS-DMA) and a COMPUTE segment (the 16 MFMAs), each closed by a raw
// s_barrier. Group 1 (waves 4-7) runs one barrier behind group 0, so on every SIMD one wave computes while
// its partner loads (MI355X_MICROARCH.md "Two waves per SIMD"; cdna_hip_programming.md §5 "The 256²
// 8-phase template"). The 16x16x32 shape holds a higher clock than 32x32x16 at the same cycles per FLOP
// (MI355X_MICROARCH.md DVFS item 7).
//
// LDS: two K-tile buffers of four 16-KiB half-tiles, 128 KiB. The half-tiles are grouped by the phase that
// first reads them, so each can be refilled as soon as its previous contents are dead:
//   XA = X rows {0-63, 128-191} (each group's first 64 rows), XB = X rows {64-127, 192-255},
//   WA = W columns {64c + 0..31}, WB = W columns {64c + 32..63} (c = 0..3, each wave's n halves).
// Phase p of K-tile t reads: 1: XA + WA, 2: WB, 3: XB, 4: WA again (re-read, so one W set is live), and
// issues the next K-tile's half-tile 1: XA, 2: WA, 3: WB, 4: XB (2 pieces of 1 KiB per wave), then waits
// vmcnt(4) in phases 1, 2, 4 -- two half-tiles stay in flight and each lands >= 3 phases before its first
// read. A wave's wait + the barrier that closes its load segment publish its pieces; with the one-barrier
// group stagger every read still follows both groups' waits (the reader's load segment starts after the
// other group's next barrier). Refills reuse a half-tile >= 2 phases after its last read.
// K-contiguous images [128 rows][64 k] (128-B rows, kc_swz<64>); an MN-contiguous operand (B_KC = false: the
// backward-data product, W stored [K][N]; A_KC = B_KC = false: the weight gradient dW = dY^T X, both stored
// [K][rows]) as [64 k][128 cols] (256-B rows, chunk ^ ((k & 3) << 2 | (k >> 3 & 1) << 1), conflict-free
// ds_read_b64_tr_b16 reads). Split-K (weight gradients): blockIdx.y = K slice, each writing its own fp32 slab
// (o32 + slice * split_stride), with the XCD-major (tile, slice, problem) order of gemm_kernel.
// ---------------------------------------------------------------------------------------------
template <int SUB, bool IS_W, bool KC>
__device__ __forceinline__ void issue_half(const i32x4& rsrc, uint32_t img, int ld, int rows_total, int K, int r0, int k0,
                                           int wave, int lane) {
  // (img: the half-tile's LDS byte address, wave-uniform; ld / rows_total / K / r0 in registers: a value
  // read through the GemmProblem reference is re-loaded after every asm "memory" clobber)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = wave * 2 + u;  // piece 0..15 of the half-tile
    int voff;
    if (KC) {
      const int irow = 8 * i + (lane >> 3);                     // image row
      const int chunk = kc_swz<64>(lane & 7, irow);
      const int trow = IS_W ? ((irow >> 5) * 64 + (irow & 31) + SUB * 32) : ((irow >> 6) * 128 + (irow & 63) + SUB * 64);
      const int gk = k0 + chunk * 8;
      voff = (r0 + trow < rows_total && gk < K) ? (trow * ld + gk) * 2 : 0x7fffffff;
    } else {  // operand stored [K][rows] (rsrc based at row k0): image [64 k][128 cols]
      const int kr = 4 * i + (lane >> 4);
      const int c = (lane & 15) ^ (((kr & 3) << 2) | (((kr >> 3) & 1) << 1));  // image chunk stored at slot lane & 15
      const int tcol = IS_W ? (c >> 2) * 64 + (c & 3) * 8 + SUB * 32 : (c >> 3) * 128 + (c & 7) * 8 + SUB * 64;
      voff = (k0 + kr < K && r0 + tcol < rows_total) ? (kr * ld + r0 + tcol) * 2 : 0x7fffffff;
    }
    dma16(rsrc, img + i * 1024, voff);
  }
}

// 16x16x32 operand fragment: lane l holds rows irow0 + (l & 15), k = 32 s + 8 (l >> 4) + 0..7
__device__ __forceinline__ bf16x8 frag16_kc(const char* img, int irow0, int s, int lane) {
  const int irow = irow0 + (lane & 15);
  return *reinterpret_cast<const bf16x8*>(img + irow * 128 + kc_swz<64>(4 * s + (lane >> 4), irow) * 16);
}
// the same from an MN-contiguous image [64 k][128 n]: columns icol0 + (l & 15), two transposed 4-row reads
__device__ __forceinline__ bf16x8 frag16_mn(const char* img, int icol0, int s, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = icol0 + 4 * p;
  const int k1 = 32 * s + 8 * g + q, k2 = k1 + 4;  // (k2 & 3) == q, bit 3 equal
  const int f = (q << 2) | (((k1 >> 3) & 1) << 1);
  const char* a = img + ((col >> 3) ^ f) * 16 + (col & 7) * 2;
  return join4(lds_tr16(a + k1 * 256), lds_tr16(a + k2 * 256));
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int EPI, bool A_KC, bool B_KC>
__global__ __launch_bounds__(512, 1) void gemm8_kernel(GemmBatch batch) {
  using TL = TileL;  // 256 x 256, 8 waves 2 (m) x 4 (n): epilogue geometry
  constexpr int HT = 16384;          // half-tile bytes
  constexpr int EPI_ROWS = 64;
  int tile = blockIdx.x, split = blockIdx.y, prob = blockIdx.z;
  const int nsplit = gridDim.y;
  if (batch.xcd_plane) {  // XCD-major order of the whole (tile, split, problem) grid (as gemm_kernel)
    const int nwg = gridDim.x * nsplit * gridDim.z;
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + nsplit * blockIdx.z);
    const int x = lin % 8, q = nwg / 8, rr = nwg % 8;
    const int l2 = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + lin / 8;
    tile = l2 % gridDim.x;
    split = (l2 / gridDim.x) % nsplit;
    prob = l2 / (gridDim.x * nsplit);
  } else {
    const int nwg = gridDim.x;
    const int x = tile % 8, q = nwg / 8, rr = nwg % 8;
    tile = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + tile / 8;
  }
  const GemmProblem& P = batch.p[prob];
  // (readfirstlane: keep them in SGPRs -- the compiler re-loads kernel-argument values inside the K loop
  // otherwise, and each such s_load's lgkmcnt(0) wait also drains the phase's LDS fragment reads)
  const int M = __builtin_amdgcn_readfirstlane(P.M), N = __builtin_amdgcn_readfirstlane(P.N);
  const int K = __builtin_amdgcn_readfirstlane(P.K);
  const int tiles_n = (N + 255) / 256, tiles_m = (M + 255) / 256;
  if (tile >= tiles_m * tiles_n) return;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * 256, n0 = tn * 256;
  const int ktiles = (K + 63) / 64;
  const int kper = (ktiles + nsplit - 1) / nsplit;
  const int kt0 = split * kper;
  const int nk = max(0, min(ktiles, kt0 + kper) - kt0);
  if (EPI == EPI_ATOMIC_F32 && nk == 0) return;
  __shared__ __attribute__((aligned(1024))) char lds[8 * HT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    const int lda = __builtin_amdgcn_readfirstlane(P.lda), ldb = __builtin_amdgcn_readfirstlane(P.ldb);
    const bf16_t* const Ap = P.A;
    const bf16_t* const Bp = P.B;
    const i32x4 rx_kc = A_KC ? op_rsrc<true>(Ap, lda, M, K, m0, 0) : i32x4{0, 0, 0, 0};
    const i32x4 rw_kc = B_KC ? op_rsrc<true>(Bp, ldb, N, K, n0, 0) : i32x4{0, 0, 0, 0};
    // rsrc of an MN-contiguous operand from row k0 (32-bit offsets: op_rsrc); column offsets stay absolute there
    auto rx = [&](int k0) { return A_KC ? rx_kc : op_rsrc<false>(Ap, lda, M, K, 0, k0); };
    auto rw = [&](int k0) { return B_KC ? rw_kc : op_rsrc<false>(Bp, ldb, N, K, 0, k0); };
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(lds_u32(lds));
    auto issue = [&](int which, int buf, int t) {  // which: 0 XA, 1 WA, 2 WB, 3 XB; t: K-tile of this slice
      const uint32_t base = lbase + buf * 4 * HT;
      const int k0 = (kt0 + t) * 64;
      if (which == 0) issue_half<0, false, A_KC>(rx(k0), base + 0 * HT, lda, M, K, m0, k0, wave, lane);
      else if (which == 3) issue_half<1, false, A_KC>(rx(k0), base + 1 * HT, lda, M, K, m0, k0, wave, lane);
      else if (which == 1) issue_half<0, true, B_KC>(rw(k0), base + 2 * HT, ldb, N, K, n0, k0, wave, lane);
      else issue_half<1, true, B_KC>(rw(k0), base + 3 * HT, ldb, N, K, n0, k0, wave, lane);
    };
    bf16x8 xf[4][2], wf[2][2];
    auto read_x = [&](const char* img) {
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          xf[mb][s] = A_KC ? frag16_kc(img, wr * 64 + 16 * mb, s, lane) : frag16_mn(img, wr * 64 + 16 * mb, s, lane);
    };
    auto read_w = [&](const char* img) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          wf[nb][s] = B_KC ? frag16_kc(img, wc * 32 + 16 * nb, s, lane) : frag16_mn(img, wc * 32 + 16 * nb, s, lane);
    };
    auto compute = [&](int msub, int nsub) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[nsub * 2 + nb][msub * 4 + mb] = mfma16(wf[nb][s], xf[mb][s], acc[nsub * 2 + nb][msub * 4 + mb]);
      __builtin_amdgcn_s_setprio(0);
    };
    auto bar = [] {
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    // prologue: K-tile 0's four half-tiles; XA and WA landed (two half-tiles in flight) + a barrier
    issue(0, 0, 0);
    issue(1, 0, 0);
    issue(2, 0, 0);
    issue(3, 0, 0);
    wait_vm(4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    if (wr == 1) bar();  // the group stagger: waves 4-7 one barrier behind
    // one K-tile (buffer BUF compile-time: static LDS offsets)
    auto ktile = [&](int t, auto BUFC) {
      constexpr int BUF = decltype(BUFC)::value;
      const char* cur = lds + BUF * 4 * HT;
      const bool more = t + 1 < nk;
      // phase 1: XA + WA, issue XA(t+1), retire WB(t)
      read_x(cur + 0 * HT);
      read_w(cur + 2 * HT);
      if (more) { issue(0, BUF ^ 1, t + 1); wait_vm(4); } else wait_vm(2);
      bar();
      compute(0, 0);
      bar();
      // phase 2: WB, issue WA(t+1), retire XB(t)
      read_w(cur + 3 * HT);
      if (more) { issue(1, BUF ^ 1, t + 1); wait_vm(4); } else wait_vm(0);
      bar();
      compute(0, 1);
      bar();
      // phase 3: XB, issue WB(t+1)
      read_x(cur + 1 * HT);
      if (more) issue(2, BUF ^ 1, t + 1);
      bar();
      compute(1, 1);
      bar();
      // phase 4: WA again, issue XB(t+1), retire XA(t+1) and WA(t+1)
      read_w(cur + 2 * HT);
      if (more) { issue(3, BUF ^ 1, t + 1); wait_vm(4); }
      bar();
      compute(1, 0);
      bar();
    };
    int t = 0;
    for (; t + 2 <= nk; t += 2) {
      ktile(t, std::integral_constant<int, 0>{});
      ktile(t + 1, std::integral_constant<int, 1>{});
    }
    if (t < nk) ktile(t, std::integral_constant<int, 0>{});
    if (wr == 0) bar();  // balance the stagger before the epilogue's block barriers
  }
  float alpha = P.alpha;
  if (P.alpha_ptr) alpha *= *P.alpha_ptr;
  float* o32 = P.o32 + (P.split_stride ? (int64_t)split * P.split_stride : (int64_t)0);
  epilogue_swap<TL, EPI, EPI_ROWS>(P, acc, lds, o32, alpha, m0, n0, tid, lane, wave);
}

template <int EPI, bool A_KC, bool B_KC>
static hipError_t launch8(const GemmBatch& b, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((gemm8_kernel<EPI, A_KC, B_KC>), grid, dim3(512), 0, s, b);
  return hipGetLastError();
}

// grid = (256 x 256 tiles of the largest problem, K slices, problems). The forward (a_kc, b_kc), backward-data
// (a_kc, !b_kc: W stored [K][N]) and weight-gradient (!a_kc, !b_kc: slab or accumulate) products;
// hipErrorInvalidValue for an epilogue the kernel does not instantiate.
hipError_t mmt_launch_gemm8(const GemmBatch& b, int epi, bool a_kc, bool b_kc, dim3 grid, hipStream_t s) {
  if (a_kc && b_kc) {
    switch (epi) {
      case EPI_STORE_BF16: return launch8<EPI_STORE_BF16, true, true>(b, grid, s);
      case EPI_BIAS_TANH_BF16: return launch8<EPI_BIAS_TANH_BF16, true, true>(b, grid, s);
      case EPI_BIAS_RELU_BF16: return launch8<EPI_BIAS_RELU_BF16, true, true>(b, grid, s);
      case EPI_BIAS_RESID_F32: return launch8<EPI_BIAS_RESID_F32, true, true>(b, grid, s);
      case EPI_STORE_F32: return launch8<EPI_STORE_F32, true, true>(b, grid, s);
      case EPI_ACC_F32: return launch8<EPI_ACC_F32, true, true>(b, grid, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (a_kc) {
    switch (epi) {
      case EPI_LN_BWD_F32: return launch8<EPI_LN_BWD_F32, true, false>(b, grid, s);
      case EPI_STORE_BF16: return launch8<EPI_STORE_BF16, true, false>(b, grid, s);
      case EPI_DTANH_BF16: return launch8<EPI_DTANH_BF16, true, false>(b, grid, s);
      case EPI_DRELU_BF16: return launch8<EPI_DRELU_BF16, true, false>(b, grid, s);
      case EPI_STORE_F32: return launch8<EPI_STORE_F32, true, false>(b, grid, s);
      case EPI_ACC_F32: return launch8<EPI_ACC_F32, true, false>(b, grid, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (!b_kc) {
    switch (epi) {
      case EPI_STORE_F32: return launch8<EPI_STORE_F32, false, false>(b, grid, s);
      case EPI_ACC_F32: return launch8<EPI_ACC_F32, false, false>(b, grid, s);
      default: return hipErrorInvalidValue;
    }
  }
  return hipErrorInvalidValue;
}
