// bf16 MFMA GEMM for gfx950 with fused epilogues (forward linear, backward data, weight grad).
//
// Tile 128x128, K-step 64, 256 threads = 4 waves (2x2), each wave a 64x64 sub-tile as 2x2
// v_mfma_f32_32x32x16_bf16 accumulators (fp32).
//
// Operand staging is direct global->LDS (buffer_load_dwordx4 ... lds), no VGPR round trip, into
// an S-stage LDS ring: the loads of K-step t+S-1 are in flight while step t computes; each step
// starts with a counted `s_waitcnt vmcnt` (never 0 while later stages are in flight) and one raw
// s_barrier. Out-of-range chunks (M/N/K edges) get an out-of-bounds buffer offset and land as
// zeros (the buffer descriptor's range check), so edge tiles need no branches.
//   K-contiguous operand  -> image [128 rows][64 k], 128-B rows, 16-B chunk XOR swizzle
//                            chunk ^= (row>>1)&7 (conflict-free ds_read_b128 fragments)
//   MN-contiguous operand -> image [64 k][128], 256-B rows, chunk ^= (k&3)<<2 (conflict-free
//                            ds_read_b64_tr_b16 transposed fragments)
// The swizzle is applied on the per-lane GLOBAL source address (the LDS destination of an
// LDS-DMA is lane-linear) and again on the fragment read.
// SWAP=true computes C^T tiles (N on accumulator rows, M on lanes): each lane owns one output row
// and 4 consecutive columns per register group -> 8/16-B vector epilogue stores.
// SWAP=false keeps N on lanes: 32 lanes hit 128 contiguous bytes of one row, the shape fp32
// atomics need (weight-grad split-K accumulate).
#include "mmt_common.h"
#include "mmt_kernels.h"

#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "mmt_gemm_dev.h"


// tuning knob (mmt_gemm_set_variant): pipeline variant of the forward / backward-data GEMMs in
// bits 0-3 and of the weight-grad (split-K, atomic) GEMMs in bits 4-7:
//   0 = BK 64 x 2 stages, 1 = BK 32 x 2, 2 = BK 32 x 3, 3 = BK 32 x 4, 4 = BK 64 x 3,
//   5 = BK 32 x 3 and 6 = BK 32 x 2 at 3 blocks per CU (64-row epilogue passes)
static int g_gemm_variant = -1;     // forward / backward-data (-1: per-epilogue policy, launch_t)

static int g_gemm_big_variant_rt = 0;  // bits 8-11 of mmt_gemm_set_variant: 256x256 pipeline (0: env / default)
static int g_force_big_rt = 0;         // bit 16: the 256x256 tile whatever K (M, N >= 256), for tests / benches
static int g_gemm8_rt = -1;            // bit 17 / 18: ping-pong 256x256 kernel (gemm8_kernel) on / off (-1: env / default)
static int g_gemm_variant_dw = 0;   // weight grad (split-K atomic)
extern "C" int mmt_gemm_set_variant(int v) {
  if (v < 0) {  // back to the default policy
    g_gemm_variant = -1; g_gemm_variant_dw = 0; g_gemm_big_variant_rt = 0; g_force_big_rt = 0; g_gemm8_rt = -1;
    return 0;
  }
  if ((v & 15) > 6 || ((v >> 4) & 15) > 6 || ((v >> 8) & 15) > 3) return -1;
  g_gemm_variant = v & 15;
  g_gemm_variant_dw = (v >> 4) & 15;
  g_gemm_big_variant_rt = (v >> 8) & 15;
  g_force_big_rt = (v >> 16) & 1;
  g_gemm8_rt = ((v >> 17) & 1) ? 1 : ((v >> 18) & 1) ? 0 : -1;
  return 0;
}


// Diagnostic timestamps (-DMMT_GEMM_STAMPS builds only; tools/gemm_stamps.py): thread 0 of each block
// records s_memtime at phase boundaries into batch.stamps[block * 8 + k]: 0 start, 1 prologue issued,
// 2 first K-step's stage landed (after its barrier), 3 K loop done, 4 epilogue done, 5 HW_ID, 6 XCC_ID.
#ifdef MMT_GEMM_STAMPS
static unsigned long long* g_stamps = nullptr;
extern "C" int mmt_gemm_set_stamps(void* p) { g_stamps = (unsigned long long*)p; return 0; }
#define GEMM_STAMP(k)                                                                                   \
  do {                                                                                                \
    if (batch.stamps && threadIdx.x == 0)                                                             \
      batch.stamps[((size_t)blockIdx.z * gridDim.y * gridDim.x + (size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (k)] = \
          (k) == 5   ? (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11))  \
          : (k) == 6 ? (unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) \
                     : (unsigned long long)__builtin_amdgcn_s_memtime();                             \
  } while (0)
#else
#define GEMM_STAMP(k) \
  do {                \
  } while (0)
#endif


// Per-head Q/K/V stage 2 fused into the stage-1 GEMM's epilogue (reference model.py:36-50,
// each head's key / query / value = Linear(hs/2, hs, no bias) of tanh(Linear(C, hs/2))). acc holds
// this wave's TN x TM 32x32 sub-tiles of h1^T (stage-1 column n on accumulator rows, row m on lanes).
// First, in place, acc = h1 = tanh(alpha acc + bias) (what the epilogue then stores as o16, PRE).
// Each hh-wide column block blk of h1 (hh = 16 or 32) is one head's K, Q or V stage-1 output; its
// stage 2 out[m][blk*2hh + o] = sum_k W2[blk][o][k] h1[m][blk*hh + k] runs on MFMA straight from
// the accumulator registers: lane (r, h) holds h1[r][4h + 0..3] and h1[r][8 + 4h + 0..3] of a
// 16-column block (accumulator groups g and g + 1), which is a K-16 B operand with K permuted
// (slot j <-> k = 4h + j, j < 4; 8 + 4h + j - 4, j >= 4) -- the W2 fragment takes the same
// permutation. A 32 x 32 stage-1 sub-tile yields 64 consecutive output columns (2 n0 + ...) of 32
// rows: they cross a wave-private LDS slot (no block barrier) so they leave as 128-B row segments,
// 8 rows per store instruction (storing the MFMA layout directly touches 32 rows x 32 B per store
// and ran the target's qkv1 launch 169 us against 78 + 65 for the unfused pair).
// The W2 fragments of the tile's stage-1 column blocks, converted to bf16 and permuted once per block
// into LDS at kernel start (before the K loop; the epilogue reads them with one ds_read_b128 each):
// fragment (b, ot, kh) of local block b = lane-ordered 16-B pieces at ((b * 2 + ot) * 2 + kh) KiB
// (HH = 16: ot = kh = 0, fragment b at b KiB). Fetching them from global fp32 inside the epilogue
// put two dependent global loads in front of every sub-tile's MFMAs.
constexpr int QKV2_W2_LDS = 16384;
template <class TL>
__device__ __forceinline__ void qkv2_stage_w2(const GemmProblem& P, char* w2l, int n0, int tid) {
  const int HH = P.qkv2_hh, HS = 2 * HH;
  const int nfrag = HH == 32 ? (TL::BN / 32) * 4 : TL::BN / 16;  // 16 (HH 32) or 8 (HH 16)
  const int blk0 = n0 / HH, nblk = P.N / HH;
  for (int q = tid; q < nfrag * 64; q += TL::NT) {
    const int f = q >> 6, ln = q & 63, r = ln & 31, h = ln >> 5;
    const int b = HH == 32 ? f >> 2 : f, ot = HH == 32 ? (f >> 1) & 1 : 0, kh = HH == 32 ? f & 1 : 0;
    u32x4 u = {0u, 0u, 0u, 0u};
    if (blk0 + b < nblk) {
      const float* w = P.qkv2_w2 + ((int64_t)(blk0 + b) * HS + ot * 32 + r) * HH + 16 * kh + 4 * h;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(w);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(w + 8);
      u = u32x4{pack2bf(lo[0], lo[1]), pack2bf(lo[2], lo[3]), pack2bf(hi[0], hi[1]), pack2bf(hi[2], hi[3])};
    }
    *reinterpret_cast<u32x4*>(w2l + f * 1024 + ln * 16) = u;
  }
}

template <class TL>
__device__ __forceinline__ void qkv2_fused(const GemmProblem& P, f32x16 (&acc)[TL::TN][TL::TM], char* lds, char* w2l,
                                           float alpha, int m0, int n0, int lane, int wave) {
  constexpr int TM = TL::TM, TN = TL::TN;
  constexpr int SROW = 144;  // slot row pitch (128 B of bf16 + 16 B pad)
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int h = lane >> 5, r = lane & 31;
  const int M = P.M, N = P.N, HH = P.qkv2_hh, HS = 2 * HH;
  const int nw = n0 + wn * TN * 32;  // first stage-1 column of this wave
  char* slot = lds + wave * 32 * SROW;
  // W2 fragment of block blk, output tile ot, K-16 half kh (HH = 32: two halves): lane (o, h), slot j
  // (staged in LDS by qkv2_stage_w2)
  const int blk0 = n0 / HH;
  auto w2frag = [&](int blk, int ot, int kh) {
    const int f = HH == 32 ? ((blk - blk0) * 2 + ot) * 2 + kh : blk - blk0;
    return *reinterpret_cast<const bf16x8*>(w2l + f * 1024 + lane * 16);
  };
  // accumulator elements [8q, 8q + 8) of a sub-tile as a bf16 B operand (16 columns of h1)
  auto hfrag = [&](const f32x16& a, int q) {
    const u32x4 u = {pack2bf(a[8 * q], a[8 * q + 1]), pack2bf(a[8 * q + 2], a[8 * q + 3]),
                     pack2bf(a[8 * q + 4], a[8 * q + 5]), pack2bf(a[8 * q + 6], a[8 * q + 7])};
    return __builtin_bit_cast(bf16x8, u);
  };
  // D[o][m] (32 output columns c0 + o of the sub-tile's 64, rows m = lanes) into the slot: 16-B row
  // pieces after a v_permlane32_swap of the two halves
  auto put = [&](const f32x16& d, int c0) {
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int ga = 2 * pr, gb = 2 * pr + 1;
      const auto s0 = __builtin_amdgcn_permlane32_swap(pack2bf(d[4 * ga], d[4 * ga + 1]), pack2bf(d[4 * gb], d[4 * gb + 1]),
                                                       false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(pack2bf(d[4 * ga + 2], d[4 * ga + 3]),
                                                       pack2bf(d[4 * gb + 2], d[4 * gb + 3]), false, false);
      *reinterpret_cast<u32x4*>(slot + r * SROW + (c0 + 16 * pr + 8 * h) * 2) = u32x4{s0[0], s1[0], s0[1], s1[1]};
    }
  };
  // the slot's 32 rows x 64 columns to out[m0j + row][2 nb + col]: 8 rows of 128 B per store
  auto drain = [&](int nb, int j) {
    const int mj = m0 + wm * TM * 32 + 32 * j;
    const int cc = (lane & 7) * 8, cg = 2 * nb + cc;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = 8 * it + (lane >> 3);
      const u32x4 v = *reinterpret_cast<const u32x4*>(slot + row * SROW + cc * 2);
      if (mj + row < M && cg < 2 * N)
        *reinterpret_cast<u32x4*>(P.qkv2_out + (int64_t)(mj + row) * P.qkv2_ld + cg) = v;
    }
  };
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;
  __syncthreads();  // the slots overlay the stage ring: every wave's last K-step reads are done
  // one 32x32 sub-tile at a time (activation, then its stage-2 MFMAs, slot, stores): every value is
  // produced right before its use, so the epilogue stays inside the main loop's register budget
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int nb = nw + 32 * i;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      // (the bias is already in the accumulators: gemm_kernel starts them at bias / alpha)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = fast_tanh(alpha * acc[i][j][e]);
      if (nb < N) {
        if (HH == 16) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
            if (nb + 16 * q < N) put(mfma32(w2frag((nb + 16 * q) / 16, 0, 0), hfrag(acc[i][j], q), z), 32 * q);
        } else {  // HH == 32: K = 32 in two halves, two output tiles
          const bf16x8 h0 = hfrag(acc[i][j], 0), h1 = hfrag(acc[i][j], 1);
#pragma unroll
          for (int ot = 0; ot < 2; ++ot) put(mfma32(w2frag(nb / 32, ot, 1), h1, mfma32(w2frag(nb / 32, ot, 0), h0, z)), 32 * ot);
        }
        drain(nb, j);  // (LDS ops of one wave complete in order: the next put cannot pass these reads)
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}


// MINB > 1 (128x128 tile only): a launch-bounds hint of MINB blocks per CU, with the epilogue staged in
// 64-row passes so the LDS footprint leaves room for them (variants 5 and 6)
template <class TL, int BK, int ST, bool A_KC, bool B_KC, bool SWAP, int EPI, int MINB = 1>
__global__ __launch_bounds__(TL::NT, MINB) void gemm_kernel(GemmBatch batch) {
  constexpr int GBM = TL::BM, GBN = TL::BN, NW = TL::NW, NT = TL::NT, TM = TL::TM, TN = TL::TN;
  constexpr int IMG_A = GBM * BK * 2, IMG_B = GBN * BK * 2;  // per operand per stage (both layouts)
  constexpr int STAGE_BYTES = IMG_A + IMG_B;
  constexpr int PIECES = (GBM + GBN) * BK / 512 / NW;        // LDS-DMA pieces per wave per stage (A + B)
  constexpr int AI = SWAP ? TN : TM, AJ = SWAP ? TM : TN;    // accumulator sub-tile grid
  // XCD-aware remap (bijective): blocks b and b+8 share an XCD; give each XCD a contiguous run
  // of tiles so neighbouring tiles (same A row panel) share that XCD's L2
  int tile = blockIdx.x;
  int split = blockIdx.y;
  int prob = blockIdx.z;
  const int nsplit = gridDim.y;
  if (batch.xcd_plane) {
    // weight gradients: remap the whole (tile, split, problem) grid XCD-major, so the tiles of one
    // (K slice, problem) -- which share its dY / X panels -- run on one XCD's L2 instead of being
    // spread over the eight (C1: dW fetch bytes per launch 214 -> 166 MB)
    const int nwg = gridDim.x * nsplit * gridDim.z;
    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + nsplit * blockIdx.z);
    const int x = lin % 8, q = nwg / 8, rr = nwg % 8;
    const int l2 = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + lin / 8;
    tile = l2 % gridDim.x;
    split = (l2 / gridDim.x) % nsplit;
    prob = l2 / (gridDim.x * nsplit);
  }
  const GemmProblem& P = batch.p[prob];
  // (readfirstlane: values the compiler cannot rematerialise by re-loading the kernel argument; as plain
  // P.* reads it re-loaded lda in front of every K-step's DMA, an s_load plus a full lgkmcnt wait)
  const int M = __builtin_amdgcn_readfirstlane(P.M), N = __builtin_amdgcn_readfirstlane(P.N);
  const int K = __builtin_amdgcn_readfirstlane(P.K);
  const int tiles_n = (N + GBN - 1) / GBN;
  const int tiles_m = (M + GBM - 1) / GBM;
  const int ntiles = tiles_m * tiles_n;
  if (!batch.xcd_plane) {
    const int nwg = gridDim.x;
    const int x = tile % 8, q = nwg / 8, rr = nwg % 8;
    tile = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + tile / 8;
  }
  if (tile >= ntiles) return;
  GEMM_STAMP(0);
  GEMM_STAMP(5);
  GEMM_STAMP(6);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int ksteps = (K + BK - 1) / BK;
  const int kper = (ksteps + nsplit - 1) / nsplit;
  const int ks0 = split * kper;
  const int ks1 = min(ksteps, ks0 + kper);
  if (EPI == EPI_ATOMIC_F32 && ks0 >= ks1) return;  // nothing to add (a slab split still writes its zeros)

  // one LDS array (a second __shared__ object can make hipcc drain vmcnt before ds_reads):
  // the stage ring during the K loop, the fp32 output tile (EPI_ROWS x (GBN + 4)) in the epilogue
  constexpr int EPI_ROWS = (GBN >= 512 || (GBM == 128 && GBN == 256)) ? 32 : (GBM == 128 && MINB == 1) ? 128 : 64;
  constexpr int RING = ST * STAGE_BYTES, CTILE = EPI_ROWS * (GBN + 4) * 4;
  constexpr int LDS_MAIN = RING > CTILE ? RING : CTILE;
  // + the fused Q/K/V stage 2's W2 fragments (qkv2_stage_w2)
  constexpr int LDS_W2 = (SWAP && EPI == EPI_BIAS_TANH_BF16 && TL::NW == 4 && TL::BN == 128) ? QKV2_W2_LDS : 0;
  __shared__ __attribute__((aligned(1024))) char lds[LDS_MAIN + LDS_W2];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / TL::WN, wn = wave % TL::WN;

  f32x16 acc[AI][AJ];
#pragma unroll
  for (int i = 0; i < AI; ++i)
#pragma unroll
    for (int j = 0; j < AJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  if constexpr (SWAP && EPI == EPI_BIAS_TANH_BF16 && TL::NW == 4 && TL::BN == 128) {
    // fused Q/K/V stage 2: the accumulators start at bias / alpha, so the epilogue (short of
    // registers at 3 blocks per CU) holds no bias values
    if (P.qkv2_out) qkv2_stage_w2<TL>(P, lds + LDS_MAIN, n0, tid);  // read after the epilogue's barrier
    if (P.qkv2_out && P.bias) {
      const float ia = 1.0f / P.alpha;
      const int hh = (tid & 63) >> 5;
#pragma unroll
      for (int i = 0; i < AI; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int n = n0 + wn * TL::TN * 32 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * hh;
          const float bv = n < N ? P.bias[n] * ia : 0.0f;
#pragma unroll
          for (int j = 0; j < AJ; ++j) acc[i][j][e] = bv;
        }
    }
  }

  if (ks0 < ks1) {
    const int lda = __builtin_amdgcn_readfirstlane(P.lda), ldb = __builtin_amdgcn_readfirstlane(P.ldb);
    // (the operand base pointers likewise: an MN-contiguous operand's descriptor is rebuilt per K-step)
    auto sgpr_ptr = [](const bf16_t* q) {
      const uint64_t v = (uint64_t)(uintptr_t)q;
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
      return (const bf16_t*)(uintptr_t)(((uint64_t)hi << 32) | lo);
    };
    const bf16_t* const Ap = sgpr_ptr(P.A);
    const bf16_t* const Bp = sgpr_ptr(P.B);
    // buffer descriptors (range-checked: OOB pieces read 0) from the tile's first row for a
    // K-contiguous operand; an MN-contiguous operand's descriptor is made per K-step (op_rsrc)
    const i32x4 ra_kc = A_KC ? op_rsrc<true>(Ap, lda, M, K, m0, 0) : i32x4{0, 0, 0, 0};
    const i32x4 rb_kc = B_KC ? op_rsrc<true>(Bp, ldb, N, K, n0, 0) : i32x4{0, 0, 0, 0};
    auto ra = [&](int k0) { return A_KC ? ra_kc : op_rsrc<false>(Ap, lda, M, K, m0, k0); };
    auto rb = [&](int k0) { return B_KC ? rb_kc : op_rsrc<false>(Bp, ldb, N, K, n0, k0); };
    const int nk = ks1 - ks0;
    // one K-step: stage U of the ring holds K-step tt (tt % ST == U), the step prefetches K-step
    // tt + ST - 1 into stage (U + ST - 1) % ST. U is a compile-time constant (the loop below is
    // unrolled by ST) so the LDS offsets of the DMA writes and of the fragment reads are static:
    // with a dynamic stage index hipcc cannot separate them and drains vmcnt(0) before the
    // fragment reads, serialising every K-step behind its own prefetch.
    auto step = [&](int tt, auto UC) {
      constexpr int U = decltype(UC)::value;
      // stage U landed for this wave: allow the younger stages' pieces to stay in flight
      wait_vm(PIECES * min(ST - 2, nk - 1 - tt));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's pieces of stage U landed; the previous stage's reads done
      if (tt == 0) GEMM_STAMP(2);
      if (tt + ST - 1 < nk) {
        char* st = lds + ((U + ST - 1) % ST) * STAGE_BYTES;
        const int k0 = (ks0 + tt + ST - 1) * BK;
        issue_tile<BK, A_KC, GBM, NW>(ra(k0), st, lda, M, K, m0, k0, wave, lane);
        issue_tile<BK, B_KC, GBN, NW>(rb(k0), st + IMG_A, ldb, N, K, n0, k0, wave, lane);
      }
      const char* imgA = lds + U * STAGE_BYTES;
      const char* imgB = imgA + IMG_A;
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int j = 0; j < TM; ++j) fa[j] = frag<BK, A_KC, GBM>(imgA, wm * TM * 32 + 32 * j, s, lane);
#pragma unroll
        for (int i = 0; i < TN; ++i) fb[i] = frag<BK, B_KC, GBN>(imgB, wn * TN * 32 + 32 * i, s, lane);
#pragma unroll
        for (int i = 0; i < AI; ++i)
#pragma unroll
          for (int j = 0; j < AJ; ++j) {
            if (SWAP) acc[i][j] = mfma32(fb[i], fa[j], acc[i][j]);
            else acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
          }
      }
    };
#pragma unroll
    for (int t = 0; t < ST - 1; ++t)
      if (t < nk) {
        char* st = lds + t * STAGE_BYTES;
        const int k0 = (ks0 + t) * BK;
        issue_tile<BK, A_KC, GBM, NW>(ra(k0), st, lda, M, K, m0, k0, wave, lane);
        issue_tile<BK, B_KC, GBN, NW>(rb(k0), st + IMG_A, ldb, N, K, n0, k0, wave, lane);
      }
    GEMM_STAMP(1);
    int t = 0;
    for (; t + ST <= nk; t += ST) {
      step(t, std::integral_constant<int, 0>{});
      step(t + 1, std::integral_constant<int, 1>{});
      if constexpr (ST > 2) step(t + 2, std::integral_constant<int, (ST > 2 ? 2 : 0)>{});
      if constexpr (ST > 3) step(t + 3, std::integral_constant<int, (ST > 3 ? 3 : 0)>{});
    }
    if (t < nk) step(t, std::integral_constant<int, 0>{});
    if (ST > 2 && t + 1 < nk) step(t + 1, std::integral_constant<int, 1>{});
    if constexpr (ST > 3) { if (t + 2 < nk) step(t + 2, std::integral_constant<int, (ST > 3 ? 2 : 0)>{}); }
  }

  GEMM_STAMP(3);
  float alpha = P.alpha;
  if (P.alpha_ptr) alpha *= *P.alpha_ptr;
  // split-K into slabs: split s of the K loop writes its own fp32 slab (reduced by mmt_gemm_slab_reduce)
  float* o32 = P.o32 + (P.split_stride ? (int64_t)split * P.split_stride : (int64_t)0);
  const int h = lane >> 5, r = lane & 31;
  // the fused per-head Q/K/V stage 2 on the 128 x 128 tile only: next to the 256 x 256 tile's 128
  // accumulators it spills (the launcher refuses qkv2_out there; the engine then runs qkv2_fwd)
  if constexpr (SWAP && EPI == EPI_BIAS_TANH_BF16 && TL::NW == 4 && TL::BN == 128) {
    if (P.qkv2_out) {  // the per-head stage 2 of Q/K/V (uniform per problem)
      qkv2_fused<TL>(P, acc, lds, lds + LDS_MAIN, alpha, m0, n0, lane, wave);
      epilogue_swap<TL, EPI, EPI_ROWS, true>(P, acc, lds, o32, alpha, m0, n0, tid, lane, wave);
    } else {
      epilogue_swap<TL, EPI, EPI_ROWS>(P, acc, lds, o32, alpha, m0, n0, tid, lane, wave);
    }
  } else if constexpr (SWAP) {
    epilogue_swap<TL, EPI, EPI_ROWS>(P, acc, lds, o32, alpha, m0, n0, tid, lane, wave);
  } else {
    // acc[i][j]: rows = m (sub-tile i), cols = n (sub-tile j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * TN * 32 + 32 * j + r;
        if (n >= N) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * TM * 32 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (m < M) epi_scalar<EPI>(P, o32, alpha, m, n, acc[i][j][e]);
        }
      }
  }
  GEMM_STAMP(4);
}

// ---------------------------------------------------------------------------------------------
// MX-fp8 forward GEMM (C4's fp8 path): Y = X W^T with X [M][K], W [N][K] e4m3fn bytes and E8M0
// block exponents per 32 K elements, on v_mfma_scale_f32_32x32x64_f8f6f4 (2x the bf16 MFMA rate).
// Same structure as gemm_kernel (SWAP layout, LDS-DMA ring, XCD tile order, fused epilogues); a
// K-step is 128 fp8 = the 128-B image rows of the bf16 kernel's 64-element step, so the image
// geometry and swizzle are unchanged. Operand lane map (probed on gfx950: tools/probe/probe_mx.py):
// lane r + 32h of a 64-deep MFMA holds K elements [16h, 16h+16) and [32+16h, 48+16h) of row r in
// its 32 bytes, and its scale byte is the exponent of block h (K elements [32h, 32h+32)) of row r
// -> image chunks 4s + h and 4s + 2 + h, scale byte 2s + h of the row's K-step dword.
// ---------------------------------------------------------------------------------------------
template <int ROWS, int NW>
__device__ __forceinline__ void issue_tile_f8(const i32x4& rsrc, char* img, int ld, int rows_total, int K, int r0,
                                              int k0, int wave, int lane) {
  constexpr int PPW = ROWS * 128 / 1024 / NW;  // 1-KiB pieces per wave: 8 rows of 128 B
#pragma unroll
  for (int u = 0; u < PPW; ++u) {
    const int i = wave * PPW + u;
    const int row = 8 * i + lane / 8;
    const int chunk = kc_swz<64>(lane % 8, row);
    const int grow = r0 + row, gk = k0 + chunk * 16;
    const int voff = (grow < rows_total && gk < K) ? row * ld + gk : 0x7fffffff;  // rsrc from row r0
    dma16(rsrc, __builtin_amdgcn_readfirstlane(lds_u32(img + i * 1024)), voff);
  }
}

__device__ __forceinline__ i32x8 frag_f8(const char* img, int sb, int s, int lane) {
  const int row = sb + (lane & 31), h = lane >> 5;
  const u32x4 lo = *reinterpret_cast<const u32x4*>(img + row * 128 + kc_swz<64>(4 * s + h, row) * 16);
  const u32x4 hi = *reinterpret_cast<const u32x4*>(img + row * 128 + kc_swz<64>(4 * s + 2 + h, row) * 16);
  return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

// one 4-B-per-lane LDS-DMA (buffer_load_dword ... lds): LDS[lds_addr + 4*lane] = buffer[voff]
__device__ __forceinline__ void dma4(const i32x4& rsrc, uint32_t lds_addr, int voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :
               : "s"(lds_addr), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}

template <class TL, int EPI>
__global__ __launch_bounds__(TL::NT) void gemm_f8_kernel(GemmBatch batch) {
  constexpr int GBM = TL::BM, GBN = TL::BN, NW = TL::NW, NT = TL::NT, TM = TL::TM, TN = TL::TN;
  constexpr int ST = 2, KS = 128;                           // stages, K elements per step
  constexpr int IMG_A = GBM * 128, IMG_B = GBN * 128;       // e4m3 tiles
  constexpr int SC_A = GBM * 4, SC_B = GBN * 4;             // E8M0 dwords of the step, one per row
  constexpr int STAGE_BYTES = IMG_A + IMG_B + SC_A + SC_B;
  constexpr int SCDMA = (GBM + GBN) / 64;                   // dword LDS-DMAs of the exponents per stage
  static_assert(SCDMA <= NW, "one exponent DMA per wave at most");
  const GemmProblem& P = batch.p[blockIdx.z];
  const int M = P.M, N = P.N, K = P.K;
  const int tiles_n = (N + GBN - 1) / GBN, tiles_m = (M + GBM - 1) / GBM;
  int tile = blockIdx.x;
  {
    const int nwg = gridDim.x;
    const int x = tile % 8, q = nwg / 8, rr = nwg % 8;
    tile = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + tile / 8;
  }
  if (tile >= tiles_m * tiles_n) return;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int nk = (K + KS - 1) / KS;
  constexpr int EPI_ROWS = GBM == 128 ? 128 : 64;
  constexpr int RING = ST * STAGE_BYTES, CTILE = EPI_ROWS * (GBN + 4) * 4;
  __shared__ __attribute__((aligned(1024))) char lds[RING > CTILE ? RING : CTILE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / TL::WN, wn = wave % TL::WN;
  const int h = lane >> 5, r = lane & 31;
  f32x16 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  // descriptors from the tile's first rows (32-bit offsets: see op_rsrc)
  const i32x4 ra = op_rsrc<true>(P.A, P.lda, M, K, m0, 0, 1);
  const i32x4 rb = op_rsrc<true>(P.B, P.ldb, N, K, n0, 0, 1);
  const i32x4 rsa = op_rsrc<true>(P.sa, P.lds_a, M, K, m0, 0, 1);
  const i32x4 rsb = op_rsrc<true>(P.sb, P.lds_b, N, K, n0, 0, 1);
  // the E8M0 dwords of a K-step ride the ring next to the tiles: wave w < SCDMA brings 64 rows' dwords
  // (rows past M / N land as zeros: exponent 2^-127 on zero-filled values)
  auto issue_scales = [&](char* st, int t) {
    if (wave >= SCDMA) return;
    const bool isa = wave < GBM / 64;
    const int row = (isa ? wave : wave - GBM / 64) * 64 + lane;
    const int grow = (isa ? m0 : n0) + row;
    const int voff = grow < (isa ? M : N) ? row * (isa ? P.lds_a : P.lds_b) + 4 * t : 0x7fffffff;
    char* dst = st + IMG_A + IMG_B + (isa ? 0 : SC_A) + (isa ? wave : wave - GBM / 64) * 256;
    dma4(isa ? rsa : rsb, __builtin_amdgcn_readfirstlane(lds_u32(dst)), voff);
  };
  issue_tile_f8<GBM, NW>(ra, lds, P.lda, M, K, m0, 0, wave, lane);
  issue_tile_f8<GBN, NW>(rb, lds + IMG_A, P.ldb, N, K, n0, 0, wave, lane);
  issue_scales(lds, 0);
  for (int t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage t landed for every wave; stage t-1's reads are done
    if (t + 1 < nk) {
      char* st = lds + ((t + 1) & 1) * STAGE_BYTES;
      issue_tile_f8<GBM, NW>(ra, st, P.lda, M, K, m0, (t + 1) * KS, wave, lane);
      issue_tile_f8<GBN, NW>(rb, st + IMG_A, P.ldb, N, K, n0, (t + 1) * KS, wave, lane);
      issue_scales(st, t + 1);
    }
    const char* imgA = lds + (t & 1) * STAGE_BYTES;
    const char* imgB = imgA + IMG_A;
    const uint32_t* scA = reinterpret_cast<const uint32_t*>(imgB + IMG_B);
    const uint32_t* scB = scA + GBM;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      // B fragments for the sub-step, A fragments one at a time (32-byte fragments)
      i32x8 fb[TN];
      uint32_t sb[TN];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        fb[i] = frag_f8(imgB, wn * TN * 32 + 32 * i, s, lane);
        sb[i] = scB[wn * TN * 32 + 32 * i + r] >> (8 * (2 * s + h));
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const i32x8 fa = frag_f8(imgA, wm * TM * 32 + 32 * j, s, lane);
        const uint32_t sa = scA[wm * TM * 32 + 32 * j + r] >> (8 * (2 * s + h));
#pragma unroll
        for (int i = 0; i < TN; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fb[i], fa, acc[i][j], 0, 0, 0, (int)sb[i], 0,
                                                                       (int)sa);
      }
    }
  }
  float alpha = P.alpha;
  if (P.alpha_ptr) alpha *= *P.alpha_ptr;
  epilogue_swap<TL, EPI, EPI_ROWS>(P, acc, lds, P.o32, alpha, m0, n0, tid, lane, wave);
}


template <class TL, int BK, int ST, bool A_KC, bool B_KC, bool SWAP, int EPI, int MINB = 1>
static void launch_v(const GemmBatch& b, dim3 grid, hipStream_t s) {
#ifdef MMT_GEMM_STAMPS
  GemmBatch bs = b;
  bs.stamps = g_stamps;
  hipLaunchKernelGGL((gemm_kernel<TL, BK, ST, A_KC, B_KC, SWAP, EPI, MINB>), grid, dim3(TL::NT), 0, s, bs);
#else
  hipLaunchKernelGGL((gemm_kernel<TL, BK, ST, A_KC, B_KC, SWAP, EPI, MINB>), grid, dim3(TL::NT), 0, s, b);
#endif
}

template <class TL>
static int max_tiles(const GemmBatch& b, int* total) {
  int maxtiles = 0, sum = 0;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    const int t = ((P.M + TL::BM - 1) / TL::BM) * ((P.N + TL::BN - 1) / TL::BN);
    maxtiles = t > maxtiles ? t : maxtiles;
    sum += t;
  }
  if (total) *total = sum;
  return maxtiles;
}

// split-K factor of a weight-gradient launch (splits <= 0: automatic). Every split adds one fp32
// atomic per output element and an epilogue, so aim at ~2 blocks per CU for the 128x128 tile and
// ~1 for the 256x256 one, keeping >= 8 K-steps per split. Measured at C1 (128x128, grouped
// launches): 8 tiles 44.5 -> 29.2 us going from 8 to 32 splits, 24 tiles 50.7 -> 64.9 us from 8 to 22.
template <class TL>
static int auto_splits(const GemmBatch& b, int splits) {
  if (splits > 0) return splits;
  int tiles = 0, maxk = 0;
  max_tiles<TL>(b, &tiles);
  for (int g = 0; g < b.count; ++g) maxk = b.p[g].K > maxk ? b.p[g].K : maxk;
  if (tiles <= 0) return 1;
  static const int env_target = [] {
    const char* e = getenv("MMT_WGRAD_BLOCKS");  // tuning knob: blocks per weight-gradient launch
    return e ? atoi(e) : 0;
  }();
  // ~128 blocks: the weight gradients run on the side stream next to the data-gradient chain, so
  // half the chip for longer beats the whole chip with twice the split-K slab traffic (measured at
  // C1: 128 -> 9.97-10.28 ms/step, 256 -> 10.21-10.50, 64 -> 10.6)
  const int target = env_target > 0 ? env_target : b.dw_blocks > 0 ? b.dw_blocks : 128;
  const int cap = 32;
  const int s = target / tiles;
  const int maxs = std::max(1, std::min(cap, maxk / 512));
  return std::max(1, std::min(s, maxs));
}

// 256x256 pipeline (MMT_GEMM_BIG_VARIANT): 0 = BK 64 x 2 stages, 1 = BK 32 x 4 (three K-steps in
// flight), 2 = BK 32 x 3. Round 4 also built a software-pipelined K-step (the next sub-step's fragments
// read while this one's MFMAs issue, the prefetch pieces spread between MFMAs) and a persistent
// 256 x 256 kernel that prefetches the next tile's first stage under the last K-step and the epilogue.
// Both won standalone (tools/gemm_bench.py: 4096^3 1136 -> 1180 TF/s, C4 ffn0 889 -> 915) and lost in
// the training step beside the side stream (C1 8.78 -> 8.88 ms/step, target 20.47 -> 20.98), so they
// were removed at the end of round 4.
// Default: BK 32 x 4 for the weight gradients (both operands MN-contiguous, K = B*T: 128+ K-steps, the
// deeper ring keeps three in flight; C1 *_dw family 3.44 -> 3.20 ms/step live, C3 73.8 -> 69.4),
// BK 64 x 2 for the rest (the forward / data-gradient 256 x 256 launches measured 0.3-0.9 % slower
// at BK 32 x 4 in C3 / C4: profiles/r4z_big_variant_ab.txt). MMT_GEMM_BIG_VARIANT sets all of them.
static int g_big_variant = [] {
  const char* e = getenv("MMT_GEMM_BIG_VARIANT");
  return e ? atoi(e) : -1;
}();

// default 128 x 128 pipelines (build-time, tools/build_variant.py A/B): bf16-output epilogues at 3
// blocks per CU (variant 6: BK 32 x 2), the others at 2 (variant 0: BK 64 x 2). Deeper rings lose
// in the step (round 4, profiles/r4m_ab.txt: variant 5 for the former C1 +0.6 %, variants 2 / 4 for
// the latter C1 +0.6 / +5.5 %, target +0.5 / +5.3 %)
#ifndef MMT_OCC3_VARIANT
#define MMT_OCC3_VARIANT 6
#endif
#ifndef MMT_DEF_VARIANT
#define MMT_DEF_VARIANT 0
#endif
hipError_t mmt_launch_gemm8(const GemmBatch& b, int epi, bool a_kc, bool b_kc, dim3 grid, hipStream_t s);  // mmt_gemm8.hip
// the (operand layouts, epilogue) pairs mmt_gemm8.hip instantiates
constexpr bool gemm8_supports(bool akc, bool bkc, int epi) {
  return (akc && bkc && (epi == EPI_STORE_BF16 || epi == EPI_BIAS_TANH_BF16 || epi == EPI_BIAS_RELU_BF16 ||
                         epi == EPI_BIAS_RESID_F32 || epi == EPI_STORE_F32 || epi == EPI_ACC_F32)) ||
         (akc && !bkc && (epi == EPI_STORE_BF16 || epi == EPI_DTANH_BF16 || epi == EPI_DRELU_BF16 ||
                          epi == EPI_STORE_F32 || epi == EPI_ACC_F32 || epi == EPI_LN_BWD_F32)) ||
         (!akc && !bkc && (epi == EPI_STORE_F32 || epi == EPI_ACC_F32));
}

static bool gemm8_ln_on();

static bool gemm8_on() {
  // default on (round 5): C4 355 -> 350 ms/step, C3 153.3 -> 152.4, target / C1 neutral (same-box A/B,
  // profiles/r5_gemm8_mlp2_ab.txt); MMT_GEMM8=0 restores the 2-stage 256 x 256 ring everywhere
  static const int env = [] {
    const char* e = getenv("MMT_GEMM8");
    return e ? atoi(e) : 1;
  }();
  return g_gemm8_rt >= 0 ? g_gemm8_rt != 0 : env != 0;
}

// the row-wide (N = 256) LayerNorm-fused launches on the ping-pong kernel: MMT_GEMM8_LN=0 keeps them on the
// 2-stage ring (variant bit 17 / 18 still force the ping-pong kernel on / off for the tests)
static bool gemm8_ln_on() {
  static const bool env = [] {
    const char* e = getenv("MMT_GEMM8_LN");
    return e ? atoi(e) != 0 : true;
  }();
  if (g_gemm8_rt >= 0) return g_gemm8_rt == 1;
  return gemm8_on() && env;
}

// K threshold 1024 (round 2 c): at K = 512 (d512 forward GEMMs and data gradients) the 128x128 tile at
// 2-3 blocks per CU overlaps one block's epilogue with the others' K loops and shares the chip with
// the side stream better than the single 256x256 block per CU (target step 23.13 -> 22.73 ms)
static int g_big_kmin = [] {
  const char* e = getenv("MMT_GEMM_BIG_KMIN");
  return e ? atoi(e) : 1024;
}();
// MMT_GEMM_T2=1: the big launches with K below the 256 x 256 tile's threshold (K = 512: the d512 FFN and
// cross-attention K/V products the ping-pong kernel takes by default) on a 128 x 256 tile of 4 waves (TileL's
// per-wave 128 x 64) at two workgroups per CU (BK 32 x 3 stages: 72 KiB each), so one workgroup's prologue /
// epilogue overlaps the other's K loop
using TileM = TileCfg<1, 4, 4, 2>;
static int g_gemm_t2 = [] {
  const char* e = getenv("MMT_GEMM_T2");
  return e ? atoi(e) : 0;
}();
extern "C" int mmt_gemm_set_t2(int v) {
  const int old = g_gemm_t2;
  g_gemm_t2 = v;
  return old;
}

template <bool A_KC, bool B_KC, bool SWAP, int EPI>
static hipError_t launch_t(const GemmBatch& b, int splits, bool big, hipStream_t s) {
  if (b.count == 0) return hipSuccess;
  if constexpr (SWAP && EPI != EPI_ATOMIC_F32) {
    if (big && (g_gemm_t2 || b.tile_hint == 1)) {
      int maxk = 0;
      for (int g = 0; g < b.count; ++g) maxk = std::max(maxk, b.p[g].K);
      if (maxk < g_big_kmin) {
        const int mt = max_tiles<TileM>(b, nullptr);
        if (mt == 0) return hipSuccess;
        launch_v<TileM, 32, 3, A_KC, B_KC, SWAP, EPI, 2>(b, dim3(mt, std::max(1, splits), b.count), s);
        return hipGetLastError();
      }
    }
  }
  if (big) {
    const int mt = max_tiles<TileL>(b, nullptr);
    if (mt == 0) return hipSuccess;
    dim3 grid(mt, EPI == EPI_ATOMIC_F32 ? auto_splits<TileL>(b, splits) : std::max(1, splits), b.count);
    // forward / backward-data products on the ping-pong kernel; the weight gradients (both operands
    // MN-contiguous) only with MMT_GEMM8_DW=1: standalone 2-4 % faster, but on the side stream beside the
    // main stream's attention backward the step measured slower (C1 attention backward 198 -> 207 us live,
    // the *_dw family 107 -> 113 us; profiles/r5_gemm8_mlp2_ab.txt)
    if constexpr (SWAP && gemm8_supports(A_KC, B_KC, EPI)) {
      static const bool dw8 = [] {
        const char* e = getenv("MMT_GEMM8_DW");
        return e ? atoi(e) != 0 : false;
      }();
      // (mmt_gemm_set_variant bit 17 forces it everywhere: the kernel tests)
      if (gemm8_on() && (A_KC || dw8 || g_gemm8_rt == 1)) return mmt_launch_gemm8(b, EPI, A_KC, B_KC, grid, s);
    }
    const int bv = g_gemm_big_variant_rt ? g_gemm_big_variant_rt
                   : g_big_variant >= 0  ? g_big_variant
                   : (!A_KC && !B_KC)    ? 1
                                         : 0;
    switch (bv) {
      case 1: launch_v<TileL, 32, 4, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
      case 2: launch_v<TileL, 32, 3, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
      // BK 32 x 2 (66.5 KiB with the epilogue tile): leaves room on its CU for an 80 KiB attention-backward
      // workgroup beside it (measured for the weight gradients)
      case 3: launch_v<TileL, 32, 2, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
      default: launch_v<TileL, 64, 2, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
    }
    return hipGetLastError();
  }
  const int mt = max_tiles<TileS>(b, nullptr);
  if (mt == 0) return hipSuccess;
  dim3 grid(mt, EPI == EPI_ATOMIC_F32 ? auto_splits<TileS>(b, splits) : std::max(1, splits), b.count);
  // default policy (variant knob unset): bf16-output epilogues with no aux operand stage 64 rows
  // per epilogue pass and run 3+ blocks per CU (variant 6: 33 KB of LDS instead of 66 KB), which
  // overlaps one block's short K loop with the others' prologue / stores; epilogues that read an aux
  // or residual operand or store fp32 measured faster at 2 blocks per CU with the 64-deep ring
  // (profiles/r2_gemm_bench.txt)
  constexpr bool occ3 = EPI == EPI_STORE_BF16 || EPI == EPI_BIAS_TANH_BF16 || EPI == EPI_BIAS_RELU_BF16;
  static const int env_dw = [] {  // tuning knob: pipeline variant of the 128x128 weight-gradient GEMMs
    const char* e = getenv("MMT_GEMM_DW_VARIANT");
    return e ? atoi(e) : -1;
  }();
  // (a 256 x 128 tile at two blocks per CU won standalone on the target ffn0, 214 -> 194 us, but not in
  // the step beside the side stream, 20.21 -> 20.37 ms: profiles/r3y_tilem_ab.txt; removed in round 4)
  // (the ReLU' epilogue reading bits has no 16-B aux operand left, but at 3 blocks per CU it measured
  // neutral: C1 8.558 vs 8.555, target 19.937 vs 19.935 ms, profiles/r5ac_drelu_occ3_ab.txt)
  const int var = EPI == EPI_ATOMIC_F32 ? g_gemm_variant_dw
                  : (!A_KC && !B_KC && env_dw >= 0) ? env_dw
                  : (g_gemm_variant >= 0 ? g_gemm_variant : occ3 ? MMT_OCC3_VARIANT : MMT_DEF_VARIANT);
  switch (var) {
    case 1: launch_v<TileS, 32, 2, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
    case 2: launch_v<TileS, 32, 3, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
    case 3: launch_v<TileS, 32, 4, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
    case 4: launch_v<TileS, 64, 3, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
    case 5: launch_v<TileS, 32, 3, A_KC, B_KC, SWAP, EPI, 3>(b, grid, s); break;
    case 6: launch_v<TileS, 32, 2, A_KC, B_KC, SWAP, EPI, 3>(b, grid, s); break;
    default: launch_v<TileS, 64, 2, A_KC, B_KC, SWAP, EPI>(b, grid, s); break;
  }
  return hipGetLastError();
}

// tile policy: the 256x256 tile where every problem of the launch fills it (M, N >= 256) and the
// K loop is long enough to amortise its prologue/epilogue (K >= g_big_kmin; weight gradients
// always qualify: K = B*T). MMT_GEMM_BIG=0 disables it, MMT_GEMM_BIG_KMIN sets the K threshold.
static int g_big_mode = [] {
  const char* e = getenv("MMT_GEMM_BIG");
  return e ? atoi(e) : 1;
}();

// K threshold of the ping-pong 256 x 256 kernel for launches with many tiles: at K = 512 it wins where
// the launch has >= 4 tiles per CU (the target's ffn0 and ffn2 dX: 221 -> 177 and 252 -> 230 us
// standalone; smaller launches leave CUs idle or lose the 128 x 128 tile's 2-3 blocks per CU beside the
// side stream: every K = 512 launch on it measured +1 % on the target step)
static int g_gemm8_kmin = [] {
  const char* e = getenv("MMT_GEMM8_KMIN");
  return e ? atoi(e) : 512;
}();
static int g_gemm8_min_tiles = [] {
  const char* e = getenv("MMT_GEMM8_MIN_TILES");
  return e ? atoi(e) : 1024;
}();
static bool use_big(const GemmBatch& b) {
  if (!g_big_mode || b.count == 0) return false;
  bool big = true, qkv2 = false;
  int tiles = 0;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    if (P.M < TileL::BM || P.N < TileL::BN) return false;
    if (P.K < g_big_kmin && !g_force_big_rt) big = false;
    qkv2 = qkv2 || P.qkv2_out != nullptr;
    tiles += ((P.M + 255) / 256) * ((P.N + 255) / 256);
  }
  if (big) return true;
  // shorter K on the ping-pong kernel: only big launches, and never the fused Q/K/V stage 2 (128 x 128 only)
  if (!gemm8_on() || qkv2 || tiles < g_gemm8_min_tiles) return false;
  for (int g = 0; g < b.count; ++g)
    if (b.p[g].K < g_gemm8_kmin) return false;
  return true;
}

// the fused per-head Q/K/V stage 2 (qkv2_fused): forward tanh epilogue only, hh 16 or 32, 16-B stores,
// whole hh-blocks (N % hh == 0)
static bool qkv2_ok(const GemmProblem& P, int epi, bool fwd) {
  if (!P.qkv2_out) return true;
  // (no alpha_ptr, alpha != 0: the accumulators start at bias / alpha)
  return epi == EPI_BIAS_TANH_BF16 && fwd && (P.qkv2_hh == 16 || P.qkv2_hh == 32) && P.N % P.qkv2_hh == 0 &&
         !P.alpha_ptr && P.alpha != 0.0f &&
         P.qkv2_w2 && !(P.qkv2_ld & 7) && !((uintptr_t)P.qkv2_out & 15) && !((uintptr_t)P.qkv2_w2 & 15);
}

// tile-local operand spans (op_rsrc) must stay below 2^31 bytes: at most 512 rows (or a 64-deep K-step)
// of the leading dimension plus K (weight-gradient slabs and outputs use 64-bit offsets)
static bool gemm_span_ok(const GemmBatch& b) {
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    if (P.M < 0 || P.N < 0 || P.K < 0 || P.lda < 0 || P.ldb < 0) return false;
    if ((int64_t)(512 + 1) * std::max(P.lda, P.ldb) * 2 + (int64_t)P.K * 2 >= ((int64_t)1 << 31)) return false;
  }
  return true;
}

hipError_t mmt_launch_gemm(const GemmBatch& b, bool a_kc, bool b_kc, int epi, int splits, hipStream_t s) {
  if (!gemm_span_ok(b)) return hipErrorInvalidValue;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    // 16-byte LDS-DMA pieces need 8-element-aligned leading dimensions and 16-byte aligned bases
    if ((P.lda & 7) || (P.ldb & 7) || (((uintptr_t)P.A | (uintptr_t)P.B) & 15)) return hipErrorInvalidValue;
    if (!qkv2_ok(P, epi, a_kc && b_kc)) return hipErrorInvalidValue;
  }
  const bool big = use_big(b);
  for (int g = 0; g < b.count; ++g)
    if (big && b.p[g].qkv2_out) return hipErrorInvalidValue;  // fused stage 2: 128 x 128 tile only
  if (a_kc && b_kc) {
    switch (epi) {
      case EPI_STORE_BF16: return launch_t<true, true, true, EPI_STORE_BF16>(b, 1, big, s);
      case EPI_BIAS_TANH_BF16: return launch_t<true, true, true, EPI_BIAS_TANH_BF16>(b, 1, big, s);
      case EPI_BIAS_RELU_BF16: return launch_t<true, true, true, EPI_BIAS_RELU_BF16>(b, 1, big, s);
      case EPI_BIAS_RESID_F32: return launch_t<true, true, true, EPI_BIAS_RESID_F32>(b, 1, big, s);
      case EPI_STORE_F32: return launch_t<true, true, true, EPI_STORE_F32>(b, 1, big, s);
      case EPI_ACC_F32: return launch_t<true, true, true, EPI_ACC_F32>(b, 1, big, s);
      default: break;
    }
  } else if (a_kc && !b_kc) {
    switch (epi) {
      case EPI_STORE_BF16: return launch_t<true, false, true, EPI_STORE_BF16>(b, 1, big, s);
      case EPI_DTANH_BF16: return launch_t<true, false, true, EPI_DTANH_BF16>(b, 1, big, s);
      case EPI_DRELU_BF16: return launch_t<true, false, true, EPI_DRELU_BF16>(b, 1, big, s);
      case EPI_STORE_F32: return launch_t<true, false, true, EPI_STORE_F32>(b, 1, big, s);
      case EPI_ACC_F32: return launch_t<true, false, true, EPI_ACC_F32>(b, 1, big, s);
      default: break;
    }
  } else if (!a_kc && !b_kc) {
    switch (epi) {
      case EPI_ATOMIC_F32: return launch_t<false, false, false, EPI_ATOMIC_F32>(b, splits, big, s);
      case EPI_STORE_F32: return launch_t<false, false, true, EPI_STORE_F32>(b, splits, big, s);
      case EPI_ACC_F32: return launch_t<false, false, true, EPI_ACC_F32>(b, 1, big, s);
      default: break;
    }
  } else {
    switch (epi) {
      case EPI_ATOMIC_F32: return launch_t<false, true, false, EPI_ATOMIC_F32>(b, splits, big, s);
      case EPI_STORE_F32: return launch_t<false, true, true, EPI_STORE_F32>(b, 1, big, s);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------
// Weight gradients dW[M, N] += alpha * dY[K, M]^T X[K, N] (both operands MN-contiguous, K = rows).
// K = B*T is long and M x N small, so the K loop is split over workgroups. Each split writes a
// plain fp32 slab (row-coalesced 16-B stores of the staged epilogue) and one reduce pass adds the
// slabs into the gradient. Measured alternatives (C1, same box): per-element fp32
// atomics (16.7 M per FFN launch, ~60 of its ~85 us), and three in-kernel reductions with no
// reduce launch (pairwise tree, every-split slice combine behind a per-tile arrival barrier, last
// arriver) were all slower than this: the reduce launch runs on the side stream beside the
// data-gradient chain, while an in-kernel reduction holds CUs waiting or reading serially.
// ---------------------------------------------------------------------------------------------
struct SlabProblem {
  const float* slab;  // [splits][M * N]
  float* out;         // [M][ldc]
  int M, N, ldc;
  int64_t stride;     // elements per slab
};
struct SlabBatch {
  SlabProblem p[MMT_MAX_GROUP];
  int count, splits;
};

__global__ __launch_bounds__(256) void slab_reduce_kernel(SlabBatch b) {
  const SlabProblem& P = b.p[blockIdx.y];
  const bool vec = (P.N % 4 == 0) && (P.ldc % 4 == 0) && (((uintptr_t)P.out & 15) == 0);
  // kernel arguments the split loop reads, as values (read through P they were re-loaded per split group)
  const int splits = __builtin_amdgcn_readfirstlane(b.splits);
  const int64_t stride = P.stride;
  const float* const slab = P.slab;
  if (vec) {
    const int64_t n4 = (int64_t)P.M * P.N / 4;
    const int N4 = P.N / 4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
      // 8 slab loads in flight per thread (independent partial sums)
      f32x4 part[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) part[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      int sp = 0;
      for (; sp + 8 <= splits; sp += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) part[u] += reinterpret_cast<const f32x4*>(slab + (sp + u) * stride)[i];
      }
      for (; sp < splits; ++sp) part[0] += reinterpret_cast<const f32x4*>(slab + sp * stride)[i];
      const f32x4 acc = ((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]));
      const int m = (int)(i / N4), c = (int)(i % N4) * 4;
      float* o = P.out + (int64_t)m * P.ldc + c;
      *reinterpret_cast<f32x4*>(o) = *reinterpret_cast<const f32x4*>(o) + acc;
    }
  } else {
    const int64_t n = (int64_t)P.M * P.N;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
      float acc = P.slab[i];
      for (int sp = 1; sp < b.splits; ++sp) acc += P.slab[sp * P.stride + i];
      P.out[(int64_t)(i / P.N) * P.ldc + i % P.N] += acc;
    }
  }
}

// MMT_DW_SMALL=1: every weight gradient on the 128 x 128 tile (4x the tiles of the 256 x 256 one, so a
// quarter of the K splits and of the split-K slab traffic at the ~128-block side-stream target)
static const int g_dw_small = [] {
  const char* e = getenv("MMT_DW_SMALL");
  return e ? atoi(e) : 0;
}();
// (GemmBatch::tile_hint 2: this launch on the 128 x 128 tile, 64 KiB of LDS, which fits on a CU beside the
// main stream's 80 KiB attention-backward workgroups where the 256 x 256 one's 128 KiB does not)
static bool use_big_dw(const GemmBatch& b) { return !g_dw_small && b.tile_hint != 2 && use_big(b); }

hipError_t mmt_launch_gemm_wgrad(const GemmBatch& b, float* slab, int64_t slab_bytes, hipStream_t s) {
  if (b.count == 0) return hipSuccess;
  if (!gemm_span_ok(b)) return hipErrorInvalidValue;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    if ((P.lda & 7) || (P.ldb & 7) || (((uintptr_t)P.A | (uintptr_t)P.B) & 15)) return hipErrorInvalidValue;
  }
  const bool big = use_big_dw(b);
  int splits = big ? auto_splits<TileL>(b, 0) : auto_splits<TileS>(b, 0);
  int64_t per = 0;  // slab elements of one split over all problems (each slab 16-B aligned)
  for (int g = 0; g < b.count; ++g) per += ((int64_t)b.p[g].M * b.p[g].N + 3) / 4 * 4;
  if (slab) {
    const int64_t cap = slab_bytes / (int64_t)sizeof(float) / std::max<int64_t>(1, per);
    if (splits > cap) splits = (int)cap;
  } else {
    splits = 1;
  }
  // XCD-major remap of the (tile, split, problem) grid (MMT_DW_XCD_PLANE=0 turns it off)
  static const int xcd_plane = [] {
    const char* e = getenv("MMT_DW_XCD_PLANE");
    return e ? atoi(e) : 1;
  }();
  if (splits <= 1) {  // one K pass: accumulate straight into the gradient
    GemmBatch d = b;
    d.xcd_plane = xcd_plane;
    for (int g = 0; g < d.count; ++g) d.p[g].split_stride = 0;
    return launch_t<false, false, true, EPI_ACC_F32>(d, 1, big, s);
  }
  GemmBatch d = b;
  d.xcd_plane = xcd_plane;
  SlabBatch sb{};
  sb.count = b.count;
  sb.splits = splits;
  int64_t off = 0;
  for (int g = 0; g < d.count; ++g) {
    GemmProblem& P = d.p[g];
    const int64_t mn = ((int64_t)P.M * P.N + 3) / 4 * 4;
    sb.p[g] = SlabProblem{slab + off, P.o32, P.M, P.N, P.ldc, per};
    P.o32 = slab + off;
    P.ldc = P.N;
    P.split_stride = per;
    off += mn;
  }
  hipError_t e = launch_t<false, false, true, EPI_STORE_F32>(d, splits, big, s);
  if (e != hipSuccess) return e;
  int64_t maxn4 = 0;
  for (int g = 0; g < b.count; ++g) maxn4 = std::max<int64_t>(maxn4, ((int64_t)b.p[g].M * b.p[g].N + 3) / 4);
  const int blocks = (int)std::min<int64_t>(4096, (maxn4 + 255) / 256);
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(blocks, b.count), dim3(256), 0, s, sb);
  return hipGetLastError();
}



bool mmt_gemm_wgrad_big(const GemmBatch& b) { return use_big_dw(b); }

bool mmt_gemm_resid_ln_ok(const GemmBatch& b) {
  if (b.count == 0) return false;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    if ((P.N != TileL::BN && P.N != TileW::BN) || P.N != b.p[0].N || !P.resid || !P.o32 || (P.ldc & 3) ||
        (P.ldres & 3) || (P.o16 && (P.ldo16 & 7)) || (P.lda & 7) || (P.ldb & 7) ||
        (((uintptr_t)P.A | (uintptr_t)P.B | (uintptr_t)P.o32 | (uintptr_t)P.resid) & 15))
      return false;
    if (P.lnf_y && (!P.lnf_gamma || !P.lnf_beta || !P.lnf_mean || !P.lnf_rstd ||
                    (((uintptr_t)P.lnf_y | (uintptr_t)P.lnf_gamma | (uintptr_t)P.lnf_beta) & 15)))
      return false;
  }
  return true;
}

// ring depth of the 128 x 512 row-wide GEMMs (LayerNorm backward / forward fused): 3 stages of BK 32
// (120 KiB, one block per CU) against 2 (80 KiB, two blocks per CU): target step 20.39 -> 19.64 ms
// with the LayerNorm-backward GEMMs on it, 4 stages equal to 3 (profiles/r4k_ab.txt); at 2 stages the
// next K-step's DMA had one 32-deep step of MFMAs to hide under
#ifndef MMT_GEMM_W_ST
#define MMT_GEMM_W_ST 3
#endif
hipError_t mmt_launch_gemm_resid_ln(const GemmBatch& b, hipStream_t s) {
  if (!mmt_gemm_resid_ln_ok(b) || !gemm_span_ok(b)) return hipErrorInvalidValue;
  // a tile as wide as the row whatever K (its block owns whole rows): 256 x 256 (as launch_t's big
  // path, variant 0) at C = 256, 128 x 512 at C = 512
  if (b.p[0].N == TileW::BN) {
    const int mt = max_tiles<TileW>(b, nullptr);
    if (mt == 0) return hipSuccess;
    launch_v<TileW, 32, MMT_GEMM_W_ST, true, true, true, EPI_BIAS_RESID_F32>(b, dim3(mt, 1, b.count), s);
  } else {
    const int mt = max_tiles<TileL>(b, nullptr);
    if (mt == 0) return hipSuccess;
    // the ping-pong kernel takes the 256 x 256 row-wide tile too (same epilogue, LayerNorm included)
    if (gemm8_ln_on()) return mmt_launch_gemm8(b, EPI_BIAS_RESID_F32, true, true, dim3(mt, 1, b.count), s);
    launch_v<TileL, 64, 2, true, true, true, EPI_BIAS_RESID_F32>(b, dim3(mt, 1, b.count), s);
  }
  return hipGetLastError();
}

bool mmt_gemm_ln_bwd_ok(const GemmBatch& b) {
  if (b.count == 0) return false;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    if ((P.N != TileL::BN && P.N != TileW::BN) || P.N != b.p[0].N || !P.resid || !P.o32 || !P.ln_gamma || !P.ln_mean || !P.ln_rstd || !P.ln_dgamma ||
        !P.ln_dbeta || (P.ldc & 3) || (P.ldres & 3) || (P.o16 && (P.ldo16 & 7)) || (P.lda & 7) || (P.ldb & 7) ||
        (((uintptr_t)P.A | (uintptr_t)P.B | (uintptr_t)P.o32 | (uintptr_t)P.resid | (uintptr_t)P.ln_gamma |
          (uintptr_t)P.o16) & 15))  // (o16: the epilogue's 16-B dropout-masked copy stores)
      return false;
  }
  return true;
}

hipError_t mmt_launch_gemm_ln_bwd(const GemmBatch& b, hipStream_t s) {
  if (!mmt_gemm_ln_bwd_ok(b) || !gemm_span_ok(b)) return hipErrorInvalidValue;
  // a tile as wide as the row, whatever K: its block owns whole rows of the LayerNorm (C = 256:
  // 256 x 256; C = 512: 128 x 512 at BK 32 x 2 stages = 80 KiB of ring; BK 64 measured neutral, a
  // 128 x 256 tile at C = 256 slower: 63.7 -> 92.9 us per launch, profiles/r3i_lnb_tile_ab.txt)
  if (b.p[0].N == TileW::BN) {
    const int mt = max_tiles<TileW>(b, nullptr);
    if (mt == 0) return hipSuccess;
    launch_v<TileW, 32, MMT_GEMM_W_ST, true, false, true, EPI_LN_BWD_F32>(b, dim3(mt, 1, b.count), s);
  } else {
    const int mt = max_tiles<TileL>(b, nullptr);
    if (mt == 0) return hipSuccess;
    if (gemm8_ln_on()) return mmt_launch_gemm8(b, EPI_LN_BWD_F32, true, false, dim3(mt, 1, b.count), s);
    launch_v<TileL, 64, 2, true, false, true, EPI_LN_BWD_F32>(b, dim3(mt, 1, b.count), s);
  }
  return hipGetLastError();
}

template <class TL, int EPI>
static hipError_t launch_f8(const GemmBatch& b, hipStream_t s) {
  int mt = 0;
  for (int g = 0; g < b.count; ++g)
    mt = std::max(mt, ((b.p[g].M + TL::BM - 1) / TL::BM) * ((b.p[g].N + TL::BN - 1) / TL::BN));
  if (mt == 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_f8_kernel<TL, EPI>), dim3(mt, 1, b.count), dim3(TL::NT), 0, s, b);
  return hipGetLastError();
}

template <int EPI>
static hipError_t launch_f8_tile(const GemmBatch& b, hipStream_t s) {
  // the 256x256 tile where every problem fills it and K is long (as the bf16 policy), else 128x128
  // (tile_hint 1: the 128 x 128 tile, which fits beside other streams' waves where the 256 x 256 one needs a free CU)
  bool big = g_big_mode != 0 && b.tile_hint != 1;
  for (int g = 0; g < b.count; ++g)
    if (b.p[g].M < TileL::BM || b.p[g].N < TileL::BN || b.p[g].K < g_big_kmin) big = false;
  return big ? launch_f8<TileL, EPI>(b, s) : launch_f8<TileS, EPI>(b, s);
}

hipError_t mmt_launch_gemm_f8(const GemmBatch& b, int epi, hipStream_t s) {
  if (b.count == 0) return hipSuccess;
  if (!gemm_span_ok(b)) return hipErrorInvalidValue;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    if ((P.K & 31) || (P.lda & 15) || (P.ldb & 15) || (((uintptr_t)P.A | (uintptr_t)P.B) & 15) || (P.lds_a & 3) ||
        (P.lds_b & 3) || (((uintptr_t)P.sa | (uintptr_t)P.sb) & 3) || P.lds_a * 32 < P.K || P.lds_b * 32 < P.K)
      return hipErrorInvalidValue;
    if (P.o8 && ((P.N & 31) || (P.ld8 & 7) || ((uintptr_t)P.o8 & 7))) return hipErrorInvalidValue;
    if (P.qkv2_out) return hipErrorInvalidValue;  // (no fused Q/K/V stage 2 on the fp8 kernel)
  }
  switch (epi) {
    case EPI_STORE_BF16: return launch_f8_tile<EPI_STORE_BF16>(b, s);
    case EPI_BIAS_TANH_BF16: return launch_f8_tile<EPI_BIAS_TANH_BF16>(b, s);
    case EPI_BIAS_RELU_BF16: return launch_f8_tile<EPI_BIAS_RELU_BF16>(b, s);
    case EPI_BIAS_RESID_F32: return launch_f8_tile<EPI_BIAS_RESID_F32>(b, s);
    case EPI_STORE_F32: return launch_f8_tile<EPI_STORE_F32>(b, s);
    default: return hipErrorInvalidValue;
  }
}

