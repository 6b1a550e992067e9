// Per-head Q/K/V stage 2 on MFMA (reference model.py:36-50: each of key/query/value of each head
// ends in Linear(hs/2, hs, bias=False) after a tanh): 3*H independent [hs/2 -> hs] maps per row.
//
// forward   out^T[o][r] = sum_i W2[o][i] h1[r][i]          one 32x32x16 MFMA per (32 rows, blk)
// backward  dh1^T[i][r] = (sum_o W2[o][i] dout[r][o]) * (1 - h1[r][i]^2)
//           dW2[o][i]  += sum_r dout[r][o] h1[r][i]        K = rows, operands by transposed LDS reads
// blk = kind*H + head; h1 / dh1 rows hold nblk*hs/2 columns, out / dout rows nblk*hs columns.

#include <cstdlib>
#include <type_traits>

#include "mmt_common.h"
#include "mmt_kernels.h"

template <int N>
__device__ __forceinline__ void ld4_guarded(const bf16_t* p, int valid, uint32_t& w0, uint32_t& w1) {
  // 4 bf16 at p (8-byte aligned); elements >= valid read as zero
  if (valid >= 4) {
    const u32x2 v = *reinterpret_cast<const u32x2*>(p);
    w0 = v[0]; w1 = v[1];
  } else {
    uint16_t e[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) e[t] = t < valid ? p[t] : (uint16_t)0;
    w0 = e[0] | ((uint32_t)e[1] << 16);
    w1 = e[2] | ((uint32_t)e[3] << 16);
  }
}

// ---------------------------------------------------------------------------------------------
// rows per forward block: qkv2_strips(HS) strips of 128 rows, the next strip's h1 loaded into
// registers while this one computes and stores (one load -> compute -> store chain per block leaves
// each block's latency exposed). hs 64: 4 strips (target 94 -> 66 us); hs <= 32 keeps one strip per
// block (4 measured 33 -> 36 us at C1: the grid already holds 12k blocks)
constexpr int qkv2_strips(int hs) { return hs >= 48 ? 4 : 1; }
template <int HS>
__global__ __launch_bounds__(256) void qkv2_fwd_mfma(Qkv2Batch batch, int R, int ld_h1, int ld_out) {
  constexpr int HH = HS / 2;
  constexpr int NOT = (HS + 31) / 32;  // output (o) tiles
  constexpr int KS = (HH + 15) / 16;   // k-steps over i
  constexpr int SHW = KS * 16 + 8;     // h1 tile row (zero padded to the k-steps; +8 de-conflicts)
  constexpr int SOW = HS + 8;          // out tile row
  constexpr int BR = 128 * qkv2_strips(HS);
  const Qkv2Problem& P = batch.p[blockIdx.z];
  // grid.x = row blocks x nblk, blk fastest in logical order (one row's blocks share its lines)
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int nblk = gridDim.x / ((R + BR - 1) / BR);
  const int blk = tile % nblk, rb = tile / nblk;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  __shared__ __attribute__((aligned(16))) bf16_t sh[128 * SHW];
  __shared__ __attribute__((aligned(16))) bf16_t so[128 * SOW];
  // h1 strip [128][HH] in 8-B pieces, consecutive lanes along a row; pad columns zero
  constexpr int HPC = HH / 4, PPC = (KS * 16 - HH) / 4;
  constexpr int NL = (128 * HPC + 255) / 256;
  u32x2 hv[NL];  // every load of a strip in flight before its LDS stores
  auto load = [&](int r0) {
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int c = tid + 256 * u, row = c / HPC, col = (c % HPC) * 4;
      hv[u] = u32x2{0u, 0u};
      if (c < 128 * HPC && r0 + row < R)
        hv[u] = *reinterpret_cast<const u32x2*>(P.h1 + (int64_t)(r0 + row) * ld_h1 + blk * HH + col);
    }
  };
  if (PPC > 0)  // pad columns: zero once (the strips only rewrite columns < HH)
    for (int c = tid; c < 128 * PPC; c += 256) {
      const int row = c / PPC, col = HH + (c % PPC) * 4;
      *reinterpret_cast<u32x2*>(sh + row * SHW + col) = u32x2{0u, 0u};
    }
  // this wave's W2 fragments (the same for every strip)
  const float* w2 = P.w2 + (int64_t)blk * HS * HH;
  bf16x8 wa[NOT][KS];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int o = ot * 32 + r, i = 16 * s + 8 * h + j;
        wa[ot][s][j] = (__bf16)((o < HS && i < HH) ? w2[o * HH + i] : 0.f);
      }
  const int lr = w * 32;
  const int rend = min(R, rb * BR + BR);
  load(rb * BR);
  for (int r0 = rb * BR; r0 < rend; r0 += 128) {
    if (r0 > rb * BR) __syncthreads();  // the previous strip's LDS reads (sh, so) are done
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int c = tid + 256 * u;
      if (c < 128 * HPC) *reinterpret_cast<u32x2*>(sh + (c / HPC) * SHW + (c % HPC) * 4) = hv[u];
    }
    __syncthreads();
    if (r0 + 128 < rend) load(r0 + 128);
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot) {
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8 hb = *reinterpret_cast<const bf16x8*>(sh + (lr + r) * SHW + 16 * s + 8 * h);
        acc = mfma32(wa[ot][s], hb, acc);  // D[o][row]
      }
      // lane owns row (r) and o = ot*32 + (e&3) + 8(e>>2) + 4h
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int o0 = ot * 32 + 8 * g + 4 * h;
        if (o0 < HS)
          *reinterpret_cast<u32x2*>(so + (lr + r) * SOW + o0) =
              u32x2{pack2bf(acc[4 * g], acc[4 * g + 1]), pack2bf(acc[4 * g + 2], acc[4 * g + 3])};
      }
    }
    __syncthreads();
    // out strip [128][HS] in 16-B pieces, consecutive lanes along a row
    constexpr int OPC = HS / 8;
    for (int c = tid; c < 128 * OPC; c += 256) {
      const int row = c / OPC, col = (c % OPC) * 8;
      if (r0 + row < R)
        *reinterpret_cast<u32x4*>(P.out + (int64_t)(r0 + row) * ld_out + blk * HS + col) =
            *reinterpret_cast<const u32x4*>(so + row * SOW + col);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// tr fragment of an LDS image [rows][ld] (ld elements per row): lane gets column
// cb + (lane&31) and rows kb + 16s + 8(lane>>5) + 0..7 (B/A operand with k along rows)
__device__ __forceinline__ bf16x8 tr_rows(const bf16_t* img, int ld, int kb, int cb, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int kr = kb + 8 * (g >> 1) + q;
  return join4(lds_tr16(img + kr * ld + col), lds_tr16(img + (kr + 4) * ld + col));
}

// rows per backward block (a multiple of 256)
#ifndef QKV2_BWD_ROWS
#define QKV2_BWD_ROWS 2048
#endif
template <int HS>
__global__ __launch_bounds__(256) void qkv2_bwd_mfma(Qkv2Batch batch, int R, int ld_h1, int ld_out) {
  constexpr int HH = HS / 2;
  constexpr int NOT = (HS + 31) / 32;
  constexpr int SDW = (HS < 32 ? 32 : HS) + 16;  // sd row: HS cols (>= 32 for tr reads) + pad
  constexpr int SHW = 32 + 16;                    // sh row: 32 cols (HH valid) + pad
  constexpr int KSD = (HS + 15) / 16;             // k-steps over o for dh1
  const Qkv2Problem& P = batch.p[blockIdx.z];
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int nblk = gridDim.x / ((R + QKV2_BWD_ROWS - 1) / QKV2_BWD_ROWS);
  const int blk = tile % nblk;
  const int rbase = (tile / nblk) * QKV2_BWD_ROWS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  __shared__ __attribute__((aligned(16))) bf16_t sd[256 * SDW];
  __shared__ __attribute__((aligned(16))) bf16_t sh[256 * SHW];
  __shared__ __attribute__((aligned(16))) bf16_t w2t[32 * SDW];
  const float* w2 = P.w2 + (int64_t)blk * HS * HH;
  // W2^T (bf16) : w2t[i][o]
  for (int q = tid; q < 32 * SDW; q += 256) {
    const int i = q / SDW, o = q % SDW;
    w2t[q] = f2bf((i < HH && o < HS) ? w2[o * HH + i] : 0.f);
  }
  // dW2 partials accumulate over QKV2_BWD_ROWS / 256 chunks: one atomic add per element per block
  // (blocks of one blk all add into the same [HS][HH] table, so fewer blocks = less contention)
  f32x16 dw[NOT];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
    for (int e = 0; e < 16; ++e) dw[ot][e] = 0.f;
  // fused stage-1 bias gradient: this lane's running column sums of dh1 (columns 8g + 4h + e)
  float cs[4][4] = {};
  // chunks of 256 rows, row per thread. The next chunk's dout / h1 pieces are loaded into registers
  // before this chunk's MFMA work (software pipeline: every wave keeps its loads in flight through
  // the compute; the block runs 8 chunks back to back)
  // 16-B pieces of a dout / h1 row slice (8-B pieces when the h1 slice is not a multiple of 8)
  constexpr int PW = (HH % 8 == 0) ? 8 : 4;  // elements per piece
  constexpr int ND = HS / PW, NH = HH / PW;
  using Piece = typename std::conditional<PW == 8, u32x4, u32x2>::type;
  Piece dv[ND], hv[NH];
  auto load = [&](int r0) {
    const int rr = r0 + tid;
    const bool ok = rr < R;
    const Piece* d = reinterpret_cast<const Piece*>(P.dout + (int64_t)rr * ld_out + blk * HS);
    const Piece* hp = reinterpret_cast<const Piece*>(P.h1 + (int64_t)rr * ld_h1 + blk * HH);
#pragma unroll
    for (int c = 0; c < ND; ++c) dv[c] = ok ? d[c] : Piece{};
#pragma unroll
    for (int c = 0; c < NH; ++c) hv[c] = ok ? hp[c] : Piece{};
  };
  const int rend = min(R, rbase + QKV2_BWD_ROWS);
  load(rbase);
  for (int r0 = rbase; r0 < rend; r0 += 256) {
  if (r0 > rbase) __syncthreads();  // the previous chunk's LDS reads are done
  {
    Piece* dd = reinterpret_cast<Piece*>(sd + tid * SDW);
#pragma unroll
    for (int c = 0; c < SDW / PW; ++c) dd[c] = c < ND ? dv[c] : Piece{};
    Piece* hd = reinterpret_cast<Piece*>(sh + tid * SHW);
#pragma unroll
    for (int c = 0; c < SHW / PW; ++c) hd[c] = c < NH ? hv[c] : Piece{};
  }
  if (r0 + 256 < rend) load(r0 + 256);
  __syncthreads();
  // ---- dh1 for this wave's 64 rows (2 sub-tiles of 32) ----
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const int lr = w * 64 + st * 32;  // local row base
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int s = 0; s < KSD; ++s) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(w2t + r * SDW + 16 * s + 8 * h);  // W2^T[i=r][o]
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(sd + (lr + r) * SDW + 16 * s + 8 * h);  // dout[row][o]
      acc = mfma32(a, b, acc);  // D[i][row]
    }
    const int grow = r0 + lr + r;
    if (grow < R) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // D rows i = 8g + 4h + 0..3 cover i < 32 >= HH
        const int i0 = 8 * g + 4 * h;
        if (i0 < HH) {
          const bf16_t* hv = sh + (lr + r) * SHW + i0;
          float t[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) { const float x = bf2f(hv[e]); t[e] = acc[4 * g + e] * (1.f - x * x); }
#pragma unroll
          for (int e = 0; e < 4; ++e) cs[g][e] += t[e];
          *reinterpret_cast<u32x2*>(P.dh1 + (int64_t)grow * ld_h1 + blk * HH + i0) =
              u32x2{pack2bf(t[0], t[1]), pack2bf(t[2], t[3])};
        }
      }
    }
  }
  // ---- dW2 partial over this wave's 64 rows: D[o][i] = sum_r dout[r][o] h1[r][i] ----
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int kb = w * 64 + 16 * s;
      const bf16x8 a = tr_rows(sd, SDW, kb, ot * 32, lane);  // A[o][r]
      const bf16x8 b = tr_rows(sh, SHW, kb, 0, lane);        // B[r][i]
      dw[ot] = mfma32(a, b, dw[ot]);
    }
  }
  }  // chunks
  __shared__ float dbr[4][32];
  if (P.db1) {  // column sums: over the 32 row lanes of each half, then the 4 waves, one atomic per column
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = cs[g][e];
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
        if (r == 0 && 8 * g + 4 * h + e < 32) dbr[w][8 * g + 4 * h + e] = v;
      }
  }
  __syncthreads();
  if (P.db1 && tid < HH)
    atomicAdd(P.db1 + (int64_t)blk * HH + tid, (dbr[0][tid] + dbr[1][tid]) + (dbr[2][tid] + dbr[3][tid]));
  float* red = reinterpret_cast<float*>(sd);  // reuse: [4 waves][NOT*32 o][32 i] floats
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int o = ot * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      red[(w * NOT * 32 + o) * 32 + r] = dw[ot][e];
    }
  __syncthreads();
  for (int q = tid; q < HS * HH; q += 256) {
    const int o = q / HH, i = q % HH;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) s += red[(ww * NOT * 32 + o) * 32 + i];
    atomicAdd(P.dw2 + (int64_t)blk * HS * HH + q, s);
  }
}

// ---------------------------------------------------------------------------------------------
// Backward at hs 32 / 64 (hh = 16 / 32), the head sizes of C1 and the target / C3 / C4 shapes. The op
// is HBM-bound (read dout and h1, write dh1), so the dh1 product takes its operands straight from
// global memory: a wave owns 32-row tiles of one block blk, lane (r, h) loads dout[r][16 s + 8 h ..
// + 8] as the K = o slice of an MFMA B operand and h1[r][8 h .. + 8] (and [16 + 8 h ..] at hh 32) with
// one 16-B load each. The A operand is W2^T with its rows permuted (physical row p <-> i = p with bits
// 2 and 3 swapped) so the accumulator hands lane (r, h) exactly dh1[r][8 h + 0..7] (+ [16 + 8 h ..]):
// tanh' from the h1 registers, one 16-B store, column sums for the stage-1 bias gradient in registers.
// dW2 (K = rows) needs the tile transposed: the wave writes its dout / h1 registers into its own LDS
// images (32 rows x 32 columns, 64-B rows, 16-B chunk c of row r at c ^ ((r >> 2) & 3): conflict-free
// for the 8-lane ds_write_b128 groups and the 4-row ds_read_b64_tr_b16 groups alike) and reads
// them back transposed. No block barrier in the row loop; the next tile's loads are in flight while
// the current one computes.
// ---------------------------------------------------------------------------------------------
constexpr int QKV2B_TILES = 8;  // 32-row tiles per wave (a block of 4 waves: 1024 rows)
__device__ __forceinline__ int q2_swz(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// COAL: each load instruction reads whole row slices (lane l: row l / CPR, 16-B chunk l % CPR), so one
// instruction touches 64 / CPR rows instead of 32 row pieces; the tile goes through the wave's LDS
// images (which the dW2 product reads anyway) and the MFMA fragments are read back from there. At
// hs 64 the dh1 tile is restaged the same way before its store.
#ifndef MMT_QKV2B_OCC
#define MMT_QKV2B_OCC 2
#endif
template <int HS, bool COAL>
__global__ __launch_bounds__(256, MMT_QKV2B_OCC) void qkv2_bwd_v2(Qkv2Batch batch, int R, int ld_h1, int ld_out) {
  constexpr int HH = HS / 2;
  constexpr int NOT = HS / 32;  // 32-column output tiles of dout (o)
  constexpr int KSO = HS / 16;  // k-steps over o for dh1
  constexpr int NI = HH / 16;   // 16-column slices of h1 per lane group (1 or 2)
  constexpr int RPB = 4 * 32 * QKV2B_TILES;
  const Qkv2Problem& P = batch.p[blockIdx.z];
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int nblk = gridDim.x / ((R + RPB - 1) / RPB);
  const int blk = tile % nblk, rb = tile / nblk;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  // per-wave images: NOT dout sub-images + one h1 image, each 32 x 32 bf16 (2 KiB)
  __shared__ __attribute__((aligned(16))) char lds[4 * (NOT + 1) * 2048];
  char* img = lds + w * (NOT + 1) * 2048;
  char* himg = img + NOT * 2048;
  if (HH == 16)  // h1 image columns 16..31 stay zero (the dW2 B operand's unused half)
    *reinterpret_cast<u32x4*>(himg + q2_swz(r, 2 + h)) = u32x4{0u, 0u, 0u, 0u};
  // A operand of dh1^T = W2^T dout^T: lane (p, h), k-step s -> W2[o = 16 s + 8 h + j][i = pi(p)]
  const float* w2 = P.w2 + (int64_t)blk * HS * HH;
  const int ip = (r & 16) | ((r & 4) << 1) | ((r & 8) >> 1) | (r & 3);  // bits 2 and 3 of p swapped
  bf16x8 wa[KSO];
#pragma unroll
  for (int s = 0; s < KSO; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) wa[s][j] = (__bf16)(ip < HH ? w2[(16 * s + 8 * h + j) * HH + ip] : 0.f);
  f32x16 dw[NOT];
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
    for (int e = 0; e < 16; ++e) dw[ot][e] = 0.f;
  float cs[8 * NI];
#pragma unroll
  for (int e = 0; e < 8 * NI; ++e) cs[e] = 0.f;
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;

  constexpr int CPR = HS / 8, RPI = 64 / CPR;  // COAL: dout chunks per row, rows per load instruction
  constexpr int HPR = HH / 8, HRPI = 64 / HPR;  // the same for h1 / dh1
  static_assert(!COAL || (KSO * RPI == 32 && NI * HRPI == 32), "coalesced loads cover the 32-row tile");
  // kernel arguments of the tile loop pinned (read through P they were re-loaded on every tile)
  const bf16_t* const dout = sgpr_ptr(P.dout);
  const bf16_t* const h1 = sgpr_ptr(P.h1);
  bf16_t* const dh1 = sgpr_ptr(P.dh1);
  ld_h1 = __builtin_amdgcn_readfirstlane(ld_h1);
  ld_out = __builtin_amdgcn_readfirstlane(ld_out);
  R = __builtin_amdgcn_readfirstlane(R);
  u32x4 dv[KSO], hv[NI];
  auto load = [&](int row0) {  // row0: the tile's first row
    const u32x4 zz = {0u, 0u, 0u, 0u};
    if (COAL) {
#pragma unroll
      for (int s = 0; s < KSO; ++s) {
        const int rr = row0 + s * RPI + lane / CPR;
        dv[s] = rr < R ? *reinterpret_cast<const u32x4*>(dout + (int64_t)rr * ld_out + blk * HS + 8 * (lane % CPR)) : zz;
      }
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const int rr = row0 + q * HRPI + lane / HPR;
        hv[q] = rr < R ? *reinterpret_cast<const u32x4*>(h1 + (int64_t)rr * ld_h1 + blk * HH + 8 * (lane % HPR)) : zz;
      }
      return;
    }
    const int row = row0 + r;
    const bool ok = row < R;
    const bf16_t* d = dout + (int64_t)row * ld_out + blk * HS + 8 * h;
    const bf16_t* hp = h1 + (int64_t)row * ld_h1 + blk * HH + 8 * h;
#pragma unroll
    for (int s = 0; s < KSO; ++s) dv[s] = ok ? *reinterpret_cast<const u32x4*>(d + 16 * s) : zz;
#pragma unroll
    for (int q = 0; q < NI; ++q) hv[q] = ok ? *reinterpret_cast<const u32x4*>(hp + 16 * q) : zz;
  };
  const int r0 = rb * RPB + w * 32 * QKV2B_TILES;
  load(r0);
#pragma unroll 1
  for (int t = 0; t < QKV2B_TILES; ++t) {
    const int row = r0 + 32 * t + r;
    if (r0 + 32 * t >= R) break;  // wave-uniform
    u32x4 dc[KSO], hc[NI];
    if (COAL) {  // rows past R hold zeros (their loads returned 0)
#pragma unroll
      for (int s = 0; s < KSO; ++s) {
        const int c = lane % CPR;
        *reinterpret_cast<u32x4*>(img + (c >> 2) * 2048 + q2_swz(s * RPI + lane / CPR, c & 3)) = dv[s];
      }
#pragma unroll
      for (int q = 0; q < NI; ++q) *reinterpret_cast<u32x4*>(himg + q2_swz(q * HRPI + lane / HPR, lane % HPR)) = hv[q];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int s = 0; s < KSO; ++s) dc[s] = *reinterpret_cast<const u32x4*>(img + (s >> 1) * 2048 + q2_swz(r, 2 * (s & 1) + h));
#pragma unroll
      for (int q = 0; q < NI; ++q) hc[q] = *reinterpret_cast<const u32x4*>(himg + q2_swz(r, 2 * q + h));
    } else {
#pragma unroll
      for (int s = 0; s < KSO; ++s) dc[s] = dv[s];
#pragma unroll
      for (int q = 0; q < NI; ++q) hc[q] = hv[q];
    }
    if (t + 1 < QKV2B_TILES) load(r0 + 32 * t + 32);  // the next tile's loads fly while this one computes
    // dh1 (accumulator rows = i in the permuted order: lane (r, h) gets i = 8 h + e, 16 + 8 h + e - 8)
    f32x16 acc = z;
#pragma unroll
    for (int s = 0; s < KSO; ++s) acc = mfma32(wa[s], __builtin_bit_cast(bf16x8, dc[s]), acc);
    u32x4 dz[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      float t8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t wd = hc[q][e >> 1];
        const float x = bf2f((bf16_t)((e & 1) ? (wd >> 16) : (wd & 0xffff)));
        t8[e] = acc[8 * q + e] * (1.f - x * x);
      }
      dz[q] = u32x4{pack2bf(t8[0], t8[1]), pack2bf(t8[2], t8[3]), pack2bf(t8[4], t8[5]), pack2bf(t8[6], t8[7])};
      if (row < R) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[8 * q + e] += t8[e];
        if (!(COAL && HPR >= 4))
          *reinterpret_cast<u32x4*>(dh1 + (int64_t)row * ld_h1 + blk * HH + 16 * q + 8 * h) = dz[q];
      }
    }
    // dW2 over this tile's 32 rows: LDS images (rows past R hold zeros: their loads returned 0)
    if (!COAL) {
#pragma unroll
      for (int s = 0; s < KSO; ++s)  // dout columns 16 s + 8 h: sub-image s / 2, chunk 2 (s & 1) + h
        *reinterpret_cast<u32x4*>(img + (s >> 1) * 2048 + q2_swz(r, 2 * (s & 1) + h)) = dc[s];
#pragma unroll
      for (int q = 0; q < NI; ++q) *reinterpret_cast<u32x4*>(himg + q2_swz(r, 2 * q + h)) = hc[q];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own wave's writes visible to its reads
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {  // rows 16 ks .. 16 ks + 15
      // tr read: lane gets column (l & 31) and rows 16 ks + 8 h + 0..7 of an image
      auto trd = [&](const char* im) {
        const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
        const int col = 16 * (g & 1) + 4 * pp;
        const int kr = 16 * ks + 8 * (g >> 1) + qq;
        const s16x4 lo = lds_tr16(im + q2_swz(kr, col >> 3) + (col & 7) * 2);
        const s16x4 hi = lds_tr16(im + q2_swz(kr + 4, col >> 3) + (col & 7) * 2);
        return join4(lo, hi);
      };
      const bf16x8 bh = trd(himg);
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot) dw[ot] = mfma32(trd(img + ot * 2048), bh, dw[ot]);
    }
    if (COAL && HPR >= 4) {  // dh1 through the h1 image (its reads above come first: LDS is in order per wave)
#pragma unroll
      for (int q = 0; q < NI; ++q) *reinterpret_cast<u32x4*>(himg + q2_swz(r, 2 * q + h)) = dz[q];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const int rr = r0 + 32 * t + q * HRPI + lane / HPR;
        const u32x4 v = *reinterpret_cast<const u32x4*>(himg + q2_swz(q * HRPI + lane / HPR, lane % HPR));
        if (rr < R) *reinterpret_cast<u32x4*>(dh1 + (int64_t)rr * ld_h1 + blk * HH + 8 * (lane % HPR)) = v;
      }
    }
  }
  // block reductions: db1 (column sums) and dW2, then one atomic per element per block
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);  // [HS][HH] floats over the (now dead) images
  if (P.db1) {
#pragma unroll
    for (int e = 0; e < 8 * NI; ++e) {
      float v = cs[e];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
      cs[e] = v;
    }
  }
  __shared__ float dbr[4][32];
  if (P.db1 && r == 0) {
#pragma unroll
    for (int q = 0; q < NI; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) dbr[w][16 * q + 8 * h + e] = cs[8 * q + e];
  }
  __syncthreads();
  if (P.db1 && tid < HH) atomicAdd(P.db1 + (int64_t)blk * HH + tid, (dbr[0][tid] + dbr[1][tid]) + (dbr[2][tid] + dbr[3][tid]));
  // dW2 partials: D[o][i], o = ot*32 + (e&3) + 8(e>>2) + 4h, i = lane r (< HH valid)
  static_assert(HS * HH * 4 <= 4 * (NOT + 1) * 2048, "dW2 reduction fits the images");
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int o = ot * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (r < HH) {
            float* q = red + o * HH + r;
            *q = (ww == 0 ? 0.f : *q) + dw[ot][e];
          }
        }
    }
    __syncthreads();
  }
  for (int q = tid; q < HS * HH; q += 256) atomicAdd(P.dw2 + (int64_t)blk * HS * HH + q, red[q]);
}

static int g_qkv2_coal = [] {
  const char* e = getenv("MMT_QKV2_COAL");
  return e ? atoi(e) : 2;  // bit 0: hs 32, bit 1: hs 64 (hs 32: C1 +0.13 %, hs 64: target -0.25 %, r5y)
}();
extern "C" int mmt_qkv2_set_coal(int on) {
  const int old = g_qkv2_coal;
  g_qkv2_coal = on;
  return old;
}

template <int HS>
static void qkv2_launch(const Qkv2Batch& b, int R, int nblk, int ld_h1, int ld_out, bool bwd, hipStream_t s) {
  constexpr int RPB = 4 * 32 * QKV2B_TILES;
  // (v2 against qkv2_bwd_mfma in the step: C1 8.818 vs 8.832 ms, target 20.39 vs 20.48: profiles/r4k_ab.txt)
  constexpr int HV = HS == 64 ? 64 : 32;
  if (bwd && (HS == 32 || HS == 64)) {
    const dim3 grid((R + RPB - 1) / RPB * nblk, 1, b.count);
    if (g_qkv2_coal & (HV == 64 ? 2 : 1))
      hipLaunchKernelGGL((qkv2_bwd_v2<HV, true>), grid, dim3(256), 0, s, b, R, ld_h1, ld_out);
    else
      hipLaunchKernelGGL((qkv2_bwd_v2<HV, false>), grid, dim3(256), 0, s, b, R, ld_h1, ld_out);
  }
  else if (bwd)
    hipLaunchKernelGGL(qkv2_bwd_mfma<HS>, dim3((R + QKV2_BWD_ROWS - 1) / QKV2_BWD_ROWS * nblk, 1, b.count), dim3(256), 0, s,
                       b, R, ld_h1, ld_out);
  else
    hipLaunchKernelGGL(qkv2_fwd_mfma<HS>, dim3((R + 128 * qkv2_strips(HS) - 1) / (128 * qkv2_strips(HS)) * nblk, 1, b.count),
                       dim3(256), 0, s, b, R, ld_h1, ld_out);
}

static hipError_t qkv2_dispatch(const Qkv2Batch& b, int R, int nblk, int hs, int ld_h1, int ld_out, bool bwd,
                                hipStream_t s) {
  if (b.count == 0 || R == 0) return hipSuccess;
  if (!bwd) {  // the forward stores 16-B row pieces of out
    if (ld_out & 7) return hipErrorInvalidValue;
    for (int g = 0; g < b.count; ++g)
      if ((uintptr_t)b.p[g].out & 15) return hipErrorInvalidValue;
  }
  if (bwd) {  // the backward stages dout / h1 row slices as 16-B pieces
    if ((ld_h1 | ld_out) & 7) return hipErrorInvalidValue;
    for (int g = 0; g < b.count; ++g)
      if (((uintptr_t)b.p[g].h1 | (uintptr_t)b.p[g].dout) & 15) return hipErrorInvalidValue;
  }
  switch (hs) {
    case 8: qkv2_launch<8>(b, R, nblk, ld_h1, ld_out, bwd, s); break;
    case 16: qkv2_launch<16>(b, R, nblk, ld_h1, ld_out, bwd, s); break;
    case 24: qkv2_launch<24>(b, R, nblk, ld_h1, ld_out, bwd, s); break;
    case 32: qkv2_launch<32>(b, R, nblk, ld_h1, ld_out, bwd, s); break;
    case 48: qkv2_launch<48>(b, R, nblk, ld_h1, ld_out, bwd, s); break;
    case 64: qkv2_launch<64>(b, R, nblk, ld_h1, ld_out, bwd, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t mmt_launch_qkv2_fwd(const Qkv2Batch& b, int R, int nblk, int hs, int ld_h1, int ld_out, hipStream_t s) {
  return qkv2_dispatch(b, R, nblk, hs, ld_h1, ld_out, false, s);
}
hipError_t mmt_launch_qkv2_bwd(const Qkv2Batch& b, int R, int nblk, int hs, int ld_h1, int ld_out, hipStream_t s) {
  return qkv2_dispatch(b, R, nblk, hs, ld_h1, ld_out, true, s);
}
