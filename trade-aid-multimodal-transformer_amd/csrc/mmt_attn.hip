// Causal self-attention and multi-stream selective cross-attention for gfx950.
//
// Reference semantics (model.py:60-73, 136-159): per head, aff = q k^T * hs^-0.5, causal mask,
// softmax, @ v. Cross-attention runs one independent causal softmax per KV modality ("stream")
// and SUMS the per-stream outputs (no joint softmax).
//
// Structure: a 256-thread workgroup (4 waves) owns 8 32-row tiles of one (batch, head) (wave w
// takes tiles w and 7-w: balanced causal work). The operand the tiles share (K/V in the forward
// and dQ pass, Q/dO/LSE/D in the dK/dV pass) is staged into LDS in chunks of up to 256 rows; at
// T <= chunk the whole sequence lands with one barrier (see "Chunked staging" below).
// All products are v_mfma_f32_32x32x16_bf16 with fp32 accumulation:
//   forward  S^T = K Q^T (keys on accumulator rows, queries on lanes) -> online softmax per lane;
//            O^T += V^T P^T with P^T straight from the accumulator registers as the B operand and
//            V^T by ds_read_b64_tr_b16 from the V tile.
//   dQ       S^T, dP^T recomputed per key tile; dQ^T += K^T dS^T (K^T by transposed LDS reads).
//   dK, dV   S = Q K^T, dP = dO V^T (queries on rows); dV += P^T dO, dK += dS^T Q with P and dS
//            taken from registers as the A operand and dO / Q by transposed LDS reads.
// Head sizes 8..64: padded to 16 on the reduction side and to 32 on the output side.
// Dropout (model.py:69, 151: applied to the normalised probabilities): a counter-hash mask,
// O = (P.Z) V with Z = mask / (1 - p), so dV = (P.Z)^T dO, dS = P.(Z.dP - D) with D = rowsum(dO.O)
// unchanged. The hash runs once, in attn_mask_kernel (launched on a side stream, overlapping the
// GEMMs before the attention), which stores one keep bit per element in the S^T accumulator order
// (AttnProblem::dmask). The three attention kernels stage the bits of their chunk in LDS next to
// K/V (Q/dO) and apply them with no hashing: the forward and dQ pass turn a pair of mask dwords
// into the lane mask of a v_cndmask (inverse ballot), the dK/dV pass (keys on lanes) extracts its
// bit per element. 1/(1-p) is folded into the output normalisation / dV write-out.
#include <stdlib.h>

#include <algorithm>

#include <type_traits>

#include "mmt_common.h"
#include "mmt_kernels.h"

namespace {

__device__ __forceinline__ bf16x8 zero8() {
  const u32x4 z = {0u, 0u, 0u, 0u};
  return __builtin_bit_cast(bf16x8, z);
}

__device__ __forceinline__ bf16x8 ld8(const bf16_t* p, bool ok) {
  if (!ok) return zero8();
  return *reinterpret_cast<const bf16x8*>(p);
}

template <int HS>
struct Geo {
  static constexpr int NKS = (HS + 15) / 16;           // k-steps over the head dim
  static constexpr int ND = (HS + 31) / 32;            // 32-wide output tiles over the head dim
  static constexpr int W = ND * 32;                    // padded head width in LDS tiles
  static constexpr int RW = W + 8;                     // row-read tile stride (16-B pad: no b128 conflicts)
  static constexpr int TW = (W == 64) ? 96 : W;        // transposed-read tile stride (conflict-free)
  static constexpr int CH = HS / 8;                    // 16-byte chunks per row
};

// one 16-B chunk (8 bf16) of a 32-row tile: row r0+row, columns col..col+7 of the head (zero padded)
__device__ __forceinline__ u32x4 tile_chunk(const bf16_t* base, int64_t rowbase, int r0, int row, int col, int T,
                                            int ld) {
  u32x4 v = {0u, 0u, 0u, 0u};
  if (r0 + row < T) v = *reinterpret_cast<const u32x4*>(base + (rowbase + r0 + row) * ld + col);
  return v;
}

// A-operand fragment of X^T where X is a [32 rows][stride] LDS tile: lane gets column
// d = dt*32 + (lane&31) and rows {16s+4h+0..3, 16s+8+4h+0..3} (the accumulator-as-operand k order)
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* lds, int stride, int dt, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int col = dt * 32 + 16 * (g & 1) + 4 * p;
  const int kb = 16 * s + 4 * (g >> 1) + q;
  return join4(lds_tr16(lds + kb * stride + col), lds_tr16(lds + (kb + 8) * stride + col));
}

// hs-32 slice image of the backward's shared operands (round 5, as the hs-64 rings' images of
// mmt_attn2.hip): 32-row slices of two 16-column sub-images 1152 B apart (1 KiB + 128 B pad), the two
// 16-B halves of a row swapped when bit 3 of the row is set. Row reads (ds_read_b128, a row per lane)
// and transposed reads (ds_read_b64_tr_b16, 4 rows x 16 columns per 16-lane group) are both
// conflict-free; the [row][40] image of Geo<32>::RW took 2-way conflicts on every transposed read
// (SQ_LDS_BANK_CONFLICT 0.31 / 0.25 of the dQ / dK-dV passes' LDS cycles at C1, round 4)
constexpr int SL_SUB = 1152, SL_SLICE = 2 * SL_SUB;
template <int HS>
struct SliceImg {
  static constexpr bool on = HS == 32;
};
// byte offset of 16-B chunk `chunk` (8 columns, 0..3) of row `row`
__device__ __forceinline__ int sl_off(int row, int chunk) {
  return (row >> 5) * SL_SLICE + (chunk >> 1) * SL_SUB + (row & 31) * 32 + (((chunk & 1) ^ ((row >> 3) & 1)) << 4);
}
// row fragment: row row0 + r of the slice at row0 (a multiple of 32), columns 16 s + 8 h .. + 7
// (per-lane part r 32 + swapped half: one register; the slice and s are immediates / scalars)
__device__ __forceinline__ bf16x8 sl_row(const bf16_t* img, int row0, int r, int s, int h) {
  const int o = (row0 >> 5) * SL_SLICE + s * SL_SUB + r * 32 + ((h ^ ((r >> 3) & 1)) << 4);
  return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(img) + o);
}
// transposed fragment of the slice at row0 (as tr_frag: column 16 (g & 1) + 4 p of rows
// 16 s + 4 (g >> 1) + q and + 8): the first row set has bit 3 clear, the second set, so the swap is
// fixed per set and the per-lane parts are two registers
__device__ __forceinline__ bf16x8 sl_tr(const bf16_t* img, int row0, int s, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int L = (g & 1) * SL_SUB + (p & 1) * 8 + (4 * (g >> 1) + q) * 32;
  const char* b = reinterpret_cast<const char*>(img) + (row0 >> 5) * SL_SLICE + 512 * s;
  return join4(lds_tr16(b + L + ((p >> 1) << 4)), lds_tr16(b + L + 256 + (((p >> 1) ^ 1) << 4)));
}

// accumulator registers 8s..8s+7 -> bf16 operand fragment
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  const u32x4 v = {pack2bf(a[8 * s], a[8 * s + 1]), pack2bf(a[8 * s + 2], a[8 * s + 3]),
                   pack2bf(a[8 * s + 4], a[8 * s + 5]), pack2bf(a[8 * s + 6], a[8 * s + 7])};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void zero16(f32x16& a) {
#pragma unroll
  for (int e = 0; e < 16; ++e) a[e] = 0.f;
}

__device__ __forceinline__ float keep_f(float v, int m) { return __int_as_float(__float_as_int(v) & m); }

// dword of an S^T mask tile that holds key r's keep bits over the tile's 32 queries
__device__ __forceinline__ int key_dword(int r) { return 2 * ((r & 3) + 4 * (r >> 3)) + ((r >> 2) & 1); }

}  // namespace

// =============================================================================================
// Chunked staging. A workgroup (4 waves) owns 8 consecutive 32-row tiles of one (batch, head);
// wave w takes tiles w and 7-w, so the causal work of the 4 waves is balanced. The operand the
// tiles share (K/V in the forward and dQ pass, Q/dO in the dK/dV pass) is staged into LDS in
// chunks of ROWS rows (32 KiB of bf16 per operand pair): at T <= ROWS the whole sequence lands with
// one barrier and the waves then run barrier-free; longer sequences reload between chunks (the
// other resident workgroups of the CU cover that latency; a register prefetch would cost the
// occupancy it buys). Softmax runs in the log2 domain (scale * log2(e) folded into
// one multiply, exp2 on v_exp_f32); only tiles on the causal diagonal (and a ragged last query
// tile) evaluate the mask.
// =============================================================================================
template <int HS>
struct Chunk {
  static constexpr int ROWS = (HS <= 32) ? 256 : 128;
  static constexpr int HALF = ROWS * Geo<HS>::CH;  // 16-B pieces of one operand
  static constexpr int NSTG = 2 * HALF / 256;      // pieces per thread (two operands)
};

template <int HS>
struct Stager {
  u32x4 v[Chunk<HS>::NSTG];
  // rows [r0, r0 + ROWS) of operands a, b (columns 0..HS-1); rows >= T read as zeros
  __device__ __forceinline__ void load(const bf16_t* a, int lda, const bf16_t* b, int ldb, int64_t rowbase, int r0,
                                       int T, int tid) {
    constexpr int CH = Geo<HS>::CH, HALF = Chunk<HS>::HALF;
#pragma unroll
    for (int u = 0; u < Chunk<HS>::NSTG; ++u) {
      const int c = tid + 256 * u;
      const bool isb = c >= HALF;
      const int cc = isb ? c - HALF : c;
      v[u] = tile_chunk(isb ? b : a, rowbase, r0, cc / CH, (cc % CH) * 8, T, isb ? ldb : lda);
    }
  }
  // operand a's chunks only (a second image of it at another stride)
  __device__ __forceinline__ void store_a(bf16_t* la, int sa, int tid) const {
    constexpr int CH = Geo<HS>::CH, HALF = Chunk<HS>::HALF;
#pragma unroll
    for (int u = 0; u < Chunk<HS>::NSTG; ++u) {
      const int c = tid + 256 * u;
      if (c < HALF) *reinterpret_cast<u32x4*>(la + (c / CH) * sa + (c % CH) * 8) = v[u];
    }
  }
  __device__ __forceinline__ void store(bf16_t* la, int sa, bf16_t* lb, int sb, int tid) const {
    constexpr int CH = Geo<HS>::CH, HALF = Chunk<HS>::HALF;
#pragma unroll
    for (int u = 0; u < Chunk<HS>::NSTG; ++u) {
      const int c = tid + 256 * u;
      const bool isb = c >= HALF;
      const int cc = isb ? c - HALF : c;
      const int row = cc / CH, col = (cc % CH) * 8;
      *reinterpret_cast<u32x4*>(isb ? lb + row * sb + col : la + row * sa + col) = v[u];
    }
  }
  // both operands as slice images (SliceImg; HS == 32: 4 chunks per row)
  __device__ __forceinline__ void store_slices(bf16_t* la, bf16_t* lb, int tid) const {
    constexpr int CH = Geo<HS>::CH, HALF = Chunk<HS>::HALF;
    static_assert(CH == 4, "slice images hold 32 columns");
#pragma unroll
    for (int u = 0; u < Chunk<HS>::NSTG; ++u) {
      const int c = tid + 256 * u;
      const bool isb = c >= HALF;
      const int cc = isb ? c - HALF : c;
      *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(isb ? lb : la) + sl_off(cc / CH, cc % CH)) = v[u];
    }
  }
};

// Dropout keep bits of one staged chunk: LDS [8 block tiles][KT chunk tiles][32 dwords]. The block
// tiles are the block's 8 query tiles (forward, dQ) or key tiles (dK/dV); the chunk tiles are the
// key (query) tiles of the staged chunk. Tiles above the causal diagonal are left as zeros.
template <int HS, int KT_ = Chunk<HS>::ROWS / 32>
struct MaskStager {
  static constexpr int KT = KT_;
  static constexpr int N4 = 8 * KT * 8;  // 16-B pieces
  static constexpr int PER = (N4 + 255) / 256;
  static constexpr int DWORDS = 8 * KT * 32;
  u32x4 v[PER];
  // b0: first block tile, c0: first chunk tile; blk_q: block tiles are query tiles
  __device__ __forceinline__ void load(const uint32_t* base, int bh, int nt, int b0, int c0, bool blk_q, int tid) {
    const int64_t ntri = (int64_t)nt * (nt + 1) / 2;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + 256 * u;
      v[u] = u32x4{0u, 0u, 0u, 0u};
      if (N4 % 256 == 0 || c < N4) {
        const int i = c / (KT * 8), k = (c / 8) % KT, p = c % 8;
        const int qt = blk_q ? b0 + i : c0 + k, kt = blk_q ? c0 + k : b0 + i;
        if (qt < nt && kt <= qt)
          v[u] = *reinterpret_cast<const u32x4*>(base + ((int64_t)bh * ntri + qt * (qt + 1) / 2 + kt) * 32 + p * 4);
      }
    }
  }
  __device__ __forceinline__ void store(uint32_t* lds, int tid) const {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + 256 * u;
      if (N4 % 256 == 0 || c < N4) *reinterpret_cast<u32x4*>(lds + 4 * c) = v[u];
    }
  }
};

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// Softmax / dS arithmetic is scalar fp32 on purpose: v_pk_*_f32 beside MFMAs costs more issue
// cycles than the two scalar instructions it replaces (MI355X_MICROARCH.md, constants table), and
// this file is compiled with -fno-slp-vectorize so the compiler does not re-pack them.

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kTau = 8.0f;  // lazy-rescale threshold of the forward's running max (log2 units)

// waves per SIMD the forward / dQ kernels are compiled for (hs <= 32 fits two at no spill; at hs
// = 64 the forward fits two without AGPRs; the dQ pass spills ~25 VGPRs there and is still faster)
#ifndef MMT_FWD_MINB
#define MMT_FWD_MINB(hs) 2
#endif
#ifndef MMT_DQ_MINB
#define MMT_DQ_MINB(hs) 2
#endif
// single-tile dK/dV: at hs <= 32 the default bound (the compiler keeps the accumulators in AGPRs
// and still reaches 2 waves) measured faster than forcing 2; at hs = 64 forcing 2 fits without AGPRs
#ifndef MMT_DKDV1_MINB
#define MMT_DKDV1_MINB(hs) ((hs) <= 32 ? 1 : 2)
#endif

// cross-half reductions (lanes l and l ^ 32) in one v_permlane32_swap: no LDS round trip
__device__ __forceinline__ float xhalf_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  float m;
  asm("v_max_f32 %0, %1, %2" : "=v"(m) : "v"(__uint_as_float(r[0])), "v"(__uint_as_float(r[1])));
  return m;
}
__device__ __forceinline__ float xhalf_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Lane word of an S^T keep tile (attn_mask_kernel): bit i = element 2i, bit 8 + i = element 2i + 1
// of the lane's 16 accumulator elements. keep_spread moves the odd byte to bits 16..23 (one
// v_perm_b32); pair_keep then turns pair i (the two elements one v_cvt_pk_bf16_f32 packs) into a
// 0x0000 / 0xFFFF half mask with one shift and one packed arithmetic shift: 1.5 VALU per element
// including the AND on the packed bf16 pair.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t keep_spread(uint32_t w16) { return __builtin_amdgcn_perm(0u, w16, 0x0c010c00u); }
__device__ __forceinline__ uint32_t pair_keep(uint32_t w32, int i) {
  s16x2 v = __builtin_bit_cast(s16x2, w32 << (15 - i));
  v = v >> (s16x2){15, 15};
  return __builtin_bit_cast(uint32_t, v);
}
// keep mask (all ones / zero) of element e of a lane word (fp32 selects in the dQ pass)
__device__ __forceinline__ int elem_keep(uint32_t w16, int e) {
  return __builtin_amdgcn_sbfe((int)w16, (e & 1) * 8 + (e >> 1), 1);
}

// accumulator registers 8s..8s+7 -> bf16 operand fragment, dropped elements zeroed
__device__ __forceinline__ bf16x8 acc_frag_keep(const f32x16& a, int s, uint32_t w32) {
  const u32x4 v = {pack2bf(a[8 * s], a[8 * s + 1]) & pair_keep(w32, 4 * s),
                   pack2bf(a[8 * s + 2], a[8 * s + 3]) & pair_keep(w32, 4 * s + 1),
                   pack2bf(a[8 * s + 4], a[8 * s + 5]) & pair_keep(w32, 4 * s + 2),
                   pack2bf(a[8 * s + 6], a[8 * s + 7]) & pair_keep(w32, 4 * s + 3)};
  return __builtin_bit_cast(bf16x8, v);
}

// per query tile state of the forward walk: Q fragments, running max / sum, O^T accumulators.
// l is this lane's HALF of the row sum (keys 4h + ..., combined across halves at the end): the
// two halves always share m (the max is reduced across them every tile)
template <int HS>
struct FwdQ {
  bf16x8 qf[Geo<HS>::NKS];
  f32x16 o[Geo<HS>::ND];
  float m, l;
  int tq;
};

// online softmax of one S^T tile for one query tile (log2 domain, lazy rescale)
template <int HS, bool diag>
__device__ __forceinline__ void fwd_softmax(f32x16& sacc, FwdQ<HS>& q, int k0, float c2, int h) {
  using G = Geo<HS>;
  // row max on the raw scores (c2 > 0 commutes with max), then into the log2 domain
  float tmax = -INFINITY;
  if (diag) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int key = k0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (key > q.tq) sacc[e] = -INFINITY;
    }
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) tmax = fmaxf(tmax, sacc[e]);
  tmax = xhalf_max(tmax) * c2;
  // lazy rescale: the running max m moves only when a tile's max exceeds it by more than kTau
  // (log2 units; always on the first tile, m = -inf). Until then exp2(s - m) <= 2^kTau keeps P, l
  // and O comfortably in fp32/bf16 range and the O accumulators are not touched on the common
  // path. l and O share m, so the normalised output and the LSE m + log2(l) are unchanged.
  const bool up = tmax > q.m + kTau;
  if (__builtin_amdgcn_ballot_w64(up)) {  // wave-uniform
    const float alpha = up ? ex2(q.m - tmax) : 1.f;
    q.m = up ? tmax : q.m;
    q.l *= alpha;
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) q.o[dt][e] *= alpha;
  }
  const float nm = -q.m;
#pragma unroll
  for (int e = 0; e < 16; ++e) sacc[e] = ex2(__builtin_fmaf(sacc[e], c2, nm));
  // the row sum keeps every term (dropout acts on the normalised probabilities); four partial
  // chains, no cross-half reduction per tile
  float r0 = sacc[0] + sacc[1], r1 = sacc[2] + sacc[3], r2 = sacc[4] + sacc[5], r3 = sacc[6] + sacc[7];
  r0 += sacc[8] + sacc[9]; r1 += sacc[10] + sacc[11]; r2 += sacc[12] + sacc[13]; r3 += sacc[14] + sacc[15];
  q.l += (r0 + r1) + (r2 + r3);
}

// forward step over one 32-key tile for one or two query tiles (NQ): the K fragments and the
// transposed V fragments are read from LDS once and feed both tiles' MFMAs; the V reads are
// issued before the softmax so their latency hides under it
template <int HS, int NQ, bool DA, bool DB, bool DROP>
__device__ __forceinline__ void fwd_step(const bf16_t* ks, const bf16_t* vs, int kl, int k0, FwdQ<HS>& a, FwdQ<HS>& b,
                                         const uint32_t* mta, const uint32_t* mtb, float c2, int lane) {
  using G = Geo<HS>;
  const int r = lane & 31, h = lane >> 5;
  const uint32_t wa = DROP ? keep_spread(reinterpret_cast<const uint16_t*>(mta)[lane]) : 0u;
  const uint32_t wb = (DROP && NQ == 2) ? keep_spread(reinterpret_cast<const uint16_t*>(mtb)[lane]) : 0u;
  f32x16 sa, sb;
  zero16(sa);
  if (NQ == 2) zero16(sb);
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ks + (kl + r) * G::RW + 16 * s + 8 * h);
    sa = mfma32(kf, a.qf[s], sa);
    if (NQ == 2) sb = mfma32(kf, b.qf[s], sb);
  }
  bf16x8 vf[2][G::ND];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt) vf[s][dt] = tr_frag(vs + kl * G::TW, G::TW, dt, s, lane);
  fwd_softmax<HS, DA>(sa, a, k0, c2, h);
  if (NQ == 2) fwd_softmax<HS, DB>(sb, b, k0, c2, h);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 pa = DROP ? acc_frag_keep(sa, s, wa) : acc_frag(sa, s);
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt) a.o[dt] = mfma32(vf[s][dt], pa, a.o[dt]);
    if (NQ == 2) {
      const bf16x8 pb = DROP ? acc_frag_keep(sb, s, wb) : acc_frag(sb, s);
#pragma unroll
      for (int dt = 0; dt < G::ND; ++dt) b.o[dt] = mfma32(vf[s][dt], pb, b.o[dt]);
    }
  }
}

// =============================================================================================
// forward: grid (ceil(nt/8) * B*H, 1, G). Wave w owns query tiles qa = 8*bx + w and qb = 8*bx + 7 - w
// and walks them TOGETHER: while both need a key tile the two online softmaxes run as one
// straight-line body (no branches: the diagonal and dropout variants are compile-time), so two
// independent MFMA -> softmax -> MFMA chains interleave in the wave; the resident K/V chunk of each
// (stream, chunk) is loaded once per block.
// =============================================================================================
template <int HS, bool DROP>
__global__ __launch_bounds__(256, MMT_FWD_MINB(HS)) void attn_fwd_kernel(AttnBatch batch, int T, int H, float scale) {
  using G = Geo<HS>;
  constexpr int ROWS = Chunk<HS>::ROWS;
  constexpr int MKT = ROWS / 32;     // key tiles per chunk
  constexpr int MDW = 8 * MKT * 32;  // keep-bit dwords per chunk
  const AttnProblem& P = batch.p[blockIdx.z];
  // grid.x = nb * B*H in XCD-aware logical order: the heads of one batch row (halves of the same
  // Q/K/V cache lines) run on one XCD together
  const int nb = ((T + 31) / 32 + 7) / 8;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int bh = tile / nb, b = bh / H, head = bh % H;
  const int bx = tile % nb;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int nt = (T + 31) / 32;
  const int qt0 = bx * 8;
  const int qmax = min(qt0 + 7, nt - 1);
  const int nch = (min((qmax + 1) * 32, T) + ROWS - 1) / ROWS;
  const int64_t rowbase = (int64_t)b * T;
  const float c2 = scale * kLog2e;
  __shared__ __attribute__((aligned(16))) bf16_t ks[ROWS * G::RW];
  __shared__ __attribute__((aligned(16))) bf16_t vs[ROWS * G::TW];
  using MS = MaskStager<HS>;
  __shared__ __attribute__((aligned(16))) uint32_t msk[DROP ? MDW : 4];  // keep-bit lane words
  // lane-word record of the keep bits (AttnProblem::dmask): after the key-major one
  const int BH = gridDim.x / nb;
  const int64_t lw_off = (int64_t)BH * (nt * (nt + 1) / 2) * 32;
  Stager<HS> st;
  MS mst;
  if (HS % 32 != 0) {  // pad columns are read only when HS is not a multiple of 32
    for (int q = tid; q < ROWS * G::RW; q += 256) if (q % G::RW >= HS) ks[q] = 0;
    for (int q = tid; q < ROWS * G::TW; q += 256) if (q % G::TW >= HS) vs[q] = 0;
  }
  st.load(P.k[0] + head * P.kv_hstride, P.kv_ld, P.v[0] + head * P.kv_hstride, P.kv_ld, rowbase, 0, T, tid);
  if (DROP) mst.load(P.dmask[0] + lw_off, bh, nt, qt0, 0, true, tid);
  st.store(ks, G::RW, vs, G::TW, tid);
  if (DROP) mst.store(msk, tid);

  const int qa = qt0 + w, qb = qt0 + 7 - w;  // qa < qb
  const bool la = qa < nt, lb = qb < nt;     // lb implies la
  FwdQ<HS> A, Bq;
  A.tq = qa * 32 + r;
  Bq.tq = qb * 32 + r;
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    const int d0 = 16 * s + 8 * h;
    A.qf[s] = ld8(P.q + (rowbase + A.tq) * P.q_ld + head * HS + d0, la && A.tq < T && d0 < HS);
    Bq.qf[s] = ld8(P.q + (rowbase + Bq.tq) * P.q_ld + head * HS + d0, lb && Bq.tq < T && d0 < HS);
  }
  __syncthreads();
  for (int j = 0; j < P.nstreams; ++j) {
    A.m = -INFINITY; A.l = 0.f; Bq.m = -INFINITY; Bq.l = 0.f;
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt) { zero16(A.o[dt]); zero16(Bq.o[dt]); }
    for (int c = 0; c < nch; ++c) {
      const uint32_t* mska = msk + (DROP ? w * MKT * 32 : 0);        // keep-bit tiles of qa, qb
      const uint32_t* mskb = msk + (DROP ? (7 - w) * MKT * 32 : 0);  // (chunk tile kt - kt_lo)
      const int kt_lo = c * MKT;
      const int kt_hi = min(kt_lo + MKT, nt) - 1;
#define FWD_STEP(NQ, DA, DB, KT) \
  fwd_step<HS, NQ, DA, DB, DROP>(ks, vs, ((KT) - kt_lo) * 32, (KT) * 32, A, Bq, mska + ((KT) - kt_lo) * 32, \
                                 mskb + ((KT) - kt_lo) * 32, c2, lane)
#define FWD_STEP_B(DB, KT) \
  fwd_step<HS, 1, DB, false, DROP>(ks, vs, ((KT) - kt_lo) * 32, (KT) * 32, Bq, A, mskb + ((KT) - kt_lo) * 32, \
                                   mska, c2, lane)
      if (lb) {
        int kt = kt_lo;
#pragma unroll 1
        for (; kt <= min(qa - 1, kt_hi); ++kt) FWD_STEP(2, false, false, kt);  // both tiles, off the diagonal
        if (qa >= kt_lo && qa <= kt_hi) FWD_STEP(2, true, false, qa);        // tile a's diagonal
#pragma unroll 1
        for (kt = max(kt_lo, qa + 1); kt <= min(qb - 1, kt_hi); ++kt) FWD_STEP_B(false, kt);
        if (qb >= kt_lo && qb <= kt_hi) FWD_STEP_B(true, qb);
      } else if (la) {
#pragma unroll 1
        for (int kt = kt_lo; kt <= min(qa - 1, kt_hi); ++kt) FWD_STEP(1, false, false, kt);
        if (qa >= kt_lo && qa <= kt_hi) FWD_STEP(1, true, false, qa);
      }
#undef FWD_STEP
#undef FWD_STEP_B
      // next (stream, chunk) resident for the whole block
      int nj = j, nc = c + 1;
      if (nc == nch) { nc = 0; ++nj; }
      if (nj < P.nstreams && (nj != j || nc != c)) {
        __syncthreads();
        st.load(P.k[nj] + head * P.kv_hstride, P.kv_ld, P.v[nj] + head * P.kv_hstride, P.kv_ld, rowbase, nc * ROWS,
                T, tid);
        if (DROP) mst.load(P.dmask[nj] + lw_off, bh, nt, qt0, nc * (ROWS / 32), true, tid);
        st.store(ks, G::RW, vs, G::TW, tid);
        if (DROP) mst.store(msk, tid);
        __syncthreads();
      }
    }
    // normalise this stream's outputs and keep its LSE. One stream: the output itself; several:
    // each stream's own output (the backward reads it), summed below
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool live = u == 0 ? la : lb;
      FwdQ<HS>& q = u == 0 ? A : Bq;
      const float l = xhalf_sum(q.l);
      const float inv = (l > 0.f) ? (DROP ? P.drop_scale : 1.f) / l : 0.f;
      // row-per-lane O^T halves (lane r: d 8g..8g+3, lane r + 32: 8g+4..8g+7) exchanged across the
      // wave halves by v_permlane32_swap so every lane holds 8 consecutive d of its row: 16-B stores,
      // half the store instructions of the 8-B form (the epilogue store tail is issue-bound). The
      // swaps run on every lane (both halves of a row are live or dead together).
      u32x4 ov[G::ND][2];
#pragma unroll
      for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const int ga = 2 * pr, gb = 2 * pr + 1;
          const uint32_t x0 = pack2bf(q.o[dt][4 * ga] * inv, q.o[dt][4 * ga + 1] * inv);
          const uint32_t x1 = pack2bf(q.o[dt][4 * ga + 2] * inv, q.o[dt][4 * ga + 3] * inv);
          const uint32_t y0 = pack2bf(q.o[dt][4 * gb] * inv, q.o[dt][4 * gb + 1] * inv);
          const uint32_t y1 = pack2bf(q.o[dt][4 * gb + 2] * inv, q.o[dt][4 * gb + 3] * inv);
          const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
          ov[dt][pr] = u32x4{s0[0], s1[0], s0[1], s1[1]};  // d = dt*32 + 16 pr + 8 h + 0..7
        }
      if (live && q.tq < T) {
        if (h == 0) P.lse[j][(int64_t)bh * T + q.tq] = q.m + __log2f(l);  // log2 domain
        bf16_t* dst = (P.nstreams > 1 ? P.oj[j] : P.o) + (rowbase + q.tq) * P.o_ld + head * HS;
#pragma unroll
        for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            const int d0 = dt * 32 + 16 * pr + 8 * h;
            if (d0 < HS) *reinterpret_cast<u32x4*>(dst + d0) = ov[dt][pr];
          }
      }
    }
  }
  // several streams: the output is the sum of the per-stream outputs this lane just wrote (kept
  // out of registers: a running fp32 total would pin another O-sized accumulator set)
  if (P.nstreams > 1) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool live = u == 0 ? la : lb;
      const int tq = u == 0 ? A.tq : Bq.tq;
      if (!(live && tq < T)) continue;
      const int64_t off = (rowbase + tq) * P.o_ld + head * HS;
#pragma unroll
      for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const int d0 = dt * 32 + 16 * pr + 8 * h;  // the 16-B pieces this lane wrote
          if (d0 >= HS) continue;
          float t[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          for (int jj = 0; jj < P.nstreams; ++jj) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(P.oj[jj] + off + d0);
#pragma unroll
            for (int e = 0; e < 4; ++e) { t[2 * e] += bf2f(v[e] & 0xffff); t[2 * e + 1] += bf2f(v[e] >> 16); }
          }
          *reinterpret_cast<u32x4*>(P.o + off + d0) =
              u32x4{pack2bf(t[0], t[1]), pack2bf(t[2], t[3]), pack2bf(t[4], t[5]), pack2bf(t[6], t[7])};
        }
    }
  }
}

// per query tile state of the dQ walk: Q / dO fragments, the row's log2-domain LSE and D, dQ^T
template <int HS>
struct DqQ {
  bf16x8 qf[Geo<HS>::NKS], dof[Geo<HS>::NKS];
  f32x16 dq[Geo<HS>::ND];
  float lse2, dsum;
  int tq;
};

// dS^T of one tile for one query tile (in place in sacc), packed to the two bf16 operand fragments
template <int HS, bool diag, bool DROP>
__device__ __forceinline__ void dq_ds(f32x16& sacc, const f32x16& dpacc, const DqQ<HS>& q, int k0, float c2,
                                      float dsc, uint32_t mw, int h, bf16x8 (&df)[2]) {
  const float nl = -q.lse2, nd = -q.dsum;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    float pv = ex2(__builtin_fmaf(sacc[e], c2, nl));
    if (diag) {
      const int key = k0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (key > q.tq) pv = 0.f;
    }
    float dp = dpacc[e];
    if (DROP) dp = keep_f(dp, elem_keep(mw, e));
    sacc[e] = pv * __builtin_fmaf(dp, dsc, nd);  // dS^T = P (Z.dP - D) (dropped: -P D)
  }
  df[0] = acc_frag(sacc, 0);
  df[1] = acc_frag(sacc, 1);
}

// dQ step over one 32-key tile for one or two query tiles: S^T, dP^T recomputed, dQ^T += K^T dS^T.
// The K / V row fragments and the transposed K fragments are read once for both tiles and issued
// up front (the transposed ones land behind the dS arithmetic)
template <int HS, int NQ, bool DA, bool DB, bool DROP>
__device__ __forceinline__ void dq_step(const bf16_t* ks, const bf16_t* vs, const bf16_t* kts, int kts_ld, int kl,
                                        int k0, DqQ<HS>& a, DqQ<HS>& b, const uint32_t* mta, const uint32_t* mtb,
                                        float c2, const AttnProblem& P, int lane) {
  using G = Geo<HS>;
  const int r = lane & 31, h = lane >> 5;
  const uint32_t wa = DROP ? reinterpret_cast<const uint16_t*>(mta)[lane] : 0u;  // keep bits (LDS)
  const uint32_t wb = (DROP && NQ == 2) ? reinterpret_cast<const uint16_t*>(mtb)[lane] : 0u;
  f32x16 sa, pa, sb, pb;
  zero16(sa);
  zero16(pa);
  if (NQ == 2) { zero16(sb); zero16(pb); }
  constexpr bool SL = SliceImg<HS>::on;
  if (NQ == 2) {
    bf16x8 kf[G::NKS], vf[G::NKS];
#pragma unroll
    for (int s = 0; s < G::NKS; ++s) {
      kf[s] = SL ? sl_row(ks, kl, r, s, h) : *reinterpret_cast<const bf16x8*>(ks + (kl + r) * G::RW + 16 * s + 8 * h);
      vf[s] = SL ? sl_row(vs, kl, r, s, h) : *reinterpret_cast<const bf16x8*>(vs + (kl + r) * G::RW + 16 * s + 8 * h);
    }
#pragma unroll
    for (int s = 0; s < G::NKS; ++s) {
      sa = mfma32(kf[s], a.qf[s], sa);
      pa = mfma32(vf[s], a.dof[s], pa);
      sb = mfma32(kf[s], b.qf[s], sb);
      pb = mfma32(vf[s], b.dof[s], pb);
    }
  } else {  // register-lean order (hs >= 48)
#pragma unroll
    for (int s = 0; s < G::NKS; ++s) {
      const bf16x8 kf = SL ? sl_row(ks, kl, r, s, h) : *reinterpret_cast<const bf16x8*>(ks + (kl + r) * G::RW + 16 * s + 8 * h);
      const bf16x8 vf = SL ? sl_row(vs, kl, r, s, h) : *reinterpret_cast<const bf16x8*>(vs + (kl + r) * G::RW + 16 * s + 8 * h);
      sa = mfma32(kf, a.qf[s], sa);
      pa = mfma32(vf, a.dof[s], pa);
    }
  }
  const float dsc = DROP ? P.drop_scale : 1.f;
  bf16x8 dfa[2], dfb[2];
  if (NQ == 2) {
    bf16x8 kt[2][G::ND];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < G::ND; ++dt) kt[s][dt] = SL ? sl_tr(kts, kl, s, lane) : tr_frag(kts + kl * kts_ld, kts_ld, dt, s, lane);
    dq_ds<HS, DA, DROP>(sa, pa, a, k0, c2, dsc, wa, h, dfa);
    dq_ds<HS, DB, DROP>(sb, pb, b, k0, c2, dsc, wb, h, dfb);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < G::ND; ++dt) {
        a.dq[dt] = mfma32(kt[s][dt], dfa[s], a.dq[dt]);
        b.dq[dt] = mfma32(kt[s][dt], dfb[s], b.dq[dt]);
      }
  } else {
    dq_ds<HS, DA, DROP>(sa, pa, a, k0, c2, dsc, wa, h, dfa);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < G::ND; ++dt)
        a.dq[dt] = mfma32(SL ? sl_tr(kts, kl, s, lane) : tr_frag(kts + kl * kts_ld, kts_ld, dt, s, lane), dfa[s], a.dq[dt]);
  }
}

// =============================================================================================
// backward dQ (also writes D_j = rowsum(dO * O_j) for the dK/dV pass); grid as forward, and like the
// forward each wave walks its two query tiles together
// =============================================================================================
template <int HS, bool DROP>
__global__ __launch_bounds__(256, MMT_DQ_MINB(HS)) void attn_bwd_dq_kernel(AttnBatch batch, int T, int H,
                                                                                       float scale) {
  using G = Geo<HS>;
  // chunk rows: hs >= 48 stages 256-row chunks (two 128-row register rounds; 80 KB of LDS, still two
  // blocks per CU, which is what the registers allow): half the reloads and barriers of 128-row
  // chunks, and at T = 512 each chunk holds either a whole causal triangle or a full rectangle, so
  // the four waves' work per chunk is balanced
  constexpr int SR = Chunk<HS>::ROWS;
  constexpr int ROWS = HS >= 48 ? 256 : SR;
  constexpr int NR = ROWS / SR;
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nb = ((T + 31) / 32 + 7) / 8;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int bh = tile / nb, b = bh / H, head = bh % H;
  const int bx = tile % nb;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int nt = (T + 31) / 32;
  const int qt0 = bx * 8;
  const int qmax = min(qt0 + 7, nt - 1);
  const int nch = (min((qmax + 1) * 32, T) + ROWS - 1) / ROWS;
  const int64_t rowbase = (int64_t)b * T;
  const float c2 = scale * kLog2e;
  __shared__ __attribute__((aligned(16))) bf16_t ks[ROWS * G::RW];  // K chunk: row (+ tr at hs > 32) reads
  __shared__ __attribute__((aligned(16))) bf16_t vs[ROWS * G::RW];  // V chunk: row reads
  const bf16_t* kts = ks;
  constexpr int KTS_LD = G::RW;
  using MS = MaskStager<HS, ROWS / 32>;
  __shared__ __attribute__((aligned(16))) uint32_t msk[DROP ? MS::DWORDS : 4];  // keep-bit lane words
  if (HS % 32 != 0) {  // pad columns are read only when HS is not a multiple of 32
    for (int q = tid; q < ROWS * G::RW; q += 256)
      if (q % G::RW >= HS) { ks[q] = 0; vs[q] = 0; }
  }
  Stager<HS> st;
  MS mst;
  // lane-word record of the keep bits (AttnProblem::dmask): after the key-major one
  const int64_t lw_off = (int64_t)(gridDim.x / nb) * (nt * (nt + 1) / 2) * 32;
  auto stage = [&](int jj, int cc) {  // K / V rows [cc*ROWS, +ROWS) of stream jj and their keep bits
    if (DROP) mst.load(P.dmask[jj] + lw_off, bh, nt, qt0, cc * (ROWS / 32), true, tid);
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      st.load(P.k[jj] + head * P.kv_hstride, P.kv_ld, P.v[jj] + head * P.kv_hstride, P.kv_ld, rowbase,
              cc * ROWS + rr * SR, T, tid);
      if constexpr (SliceImg<HS>::on) st.store_slices(ks + rr * SR * G::RW, vs + rr * SR * G::RW, tid);
      else st.store(ks + rr * SR * G::RW, G::RW, vs + rr * SR * G::RW, G::RW, tid);
    }
    if (DROP) mst.store(msk, tid);
  };
  stage(0, 0);
  __syncthreads();

  const int qa = qt0 + w, qb = qt0 + 7 - w;  // qa < qb; lb implies la
  const bool la = qa < nt, lb = qb < nt;
  const uint32_t* mska = msk + (DROP ? w * MS::KT * 32 : 0);        // keep-bit tiles of qa, qb
  const uint32_t* mskb = msk + (DROP ? (7 - w) * MS::KT * 32 : 0);  // (chunk tile kt - kt_lo)
  DqQ<HS> A, Bq;
  A.tq = qa * 32 + r;
  Bq.tq = qb * 32 + r;
  const bool oka = la && A.tq < T, okb = lb && Bq.tq < T;
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    const int d0 = 16 * s + 8 * h;
    A.qf[s] = ld8(P.q + (rowbase + A.tq) * P.q_ld + head * HS + d0, oka && d0 < HS);
    A.dof[s] = ld8(P.dout + (rowbase + A.tq) * P.dout_ld + head * HS + d0, oka && d0 < HS);
    Bq.qf[s] = ld8(P.q + (rowbase + Bq.tq) * P.q_ld + head * HS + d0, okb && d0 < HS);
    Bq.dof[s] = ld8(P.dout + (rowbase + Bq.tq) * P.dout_ld + head * HS + d0, okb && d0 < HS);
  }
#pragma unroll
  for (int dt = 0; dt < G::ND; ++dt) { zero16(A.dq[dt]); zero16(Bq.dq[dt]); }
  for (int j = 0; j < P.nstreams; ++j) {
    const bf16_t* oj = (P.nstreams > 1) ? P.oj[j] : P.o;
    float dsa = 0.f, dsb = 0.f;
#pragma unroll
    for (int s = 0; s < G::NKS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bf16x8 ova = ld8(oj + (rowbase + A.tq) * P.o_ld + head * HS + d0, oka && d0 < HS);
      const bf16x8 ovb = ld8(oj + (rowbase + Bq.tq) * P.o_ld + head * HS + d0, okb && d0 < HS);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dsa += (float)ova[e] * (float)A.dof[s][e];
        dsb += (float)ovb[e] * (float)Bq.dof[s][e];
      }
    }
    dsa = xhalf_sum(dsa);
    dsb = xhalf_sum(dsb);
    if (h == 0) {  // D_j / drop_scale for the dK/dV pass (dkdv_tile: dS = sc (Z P dP - P D / sc))
      const float inv = DROP ? 1.0f / P.drop_scale : 1.0f;
      if (oka) P.dvec[j][(int64_t)bh * T + A.tq] = dsa * inv;
      if (okb) P.dvec[j][(int64_t)bh * T + Bq.tq] = dsb * inv;
    }
    A.dsum = dsa;
    Bq.dsum = dsb;
    A.lse2 = oka ? P.lse[j][(int64_t)bh * T + A.tq] : 0.f;
    Bq.lse2 = okb ? P.lse[j][(int64_t)bh * T + Bq.tq] : 0.f;
    for (int c = 0; c < nch; ++c) {
      const int kt_lo = c * (ROWS / 32);
      const int kt_hi = min(kt_lo + ROWS / 32, nt) - 1;
#define DQ_STEP(NQ, DA, DB, KT) \
  dq_step<HS, NQ, DA, DB, DROP>(ks, vs, kts, KTS_LD, ((KT) - kt_lo) * 32, (KT) * 32, A, Bq, mska + ((KT) - kt_lo) * 32, \
                                mskb + ((KT) - kt_lo) * 32, c2, P, lane)
#define DQ_STEP_B(DB, KT) \
  dq_step<HS, 1, DB, false, DROP>(ks, vs, kts, KTS_LD, ((KT) - kt_lo) * 32, (KT) * 32, Bq, A, mskb + ((KT) - kt_lo) * 32, mska, \
                                  c2, P, lane)
      if (lb) {
        int kt = kt_lo;
        // hs >= 48: the two tiles' S / dP accumulators do not fit beside their Q / dO / dQ state
        // (two waves per SIMD), so the tiles take turns (each re-reads the K / V fragments)
        constexpr int NQ2 = HS >= 48 ? 1 : 2;
#pragma unroll 1
        for (; kt <= min(qa - 1, kt_hi); ++kt) {
          DQ_STEP(NQ2, false, false, kt);
          if (NQ2 == 1) DQ_STEP_B(false, kt);
        }
        if (qa >= kt_lo && qa <= kt_hi) {
          DQ_STEP(NQ2, true, false, qa);
          if (NQ2 == 1) DQ_STEP_B(false, qa);
        }
#pragma unroll 1
        for (kt = max(kt_lo, qa + 1); kt <= min(qb - 1, kt_hi); ++kt) DQ_STEP_B(false, kt);
        if (qb >= kt_lo && qb <= kt_hi) DQ_STEP_B(true, qb);
      } else if (la) {
#pragma unroll 1
        for (int kt = kt_lo; kt <= min(qa - 1, kt_hi); ++kt) DQ_STEP(1, false, false, kt);
        if (qa >= kt_lo && qa <= kt_hi) DQ_STEP(1, true, false, qa);
      }
#undef DQ_STEP
#undef DQ_STEP_B
      int nj = j, nc = c + 1;
      if (nc == nch) { nc = 0; ++nj; }
      if (nj < P.nstreams && (nj != j || nc != c)) {
        __syncthreads();
        stage(nj, nc);
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const bool ok = u == 0 ? oka : okb;
    const DqQ<HS>& q = u == 0 ? A : Bq;
    // 16-B stores of 8 consecutive d per lane after a v_permlane32_swap exchange of the row halves
    // (as the forward's O); the swaps run on every lane
    u32x4 dv[G::ND][2];
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int ga = 2 * pr, gb = 2 * pr + 1;
        const uint32_t x0 = pack2bf(q.dq[dt][4 * ga] * scale, q.dq[dt][4 * ga + 1] * scale);
        const uint32_t x1 = pack2bf(q.dq[dt][4 * ga + 2] * scale, q.dq[dt][4 * ga + 3] * scale);
        const uint32_t y0 = pack2bf(q.dq[dt][4 * gb] * scale, q.dq[dt][4 * gb + 1] * scale);
        const uint32_t y1 = pack2bf(q.dq[dt][4 * gb + 2] * scale, q.dq[dt][4 * gb + 3] * scale);
        const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        dv[dt][pr] = u32x4{s0[0], s1[0], s0[1], s1[1]};
      }
    if (ok) {
#pragma unroll
      for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const int d0 = dt * 32 + 16 * pr + 8 * h;
          if (d0 < HS) *reinterpret_cast<u32x4*>(P.dq + (rowbase + q.tq) * P.dq_ld + head * HS + d0) = dv[dt][pr];
        }
    }
  }
}

// dK, dV: one 32x32 (queries x keys) tile; S, dP recomputed, dV += P^T dO, dK += dS^T Q
template <int HS, bool MASKED, bool DROP>
__device__ __forceinline__ void dkdv_tile(const bf16_t* qs, const bf16_t* dos, const float* lsl, const float* dsl,
                                          int ql, int q0, int tk, int T,
                                          const bf16x8 (&kf)[Geo<HS>::NKS], const bf16x8 (&vf)[Geo<HS>::NKS],
                                          f32x16 (&dk)[Geo<HS>::ND], f32x16 (&dv)[Geo<HS>::ND], float c2,
                                          const AttnProblem& P, const uint32_t* mt, int lane) {
  using G = Geo<HS>;
  const int r = lane & 31, h = lane >> 5;
  // key r's keep bits over the tile's queries, this lane's half (queries 8g + 4h + e4) at bits 8g + e4
  const uint32_t mw = DROP ? mt[key_dword(r)] >> (4 * h) : 0u;
  f32x16 sacc, dpacc;
  zero16(sacc);
  zero16(dpacc);
  // every LDS read of the tile is issued up front, in the order it is consumed (row fragments for
  // S and dP, then the transposed Q / dO fragments for dK / dV behind the softmax VALU): the
  // compiler then waits on counted lgkmcnt instead of a read -> wait -> MFMA chain per fragment
  bf16x8 qr[G::NKS], dr[G::NKS];
  constexpr bool SL = SliceImg<HS>::on;
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    qr[s] = SL ? sl_row(qs, ql, r, s, h) : *reinterpret_cast<const bf16x8*>(qs + (ql + r) * G::RW + 16 * s + 8 * h);
    dr[s] = SL ? sl_row(dos, ql, r, s, h) : *reinterpret_cast<const bf16x8*>(dos + (ql + r) * G::RW + 16 * s + 8 * h);
  }
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    sacc = mfma32(qr[s], kf[s], sacc);    // S[q][key]
    dpacc = mfma32(dr[s], vf[s], dpacc);  // dP[q][key]
  }
  bf16x8 dot[2][G::ND], qtr[2][G::ND];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt) {
      dot[s][dt] = SL ? sl_tr(dos, ql, s, lane) : tr_frag(dos + ql * G::RW, G::RW, dt, s, lane);
      qtr[s][dt] = SL ? sl_tr(qs, ql, s, lane) : tr_frag(qs + ql * G::RW, G::RW, dt, s, lane);
    }
  f32x4 l4[4], d4[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    l4[g] = *reinterpret_cast<const f32x4*>(lsl + ql + 8 * g + 4 * h);
    d4[g] = *reinterpret_cast<const f32x4*>(dsl + ql + 8 * g + 4 * h);
  }
  uint32_t pp[8], dd[8];  // packed bf16 pairs of Z.P (dV operand) and dS (dK operand)
#pragma unroll
  for (int g = 0; g < 4; ++g) {
#pragma unroll
    for (int e4 = 0; e4 < 4; e4 += 2) {
      float pm[2], ds[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = 4 * g + e4 + u;
        float pv = ex2(__builtin_fmaf(sacc[e], c2, l4[g][e4 + u]));
        if (MASKED) {
          const int tq = q0 + 8 * g + 4 * h + e4 + u;
          if (!(tk <= tq && tq < T)) pv = 0.f;
        }
        const float dp = dpacc[e];
        if (DROP) {
          // Z.P without the 1/(1-p) (applied to dV at the end); dS = P (Z dP sc - D) = sc (Z P dP - P D'),
          // D' = D / sc (the dQ pass stores it so), the factor sc applied to dK at the end: one VALU
          // per element fewer than masking dP separately
          int kb = __builtin_amdgcn_sbfe((int)mw, 8 * g + e4 + u, 1);  // all ones iff kept
          // (opaque to the compiler: seen as a one-bit test it lowered bfe + and into and + cmp + cndmask)
          asm volatile("" : "+v"(kb));
          pm[u] = keep_f(pv, kb);
          ds[u] = __builtin_fmaf(pm[u], dp, pv * d4[g][e4 + u]);  // dS[q][key] / sc
        } else {
          pm[u] = pv;
          ds[u] = pv * (dp + d4[g][e4 + u]);  // dS[q][key]
        }
      }
      pp[2 * g + e4 / 2] = pack2bf(pm[0], pm[1]);
      dd[2 * g + e4 / 2] = pack2bf(ds[0], ds[1]);
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 pf = __builtin_bit_cast(bf16x8, u32x4{pp[4 * s], pp[4 * s + 1], pp[4 * s + 2], pp[4 * s + 3]});
    const bf16x8 df = __builtin_bit_cast(bf16x8, u32x4{dd[4 * s], dd[4 * s + 1], dd[4 * s + 2], dd[4 * s + 3]});
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt) {
      dv[dt] = mfma32(pf, dot[s][dt], dv[dt]);
      dk[dt] = mfma32(df, qtr[s][dt], dk[dt]);
    }
  }
}

// Block-uniform walk over (tile u, stream j, chunk c): the chunk (j, c) resident in LDS is reused
// while consecutive steps share it (T <= ROWS with one stream: a single load for the whole block).
struct ChunkWalk {
  int ns, nch;
  __device__ __forceinline__ bool next(int u, int j, int c, int& nj, int& nc) const {
    nj = j; nc = c + 1;
    int nu = u;
    if (nc == nch) { nc = 0; ++nj; if (nj == ns) { nj = 0; ++nu; } }
    return nu < 2 && (nj != j || nc != c);
  }
};

// =============================================================================================
// backward dK, dV: grid (ceil(nt/8), B*H*nstreams, G); wave w owns key tiles 8*bx + w, 8*bx + 7 - w
// =============================================================================================
template <int HS, bool DROP>
__global__ __launch_bounds__(256, MMT_DKDV1_MINB(HS)) void attn_bwd_dkdv1_kernel(AttnBatch batch, int T, int H, float scale) {
  using G = Geo<HS>;
  constexpr int ROWS = Chunk<HS>::ROWS;
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nb = ((T + 31) / 32 + 7) / 8;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int yy = tile / nb, bx = tile % nb;
  const int nbh = gridDim.x / nb / P.nstreams;
  if (yy >= nbh * P.nstreams) return;
  const int j = yy / nbh;
  const int bh = yy % nbh;
  const int b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int nt = (T + 31) / 32;
  const int kt0 = bx * 8;
  const int q_lo = kt0 * 32;
  const ChunkWalk walk{1, (T - q_lo + ROWS - 1) / ROWS};
  const bool ragged = (T & 31) != 0;
  const int qlast = ragged ? nt - 1 : nt;  // the ragged last query tile (masked); nt: none
  const int64_t rowbase = (int64_t)b * T;
  const float c2 = scale * kLog2e;
  __shared__ __attribute__((aligned(16))) bf16_t qs[ROWS * G::RW];   // Q chunk: row + tr reads
  __shared__ __attribute__((aligned(16))) bf16_t dos[ROWS * G::RW];  // dO chunk: row + tr reads
  __shared__ __attribute__((aligned(16))) float lsd[2][ROWS];        // -log2-domain LSE, -D of the chunk rows
  using MS = MaskStager<HS>;
  __shared__ __attribute__((aligned(16))) uint32_t msk[DROP ? MS::DWORDS : 4];  // [key tile][chunk q tile]
  // epilogue transpose slots, one 32-column slice at a time: per wave [dK, dV][32 keys][EPW]
  constexpr int EPW = 40;
  __shared__ __attribute__((aligned(16))) bf16_t ept[4 * 2 * 32 * EPW];
  if (HS % 32 != 0)  // pad columns are read only when HS is not a multiple of 32
    for (int q = tid; q < ROWS * G::RW; q += 256)
      if (q % G::RW >= HS) { qs[q] = 0; dos[q] = 0; }

  const bf16_t* kp = P.k[j] + head * P.kv_hstride;
  const bf16_t* vp = P.v[j] + head * P.kv_hstride;
  const float* lsep = P.lse[j] + (int64_t)bh * T;
  const float* dvp = P.dvec[j] + (int64_t)bh * T;
  const bf16_t* qp = P.q + head * HS;
  const bf16_t* dop = P.dout + head * HS;
  constexpr int NSL = 2 * ROWS / 256;
  Stager<HS> st;
  MS mst;
  float sl[NSL];
  auto load = [&](int r0) {
    st.load(qp, P.q_ld, dop, P.dout_ld, rowbase, r0, T, tid);
    if (DROP) mst.load(P.dmask[j], bh, nt, kt0, r0 / 32, false, tid);
#pragma unroll
    for (int u = 0; u < NSL; ++u) {
      const int c = tid + 256 * u;
      const int t = r0 + (c % ROWS);
      sl[u] = t < T ? ((c < ROWS) ? -lsep[t] : -dvp[t]) : 0.f;  // negated: fma addends
    }
  };
  auto store = [&]() {
    if constexpr (SliceImg<HS>::on) st.store_slices(qs, dos, tid);
    else st.store(qs, G::RW, dos, G::RW, tid);
    if (DROP) mst.store(msk, tid);
#pragma unroll
    for (int u = 0; u < NSL; ++u) {
      const int c = tid + 256 * u;
      lsd[c / ROWS][c % ROWS] = sl[u];
    }
  };
  load(q_lo);
  store();
  __syncthreads();

#pragma unroll 1
  for (int u = 0; u < 2; ++u) {
    const int kt = u == 0 ? kt0 + w : kt0 + 7 - w;
    const bool live = kt < nt;
    const int tk = kt * 32 + r;
    bf16x8 kf[G::NKS], vf[G::NKS];
    f32x16 dk[G::ND], dv[G::ND];
#pragma unroll
    for (int s = 0; s < G::NKS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bool ok = live && tk < T && d0 < HS;
      kf[s] = ld8(kp + (rowbase + tk) * P.kv_ld + d0, ok);
      vf[s] = ld8(vp + (rowbase + tk) * P.kv_ld + d0, ok);
    }
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt) { zero16(dk[dt]); zero16(dv[dt]); }
    for (int c = 0; c < walk.nch; ++c) {
      int nj, nc;
      const bool reload = walk.next(u, 0, c, nj, nc);
      const int r0 = q_lo + c * ROWS;
      if (live) {
        const int qt_lo = r0 / 32, qt_hi = min(qt_lo + ROWS / 32, nt) - 1;
        const uint32_t* mk = msk + (kt - kt0) * MS::KT * 32;
        auto tile = [&](auto mc, int qt) {
          dkdv_tile<HS, decltype(mc)::value, DROP>(qs, dos, lsd[0], lsd[1], qt * 32 - r0, qt * 32, tk, T, kf, vf, dk, dv,
                                                   c2, P, mk + (qt - qt_lo) * 32, lane);
        };
        int qt = max(kt, qt_lo);  // diagonal and ragged last tile masked, peeled (see the paired kernel)
        if (qt == kt && qt <= qt_hi) tile(std::true_type{}, qt++);
        const int qe = min(qt_hi, qlast - 1);
#pragma unroll 1
        for (; qt <= qe; ++qt) tile(std::false_type{}, qt);
        if (qt <= qt_hi) tile(std::true_type{}, qt);
      }
      if (reload) {
        __syncthreads();
        load(q_lo + nc * ROWS);
        store();
        __syncthreads();
      }
    }
    // dK/dV tiles: accumulator rows = key ((e&3)+8(e>>2)+4h), cols = d (lane). Each 32-column slice
    // is transposed through this wave's LDS slot (ds_write_b16 at immediate offsets) and leaves as
    // row-major 16-B pieces: 2 dwordx4 per lane per matrix and slice instead of 16 two-byte stores
    // with a 64-bit address computation each
    if (live) {
      bf16_t* et = ept + w * (2 * 32 * EPW);
      const int k0 = kt * 32;
      const float dks = DROP ? scale * P.drop_scale : scale;  // dS was accumulated divided by drop_scale
#pragma unroll
      for (int dt = 0; dt < G::ND; ++dt) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int kr = (e & 3) + 8 * (e >> 2) + 4 * h;
          et[kr * EPW + r] = f2bf(dk[dt][e] * dks);
          et[32 * EPW + kr * EPW + r] = f2bf(DROP ? dv[dt][e] * P.drop_scale : dv[dt][e]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = i * 16 + (lane >> 2), d0 = dt * 32 + (lane & 3) * 8;
          const u32x4 vk = *reinterpret_cast<const u32x4*>(et + row * EPW + (lane & 3) * 8);
          const u32x4 vv = *reinterpret_cast<const u32x4*>(et + 32 * EPW + row * EPW + (lane & 3) * 8);
          if (k0 + row < T && d0 < HS) {
            const int64_t off = (rowbase + k0 + row) * P.dkv_ld + d0;
            *reinterpret_cast<u32x4*>(P.dk[j] + head * P.dkv_hstride + off) = vk;
            *reinterpret_cast<u32x4*>(P.dv[j] + head * P.dkv_hstride + off) = vv;
          }
        }
      }
    }
  }
}

// =============================================================================================
// One-pass backward at hs 32 for T <= 256 and one KV stream (C1's self-attention; round 6).
// grid (B*H, 1, problems): one workgroup (4 waves; two workgroups per CU) per (batch, head) owns all
// nt <= 8 key tiles, so S and dP -- and their softmax / dropout VALU -- are computed ONCE per tile
// (the two-pass kernels above recompute both in the dQ pass: 14 products per tile instead of 10)
// and dQ needs no sum across workgroups:
//  * Q and dO of the whole sequence land in LDS by LDS-DMA as slice images (SliceImg: conflict-free
//    row AND transposed reads); D = rowsum(dO O) and the negated log2-domain LSE of every query go
//    into LDS tables (thread t: query t);
//  * wave w owns key tiles w and 7 - w (9 tile pairs of the causal walk each at nt = 8): their K / V
//    rows (keys on lanes: the B operands of S and dP) and K^T (the A operand of dQ, transposed once
//    through the wave's LDS slot) stay in registers, and so do their dK / dV accumulators;
//  * all waves walk the query tiles in step, one barrier per tile: for each owned key tile kt <= qt,
//    S = Q K^T, dP = dO V^T, P = exp2(c2 S - LSE2), dS = P (Z dP - D); dV += (Z P)^T dO and
//    dK += dS^T Q take P and dS straight from the accumulators as A operands (keys on lanes); dS
//    crosses the wave's LDS slot once and dQ_w^T += K^T dS^T runs on MFMA;
//  * each wave's fp32 dQ partial of the step goes to an LDS tile (double-buffered by step parity, so
//    one barrier per step suffices); after the barrier wave w sums rows 8w .. 8w+7 over the waves
//    that had tiles, scales, converts and stores them.
// LDS 78 KiB (two workgroups per CU): Q / dO images 2 x 18 KiB, tables 2 KiB, slots 4 x 2 KiB, dQ
// partials 2 x 4 x 4 KiB. dS is accumulated divided by the dropout scale sc (as the dK/dV pass:
// dS / sc = Z P dP - P D'), so dK and dQ take the factor sc at the end.
// =============================================================================================
namespace {
typedef int32_t ai32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ ai32x4 a_rsrc(const void* base, int64_t bytes) {
  const uint64_t a = (uint64_t)base;
  ai32x4 rs;
  rs[0] = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
  rs[1] = __builtin_amdgcn_readfirstlane((int32_t)((a >> 32) & 0xffffu));
  rs[2] = __builtin_amdgcn_readfirstlane((int32_t)min(bytes, (int64_t)0x7ffffff0));
  rs[3] = 0x00020000;
  return rs;
}
__device__ __forceinline__ uint32_t a_lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
// 16 B per lane: LDS[lds + 16 lane] = buffer[voff] (zeros when voff is out of range)
__device__ __forceinline__ void a_dma16(const ai32x4& rsrc, uint32_t lds, int voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" : : "s"(lds), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}
// 8 B per lane: buffer[voff] = v (dropped when voff is out of range): one store instruction whatever
// the lanes' rows, so counted vmcnt waits can include it
__device__ __forceinline__ void a_bst8(const ai32x4& rsrc, int voff, u32x2 v) {
  asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen" : : "v"(v), "v"(voff), "s"(rsrc) : "memory");
}
__device__ __forceinline__ void a_bst16(const ai32x4& rsrc, int voff, f32x4 v) {
  asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" : : "v"(v), "v"(voff), "s"(rsrc) : "memory");
}
// counted wait on this wave's outstanding vector-memory operations (immediate operand, n <= 8)
__device__ __forceinline__ void a_wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}
constexpr int A_OOB = 0x7fffffff;
// sum over the 32 lanes of each wave half: quad and row rotations by DPP, one cross-row shuffle
__device__ __forceinline__ float a_dpp(float v, int ctl) {
  return __builtin_bit_cast(float, ctl == 0xB1 ? __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true)
                                  : ctl == 0x4E ? __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true)
                                  : ctl == 0x124 ? __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, true)
                                                 : __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, true));
}
__device__ __forceinline__ float a_sum32(float v) {
  v += a_dpp(v, 0xB1);   // quad_perm [1, 0, 3, 2]
  v += a_dpp(v, 0x4E);   // quad_perm [2, 3, 0, 1]
  v += a_dpp(v, 0x124);  // row_ror 4
  v += a_dpp(v, 0x128);  // row_ror 8
  return v + __shfl_xor(v, 16, 64);
}
}  // namespace

#ifndef MMT_F32_BRANCH
#define MMT_F32_BRANCH 0
#endif
#ifndef MMT_F32_REV
#define MMT_F32_REV 0
#endif
#ifndef MMT_F32_Q2_NOATOM
#define MMT_F32_Q2_NOATOM 0  // timing experiment: the stage-2 dW2 sums not added (wrong gradient)
#endif
#ifndef MMT_F32_PAIR
#define MMT_F32_PAIR 0  // 1: the two-tile body where both owned key tiles are active (register copies: slower)
#endif
// MS: several KV streams (cross-attention); Q2: the Q/K/V stage-2 backward fused into the epilogue
// (AttnProblem::q2_*, self-attention only)
#ifndef MMT_F32_NB
// 1: one KV stream walked without per-step barriers, dQ summed by LDS float atomics (ds_add_f32). Measured
// (tools/attn_bench.py c1, profiles/r6pq_fused32_nb.txt): 93 -> 309 us with the atomics, 80 us with plain
// stores in their place (wrong sums: the walk itself would gain 14 %); the LDS float atomics cost the
// difference. 2: the free walk with per-step partials summed by each query tile's last contributor
// (correct; 93.9 -> 111.8 us: the one-wave sum sits on the critical path). The per-step partials and
// barrier stay
#define MMT_F32_NB 0
#endif
template <bool DROP, bool MS, bool Q2>
__global__ __launch_bounds__(256, 2) void attn_bwd_fused32(AttnBatch batch, int T, int H, float scale) {
  static_assert(!(MS && Q2), "the stage-2 backward follows the self-attention only");
  // NB (off: see MMT_F32_NB): every wave walks its own (query tile, key tile) products without waiting for the others: the
  // Q / dO images are complete before the walk, and the dQ contributions go into per-tile fp32 sums
  // in LDS ([8 tiles][32 d][32 q], ds_add_f32) instead of per-step partials reduced behind a barrier.
  // The per-step barrier held every wave to the step's slowest (2 tiles against 0-1 elsewhere: 12
  // tile times per walk where each wave owns 9)
  constexpr bool NB = !MS && MMT_F32_NB == 1;
  // NB2 (MMT_F32_NB=2): the same free walk with the per-step partials kept (two slots per wave, tile qt in
  // slot (qt - w) & 1) and summed by the LAST contributor of each query tile (an LDS arrival counter per
  // tile); a wave reuses a slot only after the tile that held it was summed (a done flag per tile)
  constexpr bool NB2 = !MS && MMT_F32_NB == 2;
  constexpr int IMG = 8 * SL_SLICE;               // 256 rows x 32 columns as slice images
  constexpr int OFF_DO = IMG, OFF_TAB = 2 * IMG;  // tables: -LSE2 [256], -D (-D / sc under dropout) [256]
  constexpr int OFF_DS = OFF_TAB + 2048;          // per-wave [32][32] bf16 transpose slots
  constexpr int OFF_DQ = OFF_DS + 4 * 2048;       // dQ partials [2 steps][4 waves][32 q][32 d] fp32
  constexpr int OFF_SYNC = OFF_DQ + 8 * 4096;     // NB2: arrival counters [8], done flags [8]
  constexpr int BYTES = OFF_SYNC + (MMT_F32_NB == 2 ? 64 : 0);
  static_assert(2 * BYTES <= 160 * 1024, "two workgroups per CU");
  constexpr int EPW = 40;                          // epilogue transpose row stride (bf16)
  static_assert(4 * 32 * EPW * 2 <= 4 * 4096, "epilogue transposes alias one parity of the dQ partials");
  __shared__ __attribute__((aligned(1024))) char lds[BYTES];
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nt = (T + 31) / 32;
  const int bh = xcd_tile(blockIdx.x, gridDim.x);
  const int b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int64_t rowbase = (int64_t)b * T;
  const float c2 = scale * kLog2e;
  const bool ragged = (T & 31) != 0;
  const int kts[2] = {w, 7 - w};
  // walk direction: MMT_F32_REV sends the second slot's workgroups of the first generation (blocks
  // 256 .. 511: one per CU) down from the last query tile, so the two co-resident workgroups are in
  // opposite phases of the causal imbalance (light first steps vs heavy last steps)
  const bool rev = MMT_F32_REV && ((blockIdx.x >> 8) & 1);
  auto step_qt = [&](int i) { return rev ? nt - 1 - i : i; };

  // Prologue. Every global load of the kernel is issued here and waited for (pinned) BEFORE the Q / dO
  // slices go out by LDS-DMA (the compiler counts only its own loads, so a wait it places while DMAs it
  // cannot see are in flight would drain them): the keep-bit words of the wave's (step, tile) slots, the
  // K / V rows of its key tiles, this thread's LSE / O / dO row. The slices then land while D, the
  // tables and K^T are built and while the first steps run: step qt waits (counted vmcnt) only for its
  // own piece of slice qt + 1, so the loop issues no other vector-memory operation but one dQ store per
  // step (a buffer store with out-of-range rows dropped: the count is fixed).
  const int64_t ntri = (int64_t)nt * (nt + 1) / 2;
  const int ns = MS ? P.nstreams : 1;
  // cross-attention (several KV streams): the workgroup walks the streams one after the other with Q / dO
  // resident; dQ sums over the streams in the caller's fp32 scratch rows (P.dq32: written by stream 0,
  // read-added by the middle streams, read and converted into dq by the last)
  const ai32x4 rdq32 = a_rsrc(MS ? P.dq32 + rowbase * P.dq32_ld + head * 32 : nullptr, MS ? (int64_t)T * P.dq32_ld * 4 : 0);
#pragma unroll 1
  for (int j = 0; j < ns; ++j) {
  const bf16_t* const oj = MS ? P.oj[j] : P.o;
  uint32_t mwq[2][8];  // keep-bit word of tile t at step q (key r; a FIFO shifted once per step)
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // step i's query tile
      const int q = step_qt(i);
      mwq[t][i] = 0u;
      if (DROP && i < nt && kts[t] <= q)
        mwq[t][i] = P.dmask[j][((int64_t)bh * ntri + q * (q + 1) / 2 + kts[t]) * 32 + key_dword(r)];
    }
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int tk = kts[t] * 32 + r;
    const bool ok = kts[t] < nt && tk < T;
    const bf16_t* kp = P.k[j] + head * P.kv_hstride + (rowbase + tk) * P.kv_ld;
    const bf16_t* vp = P.v[j] + head * P.kv_hstride + (rowbase + tk) * P.kv_ld;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      kf[t][s] = ld8(kp + 16 * s + 8 * h, ok);
      vf[t][s] = ld8(vp + 16 * s + 8 * h, ok);
    }
  }
  float lse_t = 0.f;
  u32x4 ov[4], dv4[4];
  {
    const bool ok = tid < T;
    const int64_t t0 = ok ? tid : 0;
    lse_t = P.lse[j][(int64_t)bh * T + t0];
    const bf16_t* orow = oj + (rowbase + t0) * P.o_ld + head * 32;
    const bf16_t* drow = P.dout + (rowbase + t0) * P.dout_ld + head * 32;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      ov[c] = *reinterpret_cast<const u32x4*>(orow + 8 * c);
      dv4[c] = *reinterpret_cast<const u32x4*>(drow + 8 * c);
    }
  }
  // Q2: W2^T of the head's K / Q / V stage-2 blocks as the A operand of dh1^T = W2^T dX^T (lane: i < 16,
  // k: o = 16 s + 8 h + 0..7; rows i >= 16 zero)
  // (one pinned base, unpredicated loads: lanes r >= 16 read row r - 16's words and drop them)
  bf16x8 w2t[3][2];
  const MMT_AS1 float* const w2p = Q2 ? sgpr_gptr(P.q2_w2) + head * 512 + (r & 15) + 8 * h * 16 : nullptr;
#pragma unroll
  for (int kd = 0; kd < 3; ++kd)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float wv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        wv[e] = Q2 ? w2p[(kd * H * 32 + 16 * s + e) * 16] : 0.f;
        wv[e] = r < 16 ? wv[e] : 0.f;
      }
      w2t[kd][s] = __builtin_bit_cast(bf16x8, u32x4{pack2bf(wv[0], wv[1]), pack2bf(wv[2], wv[3]), pack2bf(wv[4], wv[5]),
                                                   pack2bf(wv[6], wv[7])});
    }
  // pins: the compiler's waits for all of the above land here, ahead of the DMAs
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int q = 0; q < 8; ++q) asm volatile("" : "+v"(mwq[t][q]));
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      asm volatile("" : "+v"(kf[t][s]));
      asm volatile("" : "+v"(vf[t][s]));
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    asm volatile("" : "+v"(ov[c]));
    asm volatile("" : "+v"(dv4[c]));
  }
  asm volatile("" : "+v"(lse_t));
  if (Q2) {
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) {
      asm volatile("" : "+v"(w2t[kd][0]));
      asm volatile("" : "+v"(w2t[kd][1]));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // Q (waves 0, 2) and dO (waves 1, 3) images: wave w streams column half w >> 1 of every slice, in
  // slice order (nt pieces: the loop's counted waits); once, for the first stream
  if (j == 0) {
    const int op = w & 1, cb = w >> 1;
    const int ld = op ? P.dout_ld : P.q_ld;
    const ai32x4 rs = a_rsrc((op ? P.dout : P.q) + rowbase * ld + head * 32, (int64_t)T * ld * 2);
    const int prow = lane >> 1, pcol = 8 * ((lane & 1) ^ ((prow >> 3) & 1));
    char* dst = lds + op * OFF_DO + cb * SL_SUB;
    for (int i = 0; i < nt; ++i) {  // in step order
      const int sl = step_qt(i);
      const int grow = sl * 32 + prow;
      const int voff = grow < T ? (grow * ld + cb * 16 + pcol) * 2 : A_OOB;
      a_dma16(rs, __builtin_amdgcn_readfirstlane(a_lds_u32(dst + sl * SL_SLICE)), voff);
    }
  }
  // the LSE / D tables: thread t holds query t
  float* tab = reinterpret_cast<float*>(lds + OFF_TAB);
  {
    float dsum = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dsum += bf2f(ov[c][e] & 0xffff) * bf2f(dv4[c][e] & 0xffff);
        dsum += bf2f(ov[c][e] >> 16) * bf2f(dv4[c][e] >> 16);
      }
    const bool ok = tid < T;
    tab[tid] = ok ? -lse_t : -INFINITY;  // rows past T: P = exp2(-inf) = 0 (the ragged last tile's mask)
    tab[256 + tid] = ok ? (DROP ? -dsum / P.drop_scale : -dsum) : 0.f;
  }
  // K^T of the wave's key tiles (d on lanes, keys in the permuted k order of the transposed reads),
  // through the wave's slot: the [key][q] dS image of the dQ product uses the same layout (8-B chunk c
  // of row k at chunk c ^ ((k >> 1) & 7)) and the same reads, so the two operands' k orders agree
  char* slot = lds + OFF_DS + w * 2048;
  const int g4 = lane >> 4, qq = (lane >> 2) & 3, p4 = lane & 3;
  const int ra0 = 4 * (g4 >> 1) + qq, ra1 = ra0 + 8;
  const int o_da0 = ra0 * 64 + (((4 * (g4 & 1) + p4) ^ ((ra0 >> 1) & 7)) << 3);
  const int o_da1 = ra1 * 64 + (((4 * (g4 & 1) + p4) ^ ((ra1 >> 1) & 7)) << 3);
  auto sw = [&](int c) { return r * 64 + ((c ^ ((r >> 1) & 7)) << 3); };  // 8-B chunk c of row r
  bf16x8 ktf[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const u32x4 v = __builtin_bit_cast(u32x4, kf[t][s]);
      *reinterpret_cast<u32x2*>(slot + sw(4 * s + 2 * h)) = u32x2{v[0], v[1]};
      *reinterpret_cast<u32x2*>(slot + sw(4 * s + 2 * h + 1)) = u32x2{v[2], v[3]};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int s = 0; s < 2; ++s) ktf[t][s] = join4(lds_tr16(slot + o_da0 + 1024 * s), lds_tr16(slot + o_da1 + 1024 * s));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (NB || NB2) {  // the whole Q / dO images before the walk; the dQ sums / the sync words start at zero
    if (NB) {
#pragma unroll
      for (int k = 0; k < 8; ++k) *reinterpret_cast<f32x4*>(lds + OFF_DQ + k * 4096 + tid * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (NB2 && tid < 16) reinterpret_cast<int*>(lds + OFF_SYNC)[tid] = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (j == 0) a_wait_vm(nt - 1);  // this wave's piece of slice 0 (the younger nt - 1 pieces stay in flight)
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the previous stream's dQ-sum stores are done
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // everyone's slice-0 pieces and table entries (later streams: and every
                                 // wave is past the previous stream's epilogue)

  // element e of a tile accumulator is query row (e & 3) + 8 (e >> 2) + 4 h of the tile, key r: bit e
  // of m_diag keeps the diagonal tile's causal half, bit e of m_rows the rows of a ragged last query
  // tile that lie before T (its keys past T then lie above the diagonal)
  uint32_t m_diag = 0, m_rows = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
    m_diag |= (uint32_t)(r <= row) << e;
    m_rows |= (uint32_t)((nt - 1) * 32 + row < T) << e;
  }
  const bf16_t* qimg = reinterpret_cast<const bf16_t*>(lds);
  const bf16_t* dimg = reinterpret_cast<const bf16_t*>(lds + OFF_DO);
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) { zero16(dk[t]); zero16(dv[t]); }

  // one owned key tile (t) against query tile qt; mw: the tile's keep bits (key r, this lane's half),
  // mk: the causal / ragged mask bits of a MASKED tile
  auto tile = [&](auto mc, int qt, int t, uint32_t mw, uint32_t mk, f32x16& dqp, bool diag) {
    constexpr bool MASKED = decltype(mc)::value;
    asm volatile("" ::: "memory");  // the slot's previous reads stay ahead of this tile's writes
    const int q0 = qt * 32;
    bf16x8 qr[2], dr[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      qr[s] = sl_row(qimg, q0, r, s, h);
      dr[s] = sl_row(dimg, q0, r, s, h);
    }
    f32x16 sacc, dpacc;
    zero16(sacc);
    zero16(dpacc);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      sacc = mfma32(qr[s], kf[t][s], sacc);    // S[q][key]
      dpacc = mfma32(dr[s], vf[t][s], dpacc);  // dP[q][key]
    }
    if (!MASKED && MMT_F32_BRANCH == 0 && diag) {  // wave-uniform: the diagonal tile
      asm volatile("" ::: "memory");  // a real branch: selects on every tile cost 16 VALU
#pragma unroll
      for (int e = 0; e < 16; ++e) sacc[e] = (mk >> e) & 1 ? sacc[e] : -INFINITY;
    }
    uint32_t pp[8], dd[8];  // packed bf16 pairs of Z P (dV operand) and dS / sc (dK operand)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(tab + q0 + 8 * gg + 4 * h);
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(tab + 256 + q0 + 8 * gg + 4 * h);
#pragma unroll
      for (int e4 = 0; e4 < 4; e4 += 2) {
        float pm[2], ds[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int e = 4 * gg + e4 + u;
          float pv = ex2(__builtin_fmaf(sacc[e], c2, l4[e4 + u]));
          if (MASKED) pv = keep_f(pv, __builtin_amdgcn_sbfe((int)mk, e, 1));
          if (DROP) {
            int kb = __builtin_amdgcn_sbfe((int)mw, 8 * gg + e4 + u, 1);  // all ones iff kept
            asm volatile("" : "+v"(kb));
            pm[u] = keep_f(pv, kb);
            ds[u] = __builtin_fmaf(pm[u], dpacc[e], pv * d4[e4 + u]);  // Z P dP - P D'
          } else {
            pm[u] = pv;
            ds[u] = pv * (dpacc[e] + d4[e4 + u]);  // P (dP - D)
          }
        }
        pp[2 * gg + e4 / 2] = pack2bf(pm[0], pm[1]);
        dd[2 * gg + e4 / 2] = pack2bf(ds[0], ds[1]);
      }
    }
    // dS -> the slot as [key][q] rows (lane (r, h): queries 8 gg + 4 h .. + 3 of key r)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) *reinterpret_cast<u32x2*>(slot + sw(2 * gg + h)) = u32x2{dd[2 * gg], dd[2 * gg + 1]};
    bf16x8 dot[2], qtr[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      dot[s] = sl_tr(dimg, q0, s, lane);
      qtr[s] = sl_tr(qimg, q0, s, lane);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pf = __builtin_bit_cast(bf16x8, u32x4{pp[4 * s], pp[4 * s + 1], pp[4 * s + 2], pp[4 * s + 3]});
      const bf16x8 df = __builtin_bit_cast(bf16x8, u32x4{dd[4 * s], dd[4 * s + 1], dd[4 * s + 2], dd[4 * s + 3]});
      dv[t] = mfma32(pf, dot[s], dv[t]);
      dk[t] = mfma32(df, qtr[s], dk[t]);
    }
    // dQ_w^T[d][q] += K^T[d][key] dS^T[key][q]: both fragments in the permuted k order of the slot reads
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 da = join4(lds_tr16(slot + o_da0 + 1024 * s), lds_tr16(slot + o_da1 + 1024 * s));
      dqp = mfma32(ktf[t][s], da, dqp);
    }
  };

  // both owned key tiles against query tile qt in one straight-line body (qt >= 7 - w): the Q / dO row and
  // transposed fragments and the LSE / D rows are read once for the two tiles, and the two tiles' S / dP ->
  // softmax -> dV / dK chains are independent, so one's MFMAs overlap the other's VALU in the wave
  auto tile2 = [&](int qt, uint32_t mwa, uint32_t mwb, f32x16& dqp, bool diagA, bool diagB) {
    asm volatile("" ::: "memory");
    const int q0 = qt * 32;
    bf16x8 qr[2], dr[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      qr[s] = sl_row(qimg, q0, r, s, h);
      dr[s] = sl_row(dimg, q0, r, s, h);
    }
    f32x16 sacc[2], dpacc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      zero16(sacc[t]);
      zero16(dpacc[t]);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        sacc[t] = mfma32(qr[s], kf[t][s], sacc[t]);
        dpacc[t] = mfma32(dr[s], vf[t][s], dpacc[t]);
      }
    if (diagA || diagB) {  // wave-uniform
      asm volatile("" ::: "memory");
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          sacc[t][e] = ((t ? diagB : diagA) && !((m_diag >> e) & 1)) ? -INFINITY : sacc[t][e];
    }
    uint32_t pp[2][8], dd[2][8];
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(tab + q0 + 8 * gg + 4 * h);
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(tab + 256 + q0 + 8 * gg + 4 * h);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const uint32_t mw = t ? mwb : mwa;
#pragma unroll
        for (int e4 = 0; e4 < 4; e4 += 2) {
          float pm[2], ds[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int e = 4 * gg + e4 + u;
            const float pv = ex2(__builtin_fmaf(sacc[t][e], c2, l4[e4 + u]));
            if (DROP) {
              int kb = __builtin_amdgcn_sbfe((int)mw, 8 * gg + e4 + u, 1);
              asm volatile("" : "+v"(kb));
              pm[u] = keep_f(pv, kb);
              ds[u] = __builtin_fmaf(pm[u], dpacc[t][e], pv * d4[e4 + u]);
            } else {
              pm[u] = pv;
              ds[u] = pv * (dpacc[t][e] + d4[e4 + u]);
            }
          }
          pp[t][2 * gg + e4 / 2] = pack2bf(pm[0], pm[1]);
          dd[t][2 * gg + e4 / 2] = pack2bf(ds[0], ds[1]);
        }
      }
    }
    bf16x8 dot[2], qtr[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      dot[s] = sl_tr(dimg, q0, s, lane);
      qtr[s] = sl_tr(qimg, q0, s, lane);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      // tile t's dS through the slot (tile 1 writes after tile 0's dS^T reads: in-order LDS per wave)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        *reinterpret_cast<u32x2*>(slot + sw(2 * gg + h)) = u32x2{dd[t][2 * gg], dd[t][2 * gg + 1]};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = __builtin_bit_cast(bf16x8, u32x4{pp[t][4 * s], pp[t][4 * s + 1], pp[t][4 * s + 2], pp[t][4 * s + 3]});
        const bf16x8 df = __builtin_bit_cast(bf16x8, u32x4{dd[t][4 * s], dd[t][4 * s + 1], dd[t][4 * s + 2], dd[t][4 * s + 3]});
        dv[t] = mfma32(pf, dot[s], dv[t]);
        dk[t] = mfma32(df, qtr[s], dk[t]);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 da = join4(lds_tr16(slot + o_da0 + 1024 * s), lds_tr16(slot + o_da1 + 1024 * s));
        dqp = mfma32(ktf[t][s], da, dqp);
      }
      asm volatile("" ::: "memory");
    }
  };

  const float dqs = DROP ? scale * P.drop_scale : scale;
  const ai32x4 rdq = a_rsrc(P.dq + rowbase * P.dq_ld + head * 32, (int64_t)T * P.dq_ld * 2);
  const int R = 8 * w + (lane >> 3), cq = lane & 7;  // this wave's dQ rows / 16-B column chunk
#ifndef MMT_F32_SKIP
#define MMT_F32_SKIP 0
#endif
  if constexpr (NB) {
#pragma unroll 1
    for (int i = 0; i < nt; ++i) {
      const int qt = i;
      const uint32_t cA = mwq[0][0] >> (4 * h), cB = mwq[1][0] >> (4 * h);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 7; ++q) mwq[t][q] = mwq[t][q + 1];
      if (kts[0] > qt) continue;  // wave-uniform: no owned key tile at or below query tile qt yet
      f32x16 dqp;
      zero16(dqp);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int kt = kts[t];
        if (kt < nt && kt <= qt) tile(std::false_type{}, qt, t, t ? cB : cA, m_diag, dqp, kt == qt);
      }
      // dQ^T[d][q] of the tile: element e is d = (e & 3) + 8 (e >> 2) + 4 h, lane r is q; 32 lanes a bank row
      float* acc = reinterpret_cast<float*>(lds + OFF_DQ + qt * 4096) + 4 * h * 32 + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
#ifdef MMT_F32_NB_NOATOM  // timing experiment: plain stores (wrong sums)
        acc[((e & 3) + 8 * (e >> 2)) * 32] = dqp[e];
#else
        __hip_atomic_fetch_add(acc + ((e & 3) + 8 * (e >> 2)) * 32, dqp[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every dQ contribution is in
    // the wave's two query tiles (the rows of its key tiles): lane (r, h) row r, columns 16 h .. 16 h + 15,
    // scaled to bf16 into the spent Q image (Q2: the stage-2 operand) or stored
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int qt = kts[t];
      if (qt >= nt) continue;
      const float* acc = reinterpret_cast<const float*>(lds + OFF_DQ + qt * 4096) + 16 * h * 32 + r;
      uint32_t pk[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) pk[k] = pack2bf(acc[(2 * k) * 32] * dqs, acc[(2 * k + 1) * 32] * dqs);
      if (Q2) {
        *reinterpret_cast<u32x4*>(lds + qt * SL_SLICE + sl_off(r, 2 * h)) = u32x4{pk[0], pk[1], pk[2], pk[3]};
        *reinterpret_cast<u32x4*>(lds + qt * SL_SLICE + sl_off(r, 2 * h + 1)) = u32x4{pk[4], pk[5], pk[6], pk[7]};
      } else {
        const int tq = qt * 32 + r;
        if (tq < T) {
          u32x2* d = reinterpret_cast<u32x2*>(P.dq + (rowbase + tq) * P.dq_ld + head * 32 + 16 * h);
#pragma unroll
          for (int k = 0; k < 4; ++k) d[k] = u32x2{pk[2 * k], pk[2 * k + 1]};
        }
      }
    }
    // the dQ sums are spent before the epilogue transposes / stage-2 images reuse their LDS
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else if constexpr (NB2) {
    int* const cnt = reinterpret_cast<int*>(lds + OFF_SYNC);
    int* const done = cnt + 8;
#pragma unroll 1
    for (int i = 0; i < nt; ++i) {
      const int qt = i;
      const uint32_t cA = mwq[0][0] >> (4 * h), cB = mwq[1][0] >> (4 * h);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 7; ++q) mwq[t][q] = mwq[t][q + 1];
      if (kts[0] > qt) continue;  // wave-uniform: not a contributor of query tile qt
      f32x16 dqp;
      zero16(dqp);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int kt = kts[t];
        if (kt < nt && kt <= qt) tile(std::false_type{}, qt, t, t ? cB : cA, m_diag, dqp, kt == qt);
      }
      // the slot last held tile qt - 2: wait until its sum has read it (bounded: a lost flag cannot hang)
      if (qt - 2 >= w) {
        for (int it = 0; it < (1 << 22); ++it) {
          if (__hip_atomic_load(done + qt - 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      char* part = lds + OFF_DQ + (((qt - w) & 1) * 4 + w) * 4096;
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        *reinterpret_cast<f32x4*>(part + r * 128 + (((2 * gg + h) ^ (r & 7)) << 4)) =
            f32x4{dqp[4 * gg], dqp[4 * gg + 1], dqp[4 * gg + 2], dqp[4 * gg + 3]};
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the partial is in before the arrival counts it
      int old = 0;
      if (lane == 0) old = __hip_atomic_fetch_add(cnt + qt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      old = __builtin_amdgcn_readfirstlane(old);
      const int nc = min(qt + 1, 4);  // contributors: waves u <= qt
      if (old == nc - 1) {  // the last one: sum the tile (4 passes of 8 rows), then free the slots
#pragma unroll
        for (int ps = 0; ps < 4; ++ps) {
          const int R = 8 * ps + (lane >> 3), cq = lane & 7;
          f32x4 a = {0.f, 0.f, 0.f, 0.f};
          for (int u = 0; u < nc; ++u)
            a += *reinterpret_cast<const f32x4*>(lds + OFF_DQ + (((qt - u) & 1) * 4 + u) * 4096 + R * 128 + ((cq ^ (R & 7)) << 4));
          const int tq = qt * 32 + R;
          if (Q2) {
            *reinterpret_cast<u32x2*>(lds + qt * SL_SLICE + sl_off(R, cq >> 1) + (cq & 1) * 8) =
                u32x2{pack2bf(a[0] * dqs, a[1] * dqs), pack2bf(a[2] * dqs, a[3] * dqs)};
          } else {
            a_bst8(rdq, tq < T ? (tq * P.dq_ld + 4 * cq) * 2 : A_OOB,
                   u32x2{pack2bf(a[0] * dqs, a[1] * dqs), pack2bf(a[2] * dqs, a[3] * dqs)});
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the partial reads are done
        if (lane == 0) __hip_atomic_store(done + qt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every tile is summed (each inside its last contributor's walk)
  } else
#pragma unroll 1
  for (int i = 0; i < (MMT_F32_SKIP ? 0 : nt); ++i) {
    const int qt = step_qt(i);
    const uint32_t cA = mwq[0][0] >> (4 * h), cB = mwq[1][0] >> (4 * h);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < 7; ++q) mwq[t][q] = mwq[t][q + 1];
    f32x16 dqp;
    zero16(dqp);
    const bool last_ragged = ragged && qt == nt - 1;
#if MMT_F32_PAIR
    if (kts[1] < nt && kts[1] <= qt) {  // both tiles (kts[0] < kts[1])
      tile2(qt, cA, cB, dqp, kts[0] == qt, kts[1] == qt);
    } else if (kts[0] <= qt) {
      tile(std::false_type{}, qt, 0, cA, m_diag, dqp, kts[0] == qt);
    }
#else
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int kt = kts[t];
      if (kt < nt && kt <= qt) {
        const uint32_t mw = t ? cB : cA;
        const uint32_t mk = (kt == qt ? m_diag : 0xffffu) & (last_ragged ? m_rows : 0xffffu);
#if MMT_F32_BRANCH == 1
        // separate masked / unmasked tile bodies: the accumulators then take register copies at the joins
        if (kt == qt || last_ragged) tile(std::true_type{}, qt, t, mw, mk, dqp, false);
        else tile(std::false_type{}, qt, t, mw, mk, dqp, false);
#elif MMT_F32_BRANCH == 2
        tile(std::true_type{}, qt, t, mw, mk, dqp, false);  // one body, the mask applied on every tile
#else
        // one body; the diagonal tile's scores above the diagonal become -inf in a branch that touches
        // only the score accumulator (rows past T: -inf LSE-table entries)
        tile(std::false_type{}, qt, t, mw, m_diag, dqp, kt == qt);
#endif
      }
    }
#endif
    char* part = lds + OFF_DQ + ((i & 1) * 4 + w) * 4096;
    if (w <= qt) {  // this wave had a tile in the step (its key tile w is the lower one)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        *reinterpret_cast<f32x4*>(part + r * 128 + (((2 * gg + h) ^ (r & 7)) << 4)) =
            f32x4{dqp[4 * gg], dqp[4 * gg + 1], dqp[4 * gg + 2], dqp[4 * gg + 3]};
    }
    // this wave's piece of slice qt + 1: younger are the pieces of slices qt + 2 .. nt - 1 and the dQ
    // stores of steps 0 .. qt - 1, nt - 2 operations at every step
    if (j == 0 && i + 1 < nt) a_wait_vm(Q2 ? nt - 2 - i : nt - 2);  // Q2: no dQ stores in the loop
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every partial of step qt is written; slice qt + 1 landed
    {
      const int nw = min(qt + 1, 4);
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
      for (int u = 0; u < nw; ++u)
        a += *reinterpret_cast<const f32x4*>(lds + OFF_DQ + ((i & 1) * 4 + u) * 4096 + R * 128 + ((cq ^ (R & 7)) << 4));
      const int tq = qt * 32 + R;
      if (Q2) {  // dQ rows into the (spent) Q slice of this step, for the stage-2 backward after the walk
        *reinterpret_cast<u32x2*>(lds + qt * SL_SLICE + sl_off(R, cq >> 1) + (cq & 1) * 8) =
            u32x2{pack2bf(a[0] * dqs, a[1] * dqs), pack2bf(a[2] * dqs, a[3] * dqs)};
      } else if (!MS || j == ns - 1) {
        if (MS && j > 0 && tq < T) a += *reinterpret_cast<const f32x4*>(P.dq32 + (rowbase + tq) * P.dq32_ld + head * 32 + 4 * cq);
        a_bst8(rdq, tq < T ? (tq * P.dq_ld + 4 * cq) * 2 : A_OOB,
               u32x2{pack2bf(a[0] * dqs, a[1] * dqs), pack2bf(a[2] * dqs, a[3] * dqs)});
      } else {  // running fp32 sum over the streams (stream 0: one counted store per step, as above)
        if (j > 0 && tq < T) a += *reinterpret_cast<const f32x4*>(P.dq32 + (rowbase + tq) * P.dq32_ld + head * 32 + 4 * cq);
        a_bst16(rdq32, tq < T ? (tq * P.dq32_ld + 4 * cq) * 4 : A_OOB, a);
      }
    }
  }

  const float dks = DROP ? scale * P.drop_scale : scale;
  const float dvs = DROP ? P.drop_scale : 1.f;
  if constexpr (Q2) {
    // Q/K/V stage-2 backward of this head (model.py:36-50) on the 32-row tiles of dQ (in the Q image),
    // dK and dV (staged from the accumulators): per tile dh1^T = W2^T dX^T (2 MFMAs), times tanh' from
    // the tile's h1 rows, stored; dW2^T += dX^T h1 (2 MFMAs) and the dh1 column sums (db1) in registers
    // until the workgroup's sums go out by atomics. dQ / dK / dV never leave the kernel.
    // the h1 rows of the six tiles (key / query tiles kts[t] x K, Q, V blocks) in flight at once: the
    // tiles are worked one after the other, each wait only for its own rows
    u32x4 h1v[2][3];
    {
      const MMT_AS1 bf16_t* const h1 = sgpr_gptr(P.q2_h1);
      const int ld = __builtin_amdgcn_readfirstlane(P.q2_ld);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int kd = 0; kd < 3; ++kd) {
          const int row = kts[t] * 32 + r;
          h1v[t][kd] = u32x4{0u, 0u, 0u, 0u};
          if (kts[t] < nt && row < T)
            h1v[t][kd] = *reinterpret_cast<const MMT_AS1 u32x4*>(h1 + (rowbase + row) * ld + (kd * H + head) * 16 + 8 * h);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's dQ rows of the last step are in the Q image
    char* xs = lds + OFF_DQ + w * SL_SLICE;              // this wave's dX tile (slice image)
    char* hs_ = lds + OFF_DQ + 4 * SL_SLICE + w * SL_SLICE;  // and its h1 tile (columns 16..31 zero)
    f32x16 dwa[3];
    float dba[3][8];
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) {
      zero16(dwa[kd]);
#pragma unroll
      for (int e = 0; e < 8; ++e) dba[kd][e] = 0.f;
    }
    MMT_AS1 bf16_t* const dh1 = sgpr_gptr(P.q2_dh1);
    const int ldd = __builtin_amdgcn_readfirstlane(P.q2_ld);
    auto tile_op = [&](int kd, const char* ximg, int row0, const u32x4& hv) {
      const int blk = kd * H + head;
      const int row = row0 + r;
      *reinterpret_cast<u32x4*>(hs_ + sl_off(r, h)) = hv;
      *reinterpret_cast<u32x4*>(hs_ + sl_off(r, 2 + h)) = u32x4{0u, 0u, 0u, 0u};
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      f32x16 acc;
      zero16(acc);
#pragma unroll
      for (int s = 0; s < 2; ++s)
        acc = mfma32(w2t[kd][s], sl_row(reinterpret_cast<const bf16_t*>(ximg), 0, r, s, h), acc);  // dh1^T[i][r]
      // lane (r, h): i = 4 h + e (e < 4) and 8 + 4 h + e - 4 (4 <= e < 8)
      const u32x2 ha = *reinterpret_cast<const u32x2*>(hs_ + sl_off(r, 0) + 8 * h);
      const u32x2 hb = *reinterpret_cast<const u32x2*>(hs_ + sl_off(r, 1) + 8 * h);
      float hh8[8] = {bf2f(ha[0] & 0xffff), bf2f(ha[0] >> 16), bf2f(ha[1] & 0xffff), bf2f(ha[1] >> 16),
                      bf2f(hb[0] & 0xffff), bf2f(hb[0] >> 16), bf2f(hb[1] & 0xffff), bf2f(hb[1] >> 16)};
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        d[e] = acc[e] * (1.f - hh8[e] * hh8[e]);
        dba[kd][e] += d[e];
      }
      if (row < T) {
        MMT_AS1 bf16_t* dst = dh1 + (rowbase + row) * ldd + blk * 16 + 4 * h;
        *reinterpret_cast<MMT_AS1 u32x2*>(dst) = u32x2{pack2bf(d[0], d[1]), pack2bf(d[2], d[3])};
        *reinterpret_cast<MMT_AS1 u32x2*>(dst + 8) = u32x2{pack2bf(d[4], d[5]), pack2bf(d[6], d[7])};
      }
      // dW2^T[i][o] ... as C[m = o][n = i]: A = dX^T (lane o), B = h1 (lane i), k = rows (permuted)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        dwa[kd] = mfma32(sl_tr(reinterpret_cast<const bf16_t*>(ximg), 0, s, lane),
                         sl_tr(reinterpret_cast<const bf16_t*>(hs_), 0, s, lane), dwa[kd]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this tile's LDS reads before the next writes
    };
    // dK, dV of the wave's key tiles: accumulators (lane: column o = r, elements: rows) -> the tile image
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int kt = kts[t];
      if (kt >= nt) continue;
#pragma unroll
      for (int mtx = 0; mtx < 2; ++mtx) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int kr = (e & 3) + 8 * (e >> 2) + 4 * h;
          *reinterpret_cast<bf16_t*>(xs + sl_off(kr, r >> 3) + (r & 7) * 2) = mtx ? f2bf(dv[t][e] * dvs) : f2bf(dk[t][e] * dks);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        tile_op(mtx ? 2 : 0, xs, kt * 32, h1v[t][mtx ? 2 : 0]);
      }
    }
    // dQ tiles w and 7 - w from the Q image
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int qt = kts[t];
      if (qt < nt) tile_op(1, lds + qt * SL_SLICE, qt * 32, h1v[t][1]);
    }
    MMT_AS1 float* const db1 = sgpr_gptr(P.q2_db1);
    MMT_AS1 float* const dw2 = sgpr_gptr(P.q2_dw2);
    // db1: column sums over the 32 rows of each lane half; lane r < 24 of each half adds sum r
    {
      float mine = 0.f;
#pragma unroll
      for (int kd = 0; kd < 3; ++kd)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = a_sum32(dba[kd][e]);
          mine = r == kd * 8 + e ? v : mine;
        }
      const int kd = r >> 3, e = r & 7;
      if (r < 24)
        __hip_atomic_fetch_add(db1 + (kd * H + head) * 16 + (e < 4 ? 4 * h + e : 8 + 4 * h + e - 4), mine, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    // dW2: the four waves' partials summed through LDS, one atomic per element
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's tile images are spent
    float* red = reinterpret_cast<float*>(lds + OFF_DQ);  // [4 waves][3 kinds][32 o][16 i]
    if (r < 16) {
#pragma unroll
      for (int kd = 0; kd < 3; ++kd)
#pragma unroll
        for (int e = 0; e < 16; ++e)
          red[((w * 3 + kd) * 32 + (e & 3) + 8 * (e >> 2) + 4 * h) * 16 + r] = dwa[kd][e];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int q = tid; q < 3 * 512; q += 256) {
      const float v = (red[q] + red[1536 + q]) + (red[3072 + q] + red[4608 + q]);
      const int kd = q / 512, oi = q % 512;
#if !MMT_F32_Q2_NOATOM
      __hip_atomic_fetch_add(dw2 + (kd * H + head) * 512 + oi, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
      if (v == 12345.f) dw2[0] = v;  // timing experiment only: keeps the sums live
#endif
    }
  } else {
  // dK / dV of the wave's key tiles, transposed through LDS into row-major 16-B pieces (as the dK/dV
  // pass), one matrix at a time through the dQ partials of the parity the last step did not use (no
  // wave reads them after the last step's barrier; the next stream's first barrier retires these reads)
  bf16_t* et = reinterpret_cast<bf16_t*>(lds + OFF_DQ + (nt & 1) * 4 * 4096) + w * (32 * EPW);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int kt = kts[t];
    if (kt >= nt) continue;
    const int k0 = kt * 32;
#pragma unroll
    for (int mtx = 0; mtx < 2; ++mtx) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kr = (e & 3) + 8 * (e >> 2) + 4 * h;
        et[kr * EPW + r] = mtx ? f2bf(dv[t][e] * dvs) : f2bf(dk[t][e] * dks);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bf16_t* dst = (mtx ? P.dv[j] : P.dk[j]) + head * P.dkv_hstride;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = i * 16 + (lane >> 2), d0 = (lane & 3) * 8;
        const u32x4 v = *reinterpret_cast<const u32x4*>(et + row * EPW + d0);
        if (k0 + row < T) *reinterpret_cast<u32x4*>(dst + (rowbase + k0 + row) * P.dkv_ld + d0) = v;
      }
    }
  }
  }  // !Q2
  }  // streams
}

// attention variant knob (bit 0: the slice-streamed hs-64 dK/dV pass, bit 1: its dQ pass, bit 2: the
// dK/dV pass at 3 waves per SIMD, bit 3: the slice-streamed hs-64 forward, bit 5: the one-pass hs-64
// backward at T <= 512 with one KV stream, bit 6: the one-pass hs-32 backward at T <= 256, bit 7: that
// kernel also for several KV streams): MMT_ATTN_RING, or mmt_attn_set_ring() for in-process A/B
static int g_attn_ring = [] {
  const char* e = getenv("MMT_ATTN_RING");
  // both hs-64 passes on the rings (dQ: two query tiles per wave), dK/dV at 3 waves per SIMD
  // (standalone backward: target 277 -> 273 us, C3 cross-attention 2461 -> 2298, C4 2237 -> 2116;
  // C3 step -1.5 %: profiles/r3u_ring_ab.txt), and the forward on the ring too (round 4: target
  // 20.42 -> 20.34 ms, C3 157.3 -> 153.8 ms same box, profiles/r4m_ab.txt)
  // bit 6 (round 6): the one-pass hs-32 backward
  return e ? atoi(e) : 15 | 64;
}();
extern "C" int mmt_attn_set_ring(int v) {
  const int old = g_attn_ring;
  g_attn_ring = v;
  return old;
}

// the slice-streamed hs-64 kernels address a sequence's rows (and one (batch, head)'s keep-bit
// records) with 32-bit per-lane offsets from a per-batch-row buffer base: a sequence whose span
// reaches 2^31 bytes takes the chunked kernels (64-bit pointer math) instead
static bool ring64_fits(const AttnBatch& bt, int T) {
  const int64_t lim = (int64_t)1 << 31;
  const int64_t nt = (T + 31) / 32, ntri = nt * (nt + 1) / 2;
  if (ntri * 128 >= lim) return false;
  for (int g = 0; g < bt.count; ++g) {
    const AttnProblem& P = bt.p[g];
    if ((int64_t)T * P.q_ld * 2 >= lim || (int64_t)T * P.dout_ld * 2 >= lim || (int64_t)T * P.kv_ld * 2 >= lim)
      return false;
  }
  return true;
}

// the one-pass hs-32 backward (knob bit 6) takes the batch: T <= 256, Q / dO rows by LDS-DMA (16-B aligned
// rows, sequences whose span fits a buffer descriptor); several KV streams only with knob bit 7 and the
// fp32 dQ scratch. Every problem sets the Q/K/V stage-2 fields (AttnProblem::q2_*) or none does, and
// only with one KV stream.
static bool fused32_ok(const AttnBatch& bt, int T, int ns) {
  if (!(g_attn_ring & 64) || T > 256 || bt.count < 1) return false;
  const bool q2 = bt.p[0].q2_w2 != nullptr;
  if (q2 && ns > 1) return false;
  bool ok = true;
  for (int g = 0; g < bt.count; ++g) {
    const AttnProblem& P = bt.p[g];
    ok = ok && !(P.q_ld & 7) && !(P.dout_ld & 7) && !((uintptr_t)P.q & 15) && !((uintptr_t)P.dout & 15) &&
         !(P.kv_ld & 7) && !(P.kv_hstride & 7) && (int64_t)T * std::max(P.q_ld, P.dout_ld) * 2 < ((int64_t)1 << 31);
    // several KV streams (knob bit 7, off by default): one workgroup walks the streams in turn, and at
    // C1's cross-attention (3 streams, 512 workgroups: one generation) that measured slower than the
    // two-pass pair, which spreads the dK/dV pass over 3x the workgroups (70.7 vs 67.9 us standalone,
    // tools/attn_bench.py c1_ca)
    if (ns > 1)
      ok = ok && (g_attn_ring & 128) && P.dq32 && !(P.dq32_ld & 3) && !((uintptr_t)P.dq32 & 15) &&
           (int64_t)T * P.dq32_ld * 4 < ((int64_t)1 << 31);
    // one stream without the stage-2 fields: dQ rows leave as 8-B pieces
    if (ns == 1 && !q2) ok = ok && !(P.dq_ld & 3) && !((uintptr_t)P.dq & 7);
    if ((P.q2_w2 != nullptr) != q2) return false;
    if (q2)
      ok = ok && P.q2_h1 && P.q2_dh1 && P.q2_dw2 && P.q2_db1 && !(P.q2_ld & 7) && !((uintptr_t)P.q2_h1 & 15) &&
           !((uintptr_t)P.q2_dh1 & 7);
  }
  return ok;
}

bool mmt_attn_bwd_fuses_qkv2(const AttnBatch& bt, int T, int hs) {
  if (hs != 32 || bt.count < 1) return false;
  for (int g = 0; g < bt.count; ++g)
    if (bt.p[g].nstreams != 1) return false;
  AttnBatch t = bt;  // as the launch will see it with the stage-2 fields set
  for (int g = 0; g < t.count; ++g) {
    AttnProblem& P = t.p[g];
    P.q2_w2 = reinterpret_cast<const float*>(16); P.q2_h1 = reinterpret_cast<const bf16_t*>(16);
    P.q2_dh1 = reinterpret_cast<bf16_t*>(16); P.q2_dw2 = reinterpret_cast<float*>(16); P.q2_db1 = P.q2_dw2;
    P.q2_ld = 8;
  }
  return fused32_ok(t, T, 1);
}

template <int HS>
static hipError_t attn_launch(const AttnBatch& bt, int B, int T, int H, float scale, bool bwd, hipStream_t s) {
  const int nb = ((T + 31) / 32 + 7) / 8;
  if (!bwd) {
    bool drop = false;
    for (int g = 0; g < bt.count; ++g) drop = drop || bt.p[g].drop_thr != 0;
    // hs 64, knob bit 3: the forward on the LDS-DMA slice ring (mmt_attn2.hip)
    if (HS == 64 && (g_attn_ring & 8) && ring64_fits(bt, T)) return mmt_attn_fwd_ring64(bt, B, T, H, scale, drop, s);
    const dim3 grid(nb * B * H, 1, bt.count);
    if (drop) hipLaunchKernelGGL((attn_fwd_kernel<HS, true>), grid, dim3(256), 0, s, bt, T, H, scale);
    else hipLaunchKernelGGL((attn_fwd_kernel<HS, false>), grid, dim3(256), 0, s, bt, T, H, scale);
  } else {
    const int ns = bt.p[0].nstreams;
    bool drop = false;
    for (int g = 0; g < bt.count; ++g) drop = drop || bt.p[g].drop_thr != 0;
    // the stage-2 fields are a promise that the fused kernel writes dh1 / dW2 / db1 (and not dq / dk / dv):
    // refused rather than dropped when it cannot run (mmt_attn_bwd_fuses_qkv2 decides beforehand)
    for (int g = 0; g < bt.count; ++g)
      if (bt.p[g].q2_w2 && (HS != 32 || !fused32_ok(bt, T, ns))) return hipErrorInvalidValue;
    // hs 64: the slice-streamed kernels (mmt_attn2.hip): bit 1 of the knob the dQ pass, bit 0 the
    // dK/dV pass; MMT_ATTN_RING=0 (or mmt_attn_set_ring(0)) keeps the chunked ones
    const bool ring = HS == 64 && ring64_fits(bt, T);
    // knob bit 5: dQ, dK, dV in one pass (mmt_attn2.hip) for T <= 512 and one KV stream
    if (ring && (g_attn_ring & 32) && T <= 512 && ns == 1) return mmt_attn_bwd_fused64(bt, B, T, H, scale, drop, s);
    // knob bit 6: dQ, dK, dV in one pass at hs 32 for T <= 256 (fused32_ok)
    if (HS == 32 && fused32_ok(bt, T, ns)) {
      const dim3 grid(B * H, 1, bt.count);
      const bool q2 = bt.p[0].q2_w2 != nullptr;
      if (ns > 1) {
        if (drop) hipLaunchKernelGGL((attn_bwd_fused32<true, true, false>), grid, dim3(256), 0, s, bt, T, H, scale);
        else hipLaunchKernelGGL((attn_bwd_fused32<false, true, false>), grid, dim3(256), 0, s, bt, T, H, scale);
      } else if (q2) {
        if (drop) hipLaunchKernelGGL((attn_bwd_fused32<true, false, true>), grid, dim3(256), 0, s, bt, T, H, scale);
        else hipLaunchKernelGGL((attn_bwd_fused32<false, false, true>), grid, dim3(256), 0, s, bt, T, H, scale);
      } else {
        if (drop) hipLaunchKernelGGL((attn_bwd_fused32<true, false, false>), grid, dim3(256), 0, s, bt, T, H, scale);
        else hipLaunchKernelGGL((attn_bwd_fused32<false, false, false>), grid, dim3(256), 0, s, bt, T, H, scale);
      }
      return hipGetLastError();
    }
    if (ring && (g_attn_ring & 2)) {
      const hipError_t e = mmt_attn_bwd_dq_ring64(bt, B, T, H, scale, drop, s);
      if (e != hipSuccess) return e;  // (hipGetLastError cleared it: report it here)
    } else if (drop) hipLaunchKernelGGL((attn_bwd_dq_kernel<HS, true>), dim3(nb * B * H, 1, bt.count), dim3(256), 0, s, bt, T, H, scale);
    else hipLaunchKernelGGL((attn_bwd_dq_kernel<HS, false>), dim3(nb * B * H, 1, bt.count), dim3(256), 0, s, bt, T, H, scale);
    if (ring && (g_attn_ring & 1)) return mmt_attn_bwd_dkdv_ring64(bt, B, T, H, scale, drop, g_attn_ring, s);
    // dK/dV: one key tile per wave at 2 waves per SIMD (a paired two-key-tile walk at one wave per
    // SIMD measured slower: C1 103 vs 127 us, target step 25.4 vs 25.9 ms; removed in round 4)
    if (drop)
      hipLaunchKernelGGL((attn_bwd_dkdv1_kernel<HS, true>), dim3(nb * B * H * ns, 1, bt.count), dim3(256), 0, s, bt, T, H,
                         scale);
    else
      hipLaunchKernelGGL((attn_bwd_dkdv1_kernel<HS, false>), dim3(nb * B * H * ns, 1, bt.count), dim3(256), 0, s, bt, T,
                         H, scale);
  }
  return hipGetLastError();
}

static hipError_t attn_dispatch(const AttnBatch& b, int B, int T, int H, int hs, float scale, bool bwd,
                                hipStream_t s) {
  if (b.count == 0 || B == 0 || T == 0) return hipSuccess;
  for (int g = 0; g < b.count; ++g) {
    if (b.p[g].nstreams < 1 || b.p[g].nstreams > MMT_MAX_STREAMS) return hipErrorInvalidValue;
    for (int j = 0; j < b.p[g].nstreams && b.p[g].nstreams > 1; ++j)  // per-stream outputs (summed, and
      if (!b.p[g].oj[j]) return hipErrorInvalidValue;                   // read by the backward)
    if (b.p[g].drop_thr)  // dropout reads the keep bits of mmt_launch_attn_mask
      for (int j = 0; j < b.p[g].nstreams; ++j)
        if (!b.p[g].dmask[j]) return hipErrorInvalidValue;
  }
  for (int g = 0; g < b.count; ++g) {  // O / O_j leave the forward as 16-B row pieces
    if (b.p[g].o_ld & 7 || ((uintptr_t)b.p[g].o & 15)) return hipErrorInvalidValue;
    for (int j = 0; j < b.p[g].nstreams && b.p[g].nstreams > 1; ++j)
      if ((uintptr_t)b.p[g].oj[j] & 15) return hipErrorInvalidValue;
  }
  if (bwd) {  // all problems in a bwd batch must share nstreams (grid.y = B*H*nstreams)
    for (int g = 1; g < b.count; ++g)
      if (b.p[g].nstreams != b.p[0].nstreams) return hipErrorInvalidValue;
    // dQ, dK, dV leave the kernels as 16-B row pieces (8-element aligned rows and head offsets)
    for (int g = 0; g < b.count; ++g) {
      if ((b.p[g].dkv_ld & 7) || (b.p[g].dkv_hstride & 7)) return hipErrorInvalidValue;
      if ((b.p[g].dq_ld & 7) || ((uintptr_t)b.p[g].dq & 15)) return hipErrorInvalidValue;
      for (int j = 0; j < b.p[g].nstreams; ++j)
        if (((uintptr_t)b.p[g].dk[j] | (uintptr_t)b.p[g].dv[j]) & 15) return hipErrorInvalidValue;
    }
  }
  switch (hs) {
    case 8: return attn_launch<8>(b, B, T, H, scale, bwd, s);
    case 16: return attn_launch<16>(b, B, T, H, scale, bwd, s);
    case 24: return attn_launch<24>(b, B, T, H, scale, bwd, s);
    case 32: return attn_launch<32>(b, B, T, H, scale, bwd, s);
    case 48: return attn_launch<48>(b, B, T, H, scale, bwd, s);
    case 64: return attn_launch<64>(b, B, T, H, scale, bwd, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t mmt_launch_attn_fwd(const AttnBatch& b, int B, int T, int H, int hs, float scale, hipStream_t s) {
  return attn_dispatch(b, B, T, H, hs, scale, false, s);
}
hipError_t mmt_launch_attn_bwd(const AttnBatch& b, int B, int T, int H, int hs, float scale, hipStream_t s) {
  return attn_dispatch(b, B, T, H, hs, scale, true, s);
}

// =============================================================================================
// Dropout keep bits (AttnProblem::dmask): one wave per 32x32 (query tile, key tile <= query tile)
// tile of one (stream, bh). Lane (r, h) hashes query r's key pairs in the accumulator order of an
// S^T tile (one hash per key pair, mmt_keep on its 16-bit halves), and the ballot of each element
// is the element's two mask dwords. Pure VALU work with no inputs: launched on a side stream it
// overlaps the MFMA-bound GEMMs ahead of the attention.
// =============================================================================================
// A wave makes G consecutive tiles of the (stream, bh, row-major lower triangle) order: the index
// division, the triangle root and the row hash are paid once per wave (and per query tile) instead of
// once per tile.
// v_writelane_b32 (the LLVM intrinsic; hipcc exposes no builtin for it): a wave-uniform value into one lane
extern "C" __device__ int mmt_writelane(int v, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

template <int G>
__global__ __launch_bounds__(256) void attn_mask_kernel(AttnBatch batch, int BH, int T) {
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nt = (T + 31) / 32;
  const int ntri = nt * (nt + 1) / 2;
  const int64_t per = (int64_t)BH * ntri;  // tiles per stream
  const int64_t total = per * P.nstreams;
  const int64_t t0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G;
  if (P.drop_thr == 0 || t0 >= total) return;  // wave-uniform
  int j, bh, tri;
  int64_t tt;
  if (total <= 0x7fffffff) {  // 32-bit index arithmetic (an emulated 64-bit division costs ~150 instructions)
    const uint32_t t32 = (uint32_t)t0, p32 = (uint32_t)per;
    j = (int)(t32 / p32);
    const uint32_t r32 = t32 - (uint32_t)j * p32;
    bh = (int)(r32 / (uint32_t)ntri);
    tri = (int)(r32 - (uint32_t)bh * (uint32_t)ntri);
    tt = r32;
  } else {
    j = (int)(t0 / per);
    tt = t0 - (int64_t)j * per;
    bh = (int)(tt / ntri);
    tri = (int)(tt % ntri);
  }
  int qt = (int)((sqrtf(8.f * (float)tri + 1.f) - 1.f) * 0.5f);
  while (qt > 0 && qt * (qt + 1) / 2 > tri) --qt;
  while ((qt + 1) * (qt + 2) / 2 <= tri) ++qt;
  int kt = tri - qt * (qt + 1) / 2;
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const uint32_t thr = P.drop_thr;
  uint32_t dkey = mmt_hash(P.drop_key, (uint32_t)j, MMT_STREAM_SALT);
  uint32_t rowh = mmt_prob_row(dkey, (uint32_t)(bh * T + qt * 32 + r));
  const int ng = (int)min<int64_t>(G, total - t0);
  for (int g = 0; g < ng; ++g) {
    // key pair c = kt*16 + 2h + off(e): the row hash plus the tile's part once, the pair offsets as constants
    const uint32_t hb = rowh + (uint32_t)(kt * 16 + 2 * h) * 0x9E3779B9u;
    uint32_t out = 0;   // lane L < 32: key-major dword L = half (L & 1) of element (L >> 1)'s ballot
    uint32_t word = 0;  // this lane's own 16 bits: element 2i at bit i, element 2i + 1 at bit 8 + i
#pragma unroll
    for (int e = 0; e < 16; e += 2) {  // keys k, k+1 (k even) share one hash
      const uint32_t off = (uint32_t)(((e & 3) >> 1) + 4 * (e >> 2));
      const uint32_t hk = mmt_prob_fin(hb + off * 0x9E3779B9u);
      const bool k0 = mmt_keep(hk, 0, thr), k1 = mmt_keep(hk, 1, thr);
      const uint64_t b0 = __builtin_amdgcn_ballot_w64(k0);
      const uint64_t b1 = __builtin_amdgcn_ballot_w64(k1);
      // the wave-uniform ballots straight into their lanes (elements e, e + 1 -> dwords 2e .. 2e + 3)
      out = (uint32_t)mmt_writelane((int)(uint32_t)b0, 2 * e, (int)out);
      out = (uint32_t)mmt_writelane((int)(uint32_t)(b0 >> 32), 2 * e + 1, (int)out);
      out = (uint32_t)mmt_writelane((int)(uint32_t)b1, 2 * e + 2, (int)out);
      out = (uint32_t)mmt_writelane((int)(uint32_t)(b1 >> 32), 2 * e + 3, (int)out);
      word |= (k0 ? 1u << (e >> 1) : 0u) | (k1 ? 1u << (8 + (e >> 1)) : 0u);  // (keep_spread, elem_keep)
    }
    uint32_t* const dm = P.dmask[j];
    if (lane < 32) dm[tt * 32 + lane] = out;
    reinterpret_cast<uint16_t*>(dm + (per + tt) * 32)[lane] = (uint16_t)word;
    // next tile: key tile, then query tile, then (b, h), then stream (wave-uniform branches)
    ++tt;
    if (++kt > qt) {
      kt = 0;
      if (++qt == nt) {
        qt = 0;
        if (++bh == BH) {
          bh = 0;
          tt = 0;
          ++j;
          dkey = mmt_hash(P.drop_key, (uint32_t)j, MMT_STREAM_SALT);
        }
      }
      rowh = mmt_prob_row(dkey, (uint32_t)(bh * T + qt * 32 + r));
    }
  }
}

static int g_mask_g_rt = 0;
extern "C" int mmt_attn_set_mask_g(int g) {
  const int old = g_mask_g_rt;
  g_mask_g_rt = g;
  return old;
}

hipError_t mmt_launch_attn_mask(const AttnBatch& b, int B, int T, int H, hipStream_t s) {
  if (b.count == 0 || B == 0 || T == 0) return hipSuccess;
  int ns = 0;
  for (int g = 0; g < b.count; ++g) {
    const AttnProblem& P = b.p[g];
    if (!P.drop_thr) continue;
    if (P.nstreams < 1 || P.nstreams > MMT_MAX_STREAMS) return hipErrorInvalidValue;
    for (int j = 0; j < P.nstreams; ++j)
      if (!P.dmask[j]) return hipErrorInvalidValue;
    ns = P.nstreams > ns ? P.nstreams : ns;
  }
  if (ns == 0) return hipSuccess;
  const int64_t nt = (T + 31) / 32;
  const int64_t tiles = (int64_t)B * H * (nt * (nt + 1) / 2) * ns;
  // tiles per wave (MMT_MASK_G or mmt_attn_set_mask_g: 1, 2, 4, 8 or 16)
  static const int g_env = [] {
    const char* e = getenv("MMT_MASK_G");
    return e ? atoi(e) : 0;
  }();
  // (16 against 8 at T = 1024 / 4096: C3 140.3-140.4 -> 139.3-140.0 ms, C4 319.4-319.5 -> 317.6-318.7; at C1
  // (T = 256) equal within noise, so 8 below T = 1024: profiles/r6aq_mask_g16_ab.txt)
  const int g_def = T >= 1024 ? 16 : 8;
  // (8 against 4: C3 142.3 -> 140.9-141.1 ms, C1 / target equal; 4 against 1, the one-tile form: C3 149.2 ->
  // 143.7, target 19.40 -> 19.24, C1 7.98 -> 7.91: profiles/r6aa_mask_pileup.txt, r6ab_mask_ab.txt)
  const int gv = g_mask_g_rt ? g_mask_g_rt : g_env ? g_env : g_def;
  const int g = (gv == 1 || gv == 2 || gv == 4 || gv == 16) ? gv : 8;
  const int64_t waves = (tiles + g - 1) / g;
  const dim3 grid((unsigned)((waves + 3) / 4), 1, b.count);
  switch (g) {
    case 1: hipLaunchKernelGGL(attn_mask_kernel<1>, grid, dim3(256), 0, s, b, B * H, T); break;
    case 2: hipLaunchKernelGGL(attn_mask_kernel<2>, grid, dim3(256), 0, s, b, B * H, T); break;
    case 4: hipLaunchKernelGGL(attn_mask_kernel<4>, grid, dim3(256), 0, s, b, B * H, T); break;
    case 16: hipLaunchKernelGGL(attn_mask_kernel<16>, grid, dim3(256), 0, s, b, B * H, T); break;
    default: hipLaunchKernelGGL(attn_mask_kernel<8>, grid, dim3(256), 0, s, b, B * H, T); break;
  }
  return hipGetLastError();
}
