// Attention backward at head size 64 (target shape, C3, C4): slice-streamed kernels.
//
// The chunked kernels of mmt_attn.hip stage 128-row chunks of the shared operand through VGPRs and
// stop the whole workgroup at every chunk reload (two barriers around a global-load -> LDS-store
// round trip); at hs 64 and T >= 512 their waves sit 35-63 % of their cycles in those waits
// (profiles/r2_sq_target.txt). Here the shared operand streams through an LDS ring of 32-row slices
// filled by LDS-DMA (buffer_load ... lds, no VGPR round trip), S - 1 slices ahead of the compute,
// with one barrier per slice: each wave waits (counted vmcnt) only for its own pieces of the slice
// it is about to read, the barrier then publishes every wave's pieces and retires the reads of the
// previous slice, whose slot takes the next DMA.
//
// Slice images: a 32-row x 64-column bf16 tile is stored as four column sub-images (16 columns =
// 32 B per row, 1 KiB each = one LDS-DMA piece) 1152 B apart; the two 16-B halves of row r are
// swapped when bit 3 of r is set. The swap is applied on the DMA's per-lane SOURCE address (the LDS
// side of an LDS-DMA is lane-linear) and again on every read. Both read kinds are bank-conflict
// free: a row read (ds_read_b128, MFMA operand with the row on the lane) of one 16-lane group covers
// each (r mod 8) twice, once per half; the 32-lane half of a transposed read (ds_read_b64_tr_b16,
// the tile as a k-major operand) takes 4 rows x 2 sub-images, and the 128-B pad puts the two
// sub-images in opposite halves of the 256-B bank row. Every read address is a per-lane base plus
// an immediate (k step s: 1152 s for row reads, 512 s for transposed reads; column block: 2304),
// so the slice loop carries almost no address arithmetic.
#include "mmt_common.h"
#include "mmt_kernels.h"

namespace {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 make_rsrc(const void* base, int64_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int32_t)((a >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int32_t)min(bytes, (int64_t)0x7ffffff0));
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
// 16 B per lane: LDS[lds + 16 lane] = buffer[voff] (zeros when voff is out of range)
__device__ __forceinline__ void dma16(const i32x4& rsrc, uint32_t lds, int voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" : : "s"(lds), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}
// 4 B per lane: LDS[lds + 4 lane] = buffer[voff]
__device__ __forceinline__ void dma4(const i32x4& rsrc, uint32_t lds, int voff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds" : : "s"(lds), "v"(voff), "s"(rsrc)
               : "memory", "m0");
}
// counted wait on this wave's outstanding vector-memory operations (immediate operand)
__device__ __forceinline__ void wait_vm(int n) {
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

constexpr float kLog2e2 = 1.4426950408889634f;
constexpr int OOB = 0x7fffffff;

constexpr int SUB = 1152;          // column sub-image stride (1 KiB + 128 B pad)
constexpr int IMG64 = 4 * SUB;      // one 32 x 64 tile
// byte offset of 16-B half `half` (0/1) of the 16-column block `cb` (0..3) in row `row`
__device__ __forceinline__ int img_off(int row, int cb, int half) {
  return cb * SUB + row * 32 + ((half ^ ((row >> 3) & 1)) << 4);
}
__device__ __forceinline__ void zero16(f32x16& a) {
#pragma unroll
  for (int e = 0; e < 16; ++e) a[e] = 0.f;
}
__device__ __forceinline__ float keep_f(float v, int m) { return __int_as_float(__float_as_int(v) & m); }
__device__ __forceinline__ int key_dword(int r) { return 2 * ((r & 3) + 4 * (r >> 3)) + ((r >> 2) & 1); }

// forward helpers (as mmt_attn.hip): cross-half reductions in one v_permlane32_swap, and the
// accumulator registers 8s..8s+7 as a bf16 operand fragment with the keep bits of a lane word applied
__device__ __forceinline__ float xh_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xh_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t keep_spread2(uint32_t w16) { return __builtin_amdgcn_perm(0u, w16, 0x0c010c00u); }
__device__ __forceinline__ uint32_t pair_keep2(uint32_t w32, int i) {
  s16x2 v = __builtin_bit_cast(s16x2, w32 << (15 - i));
  v = v >> (s16x2){15, 15};
  return __builtin_bit_cast(uint32_t, v);
}
template <bool DROP>
__device__ __forceinline__ bf16x8 p_frag(const f32x16& a, int s, uint32_t w32) {
  u32x4 v = {pack2bf(a[8 * s], a[8 * s + 1]), pack2bf(a[8 * s + 2], a[8 * s + 3]), pack2bf(a[8 * s + 4], a[8 * s + 5]),
             pack2bf(a[8 * s + 6], a[8 * s + 7])};
  if (DROP) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] &= pair_keep2(w32, 4 * s + q);
  }
  return __builtin_bit_cast(bf16x8, v);
}
constexpr float kTauR = 8.0f;  // lazy-rescale threshold of the running max (log2 units), as mmt_attn.hip

}  // namespace

// =============================================================================================
// dK, dV at hs 64. grid (nkb * B*H * nstreams, 1, problems), nkb = ceil(nt / 4): a workgroup owns
// NWV = 4 or 8 key tiles (wave w: key tile NWV kb + w, its K / V in registers, dK / dV accumulated
// in registers) and walks the query tiles NWV kb .. nt-1 in lockstep; each query slice (Q, dO, the
// row's LSE and D, the slice's keep bits) arrives in an LDS ring slot by LDS-DMA. Per query tile a
// wave whose key tile is not above it computes S = Q K^T and dP = dO V^T (keys on lanes),
// P = exp2(c2 S - LSE2), dS = P (Z dP - D), dV += (Z P)^T dO, dK += dS^T Q.
// Workgroups are ordered heaviest key block first (the causal walk of key block kb is nt - NWV kb
// slices long) so the launch does not end on a tail of long blocks.
// =============================================================================================
template <bool DROP, int OCC, int S, int NWV>
__global__ __launch_bounds__(64 * NWV, OCC) void attn_bwd_dkdv_ring64(AttnBatch batch, int T, int H, float scale) {
  constexpr int NKS = 4, ND = 2;  // hs 64: 4 k-steps of 16, 2 output tiles of 32
  static_assert(S >= 3 && 4 * (S - 2) <= 16, "ring slots: S - 1 slices in flight, counted waits <= 16");
  constexpr int OFF_DO = IMG64, OFF_L = 2 * IMG64, OFF_D = OFF_L + 256, OFF_M = OFF_D + 256;
  constexpr int SLOT = OFF_M + (DROP ? 1024 : 0);
  constexpr int EPW = 40;  // epilogue transpose slot row stride (bf16)
  static_assert(NWV == 4 || NWV == 8, "4 or 8 key tiles (waves) per workgroup");
  constexpr int PPW = 8 / NWV;  // Q / dO sub-image pieces per wave per slice
  constexpr int EPI_BYTES = NWV * 2 * 32 * EPW * 2;  // per-wave epilogue transpose slots (alias the ring)
  __shared__ __attribute__((aligned(1024))) char lds[S * SLOT > EPI_BYTES ? S * SLOT : EPI_BYTES];
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nt = (T + 31) / 32;
  const int nkb = (nt + NWV - 1) / NWV;
  const int ns = P.nstreams;
  const int nbhs = gridDim.x / nkb;  // B*H*nstreams
  const int BH = nbhs / ns;
  const int kb = blockIdx.x / nbhs;  // heaviest first (no XCD remap: it would give whole XCDs the long blocks)
  const int yy = blockIdx.x % nbhs;
  const int j = yy / BH, bh = yy % BH;
  const int b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int kt0 = kb * NWV;
  const int kt = kt0 + w;
  const bool live = kt < nt;
  const int tk = kt * 32 + r;
  const int nq = nt - kt0;  // query tiles walked by the block
  const int64_t rowbase = (int64_t)b * T;
  const float c2 = scale * kLog2e2;
  const bool ragged = (T & 31) != 0;

  // this wave's K / V rows (keys on lanes): the B operands of S and dP
  bf16x8 kf[NKS], vf[NKS];
  {
    const bf16_t* kp = P.k[j] + head * P.kv_hstride + (rowbase + tk) * P.kv_ld;
    const bf16_t* vp = P.v[j] + head * P.kv_hstride + (rowbase + tk) * P.kv_ld;
    const bool ok = live && tk < T;
    u32x4 kr[NKS], vr[NKS];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const u32x4 z = {0u, 0u, 0u, 0u};
      kr[s] = ok ? *reinterpret_cast<const u32x4*>(kp + 16 * s + 8 * h) : z;
      vr[s] = ok ? *reinterpret_cast<const u32x4*>(vp + 16 * s + 8 * h) : z;
    }
    // consume them here: the compiler's own wait for these loads then sits before the DMA prologue
    // instead of at their first use inside the slice loop, where its vmcnt(0) would drain the ring
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      asm volatile("" : "+v"(kr[s]));
      asm volatile("" : "+v"(vr[s]));
      kf[s] = __builtin_bit_cast(bf16x8, kr[s]);
      vf[s] = __builtin_bit_cast(bf16x8, vr[s]);
    }
  }
  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) { zero16(dk[dt]); zero16(dv[dt]); }

  // DMA sources: Q / dO rows of batch b (rows past T are sent out of range: zeros), the stream's
  // LSE / D rows, the key-major keep-bit records of (query tile, key tiles kt0..kt0+3) (contiguous)
  // (each resource starts at batch row b: the 32-bit per-lane offsets span one sequence only)
  const i32x4 rq = make_rsrc(P.q + rowbase * P.q_ld + head * 64, (int64_t)T * P.q_ld * 2);
  const i32x4 rdo = make_rsrc(P.dout + rowbase * P.dout_ld + head * 64, (int64_t)T * P.dout_ld * 2);
  const i32x4 rl = make_rsrc(P.lse[j] + (int64_t)bh * T, (int64_t)T * 4);
  const i32x4 rd = make_rsrc(P.dvec[j] + (int64_t)bh * T, (int64_t)T * 4);
  const int64_t ntri = (int64_t)nt * (nt + 1) / 2;
  const i32x4 rm = make_rsrc(DROP ? P.dmask[j] + (int64_t)bh * ntri * 32 : P.dmask[0], ntri * 32 * 4);
  // pieces this wave issues per slice: 2 sub-images (+ LSE for wave 0, D for wave 1, the keep bits
  // for wave 2); the counted waits below count them
  const int per = PPW + (w < 2 ? 1 : 0) + (DROP && w == 2 ? 1 : 0);
  // per-lane source of a sub-image piece: row L/2, half L&1 (swapped on rows with bit 3 set)
  const int prow = lane >> 1;
  const int pcol = 8 * ((lane & 1) ^ ((prow >> 3) & 1));
  auto issue = [&](int slot, int qt) {
    char* sb = lds + slot * SLOT;
    const int q0 = qt * 32;
    const int grow = q0 + prow;
#pragma unroll
    for (int u = 0; u < PPW; ++u) {
      const int piece = PPW * w + u;  // 0..3: Q column blocks, 4..7: dO
      const int op = piece >> 2, cb = piece & 3;
      const int ld = op ? P.dout_ld : P.q_ld;
      const int voff = grow < T ? (grow * ld + cb * 16 + pcol) * 2 : OOB;
      dma16(op ? rdo : rq, __builtin_amdgcn_readfirstlane(lds_u32(sb + op * OFF_DO + cb * SUB)), voff);
    }
    if (w < 2) {
      const int voff = (lane < 32 && q0 + lane < T) ? (q0 + lane) * 4 : OOB;
      dma4(w == 0 ? rl : rd, __builtin_amdgcn_readfirstlane(lds_u32(sb + OFF_L + w * 256)), voff);
    }
    if (DROP && w == 2) {  // NWV key tiles x 128 B of the key-major records of (qt, kt0..kt0+NWV-1)
      const int voff = lane < 8 * NWV ? (int)(((int64_t)qt * (qt + 1) / 2 + kt0) * 128 + lane * 16) : OOB;
      dma16(rm, __builtin_amdgcn_readfirstlane(lds_u32(sb + OFF_M)), voff);
    }
  };
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nq) issue(i, kt0 + i);

  // per-lane read offsets (the slot base and the k step / column block are added as immediates):
  // row reads (lane row r, half h of 16-column block s), transposed reads (tr_frag geometry: rows
  // 16 s + 4 (g >> 1) + q and + 8, columns 32 dt + 16 (g & 1) + 4 p)
  const int o_row = img_off(r, 0, h);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int o_tr0 = img_off(4 * (g >> 1) + q, g & 1, p >> 1) + 8 * (p & 1);
  const int o_tr1 = img_off(8 + 4 * (g >> 1) + q, g & 1, p >> 1) + 8 * (p & 1);
  const int o_ld = (8 * 0 + 4 * h) * 4;
  const int o_mk = ((kt - kt0) * 32 + key_dword(r)) * 4;
  const float dsc = DROP ? P.drop_scale : 1.f;
  // one query tile against this wave's key tile; MASKED: the diagonal tile / a ragged last tile
  auto tile = [&](const char* sb, int qt, auto mc) {
    constexpr bool MASKED = decltype(mc)::value;
    const uint32_t mw = DROP ? *reinterpret_cast<const uint32_t*>(sb + OFF_M + o_mk) >> (4 * h) : 0u;
    f32x16 sacc, dpacc;
    zero16(sacc);
    zero16(dpacc);
    bf16x8 qr[NKS], dr[NKS];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      qr[s] = *reinterpret_cast<const bf16x8*>(sb + o_row + s * SUB);
      dr[s] = *reinterpret_cast<const bf16x8*>(sb + OFF_DO + o_row + s * SUB);
    }
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      sacc = mfma32(qr[s], kf[s], sacc);    // S[q][key]
      dpacc = mfma32(dr[s], vf[s], dpacc);  // dP[q][key]
    }
    bf16x8 dot[2][ND], qtr[2][ND];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        dot[s][dt] = join4(lds_tr16(sb + OFF_DO + o_tr0 + 512 * s + 2 * SUB * dt),
                           lds_tr16(sb + OFF_DO + o_tr1 + 512 * s + 2 * SUB * dt));
        qtr[s][dt] = join4(lds_tr16(sb + o_tr0 + 512 * s + 2 * SUB * dt), lds_tr16(sb + o_tr1 + 512 * s + 2 * SUB * dt));
      }
    uint32_t pp[8], dd[8];  // packed bf16 pairs of Z.P (dV operand) and dS (dK operand)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(sb + OFF_L + o_ld + 32 * gg);
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(sb + OFF_D + o_ld + 32 * gg);
#pragma unroll
      for (int e4 = 0; e4 < 4; e4 += 2) {
        float pm[2], ds[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int e = 4 * gg + e4 + u;
          float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[e], c2, -l4[e4 + u]));
          if (MASKED) {
            const int tq = qt * 32 + 8 * gg + 4 * h + e4 + u;
            if (!(tk <= tq && tq < T)) pv = 0.f;
          }
          const float dp = dpacc[e];
          if (DROP) {
            // dS = P (Z dP sc - D) = sc (Z P dP - P D'), D' = D / sc as the dQ pass stores it; sc is
            // applied to dK at the end (one VALU per element fewer than masking dP separately)
            const int kbit = __builtin_amdgcn_sbfe((int)mw, 8 * gg + e4 + u, 1);  // all ones iff kept
            pm[u] = keep_f(pv, kbit);
            ds[u] = __builtin_fmaf(pm[u], dp, -(pv * d4[e4 + u]));  // dS[q][key] / sc
          } else {
            pm[u] = pv;
            ds[u] = pv * (dp - d4[e4 + u]);  // dS[q][key]
          }
        }
        pp[2 * gg + e4 / 2] = pack2bf(pm[0], pm[1]);
        dd[2 * gg + e4 / 2] = pack2bf(ds[0], ds[1]);
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pf = __builtin_bit_cast(bf16x8, u32x4{pp[4 * s], pp[4 * s + 1], pp[4 * s + 2], pp[4 * s + 3]});
      const bf16x8 df = __builtin_bit_cast(bf16x8, u32x4{dd[4 * s], dd[4 * s + 1], dd[4 * s + 2], dd[4 * s + 3]});
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        dv[dt] = mfma32(pf, dot[s][dt], dv[dt]);
        dk[dt] = mfma32(df, qtr[s][dt], dk[dt]);
      }
    }
  };

  // slice i: wait for it, publish it, refill the slot slice i - 1 used, compute. Three straight
  // loops, one tile variant each (two variants merging inside one loop made the register allocator
  // copy the dK / dV accumulators every iteration): the block's 4 diagonal slices (masked: each
  // wave's own diagonal, and nothing above it), the plain slices, a ragged last slice (masked)
  auto step = [&](int i, auto mc) {
    wait_vm(per * min(S - 2, nq - 1 - i));  // this wave's pieces of slice i landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone's pieces of slice i landed; slice i - 1's reads are done
    if (i + S - 1 < nq) issue((i + S - 1) % S, kt0 + i + S - 1);
    const int qt = kt0 + i;
    if (live && qt >= kt) tile(lds + (i % S) * SLOT, qt, mc);
  };
  const int n_diag = min(NWV, nq);
  const int n_plain_end = (ragged && nq > 4) ? nq - 1 : nq;
  int i = 0;
#pragma unroll 1
  for (; i < n_diag; ++i) step(i, std::true_type{});
#pragma unroll 1
  for (; i < n_plain_end; ++i) step(i, std::false_type{});
  if (i < nq) step(i, std::true_type{});
  __syncthreads();  // the ring is free: the epilogue transposes through it

  // dK / dV tiles: accumulator rows = key ((e&3)+8(e>>2)+4h), cols = d (lane); each 32-column slice
  // is transposed through this wave's LDS slot and leaves as row-major 16-B pieces
  if (live) {
    bf16_t* et = reinterpret_cast<bf16_t*>(lds) + w * (2 * 32 * EPW);
    const int k0 = kt * 32;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kr = (e & 3) + 8 * (e >> 2) + 4 * h;
        et[kr * EPW + r] = f2bf(DROP ? dk[dt][e] * (scale * P.drop_scale) : dk[dt][e] * scale);
        et[32 * EPW + kr * EPW + r] = f2bf(DROP ? dv[dt][e] * P.drop_scale : dv[dt][e]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = i * 16 + (lane >> 2), d0 = dt * 32 + (lane & 3) * 8;
        const u32x4 vk = *reinterpret_cast<const u32x4*>(et + row * EPW + (lane & 3) * 8);
        const u32x4 vv = *reinterpret_cast<const u32x4*>(et + 32 * EPW + row * EPW + (lane & 3) * 8);
        if (k0 + row < T) {
          const int64_t off = (rowbase + k0 + row) * P.dkv_ld + d0;
          *reinterpret_cast<u32x4*>(P.dk[j] + head * P.dkv_hstride + off) = vk;
          *reinterpret_cast<u32x4*>(P.dv[j] + head * P.dkv_hstride + off) = vv;
        }
      }
    }
  }
}


// =============================================================================================
// dQ (and D_j) at hs 64, two query tiles per wave. grid (nqb * B*H, 1, problems), nqb = ceil(nt / 8):
// a workgroup owns 8 query tiles 8 qb .. 8 qb + 7 (wave w: tiles A = 8 qb + w and B = 8 qb + 7 - w,
// so every wave's causal walk is equally long) and walks (stream j, key tile 0 .. 8 qb + 7) through
// the LDS ring; a wave reads each slice's K / V fragments (rows and K transposed) ONCE and runs both
// of its query tiles on them: half the fragment reads, DMA pieces and barriers per MFMA of the
// walk with one tile per wave. Diagonal tiles are masked at run time (a uniform branch around the mask).
// =============================================================================================
template <bool DROP, int S>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_ring64x2(AttnBatch batch, int T, int H, float scale) {
  constexpr int NKS = 4, ND = 2;
  static_assert(S >= 3 && 3 * (S - 2) <= 16, "ring slots: S - 1 slices in flight, counted waits <= 16");
  constexpr int OFF_V = IMG64, OFF_M = 2 * IMG64;
  constexpr int SLOT = OFF_M + (DROP ? 1024 : 0);
  constexpr int TAB = S * SLOT;  // [wave][tile A / B][stream][query row] {lse2, D} float2
  __shared__ __attribute__((aligned(1024))) char lds[TAB + 4 * 2 * MMT_MAX_STREAMS * 32 * 8];
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nt = (T + 31) / 32;
  const int nqb = (nt + 7) / 8;
  const int ns = P.nstreams;
  const int BH = gridDim.x / nqb;
  const int qb = nqb - 1 - (int)(blockIdx.x / BH);  // heaviest (last) query block first
  const int bh = blockIdx.x % BH;
  const int b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int qt[2] = {8 * qb + w, 8 * qb + 7 - w};
  const bool live[2] = {qt[0] < nt, qt[1] < nt};
  const int tq[2] = {qt[0] * 32 + r, qt[1] * 32 + r};
  const bool okq[2] = {live[0] && tq[0] < T, live[1] && tq[1] < T};
  const int nk = min(8 * qb + 8, nt);  // key tiles walked per stream
  const int nsl = ns * nk;             // slices
  const int64_t rowbase = (int64_t)b * T;
  const float c2 = scale * kLog2e2;

  // Q, dO of both query tiles (queries on lanes: the B operands of S^T and dP^T); per stream
  // D_j = rowsum(dO * O_j) (written for the dK/dV pass) and the LSE into the LDS table
  bf16x8 qf[2][NKS], dof[2][NKS];
  float* tab = reinterpret_cast<float*>(lds + TAB) + w * (2 * MMT_MAX_STREAMS * 64);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    u32x4 qr[NKS], dr[NKS];
    const bf16_t* qp = P.q + (rowbase + tq[u]) * P.q_ld + head * 64;
    const bf16_t* dp = P.dout + (rowbase + tq[u]) * P.dout_ld + head * 64;
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      qr[s] = okq[u] ? *reinterpret_cast<const u32x4*>(qp + 16 * s + 8 * h) : z;
      dr[s] = okq[u] ? *reinterpret_cast<const u32x4*>(dp + 16 * s + 8 * h) : z;
    }
    for (int j = 0; j < ns; ++j) {
      const bf16_t* oj = (ns > 1 ? P.oj[j] : P.o) + (rowbase + tq[u]) * P.o_ld + head * 64;
      float d = 0.f;
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const u32x4 ov = okq[u] ? *reinterpret_cast<const u32x4*>(oj + 16 * s + 8 * h) : z;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          d += bf2f(ov[e] & 0xffff) * bf2f(dr[s][e] & 0xffff);
          d += bf2f(ov[e] >> 16) * bf2f(dr[s][e] >> 16);
        }
      }
      d += __shfl_xor(d, 32, 64);
      const float l2 = okq[u] ? P.lse[j][(int64_t)bh * T + tq[u]] : 0.f;
      if (h == 0) {  // D_j / drop_scale for the dK/dV pass (its dS = sc (Z P dP - P D / sc))
        if (okq[u]) P.dvec[j][(int64_t)bh * T + tq[u]] = DROP ? d / P.drop_scale : d;
        tab[(u * MMT_MAX_STREAMS + j) * 64 + 2 * r] = l2;
        tab[(u * MMT_MAX_STREAMS + j) * 64 + 2 * r + 1] = d;
      }
    }
    // consumed here: the compiler's wait for these loads sits before the DMA prologue
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      asm volatile("" : "+v"(qr[s]));
      asm volatile("" : "+v"(dr[s]));
      qf[u][s] = __builtin_bit_cast(bf16x8, qr[s]);
      dof[u][s] = __builtin_bit_cast(bf16x8, dr[s]);
    }
  }
  f32x16 dq[2][ND];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) zero16(dq[u][dt]);

  const int64_t ntri = (int64_t)nt * (nt + 1) / 2;
  const int64_t ntiles = (int64_t)BH * ntri;
  const int prow = lane >> 1;
  const int pcol = 8 * ((lane & 1) ^ ((prow >> 3) & 1));
  const int per = 2 + (DROP && w == 0 ? 1 : 0);
  // the issuing stream's K / V / keep-bit descriptors, rebuilt when the walk enters a new stream (built
  // per slice, their kernel-argument loads put an s_load latency in front of every slice's DMA)
  i32x4 rk, rv, rm;
  int jr = -1;
  auto set_stream = [&](int j) {
    rk = make_rsrc(P.k[j] + rowbase * P.kv_ld + head * P.kv_hstride, (int64_t)T * P.kv_ld * 2);
    rv = make_rsrc(P.v[j] + rowbase * P.kv_ld + head * P.kv_hstride, (int64_t)T * P.kv_ld * 2);
    rm = make_rsrc(DROP ? P.dmask[j] + (ntiles + (int64_t)bh * ntri) * 32 : P.dmask[0], ntri * 128);
    jr = j;
  };
  // the K / V row stride as a VGPR: as a kernel argument the compiler re-loaded it (s_load + a full
  // lgkmcnt wait) in front of each slice's DMA pieces rather than keep it in an SGPR
  int kvld = P.kv_ld;
  asm volatile("" : "+v"(kvld));
  auto issue = [&](int slot, int j, int kt) {  // slice (stream j, key tile kt)
    char* sb = lds + slot * SLOT;
    const int grow = kt * 32 + prow;
    if (j != jr) set_stream(j);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int piece = 2 * w + u;  // 0..3: K column block, 4..7: V
      const int op = piece >> 2, cb = piece & 3;
      const int voff = grow < T ? (grow * kvld + cb * 16 + pcol) * 2 : OOB;
      dma16(op ? rv : rk, __builtin_amdgcn_readfirstlane(lds_u32(sb + op * OFF_V + cb * SUB)), voff);
    }
    if (DROP && w == 0) {  // lane words of (query tile 8 qb + u, key tile kt), u = 0..7: 8 x 128 B
      const int u = lane >> 3, q_ = 8 * qb + u;
      const int voff = (q_ < nt && kt <= q_) ? (q_ * (q_ + 1) / 2 + kt) * 128 + (lane & 7) * 16 : OOB;
      dma16(rm, __builtin_amdgcn_readfirstlane(lds_u32(sb + OFF_M)), voff);
    }
  };
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nsl) issue(i, i / nk, i % nk);

  const int o_row = img_off(r, 0, h);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int o_tr0 = img_off(4 * (g >> 1) + q, g & 1, p >> 1) + 8 * (p & 1);
  const int o_tr1 = img_off(8 + 4 * (g >> 1) + q, g & 1, p >> 1) + 8 * (p & 1);
  const float dsc = DROP ? P.drop_scale : 1.f;
  // one key tile against query tile u of this wave, on the slice's fragments (masked: the diagonal)
  auto tile = [&](const char* sb, int u, int j, int kt, const bf16x8 (&kf)[NKS], const bf16x8 (&vf)[NKS],
                  const bf16x8 (&ktr)[2][ND], bool masked) {
    const int ut = u == 0 ? w : 7 - w;  // the tile's index in the block (keep-bit record)
    const uint32_t mw = DROP ? reinterpret_cast<const uint16_t*>(sb + OFF_M)[ut * 64 + lane] : 0u;
    const float l2 = tab[(u * MMT_MAX_STREAMS + j) * 64 + 2 * r], dsum = tab[(u * MMT_MAX_STREAMS + j) * 64 + 2 * r + 1];
    f32x16 sa, pa;
    zero16(sa);
    zero16(pa);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      sa = mfma32(kf[s], qf[u][s], sa);   // S^T[key][q]
      pa = mfma32(vf[s], dof[u][s], pa);  // dP^T[key][q]
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sa[e], c2, -l2));
      float dp = pa[e];
      if (DROP) dp = keep_f(dp, __builtin_amdgcn_sbfe((int)mw, (e & 1) * 8 + (e >> 1), 1));
      sa[e] = pv * __builtin_fmaf(dp, dsc, -dsum);  // dS^T
    }
    if (masked) {  // keys above the query (and past T) contribute nothing
      const int tqv = tq[u];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int key = kt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (key > tqv || key >= T) sa[e] = 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const u32x4 v = {pack2bf(sa[8 * s], sa[8 * s + 1]), pack2bf(sa[8 * s + 2], sa[8 * s + 3]),
                       pack2bf(sa[8 * s + 4], sa[8 * s + 5]), pack2bf(sa[8 * s + 6], sa[8 * s + 7])};
      const bf16x8 df = __builtin_bit_cast(bf16x8, v);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) dq[u][dt] = mfma32(ktr[s][dt], df, dq[u][dt]);
    }
  };
  // slice indices kept as (stream, key tile) counters: no integer division per slice
  int ji = (S - 1) / nk, kti = (S - 1) % nk, jc = 0, ktc = 0;
#pragma unroll 1
  for (int i = 0; i < nsl; ++i) {
    wait_vm(per * min(S - 2, nsl - 1 - i));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (i + S - 1 < nsl) {
      issue((i + S - 1) % S, ji, kti);
      if (++kti == nk) { kti = 0; ++ji; }
    }
    const int j = jc, kt = ktc;
    if (++ktc == nk) { ktc = 0; ++jc; }
    // tile B (the later one) may lie past the sequence's last tile while A does not
    const bool needA = live[0] && kt <= qt[0], needB = live[1] && kt <= qt[1];
    if (needA || needB) {
      const char* sb = lds + (i % S) * SLOT;
      bf16x8 kf[NKS], vf[NKS], ktr[2][ND];
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        kf[s] = *reinterpret_cast<const bf16x8*>(sb + o_row + s * SUB);
        vf[s] = *reinterpret_cast<const bf16x8*>(sb + OFF_V + o_row + s * SUB);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
          ktr[s][dt] = join4(lds_tr16(sb + o_tr0 + 512 * s + 2 * SUB * dt), lds_tr16(sb + o_tr1 + 512 * s + 2 * SUB * dt));
      if (needA) tile(sb, 0, j, kt, kf, vf, ktr, kt == qt[0]);
      if (needB) tile(sb, 1, j, kt, kf, vf, ktr, kt == qt[1]);
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int ga = 2 * pr, gb = 2 * pr + 1;
        const uint32_t x0 = pack2bf(dq[u][dt][4 * ga] * scale, dq[u][dt][4 * ga + 1] * scale);
        const uint32_t x1 = pack2bf(dq[u][dt][4 * ga + 2] * scale, dq[u][dt][4 * ga + 3] * scale);
        const uint32_t y0 = pack2bf(dq[u][dt][4 * gb] * scale, dq[u][dt][4 * gb + 1] * scale);
        const uint32_t y1 = pack2bf(dq[u][dt][4 * gb + 2] * scale, dq[u][dt][4 * gb + 3] * scale);
        const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        const int d0 = dt * 32 + 16 * pr + 8 * h;
        if (okq[u])
          *reinterpret_cast<u32x4*>(P.dq + (rowbase + tq[u]) * P.dq_ld + head * 64 + d0) = u32x4{s0[0], s1[0], s0[1], s1[1]};
      }
}

// =============================================================================================
// Forward at hs 64, two query tiles per wave, on the same LDS-DMA slice ring as the dQ pass: grid
// (nqb * B*H, 1, problems); a workgroup owns query tiles 8 qb .. 8 qb + 7 (wave w: A = 8 qb + w,
// B = 8 qb + 7 - w) and walks (stream j, key tile 0 .. 8 qb + 7); each slice brings the key tile's K
// and V images and the keep-bit lane words of the block's 8 query tiles. Per slice a wave reads K
// rows (S^T = K Q^T, keys on accumulator rows, queries on lanes) and V transposed (O^T += V^T P^T)
// once for both of its tiles. Online softmax in the log2 domain with the lazy rescale of
// mmt_attn.hip (threshold kTauR); at the last key tile of a stream the outputs are normalised and
// stored with the stream's LSE. The chunked forward (mmt_attn.hip) re-staged 128-row chunks through
// VGPRs behind two barriers per chunk; its register prefetch of the next chunk does not fit at hs 64.
// =============================================================================================
template <bool DROP, int S>
__global__ __launch_bounds__(256, 2) void attn_fwd_ring64x2(AttnBatch batch, int T, int H, float scale) {
  constexpr int NKS = 4, ND = 2;
  static_assert(S >= 3 && 3 * (S - 2) <= 16, "ring slots: S - 1 slices in flight, counted waits <= 16");
  constexpr int OFF_V = IMG64, OFF_M = 2 * IMG64;
  constexpr int SLOT = OFF_M + (DROP ? 1024 : 0);
  __shared__ __attribute__((aligned(1024))) char lds[S * SLOT];
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nt = (T + 31) / 32;
  const int nqb = (nt + 7) / 8;
  const int ns = P.nstreams;
  const int BH = gridDim.x / nqb;
  const int qb = nqb - 1 - (int)(blockIdx.x / BH);  // heaviest (last) query block first
  const int bh = blockIdx.x % BH;
  const int b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int qt[2] = {8 * qb + w, 8 * qb + 7 - w};
  const bool live[2] = {qt[0] < nt, qt[1] < nt};
  const int tq[2] = {qt[0] * 32 + r, qt[1] * 32 + r};
  const bool okq[2] = {live[0] && tq[0] < T, live[1] && tq[1] < T};
  const int nk = min(8 * qb + 8, nt);  // key tiles walked per stream
  const int nsl = ns * nk;             // slices
  const int64_t rowbase = (int64_t)b * T;
  const float c2 = scale * kLog2e2;

  // Q of both query tiles (queries on lanes: the B operand of S^T)
  bf16x8 qf[2][NKS];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const bf16_t* qp = P.q + (rowbase + tq[u]) * P.q_ld + head * 64;
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      u32x4 v = okq[u] ? *reinterpret_cast<const u32x4*>(qp + 16 * s + 8 * h) : z;
      asm volatile("" : "+v"(v));  // consumed here: the wait for these loads sits before the DMA prologue
      qf[u][s] = __builtin_bit_cast(bf16x8, v);
    }
  }
  f32x16 o[2][ND];
  float m[2], l[2];

  const int64_t ntri = (int64_t)nt * (nt + 1) / 2;
  const int64_t ntiles = (int64_t)BH * ntri;
  const int prow = lane >> 1;
  const int pcol = 8 * ((lane & 1) ^ ((prow >> 3) & 1));
  const int per = 2 + (DROP && w == 0 ? 1 : 0);
  // as the dQ pass: the issuing stream's descriptors rebuilt only when the walk enters a new stream,
  // the K / V row stride in a VGPR (no kernel-argument loads in front of each slice's DMA)
  i32x4 rk, rv, rm;
  int jr = -1;
  auto set_stream = [&](int j) {
    rk = make_rsrc(P.k[j] + rowbase * P.kv_ld + head * P.kv_hstride, (int64_t)T * P.kv_ld * 2);
    rv = make_rsrc(P.v[j] + rowbase * P.kv_ld + head * P.kv_hstride, (int64_t)T * P.kv_ld * 2);
    rm = make_rsrc(DROP ? P.dmask[j] + (ntiles + (int64_t)bh * ntri) * 32 : P.dmask[0], ntri * 128);
    jr = j;
  };
  int kvld = P.kv_ld;
  asm volatile("" : "+v"(kvld));
  auto issue = [&](int slot, int j, int kt) {  // slice (stream j, key tile kt)
    char* sb = lds + slot * SLOT;
    const int grow = kt * 32 + prow;
    if (j != jr) set_stream(j);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int piece = 2 * w + u;  // 0..3: K column block, 4..7: V
      const int op = piece >> 2, cb = piece & 3;
      const int voff = grow < T ? (grow * kvld + cb * 16 + pcol) * 2 : OOB;
      dma16(op ? rv : rk, __builtin_amdgcn_readfirstlane(lds_u32(sb + op * OFF_V + cb * SUB)), voff);
    }
    if (DROP && w == 0) {  // lane words of (query tile 8 qb + u, key tile kt), u = 0..7: 8 x 128 B
      const int u = lane >> 3, q_ = 8 * qb + u;
      const int voff = (q_ < nt && kt <= q_) ? (q_ * (q_ + 1) / 2 + kt) * 128 + (lane & 7) * 16 : OOB;
      dma16(rm, __builtin_amdgcn_readfirstlane(lds_u32(sb + OFF_M)), voff);
    }
  };
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nsl) issue(i, i / nk, i % nk);

  const int o_row = img_off(r, 0, h);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int o_tr0 = img_off(4 * (g >> 1) + q, g & 1, p >> 1) + 8 * (p & 1);
  const int o_tr1 = img_off(8 + 4 * (g >> 1) + q, g & 1, p >> 1) + 8 * (p & 1);
  // online softmax of one S^T tile of query tile u (masked: the causal diagonal)
  auto softmax = [&](f32x16& sa, int u, int kt, bool masked) {
    if (masked) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int key = kt * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (key > tq[u]) sa[e] = -INFINITY;
      }
    }
    float tmax = sa[0];
#pragma unroll
    for (int e = 1; e < 16; ++e) tmax = fmaxf(tmax, sa[e]);
    tmax = xh_max(tmax) * c2;
    const bool up = tmax > m[u] + kTauR;
    if (__builtin_amdgcn_ballot_w64(up)) {  // wave-uniform
      const float alpha = up ? __builtin_amdgcn_exp2f(m[u] - tmax) : 1.f;
      m[u] = up ? tmax : m[u];
      l[u] *= alpha;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[u][dt][e] *= alpha;
    }
    const float nm = -m[u];
#pragma unroll
    for (int e = 0; e < 16; ++e) sa[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sa[e], c2, nm));
    float r0 = sa[0] + sa[1], r1 = sa[2] + sa[3], r2 = sa[4] + sa[5], r3 = sa[6] + sa[7];
    r0 += sa[8] + sa[9]; r1 += sa[10] + sa[11]; r2 += sa[12] + sa[13]; r3 += sa[14] + sa[15];
    l[u] += (r0 + r1) + (r2 + r3);
  };
  const float dsc = DROP ? P.drop_scale : 1.f;
  // normalise and store stream j's outputs of query tile u (and its LSE, log2 domain)
  auto finish = [&](int u, int j) {
    const float lt = xh_sum(l[u]);
    const float inv = lt > 0.f ? dsc / lt : 0.f;
    u32x4 ov[ND][2];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int ga = 2 * pr, gb = 2 * pr + 1;
        const uint32_t x0 = pack2bf(o[u][dt][4 * ga] * inv, o[u][dt][4 * ga + 1] * inv);
        const uint32_t x1 = pack2bf(o[u][dt][4 * ga + 2] * inv, o[u][dt][4 * ga + 3] * inv);
        const uint32_t y0 = pack2bf(o[u][dt][4 * gb] * inv, o[u][dt][4 * gb + 1] * inv);
        const uint32_t y1 = pack2bf(o[u][dt][4 * gb + 2] * inv, o[u][dt][4 * gb + 3] * inv);
        const auto s0 = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
        ov[dt][pr] = u32x4{s0[0], s1[0], s0[1], s1[1]};  // d = dt*32 + 16 pr + 8 h + 0..7
      }
    if (okq[u]) {
      if (h == 0) P.lse[j][(int64_t)bh * T + tq[u]] = m[u] + __log2f(lt);
      bf16_t* dst = (ns > 1 ? P.oj[j] : P.o) + (rowbase + tq[u]) * P.o_ld + head * 64;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) *reinterpret_cast<u32x4*>(dst + dt * 32 + 16 * pr + 8 * h) = ov[dt][pr];
    }
  };
  int ji = (S - 1) / nk, kti = (S - 1) % nk, jc = 0, ktc = 0;  // slice counters (no division per slice)
#pragma unroll 1
  for (int i = 0; i < nsl; ++i) {
    wait_vm(per * min(S - 2, nsl - 1 - i));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (i + S - 1 < nsl) {
      issue((i + S - 1) % S, ji, kti);
      if (++kti == nk) { kti = 0; ++ji; }
    }
    const int j = jc, kt = ktc;
    if (++ktc == nk) { ktc = 0; ++jc; }
    if (kt == 0) {  // a stream's walk starts
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        m[u] = -INFINITY;
        l[u] = 0.f;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) zero16(o[u][dt]);
      }
    }
    // tile B (the later one) may need a key tile that A does not (or lie past the sequence)
    const bool needA = live[0] && kt <= qt[0], needB = live[1] && kt <= qt[1];
    if (needA || needB) {
      const char* sb = lds + (i % S) * SLOT;
      bf16x8 kf[NKS], vtr[2][ND];
#pragma unroll
      for (int s = 0; s < NKS; ++s) kf[s] = *reinterpret_cast<const bf16x8*>(sb + o_row + s * SUB);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
          vtr[s][dt] = join4(lds_tr16(sb + OFF_V + o_tr0 + 512 * s + 2 * SUB * dt),
                             lds_tr16(sb + OFF_V + o_tr1 + 512 * s + 2 * SUB * dt));
      const uint32_t wa = DROP ? keep_spread2(reinterpret_cast<const uint16_t*>(sb + OFF_M)[w * 64 + lane]) : 0u;
      const uint32_t wb = DROP ? keep_spread2(reinterpret_cast<const uint16_t*>(sb + OFF_M)[(7 - w) * 64 + lane]) : 0u;
      f32x16 sa, sb2;
      zero16(sa);
      zero16(sb2);
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        if (needA) sa = mfma32(kf[s], qf[0][s], sa);
        if (needB) sb2 = mfma32(kf[s], qf[1][s], sb2);
      }
      if (needA) softmax(sa, 0, kt, kt == qt[0]);
      if (needB) softmax(sb2, 1, kt, kt == qt[1]);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (needA) {
          const bf16x8 pa = p_frag<DROP>(sa, s, wa);
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) o[0][dt] = mfma32(vtr[s][dt], pa, o[0][dt]);
        }
        if (needB) {
          const bf16x8 pb = p_frag<DROP>(sb2, s, wb);
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) o[1][dt] = mfma32(vtr[s][dt], pb, o[1][dt]);
        }
      }
    }
    if (kt == nk - 1) {
      if (live[0]) finish(0, j);
      if (live[1]) finish(1, j);
    }
  }
  // several streams: the output is the sum of the per-stream outputs this lane just wrote
  if (ns > 1) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!okq[u]) continue;
      const int64_t off = (rowbase + tq[u]) * P.o_ld + head * 64;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const int d0 = dt * 32 + 16 * pr + 8 * h;
          float t[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          for (int jj = 0; jj < ns; ++jj) {
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

// =============================================================================================
// One-pass backward at hs 64 for T <= 512 and one KV stream (the target shape's self-attention):
// grid (B*H, 1, problems), one workgroup per (batch, head) owns ALL nt <= 16 key tiles, so dQ needs
// no sum across workgroups and S / dP are computed once (the two-pass form recomputes both in its
// dQ pass: 7 products per tile pair instead of 5). Wave w owns key tiles w, 7-w, 8+w, 15-w (every
// causal walk 17 tile pairs long at nt = 16), their V rows and dK / dV accumulators in registers
// (256 accumulator registers at one wave per SIMD), and walks the query slices 0 .. nt-1:
//   * K of the whole sequence sits in LDS as slice images (read by rows for S, transposed for dQ);
//   * each query slice (Q, dO, O images, the LSE row, the keep-bit records of key tiles 0..qt)
//     streams through an LDS-DMA ring S - 1 slices ahead, one barrier per slice;
//   * per tile: S = Q K^T, dP = dO V^T (keys on lanes), P, dS; dV += (Z P)^T dO, dK += dS^T Q;
//     dS crosses a wave-private LDS transpose image once and dQ_w += dS K runs on MFMA;
//   * each wave's dQ partial (its tiles of the slice, summed on MFMA) goes to its fp32 LDS tile; after
//     a second barrier each wave sums 8 rows over the four tiles, scales, converts and stores them
//     (LDS float atomics instead measured 5.8x slower for the whole kernel: ds_add_f32 serialises);
//   * D = rowsum(dO * O) comes from the slice's O image (every wave computes the slice's 32 rows).
// Registers: dK / dV 256 (accumulator registers), V 64, the slice's Q / dO row fragments 32, dQ partial 32.
// =============================================================================================
template <bool DROP, int S>
__global__ __launch_bounds__(256, 1) void attn_bwd_fused64(AttnBatch batch, int T, int H, float scale) {
  constexpr int NKS = 4, ND = 2, NT = 16;
  static_assert(S >= 2 && 4 * (S - 2) <= 16, "ring slots: S - 1 slices in flight");
  constexpr int KIMG = NT * IMG64;  // K of the sequence, 16 slice images
  constexpr int OFF_DO = IMG64, OFF_O = 2 * IMG64, OFF_L = 3 * IMG64, OFF_M = OFF_L + 256;
  constexpr int SLOT = OFF_M + (DROP ? NT * 128 : 0);
  // per-wave fp32 dQ partials of the slice [32 q][64 d]; the first 2 KiB of a wave's partial hold its
  // dS transpose image ([32 keys][32 q] bf16) while its tiles run
  constexpr int OFF_DQ = KIMG + S * SLOT;
  constexpr int OFF_DT = OFF_DQ + 4 * 8192;  // per-wave D of the slice's rows
  constexpr int EPW = 40;                    // epilogue transpose row stride (bf16)
  static_assert(4 * 2 * 32 * EPW * 2 <= S * SLOT, "epilogue transposes alias the ring");
  __shared__ __attribute__((aligned(1024))) char lds[OFF_DT + 4 * 128];
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nt = (T + 31) / 32;
  const int bh = blockIdx.x;
  const int b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int64_t rowbase = (int64_t)b * T;
  const float c2 = scale * kLog2e2;
  const bool ragged = (T & 31) != 0;
  const int kts[4] = {w, 7 - w, 8 + w, 15 - w};

  // V rows of the wave's key tiles (keys on lanes: the B operands of dP)
  bf16x8 vf[4][NKS];
  {
    u32x4 vr[4][NKS];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int tk = kts[t] * 32 + r;
      const bool ok = kts[t] < nt && tk < T;
      const bf16_t* vp = P.v[0] + head * P.kv_hstride + (rowbase + tk) * P.kv_ld;
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const u32x4 z = {0u, 0u, 0u, 0u};
        vr[t][s] = ok ? *reinterpret_cast<const u32x4*>(vp + 16 * s + 8 * h) : z;
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        asm volatile("" : "+v"(vr[t][s]));  // waited for here, ahead of the DMA prologue
        vf[t][s] = __builtin_bit_cast(bf16x8, vr[t][s]);
      }
  }
  f32x16 dk[4][ND], dv[4][ND];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      zero16(dk[t][dt]);
      zero16(dv[t][dt]);
      asm volatile("" : "+a"(dk[t][dt]));
      asm volatile("" : "+a"(dv[t][dt]));
    }

  const i32x4 rk = make_rsrc(P.k[0] + rowbase * P.kv_ld + head * P.kv_hstride, (int64_t)T * P.kv_ld * 2);
  const i32x4 rl = make_rsrc(P.lse[0] + (int64_t)bh * T, (int64_t)T * 4);
  const int64_t ntri = (int64_t)nt * (nt + 1) / 2;
  const i32x4 rm = make_rsrc(DROP ? P.dmask[0] + (int64_t)bh * ntri * 32 : P.dmask[0], ntri * 128);
  const int prow = lane >> 1;
  const int pcol = 8 * ((lane & 1) ^ ((prow >> 3) & 1));
  // K of the sequence (wave w: key tiles w, w+4, w+8, w+12), the oldest pieces of every wave
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int kt = (u >> 2) * 4 + w, cb = u & 3;
    if (kt < nt) {
      const int grow = kt * 32 + prow;
      const int voff = grow < T ? (grow * P.kv_ld + cb * 16 + pcol) * 2 : OOB;
      dma16(rk, __builtin_amdgcn_readfirstlane(lds_u32(lds + kt * IMG64 + cb * SUB)), voff);
    }
  }
  // slice pieces per wave: 3 of the 12 Q / dO / O sub-images, the LSE row (wave 0), the keep-bit
  // records of key tiles 8m .. 8m+7 (wave 1 + m)
  const int per = 3 + (w == 0 ? 1 : 0) + (DROP && (w == 1 || w == 2) ? 1 : 0);
  auto issue = [&](int slot, int qt) {
    char* sb = lds + KIMG + slot * SLOT;
    const int grow = qt * 32 + prow;
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int piece = 3 * w + u;
      const int op = piece >> 2, cb = piece & 3;
      // (the operand is wave-uniform: its descriptor is built here, a select of three descriptors
      // went through a scratch array)
      const int ld = op == 0 ? P.q_ld : op == 1 ? P.dout_ld : P.o_ld;
      const bf16_t* base = op == 0 ? P.q : op == 1 ? P.dout : P.o;
      const i32x4 rs = make_rsrc(base + rowbase * ld + head * 64, (int64_t)T * ld * 2);
      const int voff = grow < T ? (grow * ld + cb * 16 + pcol) * 2 : OOB;
      dma16(rs, __builtin_amdgcn_readfirstlane(lds_u32(sb + op * IMG64 + cb * SUB)), voff);
    }
    if (w == 0) {
      const int voff = (lane < 32 && qt * 32 + lane < T) ? (qt * 32 + lane) * 4 : OOB;
      dma4(rl, __builtin_amdgcn_readfirstlane(lds_u32(sb + OFF_L)), voff);
    }
    if (DROP && (w == 1 || w == 2)) {
      const int rec = 8 * (w - 1) + (lane >> 3);
      const int voff = rec <= qt ? (qt * (qt + 1) / 2 + rec) * 128 + (lane & 7) * 16 : OOB;
      dma16(rm, __builtin_amdgcn_readfirstlane(lds_u32(sb + OFF_M + (w - 1) * 1024)), voff);
    }
  };
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nt) issue(i, i);

  const int o_row = img_off(r, 0, h);
  const int g = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
  const int o_tr0 = img_off(4 * (g >> 1) + qq, g & 1, p >> 1) + 8 * (p & 1);
  const int o_tr1 = img_off(8 + 4 * (g >> 1) + qq, g & 1, p >> 1) + 8 * (p & 1);
  const int o_mk = key_dword(r) * 4;
  // dS transpose image ([key][q], 64-B rows, 8-B chunk c of row k stored at chunk c ^ ((k >> 1) & 7)):
  // lane (r, h) writes chunk 2 gg + h of row r (its dS of queries 8 gg + 4 h .. + 3); the A operand
  // of dQ (queries on lanes) comes back with the k order of the K^T fragments below (rows
  // 16 s + 4 h + qq and + 8, chunks 4 (g & 1) + p): both read kinds conflict-free
  char* dsi = lds + OFF_DQ + w * 8192;
  auto dsw = [&](int gg) { return r * 64 + (((2 * gg + h) ^ ((r >> 1) & 7)) << 3); };
  const int ra0 = 4 * (g >> 1) + qq, ra1 = ra0 + 8;
  const int o_da0 = ra0 * 64 + (((4 * (g & 1) + p) ^ ((ra0 >> 1) & 7)) << 3);
  const int o_da1 = ra1 * 64 + (((4 * (g & 1) + p) ^ ((ra1 >> 1) & 7)) << 3);
  float* dtab = reinterpret_cast<float*>(lds + OFF_DT) + w * 32;
  const float dsc = DROP ? P.drop_scale : 1.f;
  // element e of a tile accumulator is query row (e & 3) + 8 (e >> 2) + 4 h of the tile, key r:
  // bit e of m_diag keeps the diagonal tile's causal half (key <= query), bit e of m_rows the rows
  // of a ragged last query tile that lie before T (its keys past T then lie above the diagonal)
  uint32_t m_diag = 0, m_rows = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
    m_diag |= (uint32_t)(r <= row) << e;
    m_rows |= (uint32_t)((nt - 1) * 32 + row < T) << e;
  }

  // one key tile of this wave against the slice's query tile (mk: the elements kept by the mask)
  // (the transposed Q / dO fragments and the LSE / D rows are read per tile: held across the slice
  // they pushed the wave past 512 registers)
  auto tile = [&](const char* sb, int qt, int kt, f32x16 (&dkt)[ND], f32x16 (&dvt)[ND], const bf16x8 (&vft)[NKS],
                  const bf16x8 (&qr)[NKS], const bf16x8 (&dr)[NKS], f32x16 (&dqp)[ND], uint32_t mk) {
    const char* ki = lds + kt * IMG64;
    const uint32_t mw = DROP ? *reinterpret_cast<const uint32_t*>(sb + OFF_M + kt * 128 + o_mk) >> (4 * h) : 0u;
    bf16x8 kf[NKS];
#pragma unroll
    for (int s = 0; s < NKS; ++s) kf[s] = *reinterpret_cast<const bf16x8*>(ki + o_row + s * SUB);
    f32x16 sacc, dpacc;
    zero16(sacc);
    zero16(dpacc);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      sacc = mfma32(qr[s], kf[s], sacc);     // S[q][key]
      dpacc = mfma32(dr[s], vft[s], dpacc);  // dP[q][key]
    }
    uint32_t pp[8], dd[8];
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(sb + OFF_L + (8 * gg + 4 * h) * 4);
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(dtab + 8 * gg + 4 * h);
#pragma unroll
      for (int e4 = 0; e4 < 4; e4 += 2) {
        float pm[2], ds[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int e = 4 * gg + e4 + u;
          float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[e], c2, -l4[e4 + u]));
          pv = keep_f(pv, __builtin_amdgcn_sbfe((int)mk, e, 1));
          float dp = dpacc[e];
          if (DROP) {
            const int kbit = __builtin_amdgcn_sbfe((int)mw, 8 * gg + e4 + u, 1);
            pm[u] = keep_f(pv, kbit);
            dp = keep_f(dp, kbit);
          } else {
            pm[u] = pv;
          }
          ds[u] = pv * __builtin_fmaf(dp, dsc, -d4[e4 + u]);
        }
        pp[2 * gg + e4 / 2] = pack2bf(pm[0], pm[1]);
        dd[2 * gg + e4 / 2] = pack2bf(ds[0], ds[1]);
      }
    }
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) *reinterpret_cast<u32x2*>(dsi + dsw(gg)) = u32x2{dd[2 * gg], dd[2 * gg + 1]};
    bf16x8 qtr[2][ND], dot[2][ND];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        dot[s][dt] = join4(lds_tr16(sb + OFF_DO + o_tr0 + 512 * s + 2 * SUB * dt),
                           lds_tr16(sb + OFF_DO + o_tr1 + 512 * s + 2 * SUB * dt));
        qtr[s][dt] = join4(lds_tr16(sb + o_tr0 + 512 * s + 2 * SUB * dt), lds_tr16(sb + o_tr1 + 512 * s + 2 * SUB * dt));
      }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pf = __builtin_bit_cast(bf16x8, u32x4{pp[4 * s], pp[4 * s + 1], pp[4 * s + 2], pp[4 * s + 3]});
      const bf16x8 df = __builtin_bit_cast(bf16x8, u32x4{dd[4 * s], dd[4 * s + 1], dd[4 * s + 2], dd[4 * s + 3]});
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        dvt[dt] = mfma32(pf, dot[s][dt], dvt[dt]);
        dkt[dt] = mfma32(df, qtr[s][dt], dkt[dt]);
      }
    }
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {  // dK / dV live in the accumulator registers between tiles
      asm volatile("" : "+a"(dvt[dt]));
      asm volatile("" : "+a"(dkt[dt]));
    }
    // dQ_w[q][d] += dS[q][key] K[key][d]: dS (queries on lanes) from the transpose image, K^T
    // fragments (d on lanes) from the K image, both in the permuted k order of tr16 reads
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 da = join4(lds_tr16(dsi + o_da0 + 1024 * s), lds_tr16(dsi + o_da1 + 1024 * s));
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        const bf16x8 kt_ = join4(lds_tr16(ki + o_tr0 + 512 * s + 2 * SUB * dt), lds_tr16(ki + o_tr1 + 512 * s + 2 * SUB * dt));
        dqp[dt] = mfma32(da, kt_, dqp[dt]);
      }
    }
  };

  // dQ rows of slice qt: wave w sums rows 8w .. 8w+7 over the partials of the nw waves that had
  // tiles in the slice, scales, converts and stores them
  auto finish_dq = [&](int qt, int nw) {
    const int row = 8 * w + (lane >> 3), c0 = (lane & 7) * 8;
    f32x4 a = {0.f, 0.f, 0.f, 0.f}, c = {0.f, 0.f, 0.f, 0.f};
    for (int u = 0; u < nw; ++u) {
      const f32x4* src = reinterpret_cast<const f32x4*>(lds + OFF_DQ + u * 8192 + (row * 64 + c0) * 4);
      a += src[0];
      c += src[1];
    }
    const int t = qt * 32 + row;
    if (t < T)
      *reinterpret_cast<u32x4*>(P.dq + (rowbase + t) * P.dq_ld + head * 64 + c0) =
          u32x4{pack2bf(a[0] * scale, a[1] * scale), pack2bf(a[2] * scale, a[3] * scale),
                pack2bf(c[0] * scale, c[1] * scale), pack2bf(c[2] * scale, c[3] * scale)};
  };

  // the slice's tiles of this wave: D of the slice's rows, then each key tile at or below the query
  // tile; the wave's dQ partial leaves into its fp32 partial tile
  auto slice = [&](int i) {
    const char* sb = lds + KIMG + (i % S) * SLOT;
    bf16x8 qr[NKS], dr[NKS];
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      qr[s] = *reinterpret_cast<const bf16x8*>(sb + o_row + s * SUB);
      dr[s] = *reinterpret_cast<const bf16x8*>(sb + OFF_DO + o_row + s * SUB);
      const u32x4 ov = *reinterpret_cast<const u32x4*>(sb + OFF_O + o_row + s * SUB);
      const u32x4 dv4 = __builtin_bit_cast(u32x4, dr[s]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dsum = __builtin_fmaf(bf2f(ov[e] & 0xffff), bf2f(dv4[e] & 0xffff), dsum);
        dsum = __builtin_fmaf(bf2f(ov[e] >> 16), bf2f(dv4[e] >> 16), dsum);
      }
    }
    dsum = xh_sum(dsum);  // D of query row r (both halves)
    if (h == 0) dtab[r] = dsum;
    f32x16 dqp[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) zero16(dqp[dt]);
    const bool mask_all = ragged && i == nt - 1;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kt = kts[t];
      if (kt < nt && kt <= i) {
        // causal / ragged mask as a bit per accumulator element (one variant of the tile: two
        // made the register allocator shuffle the dK / dV accumulators between them)
        const uint32_t mk = (kt == i ? m_diag : 0xffffu) & (mask_all ? m_rows : 0xffffu);
        tile(sb, i, kt, dk[t], dv[t], vf[t], qr, dr, dqp, mk);
      }
    }
    float* part = reinterpret_cast<float*>(lds + OFF_DQ + w * 8192);
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) part[((e & 3) + 8 * (e >> 2) + 4 * h) * 64 + 32 * dt + r] = dqp[dt][e];
  };

#pragma unroll 1
  for (int i = 0; i < nt; ++i) {
    wait_vm(per * min(S - 2, nt - 1 - i));  // this wave's pieces of slice i landed (and K before them)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone's pieces landed; slice i - 1's reads are done
    if (i + S - 1 < nt) issue((i + S - 1) % S, i + S - 1);
    const int nw = min(i + 1, 4);  // waves with a key tile at or below this query tile (w <= i)
    if (w < nw) slice(i);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every partial of slice i is written
    finish_dq(i, nw);
  }


  // dK / dV of the wave's key tiles, transposed through its LDS slot (aliasing the ring) into
  // row-major 16-B pieces, as the dK/dV pass
  bf16_t* et = reinterpret_cast<bf16_t*>(lds + KIMG) + w * (2 * 32 * EPW);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int kt = kts[t];
    if (kt >= nt) continue;
    const int k0 = kt * 32;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kr = (e & 3) + 8 * (e >> 2) + 4 * h;
        et[kr * EPW + r] = f2bf(dk[t][dt][e] * scale);
        et[32 * EPW + kr * EPW + r] = f2bf(DROP ? dv[t][dt][e] * P.drop_scale : dv[t][dt][e]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = i * 16 + (lane >> 2), d0 = dt * 32 + (lane & 3) * 8;
        const u32x4 vk = *reinterpret_cast<const u32x4*>(et + row * EPW + (lane & 3) * 8);
        const u32x4 vv = *reinterpret_cast<const u32x4*>(et + 32 * EPW + row * EPW + (lane & 3) * 8);
        if (k0 + row < T) {
          const int64_t off = (rowbase + k0 + row) * P.dkv_ld + d0;
          *reinterpret_cast<u32x4*>(P.dk[0] + head * P.dkv_hstride + off) = vk;
          *reinterpret_cast<u32x4*>(P.dv[0] + head * P.dkv_hstride + off) = vv;
        }
      }
    }
  }
}

hipError_t mmt_attn_bwd_fused64(const AttnBatch& bt, int B, int T, int H, float scale, bool drop, hipStream_t s) {
  if (T > 512 || bt.p[0].nstreams != 1) return hipErrorInvalidValue;
  const dim3 grid(B * H, 1, bt.count);
  if (drop) hipLaunchKernelGGL((attn_bwd_fused64<true, 3>), grid, dim3(256), 0, s, bt, T, H, scale);
  else hipLaunchKernelGGL((attn_bwd_fused64<false, 3>), grid, dim3(256), 0, s, bt, T, H, scale);
  return hipGetLastError();
}

hipError_t mmt_attn_fwd_ring64(const AttnBatch& bt, int B, int T, int H, float scale, bool drop, hipStream_t s) {
  const int nt = (T + 31) / 32;
  const dim3 g2(((nt + 7) / 8) * B * H, 1, bt.count);
  if (drop) hipLaunchKernelGGL((attn_fwd_ring64x2<true, 4>), g2, dim3(256), 0, s, bt, T, H, scale);
  else hipLaunchKernelGGL((attn_fwd_ring64x2<false, 4>), g2, dim3(256), 0, s, bt, T, H, scale);
  return hipGetLastError();
}

// ring depth 4 (three slices in flight): depth 6 measured slower (target backward 294 -> 301 us, C4
// 2315 -> 2394 us: profiles/r3e_ring_slots_ab.txt); a one-query-tile-per-wave dQ ring equal at the
// target and slower at C3, 8 key tiles per dK/dV workgroup slower at C3 / C4
// (profiles/r3h_dkdv_waves_ab.txt), two plain dK/dV slices per barrier slower at C3 / C4
// (profiles/r3u_ring_ab.txt): those variants were removed in round 4.
hipError_t mmt_attn_bwd_dq_ring64(const AttnBatch& bt, int B, int T, int H, float scale, bool drop, hipStream_t s) {
  const int nt = (T + 31) / 32;
  const dim3 g2(((nt + 7) / 8) * B * H, 1, bt.count);  // two query tiles per wave (8 per workgroup)
  if (drop) hipLaunchKernelGGL((attn_bwd_dq_ring64x2<true, 4>), g2, dim3(256), 0, s, bt, T, H, scale);
  else hipLaunchKernelGGL((attn_bwd_dq_ring64x2<false, 4>), g2, dim3(256), 0, s, bt, T, H, scale);
  return hipGetLastError();
}

// variant bit 2: 3 waves per SIMD (<= 168 VGPRs; the default), else 2
hipError_t mmt_attn_bwd_dkdv_ring64(const AttnBatch& bt, int B, int T, int H, float scale, bool drop, int variant,
                                    hipStream_t s) {
  const int nt = (T + 31) / 32;
  const bool occ3 = (variant & 4) != 0;
  const dim3 grid(((nt + 3) / 4) * B * H * bt.p[0].nstreams, 1, bt.count);
  if (occ3) {
    if (drop) hipLaunchKernelGGL((attn_bwd_dkdv_ring64<true, 3, 4, 4>), grid, dim3(256), 0, s, bt, T, H, scale);
    else hipLaunchKernelGGL((attn_bwd_dkdv_ring64<false, 3, 4, 4>), grid, dim3(256), 0, s, bt, T, H, scale);
  } else {
    if (drop) hipLaunchKernelGGL((attn_bwd_dkdv_ring64<true, 2, 4, 4>), grid, dim3(256), 0, s, bt, T, H, scale);
    else hipLaunchKernelGGL((attn_bwd_dkdv_ring64<false, 2, 4, 4>), grid, dim3(256), 0, s, bt, T, H, scale);
  }
  return hipGetLastError();
}
