// Causal self-attention and multi-stream selective cross-attention for gfx950.
//
// Reference semantics (model.py:60-73, 136-159): per head, aff = q k^T * hs^-0.5, causal mask,
// softmax, @ v. Cross-attention runs one independent causal softmax per KV modality ("stream")
// and SUMS the per-stream outputs (no joint softmax).
//
// Structure: a 256-thread workgroup (4 waves) owns a 128-row block of one (batch, head); each
// wave owns one 32-row tile. The operand tiles the waves share (K/V in the forward and dQ pass,
// Q/dO/LSE/D in the dK/dV pass) are staged once per workgroup into double-buffered LDS, the next
// tile's global loads in flight while the current tile computes; one barrier per tile.
// All products are v_mfma_f32_32x32x16_bf16 with fp32 accumulation:
//   forward  S^T = K Q^T (keys on accumulator rows, queries on lanes) -> online softmax per lane;
//            O^T += V^T P^T with P^T straight from the accumulator registers as the B operand and
//            V^T by ds_read_b64_tr_b16 from the V tile.
//   dQ       S^T, dP^T recomputed per key tile; dQ^T += K^T dS^T (K^T by transposed LDS reads).
//   dK, dV   S = Q K^T, dP = dO V^T (queries on rows); dV += P^T dO, dK += dS^T Q with P and dS
//            taken from registers as the A operand and dO / Q by transposed LDS reads.
// Head sizes 8..64: padded to 16 on the reduction side and to 32 on the output side.
// Dropout (model.py:69, 151: applied to the normalised probabilities): a counter-hash mask
// regenerated identically in all three kernels; O = (P.Z) V with Z = mask / (1 - p), so
// dV = (P.Z)^T dO, dS = P.(Z.dP - D) with D = rowsum(dO.O) unchanged.
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

// accumulator registers 8s..8s+7 -> bf16 operand fragment
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)a[8 * s + j];
  return r;
}

__device__ __forceinline__ void zero16(f32x16& a) {
#pragma unroll
  for (int e = 0; e < 16; ++e) a[e] = 0.f;
}

}  // namespace

// =============================================================================================
// forward: grid (ceil(T/128), B*H, G); wave w owns query tile 4*blockIdx.x + w
// =============================================================================================
template <int HS>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnBatch batch, int T, int H, float scale) {
  using G = Geo<HS>;
  const AttnProblem& P = batch.p[blockIdx.z];
  const int bh = blockIdx.y, b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int nt = (T + 31) / 32;
  const int qt = blockIdx.x * 4 + w;
  const int last_kt = min(blockIdx.x * 4 + 3, nt - 1);
  const int q0 = qt * 32, tq = q0 + r;
  const int64_t rowbase = (int64_t)b * T;
  __shared__ __attribute__((aligned(16))) bf16_t ks[2][32 * G::RW];
  __shared__ __attribute__((aligned(16))) bf16_t vs[2][32 * G::TW];

  bf16x8 qf[G::NKS];
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    const int d0 = 16 * s + 8 * h;
    qf[s] = ld8(P.q + (rowbase + tq) * P.q_ld + head * HS + d0, tq < T && d0 < HS);
  }
  // zero the pad columns of both buffers once (never written by staging)
  for (int q = tid; q < 2 * 32 * G::RW; q += 256) { const int c = q % G::RW; if (c >= HS) (&ks[0][0])[q] = 0; }
  for (int q = tid; q < 2 * 32 * G::TW; q += 256) { const int c = q % G::TW; if (c >= HS) (&vs[0][0])[q] = 0; }

  f32x16 otot[G::ND];
#pragma unroll
  for (int dt = 0; dt < G::ND; ++dt) zero16(otot[dt]);

  const uint32_t drow = (uint32_t)(bh * T + tq);  // dropout hash row of this lane's query
  for (int j = 0; j < P.nstreams; ++j) {
    const bf16_t* kp = P.k[j] + head * P.kv_hstride;
    const bf16_t* vp = P.v[j] + head * P.kv_hstride;
    const uint32_t dkey = mmt_hash(P.drop_key, (uint32_t)j, MMT_STREAM_SALT);
    float m = -INFINITY, l = 0.f;
    f32x16 oacc[G::ND];
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt) zero16(oacc[dt]);
    // staging: chunk c < 32*CH -> K, else V
    u32x4 stg[2];
    auto issue = [&](int kt) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = tid + 256 * u;
        if (c < 64 * G::CH) {
          const bool isv = c >= 32 * G::CH;
          const int cc = isv ? c - 32 * G::CH : c;
          stg[u] = tile_chunk(isv ? vp : kp, rowbase, kt * 32, cc / G::CH, (cc % G::CH) * 8, T, P.kv_ld);
        }
      }
    };
    auto commit = [&](int buf) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = tid + 256 * u;
        if (c < 64 * G::CH) {
          const bool isv = c >= 32 * G::CH;
          const int cc = isv ? c - 32 * G::CH : c;
          const int row = cc / G::CH, col = (cc % G::CH) * 8;
          if (isv) *reinterpret_cast<u32x4*>(&vs[buf][row * G::TW + col]) = stg[u];
          else *reinterpret_cast<u32x4*>(&ks[buf][row * G::RW + col]) = stg[u];
        }
      }
    };
    __syncthreads();  // previous stream's readers are done with both buffers
    issue(0);
    commit(0);
    __syncthreads();
    for (int kt = 0; kt <= last_kt; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 <= last_kt;
      if (more) issue(kt + 1);
      if (kt <= qt) {
        const int k0 = kt * 32;
        f32x16 sacc;
        zero16(sacc);
#pragma unroll
        for (int s = 0; s < G::NKS; ++s) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(&ks[cur][r * G::RW + 16 * s + 8 * h]);
          sacc = mfma32(kf, qf[s], sacc);
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int key = k0 + (e & 3) + 8 * (e >> 2) + 4 * h;
          const float sv = (key <= tq && key < T) ? sacc[e] * scale : -INFINITY;
          sacc[e] = sv;
          tmax = fmaxf(tmax, sv);
        }
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
        const float mnew = fmaxf(m, tmax);
        const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
        const float alpha = __expf(m - msafe);
        float rs = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float pv = __expf(sacc[e] - msafe);
          sacc[e] = pv;
          rs += pv;
        }
        rs += __shfl_xor(rs, 32, 64);
        l = l * alpha + rs;
        m = mnew;
        if (P.drop_thr) {  // dropout on the probabilities (the normaliser l keeps every term)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const uint32_t key = (uint32_t)(k0 + (e & 3) + 8 * (e >> 2) + 4 * h);
            sacc[e] = (mmt_hash(dkey, drow, key) >= P.drop_thr) ? sacc[e] * P.drop_scale : 0.f;
          }
        }
#pragma unroll
        for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
          for (int e = 0; e < 16; ++e) oacc[dt][e] *= alpha;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pf = acc_frag(sacc, s);
#pragma unroll
          for (int dt = 0; dt < G::ND; ++dt) oacc[dt] = mfma32(tr_frag(vs[cur], G::TW, dt, s, lane), pf, oacc[dt]);
        }
      }
      if (more) commit(cur ^ 1);
      __syncthreads();
    }
    const float inv = (l > 0.f) ? 1.f / l : 0.f;
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        oacc[dt][e] *= inv;
        otot[dt][e] += oacc[dt][e];
      }
    if (tq < T) {
      if (h == 0) P.lse[j][(int64_t)bh * T + tq] = m + __logf(l);
      if (P.nstreams > 1 && P.oj[j]) {
#pragma unroll
        for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int d0 = dt * 32 + 8 * g + 4 * h;
            if (d0 < HS)
              *reinterpret_cast<u32x2*>(P.oj[j] + (rowbase + tq) * P.o_ld + head * HS + d0) =
                  u32x2{pack2bf(oacc[dt][4 * g], oacc[dt][4 * g + 1]), pack2bf(oacc[dt][4 * g + 2], oacc[dt][4 * g + 3])};
          }
      }
    }
  }
  if (tq < T) {
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * h;
        if (d0 < HS)
          *reinterpret_cast<u32x2*>(P.o + (rowbase + tq) * P.o_ld + head * HS + d0) =
              u32x2{pack2bf(otot[dt][4 * g], otot[dt][4 * g + 1]), pack2bf(otot[dt][4 * g + 2], otot[dt][4 * g + 3])};
      }
  }
}

// =============================================================================================
// backward dQ (also writes D_j = rowsum(dO * O_j) for the dK/dV pass); grid as forward
// =============================================================================================
template <int HS>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnBatch batch, int T, int H, float scale) {
  using G = Geo<HS>;
  const AttnProblem& P = batch.p[blockIdx.z];
  const int bh = blockIdx.y, b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int nt = (T + 31) / 32;
  const int qt = blockIdx.x * 4 + w;
  const int last_kt = min(blockIdx.x * 4 + 3, nt - 1);
  const int q0 = qt * 32, tq = q0 + r;
  const bool qok = tq < T;
  const int64_t rowbase = (int64_t)b * T;
  __shared__ __attribute__((aligned(16))) bf16_t ks[2][32 * G::RW];  // K tile: row reads + tr reads
  __shared__ __attribute__((aligned(16))) bf16_t vs[2][32 * G::RW];  // V tile: row reads

  bf16x8 qf[G::NKS], dof[G::NKS];
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    const int d0 = 16 * s + 8 * h;
    const bool ok = qok && d0 < HS;
    qf[s] = ld8(P.q + (rowbase + tq) * P.q_ld + head * HS + d0, ok);
    dof[s] = ld8(P.dout + (rowbase + tq) * P.dout_ld + head * HS + d0, ok);
  }
  for (int q = tid; q < 2 * 32 * G::RW; q += 256) {
    const int c = q % G::RW;
    if (c >= HS) { (&ks[0][0])[q] = 0; (&vs[0][0])[q] = 0; }
  }
  f32x16 dq[G::ND];
#pragma unroll
  for (int dt = 0; dt < G::ND; ++dt) zero16(dq[dt]);

  for (int j = 0; j < P.nstreams; ++j) {
    const bf16_t* oj = (P.nstreams > 1) ? P.oj[j] : P.o;
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < G::NKS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bf16x8 ov = ld8(oj + (rowbase + tq) * P.o_ld + head * HS + d0, qok && d0 < HS);
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum += (float)ov[e] * (float)dof[s][e];
    }
    dsum += __shfl_xor(dsum, 32, 64);
    if (qok && h == 0) P.dvec[j][(int64_t)bh * T + tq] = dsum;
    const float lse = qok ? P.lse[j][(int64_t)bh * T + tq] : 0.f;
    const uint32_t dkey = mmt_hash(P.drop_key, (uint32_t)j, MMT_STREAM_SALT);
    const uint32_t drow = (uint32_t)(bh * T + tq);
    const bf16_t* kp = P.k[j] + head * P.kv_hstride;
    const bf16_t* vp = P.v[j] + head * P.kv_hstride;
    u32x4 stg[2];
    auto issue = [&](int kt) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = tid + 256 * u;
        if (c < 64 * G::CH) {
          const bool isv = c >= 32 * G::CH;
          const int cc = isv ? c - 32 * G::CH : c;
          stg[u] = tile_chunk(isv ? vp : kp, rowbase, kt * 32, cc / G::CH, (cc % G::CH) * 8, T, P.kv_ld);
        }
      }
    };
    auto commit = [&](int buf) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = tid + 256 * u;
        if (c < 64 * G::CH) {
          const bool isv = c >= 32 * G::CH;
          const int cc = isv ? c - 32 * G::CH : c;
          const int row = cc / G::CH, col = (cc % G::CH) * 8;
          *reinterpret_cast<u32x4*>(isv ? &vs[buf][row * G::RW + col] : &ks[buf][row * G::RW + col]) = stg[u];
        }
      }
    };
    __syncthreads();
    issue(0);
    commit(0);
    __syncthreads();
    for (int kt = 0; kt <= last_kt; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 <= last_kt;
      if (more) issue(kt + 1);
      if (kt <= qt) {
        const int k0 = kt * 32;
        f32x16 sacc, dpacc;
        zero16(sacc);
        zero16(dpacc);
#pragma unroll
        for (int s = 0; s < G::NKS; ++s) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(&ks[cur][r * G::RW + 16 * s + 8 * h]);
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(&vs[cur][r * G::RW + 16 * s + 8 * h]);
          sacc = mfma32(kf, qf[s], sacc);
          dpacc = mfma32(vf, dof[s], dpacc);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int key = k0 + (e & 3) + 8 * (e >> 2) + 4 * h;
          const bool ok = qok && key <= tq && key < T;
          const float pv = ok ? __expf(sacc[e] * scale - lse) : 0.f;
          float dp = dpacc[e];
          if (P.drop_thr) dp = (mmt_hash(dkey, drow, (uint32_t)key) >= P.drop_thr) ? dp * P.drop_scale : 0.f;
          sacc[e] = pv * (dp - dsum);  // dS^T
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 df = acc_frag(sacc, s);
#pragma unroll
          for (int dt = 0; dt < G::ND; ++dt) dq[dt] = mfma32(tr_frag(ks[cur], G::RW, dt, s, lane), df, dq[dt]);
        }
      }
      if (more) commit(cur ^ 1);
      __syncthreads();
    }
  }
  if (qok) {
#pragma unroll
    for (int dt = 0; dt < G::ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = dt * 32 + 8 * g + 4 * h;
        if (d0 < HS)
          *reinterpret_cast<u32x2*>(P.dq + (rowbase + tq) * P.dq_ld + head * HS + d0) =
              u32x2{pack2bf(dq[dt][4 * g] * scale, dq[dt][4 * g + 1] * scale),
                    pack2bf(dq[dt][4 * g + 2] * scale, dq[dt][4 * g + 3] * scale)};
      }
  }
}

// =============================================================================================
// backward dK, dV: grid (ceil(T/128), B*H*nstreams, G); wave w owns key tile 4*blockIdx.x + w
// =============================================================================================
template <int HS>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnBatch batch, int T, int H, float scale) {
  using G = Geo<HS>;
  const AttnProblem& P = batch.p[blockIdx.z];
  const int nbh = gridDim.y / P.nstreams;
  if ((int)blockIdx.y >= nbh * P.nstreams) return;
  const int j = blockIdx.y / nbh;
  const int bh = blockIdx.y % nbh;
  const int b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int nt = (T + 31) / 32;
  const int kt = blockIdx.x * 4 + w;
  const int first_qt = blockIdx.x * 4;
  const int k0 = kt * 32, tk = k0 + r;
  const bool kok = tk < T;
  const int64_t rowbase = (int64_t)b * T;
  __shared__ __attribute__((aligned(16))) bf16_t qs[2][32 * G::RW];   // Q tile: row + tr reads
  __shared__ __attribute__((aligned(16))) bf16_t dos[2][32 * G::RW];  // dO tile: row + tr reads
  __shared__ __attribute__((aligned(16))) float lsd[2][2][32];        // LSE, D of the tile's rows

  const bf16_t* kp = P.k[j] + head * P.kv_hstride;
  const bf16_t* vp = P.v[j] + head * P.kv_hstride;
  bf16x8 kf[G::NKS], vf[G::NKS];
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    const int d0 = 16 * s + 8 * h;
    const bool ok = kok && d0 < HS;
    kf[s] = ld8(kp + (rowbase + tk) * P.kv_ld + d0, ok);
    vf[s] = ld8(vp + (rowbase + tk) * P.kv_ld + d0, ok);
  }
  for (int q = tid; q < 2 * 32 * G::RW; q += 256) {
    const int c = q % G::RW;
    if (c >= HS) { (&qs[0][0])[q] = 0; (&dos[0][0])[q] = 0; }
  }
  f32x16 dk[G::ND], dv[G::ND];
#pragma unroll
  for (int dt = 0; dt < G::ND; ++dt) { zero16(dk[dt]); zero16(dv[dt]); }

  const uint32_t dkey = mmt_hash(P.drop_key, (uint32_t)j, MMT_STREAM_SALT);
  const float* lsep = P.lse[j] + (int64_t)bh * T;
  const float* dvp = P.dvec[j] + (int64_t)bh * T;
  const bf16_t* qp = P.q + head * HS;
  const bf16_t* dop = P.dout + head * HS;
  u32x4 stg[2];
  float sl = 0.f;
  auto issue = [&](int qt) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u;
      if (c < 64 * G::CH) {
        const bool isd = c >= 32 * G::CH;
        const int cc = isd ? c - 32 * G::CH : c;
        stg[u] = isd ? tile_chunk(dop, rowbase, qt * 32, cc / G::CH, (cc % G::CH) * 8, T, P.dout_ld)
                     : tile_chunk(qp, rowbase, qt * 32, cc / G::CH, (cc % G::CH) * 8, T, P.q_ld);
      }
    }
    if (tid < 64) {
      const int t = qt * 32 + (tid & 31);
      sl = t < T ? ((tid < 32) ? lsep[t] : dvp[t]) : 0.f;
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u;
      if (c < 64 * G::CH) {
        const bool isd = c >= 32 * G::CH;
        const int cc = isd ? c - 32 * G::CH : c;
        const int row = cc / G::CH, col = (cc % G::CH) * 8;
        *reinterpret_cast<u32x4*>(isd ? &dos[buf][row * G::RW + col] : &qs[buf][row * G::RW + col]) = stg[u];
      }
    }
    if (tid < 64) lsd[buf][tid >> 5][tid & 31] = sl;
  };
  issue(first_qt);
  commit(0);
  __syncthreads();
  for (int qt = first_qt; qt < nt; ++qt) {
    const int cur = (qt - first_qt) & 1;
    const bool more = qt + 1 < nt;
    if (more) issue(qt + 1);
    if (qt >= kt) {
      const int q0 = qt * 32;
      f32x16 sacc, dpacc;
      zero16(sacc);
      zero16(dpacc);
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) {
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(&qs[cur][r * G::RW + 16 * s + 8 * h]);
        const bf16x8 da = *reinterpret_cast<const bf16x8*>(&dos[cur][r * G::RW + 16 * s + 8 * h]);
        sacc = mfma32(qa, kf[s], sacc);    // S[q][key]
        dpacc = mfma32(da, vf[s], dpacc);  // dP[q][key]
      }
      f32x16 pm;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(&lsd[cur][0][8 * g + 4 * h]);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(&lsd[cur][1][8 * g + 4 * h]);
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          const int e = 4 * g + e4;
          const int tq = q0 + 8 * g + 4 * h + e4;
          const bool ok = kok && tq < T && tk <= tq;
          const float pv = ok ? __expf(sacc[e] * scale - l4[e4]) : 0.f;
          if (P.drop_thr) {
            const bool keep = mmt_hash(dkey, (uint32_t)(bh * T + tq), (uint32_t)tk) >= P.drop_thr;
            pm[e] = keep ? pv * P.drop_scale : 0.f;
            sacc[e] = pv * ((keep ? dpacc[e] * P.drop_scale : 0.f) - d4[e4]);
          } else {
            pm[e] = pv;
            sacc[e] = pv * (dpacc[e] - d4[e4]);  // dS[q][key]
          }
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_frag(pm, s);
        const bf16x8 df = acc_frag(sacc, s);
#pragma unroll
        for (int dt = 0; dt < G::ND; ++dt) {
          dv[dt] = mfma32(pf, tr_frag(dos[cur], G::RW, dt, s, lane), dv[dt]);
          dk[dt] = mfma32(df, tr_frag(qs[cur], G::RW, dt, s, lane), dk[dt]);
        }
      }
    }
    if (more) commit(cur ^ 1);
    __syncthreads();
  }
  // dK/dV tiles: rows = key ((e&3)+8(e>>2)+4h), cols = d (lane)
  bf16_t* dkp = P.dk[j] + head * P.dkv_hstride;
  bf16_t* dvo = P.dv[j] + head * P.dkv_hstride;
#pragma unroll
  for (int dt = 0; dt < G::ND; ++dt) {
    const int d = dt * 32 + r;
    if (d >= HS) continue;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int key = k0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (key < T) {
        dkp[(rowbase + key) * P.dkv_ld + d] = f2bf(dk[dt][e] * scale);
        dvo[(rowbase + key) * P.dkv_ld + d] = f2bf(dv[dt][e]);
      }
    }
  }
}

template <int HS>
static void attn_launch(const AttnBatch& bt, int B, int T, int H, float scale, bool bwd, hipStream_t s) {
  const int nb = (T + 127) / 128;
  if (!bwd) {
    hipLaunchKernelGGL(attn_fwd_kernel<HS>, dim3(nb, B * H, bt.count), dim3(256), 0, s, bt, T, H, scale);
  } else {
    const int ns = bt.p[0].nstreams;
    hipLaunchKernelGGL(attn_bwd_dq_kernel<HS>, dim3(nb, B * H, bt.count), dim3(256), 0, s, bt, T, H, scale);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<HS>, dim3(nb, B * H * ns, bt.count), dim3(256), 0, s, bt, T, H, scale);
  }
}

static hipError_t attn_dispatch(const AttnBatch& b, int B, int T, int H, int hs, float scale, bool bwd,
                                hipStream_t s) {
  if (b.count == 0 || B == 0 || T == 0) return hipSuccess;
  for (int g = 0; g < b.count; ++g)
    if (b.p[g].nstreams < 1 || b.p[g].nstreams > MMT_MAX_STREAMS) return hipErrorInvalidValue;
  if (bwd) {  // all problems in a bwd batch must share nstreams (grid.y = B*H*nstreams)
    for (int g = 1; g < b.count; ++g)
      if (b.p[g].nstreams != b.p[0].nstreams) return hipErrorInvalidValue;
  }
  switch (hs) {
    case 8: attn_launch<8>(b, B, T, H, scale, bwd, s); break;
    case 16: attn_launch<16>(b, B, T, H, scale, bwd, s); break;
    case 24: attn_launch<24>(b, B, T, H, scale, bwd, s); break;
    case 32: attn_launch<32>(b, B, T, H, scale, bwd, s); break;
    case 48: attn_launch<48>(b, B, T, H, scale, bwd, s); break;
    case 64: attn_launch<64>(b, B, T, H, scale, bwd, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t mmt_launch_attn_fwd(const AttnBatch& b, int B, int T, int H, int hs, float scale, hipStream_t s) {
  return attn_dispatch(b, B, T, H, hs, scale, false, s);
}
hipError_t mmt_launch_attn_bwd(const AttnBatch& b, int B, int T, int H, int hs, float scale, hipStream_t s) {
  return attn_dispatch(b, B, T, H, hs, scale, true, s);
}
