// Causal self-attention and multi-stream selective cross-attention for gfx950.
//
// Reference semantics (model.py:60-73, 136-159): per head, aff = q k^T * hs^-0.5, causal mask,
// softmax, @ v. Cross-attention runs one independent causal softmax per KV modality ("stream")
// and SUMS the per-stream outputs (no joint softmax).
//
// Structure: one wave (64-thread workgroup) owns one 32-row tile of one (batch, head). All
// products are v_mfma_f32_32x32x16_bf16 with fp32 accumulation:
//   forward  S^T = K Q^T (keys on accumulator rows, queries on lanes) -> online softmax per lane
//            O^T += V^T P^T with P^T taken straight from the accumulator registers as the
//            B operand (no LDS round trip) and V^T read by ds_read_b64_tr_b16 from a V tile.
//   dQ       S^T, dP^T recomputed per key tile; dQ^T += K^T dS^T (K^T via transposed LDS reads)
//   dK, dV   S = Q K^T, dP = dO V^T (queries on rows); dV += P^T dO, dK += dS^T Q with P / dS
//            as the A operand straight from registers, dO / Q by transposed LDS reads.
// Head sizes 8..64 (padded to 16 on the reduction side and 32 on the output side).
#include "mmt_common.h"
#include "mmt_kernels.h"

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (__bf16)0.0f;
  return z;
}

__device__ __forceinline__ bf16x8 ld8(const bf16_t* p, bool ok) {
  if (!ok) return zero8();
  return *reinterpret_cast<const bf16x8*>(p);
}

// stage a [32 rows][W] tile (rows r0.., columns 0..HS-1 of the head, zero padded) into LDS
template <int HS, int W>
__device__ __forceinline__ void stage_tile(bf16_t* lds, const bf16_t* base, int64_t rowbase, int r0, int T, int ld,
                                          int lane) {
  constexpr int CPR = W / 8;  // 16-byte chunks per row
#pragma unroll
  for (int c = lane; c < 32 * CPR; c += 64) {
    const int row = c / CPR, col = (c % CPR) * 8;
    const bool ok = (r0 + row < T) && (col < HS);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (ok) v = *reinterpret_cast<const u32x4*>(base + (rowbase + r0 + row) * ld + col);
    *reinterpret_cast<u32x4*>(lds + row * W + col) = v;
  }
}

// A-operand fragment of X^T where X is a [32 rows][W] LDS tile: lane gets column
// d = dt*32 + (lane&31) and rows {16s+4h+0..3, 16s+8+4h+0..3} (the accumulator-as-operand k order)
template <int W>
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* lds, int dt, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int col = dt * 32 + 16 * (g & 1) + 4 * p;
  const int kb = 16 * s + 4 * (g >> 1) + q;
  const s16x4 lo = lds_tr16(lds + kb * W + col);
  const s16x4 hi = lds_tr16(lds + (kb + 8) * W + col);
  return join4(lo, hi);
}

// accumulator registers 8s..8s+7 -> bf16 operand fragment
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)a[8 * s + j];
  return r;
}

// =============================================================================================
// forward
// =============================================================================================
template <int HS>
__global__ __launch_bounds__(64) void attn_fwd_kernel(AttnBatch batch, int T, int H, float scale) {
  constexpr int NKS = (HS + 15) / 16;
  constexpr int ND = (HS + 31) / 32;
  constexpr int W = ND * 32;
  const AttnProblem& P = batch.p[blockIdx.z];
  const int qt = blockIdx.x;
  const int bh = blockIdx.y;
  const int b = bh / H, head = bh % H;
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int q0 = qt * 32;
  const int64_t rowbase = (int64_t)b * T;
  const int tq = q0 + r;
  __shared__ __attribute__((aligned(16))) bf16_t vt[32 * W];

  bf16x8 qf[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int d0 = 16 * s + 8 * h;
    qf[s] = ld8(P.q + (rowbase + tq) * P.q_ld + head * HS + d0, tq < T && d0 < HS);
  }
  f32x16 otot[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) otot[dt][e] = 0.f;

  for (int j = 0; j < P.nstreams; ++j) {
    const bf16_t* kp = P.k[j] + head * P.kv_hstride;
    const bf16_t* vp = P.v[j] + head * P.kv_hstride;
    float m = -INFINITY, l = 0.f;
    f32x16 oacc[ND];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) oacc[dt][e] = 0.f;

    for (int kt = 0; kt <= qt; ++kt) {
      const int k0 = kt * 32;
      f32x16 sacc;
#pragma unroll
      for (int e = 0; e < 16; ++e) sacc[e] = 0.f;
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const int d0 = 16 * s + 8 * h;
        const bf16x8 kf = ld8(kp + (rowbase + k0 + r) * P.kv_ld + d0, k0 + r < T && d0 < HS);
        sacc = mfma32(kf, qf[s], sacc);
      }
      __syncthreads();
      stage_tile<HS, W>(vt, vp, rowbase, k0, T, P.kv_ld, lane);
      // online softmax over keys (rows of S^T) for query tq (lane column)
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
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) oacc[dt][e] *= alpha;
      __syncthreads();
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_frag(sacc, s);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) oacc[dt] = mfma32(tr_frag<W>(vt, dt, s, lane), pf, oacc[dt]);
      }
    }
    const float inv = (l > 0.f) ? 1.f / l : 0.f;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        oacc[dt][e] *= inv;
        otot[dt][e] += oacc[dt][e];
      }
    if (tq < T) {
      if (h == 0) P.lse[j][(int64_t)bh * T + tq] = m + __logf(l);
      if (P.nstreams > 1 && P.oj[j]) {
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
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
    for (int dt = 0; dt < ND; ++dt)
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
// backward: dQ (also writes D_j = rowsum(dO * O_j) for the dK/dV kernel)
// =============================================================================================
template <int HS>
__global__ __launch_bounds__(64) void attn_bwd_dq_kernel(AttnBatch batch, int T, int H, float scale) {
  constexpr int NKS = (HS + 15) / 16;
  constexpr int ND = (HS + 31) / 32;
  constexpr int W = ND * 32;
  const AttnProblem& P = batch.p[blockIdx.z];
  const int qt = blockIdx.x;
  const int bh = blockIdx.y;
  const int b = bh / H, head = bh % H;
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int q0 = qt * 32;
  const int64_t rowbase = (int64_t)b * T;
  const int tq = q0 + r;
  const bool qok = tq < T;
  __shared__ __attribute__((aligned(16))) bf16_t kt_lds[32 * W];

  bf16x8 qf[NKS], dof[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int d0 = 16 * s + 8 * h;
    const bool ok = qok && d0 < HS;
    qf[s] = ld8(P.q + (rowbase + tq) * P.q_ld + head * HS + d0, ok);
    dof[s] = ld8(P.dout + (rowbase + tq) * P.dout_ld + head * HS + d0, ok);
  }
  f32x16 dq[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) dq[dt][e] = 0.f;

  for (int j = 0; j < P.nstreams; ++j) {
    // D_j for this lane's query
    const bf16_t* oj = (P.nstreams > 1) ? P.oj[j] : P.o;
    float dsum = 0.f;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bf16x8 ov = ld8(oj + (rowbase + tq) * P.o_ld + head * HS + d0, qok && d0 < HS);
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum += (float)ov[e] * (float)dof[s][e];
    }
    dsum += __shfl_xor(dsum, 32, 64);
    if (qok && h == 0) P.dvec[j][(int64_t)bh * T + tq] = dsum;
    const float lse = qok ? P.lse[j][(int64_t)bh * T + tq] : 0.f;
    const bf16_t* kp = P.k[j] + head * P.kv_hstride;
    const bf16_t* vp = P.v[j] + head * P.kv_hstride;
    for (int kt = 0; kt <= qt; ++kt) {
      const int k0 = kt * 32;
      f32x16 sacc, dpacc;
#pragma unroll
      for (int e = 0; e < 16; ++e) { sacc[e] = 0.f; dpacc[e] = 0.f; }
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        const int d0 = 16 * s + 8 * h;
        const bool ok = k0 + r < T && d0 < HS;
        const bf16x8 kf = ld8(kp + (rowbase + k0 + r) * P.kv_ld + d0, ok);
        const bf16x8 vf = ld8(vp + (rowbase + k0 + r) * P.kv_ld + d0, ok);
        sacc = mfma32(kf, qf[s], sacc);
        dpacc = mfma32(vf, dof[s], dpacc);
      }
      __syncthreads();
      stage_tile<HS, W>(kt_lds, kp, rowbase, k0, T, P.kv_ld, lane);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int key = k0 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const bool ok = qok && key <= tq && key < T;
        const float pv = ok ? __expf(sacc[e] * scale - lse) : 0.f;
        sacc[e] = pv * (dpacc[e] - dsum);  // dS^T
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 df = acc_frag(sacc, s);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) dq[dt] = mfma32(tr_frag<W>(kt_lds, dt, s, lane), df, dq[dt]);
      }
    }
  }
  if (qok) {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
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
// backward: dK, dV for one key tile of one (stream, batch, head)
// =============================================================================================
template <int HS>
__global__ __launch_bounds__(64) void attn_bwd_dkdv_kernel(AttnBatch batch, int T, int H, float scale) {
  constexpr int NKS = (HS + 15) / 16;
  constexpr int ND = (HS + 31) / 32;
  constexpr int W = ND * 32;
  const AttnProblem& P = batch.p[blockIdx.z];
  const int kt = blockIdx.x;
  const int nbh = gridDim.y / P.nstreams;
  if ((int)blockIdx.y >= nbh * P.nstreams) return;
  const int j = blockIdx.y / nbh;
  const int bh = blockIdx.y % nbh;
  const int b = bh / H, head = bh % H;
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int k0 = kt * 32;
  const int64_t rowbase = (int64_t)b * T;
  const int tk = k0 + r;
  const bool kok = tk < T;
  const int nqt = (T + 31) / 32;
  __shared__ __attribute__((aligned(16))) bf16_t q_lds[32 * W];
  __shared__ __attribute__((aligned(16))) bf16_t do_lds[32 * W];

  const bf16_t* kp = P.k[j] + head * P.kv_hstride;
  const bf16_t* vp = P.v[j] + head * P.kv_hstride;
  bf16x8 kf[NKS], vf[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int d0 = 16 * s + 8 * h;
    const bool ok = kok && d0 < HS;
    kf[s] = ld8(kp + (rowbase + tk) * P.kv_ld + d0, ok);
    vf[s] = ld8(vp + (rowbase + tk) * P.kv_ld + d0, ok);
  }
  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int e = 0; e < 16; ++e) { dk[dt][e] = 0.f; dv[dt][e] = 0.f; }

  const float* lsep = P.lse[j] + (int64_t)bh * T;
  const float* dvp = P.dvec[j] + (int64_t)bh * T;
  for (int qt = kt; qt < nqt; ++qt) {
    const int q0 = qt * 32;
    f32x16 sacc, dpacc;
#pragma unroll
    for (int e = 0; e < 16; ++e) { sacc[e] = 0.f; dpacc[e] = 0.f; }
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bool ok = q0 + r < T && d0 < HS;
      const bf16x8 qa = ld8(P.q + (rowbase + q0 + r) * P.q_ld + head * HS + d0, ok);
      const bf16x8 da = ld8(P.dout + (rowbase + q0 + r) * P.dout_ld + head * HS + d0, ok);
      sacc = mfma32(qa, kf[s], sacc);    // S[q][key]
      dpacc = mfma32(da, vf[s], dpacc);  // dP[q][key]
    }
    __syncthreads();
    stage_tile<HS, W>(q_lds, P.q + head * HS, rowbase, q0, T, P.q_ld, lane);
    stage_tile<HS, W>(do_lds, P.dout + head * HS, rowbase, q0, T, P.dout_ld, lane);
    f32x16 pm;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int tq = q0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      const bool ok = kok && tq < T && tk <= tq;
      const float lse = tq < T ? lsep[tq] : 0.f;
      const float dd = tq < T ? dvp[tq] : 0.f;
      const float pv = ok ? __expf(sacc[e] * scale - lse) : 0.f;
      pm[e] = pv;
      sacc[e] = pv * (dpacc[e] - dd);  // dS[q][key]
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pf = acc_frag(pm, s);
      const bf16x8 df = acc_frag(sacc, s);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        dv[dt] = mfma32(pf, tr_frag<W>(do_lds, dt, s, lane), dv[dt]);
        dk[dt] = mfma32(df, tr_frag<W>(q_lds, dt, s, lane), dk[dt]);
      }
    }
  }
  // dK/dV tiles: rows = key ((e&3)+8(e>>2)+4h), cols = d (lane)
  bf16_t* dkp = P.dk[j] + head * P.dkv_hstride;
  bf16_t* dvo = P.dv[j] + head * P.dkv_hstride;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
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
  const int nt = (T + 31) / 32;
  if (!bwd) {
    hipLaunchKernelGGL(attn_fwd_kernel<HS>, dim3(nt, B * H, bt.count), dim3(64), 0, s, bt, T, H, scale);
  } else {
    int maxs = 1;
    for (int g = 0; g < bt.count; ++g) maxs = bt.p[g].nstreams > maxs ? bt.p[g].nstreams : maxs;
    hipLaunchKernelGGL(attn_bwd_dq_kernel<HS>, dim3(nt, B * H, bt.count), dim3(64), 0, s, bt, T, H, scale);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<HS>, dim3(nt, B * H * maxs, bt.count), dim3(64), 0, s, bt, T, H, scale);
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
