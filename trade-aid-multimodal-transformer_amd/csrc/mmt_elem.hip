// Memory-bound kernels of the training step (gfx950): LayerNorm fwd/bwd, token+position
// embedding fwd/bwd, fused softmax-cross-entropy, bias-gradient column sums, per-head Q/K/V
// stage-2 block-diagonal maps, fp32->bf16 weight packing, fused AdamW, directional metric.
// All grouped over modalities with blockIdx.z (one launch per op per layer).
#include <stdlib.h>

#include "mmt_common.h"
#include "mmt_kernels.h"

// ============================================================================================
// LayerNorm (reference: nn.LayerNorm(n_embd), eps 1e-5; model.py:189-190, 210, 330)
// one wave per row; each lane holds NV float4 of the row in registers
// ============================================================================================
template <int NV, int RPI>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnBatch batch, int R, int C) {
  // RPI rows per wave with every row's loads issued before any reduction (memory-level parallelism)
  const LnProblem& P = batch.p[blockIdx.z];
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPI;
  if (blockIdx.x == 0 && blockIdx.z == 0) {
    if ((int)threadIdx.x < batch.nzero_f) batch.zero_f[threadIdx.x] = 0.f;
    if ((int)threadIdx.x < batch.nzero_i) batch.zero_i[threadIdx.x] = 0;
  }
  const int C4 = C >> 2;
  f32x4 v[RPI][NV];
#pragma unroll
  for (int u = 0; u < RPI; ++u) {
    const int row = row0 + u;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      v[u][i] = (row < R && c4 < C4) ? reinterpret_cast<const f32x4*>(P.x + (int64_t)row * C)[c4]
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  f32x4 g[NV], b[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = lane + 64 * i;
    g[i] = c4 < C4 ? reinterpret_cast<const f32x4*>(P.gamma)[c4] : f32x4{0.f, 0.f, 0.f, 0.f};
    b[i] = c4 < C4 ? reinterpret_cast<const f32x4*>(P.beta)[c4] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < RPI; ++u) {
    const int row = row0 + u;
    if (row >= R) break;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += v[u][i][0] + v[u][i][1] + v[u][i][2] + v[u][i][3];
    const float mean = warp_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < C4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { const float d = v[u][i][e] - mean; q += d * d; }
      }
    }
    const float rstd = rsqrtf(warp_sum(q) / C + 1e-5f);
    bf16_t* y = P.y + (int64_t)row * C;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < C4) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (v[u][i][e] - mean) * rstd * g[i][e] + b[i][e];
        reinterpret_cast<u32x2*>(y)[c4] = u32x2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
        if (P.y8) {  // MX-fp8 copy: a 32-column block is 8 consecutive lanes
          float am = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3])));
          am = fmaxf(am, __shfl_xor(am, 1, 64));
          am = fmaxf(am, __shfl_xor(am, 2, 64));
          am = fmaxf(am, __shfl_xor(am, 4, 64));
          const int ex = mx_exp(am);
          const float inv = mx_inv(ex);
          reinterpret_cast<uint32_t*>(P.y8 + (int64_t)row * P.ld8)[c4] = pack4fp8(o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
          if ((c4 & 7) == 0) P.s8[(int64_t)row * P.lds8 + (c4 >> 3)] = (uint8_t)(ex + 127);
        }
      }
    }
    if (lane == 0) { P.mean[row] = mean; P.rstd[row] = rstd; }
  }
}

// backward: dx += rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)); dgamma/dbeta column sums.
// One wave per row, RPI rows per iteration with every load issued up front (the kernel is
// HBM-bound: x, dy, dx in; dx (+ bf16 copy) out). Optional: the bf16 copy carries the dropout
// mask of the branch that consumes it and its column sums (that branch's bias gradient).
template <int NV, int RPI>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LnBatch batch, int R, int C) {
  const LnProblem& P = batch.p[blockIdx.z];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int C4 = C >> 2;
  const bool drop = P.drop_thr != 0;
  f32x4 g[NV], dgam[NV], dbet[NV], dsm[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = lane + 64 * i;
    g[i] = (c4 < C4) ? reinterpret_cast<const f32x4*>(P.gamma)[c4] : f32x4{0.f, 0.f, 0.f, 0.f};
    dgam[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    dbet[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    dsm[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int stride = gridDim.x * 4;
  for (int row0 = blockIdx.x * 4 + wave; row0 < R; row0 += stride * RPI) {
    f32x4 xv[RPI][NV], dv[RPI][NV], ov[RPI][NV];
    float mean[RPI], rstd[RPI];
#pragma unroll
    for (int u = 0; u < RPI; ++u) {
      const int row = row0 + u * stride;
      const bool ok = row < R;
      mean[u] = ok ? P.mean[row] : 0.f;
      rstd[u] = ok ? P.rstd[row] : 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c4 = lane + 64 * i;
        const bool in = ok && c4 < C4;
        const int64_t o = (int64_t)row * C4 + c4;
        xv[u][i] = in ? reinterpret_cast<const f32x4*>(P.x)[o] : f32x4{0.f, 0.f, 0.f, 0.f};
        dv[u][i] = in ? reinterpret_cast<const f32x4*>(P.dy)[o] : f32x4{0.f, 0.f, 0.f, 0.f};
        ov[u][i] = in ? reinterpret_cast<const f32x4*>(P.dx)[o] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int u = 0; u < RPI; ++u) {
      const int row = row0 + u * stride;
      if (row >= R) break;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (xv[u][i][e] - mean[u]) * rstd[u];
          const float gd = dv[u][i][e] * g[i][e];
          xv[u][i][e] = xh;
          s1 += gd;
          s2 += gd * xh;
          dgam[i][e] += dv[u][i][e] * xh;
          dbet[i][e] += dv[u][i][e];
        }
      }
      s1 = warp_sum(s1) / C;
      s2 = warp_sum(s2) / C;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c4 = lane + 64 * i;
        if (c4 < C4) {
          f32x4 o = ov[u][i];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] += rstd[u] * (dv[u][i][e] * g[i][e] - s1 - xv[u][i][e] * s2);
          const int64_t off = (int64_t)row * C4 + c4;
          reinterpret_cast<f32x4*>(P.dx)[off] = o;
          if (P.dx16) {
            if (drop) {
#pragma unroll
              for (int q = 0; q < 2; ++q) {  // columns 4*c4 .. +3: one hash per pair
                const uint32_t hq = mmt_hash(P.drop_key, (uint32_t)row, (uint32_t)(2 * c4 + q));
                o[2 * q] = mmt_keep(hq, 0, P.drop_thr) ? o[2 * q] * P.drop_scale : 0.f;
                o[2 * q + 1] = mmt_keep(hq, 1, P.drop_thr) ? o[2 * q + 1] * P.drop_scale : 0.f;
              }
            }
            reinterpret_cast<u32x2*>(P.dx16)[off] = u32x2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
#pragma unroll
            for (int e = 0; e < 4; ++e) dsm[i][e] += o[e];
          }
        }
      }
    }
  }
  // reduce the 4 waves' partial column sums through LDS, then one atomic per column
  __shared__ float red[3][4][1024];
  const int nred = P.dsum ? 3 : 2;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = lane + 64 * i;
    if (c4 < C4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[0][wave][c4 * 4 + e] = dgam[i][e];
        red[1][wave][c4 * 4 + e] = dbet[i][e];
        red[2][wave][c4 * 4 + e] = dsm[i][e];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    for (int k = 0; k < nred; ++k) {
      const float a = red[k][0][c] + red[k][1][c] + red[k][2][c] + red[k][3][c];
      atomicAdd((k == 0 ? P.dgamma : k == 1 ? P.dbeta : P.dsum) + c, a);
    }
  }
}

hipError_t mmt_launch_ln_fwd(const LnBatch& b, int R, int C, hipStream_t s) {
  if (C % 4 != 0 || C > 1024 || b.count == 0) return C % 4 ? hipErrorInvalidValue : hipSuccess;
  const int nv = (C / 4 + 63) / 64;
  if (nv <= 1) hipLaunchKernelGGL((ln_fwd_kernel<1, 4>), dim3((R + 15) / 16, 1, b.count), dim3(256), 0, s, b, R, C);
  else if (nv <= 2) hipLaunchKernelGGL((ln_fwd_kernel<2, 2>), dim3((R + 7) / 8, 1, b.count), dim3(256), 0, s, b, R, C);
  else hipLaunchKernelGGL((ln_fwd_kernel<4, 1>), dim3((R + 3) / 4, 1, b.count), dim3(256), 0, s, b, R, C);
  return hipGetLastError();
}

hipError_t mmt_launch_ln_bwd(const LnBatch& b, int R, int C, hipStream_t s) {
  if (C % 4 != 0 || C > 1024 || b.count == 0) return C % 4 ? hipErrorInvalidValue : hipSuccess;
  // 4 rows per block per pass; the grid is capped so the dgamma/dbeta atomics stay few
  static const int cap = [] {
    // blocks per problem: every block adds its dgamma/dbeta(/dsum) partials with one atomic per
    // column, so the cap bounds the same-address atomic chain (C1, 4 problems: 4096 blocks 228 us,
    // 1024 75 us, 512 52 us, 256 45 us = 5.2 TB/s)
    const char* e = getenv("MMT_LNB_CAP");
    return e ? atoi(e) : 256;
  }();
  int blocks = (R + 3) / 4;
  if (blocks > cap) blocks = cap;
  dim3 grid(blocks, 1, b.count);
  const int nv = (C / 4 + 63) / 64;
  if (nv <= 1) hipLaunchKernelGGL((ln_bwd_kernel<1, 4>), grid, dim3(256), 0, s, b, R, C);
  else if (nv <= 2) hipLaunchKernelGGL((ln_bwd_kernel<2, 2>), grid, dim3(256), 0, s, b, R, C);
  else hipLaunchKernelGGL((ln_bwd_kernel<4, 1>), grid, dim3(256), 0, s, b, R, C);
  return hipGetLastError();
}

// ============================================================================================
// Embedding: x[b,t] = tok[idx[b,t]] + pos[t]   (model.py:308-317); backward scatter-adds
// ============================================================================================
__global__ __launch_bounds__(256) void embed_fwd_kernel(EmbBatch batch, int R, int T, int C) {
  const EmbProblem& P = batch.p[blockIdx.z];
  const int C4 = C >> 2;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)R * C4) return;
  const int r = (int)(i / C4), c4 = (int)(i % C4);
  const int t = r % T;
  int64_t id = P.idx[r];
  id = id < 0 ? 0 : (id >= P.V ? P.V - 1 : id);
  const f32x4 a = reinterpret_cast<const f32x4*>(P.tok + id * C)[c4];
  const f32x4 p = reinterpret_cast<const f32x4*>(P.pos + (int64_t)t * C)[c4];
  reinterpret_cast<f32x4*>(P.x + (int64_t)r * C)[c4] = a + p;
}

// token-table gradient, privatised in LDS: a block owns one column slab (SLAB floats, the widest
// power of two with V * SLAB floats <= the launch's LDS limit) of one modality's table and a chunk of rows;
// it scatter-adds its rows into the LDS slab (ds_add_f32) and flushes the slab. Two flush forms:
//  * with a scratch buffer (EmbProblem::part, the engine's path): plain stores of the whole slab into
//    the chunk's partial table [chunk][V][C], then embed_tok_reduce_kernel adds the partial tables
//    into dtok. Chunks are then short (two passes of EMB_U loads per thread): the launch is bound by
//    its row loads' latency, and at C1 / the target it ends the step after the side stream has
//    drained (round 4: 174 us live at C1 with 64 blocks per modality of 16 dependent load rounds);
//  * without one: one global atomic per touched entry, rows per block >= 4 V so the atomics stay few.
// A vocabulary too large for a 4-float slab takes direct atomics.
// LDS per block: 32 KiB when every problem of the launch has partial-table scratch (short chunks, many
// blocks per CU), 64 KiB for the atomic-flush form (mmt_op_embedding_bwd without scratch), so
// vocabularies up to 4096 keep the LDS-privatised slab there
#define EMB_LDS_PART 8192
#define EMB_LDS_ATOMIC 16384
__host__ __device__ __forceinline__ int emb_slab(int V, int C, int lf) {
  if ((int64_t)V * C <= lf) return C;
  int p = 256;  // largest power-of-two slab dividing C that fits (4 always divides C)
  while (p > 4 && (C % p != 0 || (int64_t)V * p > lf)) p >>= 1;
  return p;
}
#ifndef EMB_U
#define EMB_U 8
#endif
// rows per chunk: with partial tables two load rounds per thread (as long as the [chunk][V][C]
// tables fit the B*T*C-float scratch), else >= 4 V rows (atomic flush)
__host__ __device__ __forceinline__ int emb_chunk(const EmbProblem& P, int R, int C, int lf) {
  const int rpp = 256 / (emb_slab(P.V, C, lf) >> 2);
  if (P.part && (int64_t)P.V * emb_slab(P.V, C, lf) <= lf) {
    int ch = rpp * EMB_U * 2;
    while ((int64_t)((R + ch - 1) / ch) * P.V > R && ch < R) ch <<= 1;
    if ((int64_t)((R + ch - 1) / ch) * P.V <= R) return ch;
  }
  int ch = 256;
  while (ch < 4 * P.V && ch < R) ch <<= 1;
  return ch;
}
__host__ __device__ __forceinline__ bool emb_use_part(const EmbProblem& P, int R, int C, int lf) {
  if (!P.part || (int64_t)P.V * emb_slab(P.V, C, lf) > lf) return false;
  const int ch = emb_chunk(P, R, C, lf);
  return (int64_t)((R + ch - 1) / ch) * P.V <= R;
}
template <int LF>
__global__ __launch_bounds__(256) void embed_tok_bwd_kernel(EmbBatch batch, int R, int C) {
  const EmbProblem& P = batch.p[blockIdx.z];
  const int V = P.V;
  const int slab = emb_slab(V, C, LF);
  const int nslab = C / slab;
  const int chunk = emb_chunk(P, R, C, LF);
  const int nchunk = (R + chunk - 1) / chunk;
  if ((int)blockIdx.x >= nslab * nchunk) return;
  const int sl = blockIdx.x % nslab, ck = blockIdx.x / nslab;
  const int c0 = sl * slab;
  const int r0 = ck * chunk, r1 = min(R, r0 + chunk);
  __shared__ float acc[LF];
  const bool priv = (int64_t)V * slab <= LF;
  if (priv) {
    for (int q = threadIdx.x; q < V * slab; q += 256) acc[q] = 0.f;
    __syncthreads();
  }
  const int s4 = slab >> 2;            // f32x4 per row slab
  const int rows_per_pass = 256 / s4;  // rows covered by the block per pass
  const int lr = threadIdx.x / s4, c4 = threadIdx.x % s4;
  constexpr int U = EMB_U;  // passes in flight per thread (idx and dx loads issued together)
  for (int rb = r0 + lr; lr < rows_per_pass && rb < r1; rb += U * rows_per_pass) {
    int64_t id[U];
    f32x4 d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = rb + u * rows_per_pass;
      id[u] = rr < r1 ? P.idx[rr] : -1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = rb + u * rows_per_pass;
      d[u] = rr < r1 ? reinterpret_cast<const f32x4*>(P.dx + (int64_t)rr * C + c0)[c4] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (rb + u * rows_per_pass >= r1) break;
      const int64_t t = id[u] < 0 ? 0 : (id[u] >= V ? V - 1 : id[u]);
      if (priv) {
#pragma unroll
        for (int e = 0; e < 4; ++e) atomicAdd(&acc[t * slab + c4 * 4 + e], d[u][e]);
      } else {
        float* dt = P.dtok + t * C + c0 + c4 * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) atomicAdd(dt + e, d[u][e]);
      }
    }
  }
  if (priv) {
    __syncthreads();
    if (emb_use_part(P, R, C, LF)) {  // the whole slab into this chunk's partial table
      float* pt = P.part + (int64_t)ck * V * C + c0;
      for (int q = threadIdx.x; q < V * slab; q += 256) pt[(int64_t)(q / slab) * C + (q % slab)] = acc[q];
    } else {
      for (int q = threadIdx.x; q < V * slab; q += 256)
        if (acc[q] != 0.f) atomicAdd(P.dtok + (int64_t)(q / slab) * C + c0 + (q % slab), acc[q]);
    }
  }
}

// dtok += the sum over the row chunks of the partial tables (embed_tok_bwd_kernel with P.part):
// thread (float4 i of the table, group y of EMB_RED chunks) sums its group with all loads in flight
// and adds it with four atomics (a thread looping over every chunk ran 256 dependent loads deep for
// the small vocabularies: 68 us at C1)
#define EMB_RED 16
template <int LF>
__global__ __launch_bounds__(256) void embed_tok_reduce_kernel(EmbBatch batch, int R, int C) {
  const EmbProblem& P = batch.p[blockIdx.z];
  if (!emb_use_part(P, R, C, LF)) return;
  const int V = P.V, C4 = C >> 2;
  const int ch = emb_chunk(P, R, C, LF);
  const int nchunk = (R + ch - 1) / ch;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int k0 = blockIdx.y * EMB_RED;
  if (i >= (int64_t)V * C4 || k0 >= nchunk) return;
  f32x4 t[EMB_RED];
#pragma unroll
  for (int k = 0; k < EMB_RED; ++k)
    t[k] = k0 + k < nchunk ? reinterpret_cast<const f32x4*>(P.part + (int64_t)(k0 + k) * V * C)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 1; k < EMB_RED; ++k) t[0] += t[k];
  float* d = P.dtok + 4 * i;
#pragma unroll
  for (int e = 0; e < 4; ++e) atomicAdd(d + e, t[0][e]);
}

// positional-table gradient, shared by all modalities: dpos[t] += sum_m sum_b dx_m[b*T + t].
// block (t, split): a slice of the M*B rows of position t, 4 rows per wave in flight; one atomic
// per column per block (EMB_POS_SPLIT per element)
#define EMB_POS_SPLIT 8
__global__ __launch_bounds__(256) void embed_pos_bwd_kernel(EmbBatch batch, int B, int T, int C) {
  const int t = blockIdx.x;
  const int C4 = C >> 2;
  const int nrows = batch.count * B;  // (modality, b) pairs
  const int per = (nrows + EMB_POS_SPLIT - 1) / EMB_POS_SPLIT;
  const int q0 = blockIdx.y * per, q1 = min(nrows, q0 + per);
  for (int c4 = threadIdx.x; c4 < C4; c4 += 256) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    int q = q0;
    for (; q + 4 <= q1; q += 4) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = (q + u) / B, b = (q + u) % B;
        v[u] = reinterpret_cast<const f32x4*>(batch.p[m].dx + ((int64_t)b * T + t) * C)[c4];
      }
      s += (v[0] + v[1]) + (v[2] + v[3]);
    }
    for (; q < q1; ++q) {
      const int m = q / B, b = q % B;
      s += reinterpret_cast<const f32x4*>(batch.p[m].dx + ((int64_t)b * T + t) * C)[c4];
    }
    float* dp = batch.p[0].dpos + (int64_t)t * C + 4 * c4;
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(dp + e, s[e]);
  }
}

// ---------------------------------------------------------------------------------------------
// Token-table gradient by a counting sort of the rows (round 5; the engine's path, EmbProblem::part
// as int scratch): the LDS-privatised slabs above scatter-add every element with ds_add_f32, and LDS
// float atomics serialise (C1: 127 + 28 us live for 67 MB of dx, 14x its HBM time; the last kernels
// of the step). Here no float atomic touches LDS:
//  * emb_sort_kernel, one workgroup per modality: the row ids in token order -> perm [R], STABLE
//    (rows of one token in increasing row order) for R <= EMB_SORT_RMAX: a bitonic sort of the keys
//    token << 14 | row in LDS, so the run sums below add a token's rows in a fixed order (round 6:
//    the round-5 histogram scatter placed a bucket's rows in atomic arrival order, so dtok's float
//    sums changed run to run). Larger R keeps that scatter (order inside a bucket = arrival order);
//  * emb_segsum_kernel: a wave walks 64 consecutive sorted rows (each dx row read once, 1 KiB per
//    wave-load), sums runs of equal tokens in registers and adds each run to dtok with one atomic per
//    column (a few runs per wave: ~V + waves adds per column in all).
// ---------------------------------------------------------------------------------------------
#define EMB_SORT_VMAX 16384
#define EMB_SORT_RMAX 16384  // rows of the stable (bitonic) form: keys tok << 14 | row
__global__ __launch_bounds__(1024) void emb_sort_kernel(EmbBatch batch, int R) {
  const EmbProblem& P = batch.p[blockIdx.z];
  const int V = P.V;
  int* perm = P.perm ? P.perm : reinterpret_cast<int*>(P.part);
  __shared__ int cnt[EMB_SORT_VMAX];  // stable form: the keys (EMB_SORT_RMAX == EMB_SORT_VMAX)
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (R <= EMB_SORT_RMAX) {
    static_assert(EMB_SORT_RMAX <= EMB_SORT_VMAX, "the key array reuses the histogram");
    uint32_t* key = reinterpret_cast<uint32_t*>(cnt);
    int N = 2;
    while (N < R) N <<= 1;
    for (int r = tid; r < N; r += 1024) {
      uint32_t k = 0xffffffffu;  // padding sorts last
      if (r < R) {
        int64_t t = P.idx[r];
        t = t < 0 ? 0 : (t >= V ? V - 1 : t);
        k = ((uint32_t)t << 14) | (uint32_t)r;
      }
      key[r] = k;
    }
    __syncthreads();
    // keys are distinct (the row is in the low bits), so the result is the unique sorted order
    for (int k = 2; k <= N; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int p = tid; p < (N >> 1); p += 1024) {
          const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1));
          const uint32_t a = key[i], b = key[i + j];
          if ((a > b) == ((i & k) == 0)) { key[i] = b; key[i + j] = a; }
        }
        __syncthreads();
      }
    for (int r = tid; r < R; r += 1024) perm[r] = (int)(key[r] & 0x3fffu);
    return;
  }
  for (int v = tid; v < V; v += 1024) cnt[v] = 0;
  __syncthreads();
  for (int r = tid; r < R; r += 1024) {
    int64_t t = P.idx[r];
    t = t < 0 ? 0 : (t >= V ? V - 1 : t);
    atomicAdd(&cnt[t], 1);
  }
  __syncthreads();
  // exclusive scan: thread tid owns entries [tid * per, tid * per + per)
  const int per = (V + 1023) / 1024;
  const int b0 = tid * per, b1 = min(V, b0 + per);
  int s = 0;
  for (int v = b0; v < b1; ++v) s += cnt[v];
  int incl = s;  // inclusive wave scan of the per-thread sums
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int wbase = 0;
  for (int u = 0; u < w; ++u) wbase += wsum[u];
  int run = wbase + incl - s;  // exclusive prefix of this thread's first entry
  for (int v = b0; v < b1; ++v) {
    const int c = cnt[v];
    cnt[v] = run;  // now the bucket's next free slot
    run += c;
  }
  __syncthreads();
  for (int r = tid; r < R; r += 1024) {
    int64_t t = P.idx[r];
    t = t < 0 ? 0 : (t >= V ? V - 1 : t);
    perm[atomicAdd(&cnt[t], 1)] = r;
  }
}

// grid (ceil(R / 64) * halves / 4, 1, problems), 256 threads: wave -> (64-row range, column half);
// lane c4 holds float4 column 4 c4 of its half (C <= 512: halves = C / 256 rounded up)
__global__ __launch_bounds__(256) void emb_segsum_kernel(EmbBatch batch, int R, int C) {
  const EmbProblem& P = batch.p[blockIdx.z];
  const int V = P.V;
  const int* perm = P.perm ? P.perm : reinterpret_cast<const int*>(P.part);
  const int halves = (C + 255) / 256;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int range = gw / halves, hf = gw % halves;
  const int p0 = range * 64;
  if (p0 >= R) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const int c4 = hf * 64 + lane;       // float4 column of this lane
  const bool col_ok = 4 * c4 < C;
  const int n = min(64, R - p0);
  // lane l fetches sorted row p0 + l and its token; the walk reads them back by readlane
  int myrow = 0, mytok = 0;
  if (lane < n) {
    myrow = perm[p0 + lane];
    int64_t t = P.idx[myrow];
    mytok = (int)(t < 0 ? 0 : (t >= V ? V - 1 : t));
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int cur = __builtin_amdgcn_readlane(mytok, 0);
  const float* const dx = sgpr_ptr(P.dx);
  float* const dtok = sgpr_ptr(P.dtok);
  constexpr int U = 8;  // rows in flight
  for (int k0 = 0; k0 < n; k0 += U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u;
      const int row = __builtin_amdgcn_readlane(myrow, k < n ? k : 0);
      v[u] = (k < n && col_ok) ? reinterpret_cast<const f32x4*>(dx + (int64_t)row * C)[c4] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u;
      if (k >= n) break;  // wave-uniform
      const int t = __builtin_amdgcn_readlane(mytok, k);
      if (t != cur) {  // wave-uniform: a run of token cur ends
        if (col_ok) {
          float* d = dtok + (int64_t)cur * C + 4 * c4;
#pragma unroll
          for (int e = 0; e < 4; ++e) atomicAdd(d + e, acc[e]);
        }
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
        cur = t;
      }
      acc += v[u];
    }
  }
  if (col_ok) {
    float* d = dtok + (int64_t)cur * C + 4 * c4;
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(d + e, acc[e]);
  }
}

// the sorted path applies when every problem has int scratch for the permutation and a vocabulary
// the histogram holds (MMT_EMB_SORT=0: the LDS-slab kernels, A/B)
static int g_emb_sort = [] {
  const char* e = getenv("MMT_EMB_SORT");
  return e ? atoi(e) : 1;
}();
extern "C" int mmt_emb_set_sort(int on) {
  const int old = g_emb_sort;
  g_emb_sort = on;
  return old;
}
static bool emb_sorted_ok(const EmbBatch& b, int R, int C) {
  if (!g_emb_sort || C > 1024) return false;
  for (int g = 0; g < b.count; ++g) {
    const EmbProblem& P = b.p[g];
    if ((!P.part && !P.perm) || P.V < 1 || P.V > EMB_SORT_VMAX || (int64_t)R * C < R) return false;
  }
  return true;
}

// the row sort alone, into every problem's perm (the engine runs it early, on the side stream: it
// reads only the token ids); false (nothing launched) when the sorted path does not apply
bool mmt_emb_sort_ok(const EmbBatch& b, int R, int C) {
  for (int g = 0; g < b.count; ++g)
    if (!b.p[g].perm) return false;
  return b.count > 0 && C % 4 == 0 && emb_sorted_ok(b, R, C);
}
hipError_t mmt_launch_emb_sort(const EmbBatch& b, int R, hipStream_t s) {
  hipLaunchKernelGGL(emb_sort_kernel, dim3(1, 1, b.count), dim3(1024), 0, s, b, R);
  return hipGetLastError();
}

hipError_t mmt_launch_embed_fwd(const EmbBatch& b, int B, int T, int C, hipStream_t s) {
  if (C % 4 || b.count == 0) return C % 4 ? hipErrorInvalidValue : hipSuccess;
  const int64_t n = (int64_t)B * T * (C / 4);
  dim3 grid((unsigned)((n + 255) / 256), 1, b.count);
  hipLaunchKernelGGL(embed_fwd_kernel, grid, dim3(256), 0, s, b, B * T, T, C);
  return hipGetLastError();
}

hipError_t mmt_launch_embed_bwd(const EmbBatch& b, int B, int T, int C, hipStream_t s) {
  if (C % 4 || b.count == 0) return C % 4 ? hipErrorInvalidValue : hipSuccess;
  const int R = B * T;
  if (C % 4 || C > 1024) return hipErrorInvalidValue;
  if (emb_sorted_ok(b, R, C)) {
    for (int g = 1; g < b.count; ++g)
      if (b.p[g].dpos != b.p[0].dpos) return hipErrorInvalidValue;
    // perm set on every problem: mmt_launch_emb_sort already ran (same stream order or an event)
    bool sorted = true;
    for (int g = 0; g < b.count; ++g) sorted = sorted && b.p[g].perm;
    if (!sorted) hipLaunchKernelGGL(emb_sort_kernel, dim3(1, 1, b.count), dim3(1024), 0, s, b, R);  // into perm / part
    const int halves = (C + 255) / 256;
    const int waves = ((R + 63) / 64) * halves;
    hipLaunchKernelGGL(emb_segsum_kernel, dim3((waves + 3) / 4, 1, b.count), dim3(256), 0, s, b, R, C);
    hipLaunchKernelGGL(embed_pos_bwd_kernel, dim3(T, EMB_POS_SPLIT), dim3(256), 0, s, b, B, T, C);
    return hipGetLastError();
  }
  // grid: the largest (slabs x row chunks) over the problems
  bool all_part = true;
  for (int g = 0; g < b.count; ++g) all_part = all_part && b.p[g].part != nullptr;
  const int lf = all_part ? EMB_LDS_PART : EMB_LDS_ATOMIC;
  int maxblocks = 1, maxv = 1;
  bool any_part = false;
  for (int g = 0; g < b.count; ++g) {
    const int ch = emb_chunk(b.p[g], R, C, lf);
    const int nb = (C / emb_slab(b.p[g].V, C, lf)) * ((R + ch - 1) / ch);
    maxblocks = nb > maxblocks ? nb : maxblocks;
    maxv = b.p[g].V > maxv ? b.p[g].V : maxv;
    any_part = any_part || emb_use_part(b.p[g], R, C, lf);
  }
  if (all_part) hipLaunchKernelGGL(embed_tok_bwd_kernel<EMB_LDS_PART>, dim3(maxblocks, 1, b.count), dim3(256), 0, s, b, R, C);
  else hipLaunchKernelGGL(embed_tok_bwd_kernel<EMB_LDS_ATOMIC>, dim3(maxblocks, 1, b.count), dim3(256), 0, s, b, R, C);
  if (any_part) {
    int maxg = 1;
    for (int g = 0; g < b.count; ++g) {
      if (!emb_use_part(b.p[g], R, C, lf)) continue;
      const int ch = emb_chunk(b.p[g], R, C, lf);
      const int ng = ((R + ch - 1) / ch + EMB_RED - 1) / EMB_RED;
      maxg = ng > maxg ? ng : maxg;
    }
    const int64_t n4 = (int64_t)maxv * (C / 4);
    const dim3 grid((unsigned)((n4 + 255) / 256), maxg, b.count);
    if (all_part) hipLaunchKernelGGL(embed_tok_reduce_kernel<EMB_LDS_PART>, grid, dim3(256), 0, s, b, R, C);
    else hipLaunchKernelGGL(embed_tok_reduce_kernel<EMB_LDS_ATOMIC>, grid, dim3(256), 0, s, b, R, C);
  }
  // all problems of one batch must share the positional table (one model): dpos of p[0]
  for (int g = 1; g < b.count; ++g)
    if (b.p[g].dpos != b.p[0].dpos) return hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_pos_bwd_kernel, dim3(T, EMB_POS_SPLIT), dim3(256), 0, s, b, B, T, C);
  return hipGetLastError();
}

// ============================================================================================
// Cross-entropy (F.cross_entropy mean over B*T; model.py:393-400), fused with dlogits:
//   loss += (logsumexp(x) - x[t]) / R ;  dlogits = softmax(x) - onehot(t)  (bf16, unscaled)
// one wave per row, the row held in registers (KV logits per lane, all loads issued at once);
// grid-strided rows so each block adds its loss share with ONE atomic (a per-4-row atomic on
// the single loss address serialised ~16 k atomics per launch)
// ============================================================================================
// rows of one problem with KV logits per lane: two rows per wave in flight (the next row's loads
// are issued before this row's reductions), so a wave's row-after-row latency chain halves
template <int KV>
__device__ __forceinline__ float ce_rows(const CeProblem& P, int R, int lane, int first, int stride) {
  const int V = P.V;
  float contrib = 0.f;
  float v[KV], nv[KV];
  auto load = [&](int row, float (&dst)[KV]) {
    const float* x = P.logits + (int64_t)row * V;
#pragma unroll
    for (int k = 0; k < KV; ++k) {
      const int i = lane + 64 * k;
      dst[k] = (row < R && i < V) ? x[i] : -INFINITY;
    }
  };
  if (first < R) load(first, v);
  for (int row = first; row < R; row += stride) {
    const int t = (int)P.tgt[row];
    const float xt = P.logits[(int64_t)row * V + t];
    if (row + stride < R) load(row + stride, nv);
    float m = v[0];
#pragma unroll
    for (int k = 1; k < KV; ++k) m = fmaxf(m, v[k]);
    m = warp_max(m);
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < KV; ++k) sum += __expf(v[k] - m);  // exp(-inf) = 0 for the padding
    const float lse = m + __logf(warp_sum(sum));
    contrib += lse - xt;
    bf16_t* d = P.dlogits + (int64_t)row * P.ld_d;
#pragma unroll
    for (int k = 0; k < KV; ++k) {
      const int i = lane + 64 * k;
      if (i < P.ld_d) d[i] = f2bf(i < V ? __expf(v[k] - lse) - (i == t ? 1.f : 0.f) : 0.f);
    }
#pragma unroll
    for (int k = 0; k < KV; ++k) v[k] = nv[k];
  }
  return contrib;
}

// KV: the largest vocabulary's logits per lane (64 k + lane); each problem runs the smallest
// instantiation that holds its own vocabulary (the V = 5 head no longer walks 16 masked groups)
template <int KV>
__global__ __launch_bounds__(256) void ce_fwd_kernel(CeBatch batch, int R) {
  const CeProblem& P = batch.p[blockIdx.z];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int V = P.V;
  __shared__ float part[4];
  float contrib = 0.f;
  const int first = blockIdx.x * 4 + wave, stride = gridDim.x * 4;
  if (KV > 0) {
    const int kv = (V + 63) / 64;  // uniform per problem
    if (kv <= 1) contrib = ce_rows<1>(P, R, lane, first, stride);
    else if (kv <= 2 && KV >= 2) contrib = ce_rows<2>(P, R, lane, first, stride);
    else if (kv <= 4 && KV >= 4) contrib = ce_rows<4>(P, R, lane, first, stride);
    else if (kv <= 8 && KV >= 8) contrib = ce_rows<8>(P, R, lane, first, stride);
    else contrib = ce_rows<(KV > 0 ? KV : 1)>(P, R, lane, first, stride);
  } else {  // V > 1024: three passes over the row
    for (int row = first; row < R; row += stride) {
      const float* x = P.logits + (int64_t)row * V;
      const int t = (int)P.tgt[row];
      bf16_t* d = P.dlogits + (int64_t)row * P.ld_d;
      float m = -INFINITY;
      for (int i = lane; i < V; i += 64) m = fmaxf(m, x[i]);
      m = warp_max(m);
      float sum = 0.f;
      for (int i = lane; i < V; i += 64) sum += __expf(x[i] - m);
      const float lse = m + __logf(warp_sum(sum));
      contrib += lse - x[t];
      for (int i = lane; i < P.ld_d; i += 64)
        d[i] = f2bf(i < V ? __expf(x[i] - lse) - (i == t ? 1.f : 0.f) : 0.f);
    }
  }
  if (lane == 0) part[wave] = contrib;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float blk = (part[0] + part[1] + part[2] + part[3]) / (float)R;
    if (P.part) P.part[blockIdx.x] = blk;  // summed in block order by ce_loss_kernel
    else atomicAdd(P.loss, blk);
    // failure detection: a non-finite loss raises this problem's bit in a device
    // flag word the host reads when it syncs anyway (reference guard: main.py:606)
    if (P.flag && !__builtin_isfinite(blk)) {
      atomicOr(P.flag, P.bit);      // this forward's word
      atomicOr(P.flag + 1, P.bit);  // sticky word (cleared only by the caller)
    }
  }
}

// the block shares of ce_fwd_kernel (CeProblem::part) added to the loss in block order: lane l sums
// blocks l, l + 64, ... in order, then a fixed xor tree over the lanes (no atomics: the loss is the
// same bits on every run)
__global__ __launch_bounds__(64) void ce_loss_kernel(CeBatch batch, int blocks) {
  const CeProblem& P = batch.p[blockIdx.z];
  if (!P.part) return;
  const int lane = threadIdx.x;
  float s = 0.f;
  for (int b = lane; b < blocks; b += 64) s += P.part[b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) *P.loss += s;
}

hipError_t mmt_launch_ce_fwd(const CeBatch& b, int R, hipStream_t s) {
  if (b.count == 0) return hipSuccess;
  int maxv = 1;
  bool any_part = false;
  for (int g = 0; g < b.count; ++g) {
    maxv = b.p[g].V > maxv ? b.p[g].V : maxv;
    any_part = any_part || b.p[g].part;
  }
  int blocks = (R + 3) / 4;
  if (blocks > 512) blocks = 512;
  dim3 grid(blocks, 1, b.count);
  const int kv = (maxv + 63) / 64;
  if (kv <= 1) hipLaunchKernelGGL(ce_fwd_kernel<1>, grid, dim3(256), 0, s, b, R);
  else if (kv <= 2) hipLaunchKernelGGL(ce_fwd_kernel<2>, grid, dim3(256), 0, s, b, R);
  else if (kv <= 4) hipLaunchKernelGGL(ce_fwd_kernel<4>, grid, dim3(256), 0, s, b, R);
  else if (kv <= 8) hipLaunchKernelGGL(ce_fwd_kernel<8>, grid, dim3(256), 0, s, b, R);
  else if (kv <= 16) hipLaunchKernelGGL(ce_fwd_kernel<16>, grid, dim3(256), 0, s, b, R);
  else hipLaunchKernelGGL(ce_fwd_kernel<0>, grid, dim3(256), 0, s, b, R);
  if (any_part) hipLaunchKernelGGL(ce_loss_kernel, dim3(1, 1, b.count), dim3(64), 0, s, b, blocks);
  return hipGetLastError();
}

// ============================================================================================
// Bias gradients: out[n] += alpha * sum_r x[r, n]   (x bf16 [R, ld])
// block = 32 column chunks of 8 x 8 row lanes; 256 rows per block
// ============================================================================================
__global__ __launch_bounds__(256) void colsum_kernel(ColsumBatch batch, int R) {
  const ColsumProblem& P = batch.p[blockIdx.z];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + cl) * 8;
  const int r0 = blockIdx.y * 256;
  __shared__ float red[8][256 + 8];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < P.N) {
    const bool full = (c0 + 8 <= P.ld) && ((P.ld & 7) == 0);
    for (int r = r0 + rl; r < min(R, r0 + 256); r += 8) {
      const bf16_t* src = P.x + (int64_t)r * P.ld + c0;
      if (full) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(src);
#pragma unroll
        for (int e = 0; e < 4; ++e) { acc[2 * e] += bf2f(v[e] & 0xffff); acc[2 * e + 1] += bf2f(v[e] >> 16); }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) if (c0 + e < P.N) acc[e] += bf2f(src[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][cl * 8 + e] = acc[e];
  __syncthreads();
  const int c = threadIdx.x;  // 256 columns of this block
  const int gc = blockIdx.x * 256 + c;
  if (gc < P.N) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += red[i][c];
    float alpha = P.alpha;
    if (P.alpha_ptr) alpha *= *P.alpha_ptr;
    atomicAdd(P.out + gc, alpha * s);
  }
}

hipError_t mmt_launch_colsum(const ColsumBatch& b, int R, hipStream_t s) {
  int maxn = 0;
  for (int g = 0; g < b.count; ++g) maxn = b.p[g].N > maxn ? b.p[g].N : maxn;
  if (maxn == 0 || b.count == 0) return hipSuccess;
  dim3 grid((maxn + 255) / 256, (R + 255) / 256, b.count);
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, s, b, R);
  return hipGetLastError();
}

// ============================================================================================
// fp32 master weights -> bf16 packed copies with padded leading dimension (pad zero-filled)
// one block per task (segment, 32-row slab); thread per 8-column chunk
// ============================================================================================
__global__ __launch_bounds__(256) void pack_kernel(const PackSeg* __restrict__ segs, int nseg,
                                                   const int* __restrict__ task_seg, const float* __restrict__ src,
                                                   bf16_t* __restrict__ dst) {
  const int seg = task_seg[2 * blockIdx.x];
  const int row0 = task_seg[2 * blockIdx.x + 1];
  const PackSeg S = segs[seg];
  const int chunks = S.dld / 8;
  const int n = 32 * chunks;
  const bool vec = ((S.cols | S.src_off) & 3) == 0;
  // up to PK chunks per thread with every load issued before the first store (the one-chunk-at-a-time
  // loop ran the launch at half the HBM rate: 124 us for 540 MB at the target shape)
  constexpr int PK = 8;
  for (int q0 = threadIdx.x; q0 < n; q0 += 256 * PK) {
    f32x4 lo[PK], hi[PK];
#pragma unroll
    for (int k = 0; k < PK; ++k) {
      const int q = q0 + 256 * k;
      const int r = row0 + q / chunks, c = (q % chunks) * 8;
      lo[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      hi[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < n && r < S.rows) {
        const float* sp = src + S.src_off + (int64_t)r * S.cols;
        if (vec && c + 8 <= S.cols) {  // interior chunk: two 16-B loads
          lo[k] = *reinterpret_cast<const f32x4*>(sp + c);
          hi[k] = *reinterpret_cast<const f32x4*>(sp + c + 4);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            lo[k][e] = (c + e < S.cols) ? sp[c + e] : 0.f;
            hi[k][e] = (c + 4 + e < S.cols) ? sp[c + 4 + e] : 0.f;
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < PK; ++k) {
      const int q = q0 + 256 * k;
      const int r = row0 + q / chunks, c = (q % chunks) * 8;
      if (q < n && r < S.rows)
        *reinterpret_cast<u32x4*>(dst + S.dst_off + (int64_t)r * S.dld + c) =
            u32x4{pack2bf(lo[k][0], lo[k][1]), pack2bf(lo[k][2], lo[k][3]), pack2bf(hi[k][0], hi[k][1]),
                  pack2bf(hi[k][2], hi[k][3])};
    }
  }
}

hipError_t mmt_launch_pack(const PackSeg* segs_dev, int nseg, int64_t ntasks, const int* task_dev, const float* src,
                           bf16_t* dst, hipStream_t s) {
  if (ntasks == 0) return hipSuccess;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)ntasks), dim3(256), 0, s, segs_dev, nseg, task_dev, src, dst);
  return hipGetLastError();
}

__global__ void f2bf_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = f2bf(src[i]);
}
// masked copy (dropout of the consuming branch) with fused column sums, grouped over modalities
__global__ __launch_bounds__(256) void drop_copy_kernel(DropCopyBatch batch, int R, int C) {
  const DropCopyProblem& P = batch.p[blockIdx.z];
  const int C4 = C >> 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int RPI = 4;  // rows per wave per iteration, loads issued together
  __shared__ float red[4][1024];
  const int stride = gridDim.x * 4;
  const f32x4* const src = reinterpret_cast<const f32x4*>(sgpr_ptr(P.src));
  u32x2* const dst = reinterpret_cast<u32x2*>(sgpr_ptr(P.dst));
  const uint32_t dkey = sgpr_u32(P.drop_key), dthr = sgpr_u32(P.drop_thr);
  const float dscale = sgpr_f32(P.drop_scale);
  for (int cb = 0; cb < C4; cb += 64) {
    const int q = cb + lane;
    f32x4 sm = {0.f, 0.f, 0.f, 0.f};
    if (q < C4) {
      for (int row0 = blockIdx.x * 4 + wave; row0 < R; row0 += stride * RPI) {
        f32x4 o[RPI];
#pragma unroll
        for (int u = 0; u < RPI; ++u) {
          const int row = row0 + u * stride;
          o[u] = row < R ? src[(int64_t)row * C4 + q] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < RPI; ++u) {
          const int row = row0 + u * stride;
          if (row >= R) break;
          if (dthr) {
#pragma unroll
            for (int pq = 0; pq < 2; ++pq) {
              const uint32_t hq = mmt_hash(dkey, (uint32_t)row, (uint32_t)(2 * q + pq));
              o[u][2 * pq] = mmt_keep(hq, 0, dthr) ? o[u][2 * pq] * dscale : 0.f;
              o[u][2 * pq + 1] = mmt_keep(hq, 1, dthr) ? o[u][2 * pq + 1] * dscale : 0.f;
            }
          }
          dst[(int64_t)row * C4 + q] =
              u32x2{pack2bf(o[u][0], o[u][1]), pack2bf(o[u][2], o[u][3])};
          sm += o[u];
        }
      }
      *reinterpret_cast<f32x4*>(&red[wave][4 * q]) = sm;
    }
  }
  if (!P.dsum) return;
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) atomicAdd(P.dsum + c, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
}

hipError_t mmt_launch_drop_copy(const DropCopyBatch& b, int R, int C, hipStream_t s) {
  if (C % 4 != 0 || C > 1024) return hipErrorInvalidValue;
  if (b.count == 0 || R == 0) return hipSuccess;
  // one dsum atomic per column per block: cap the blocks (see mmt_launch_ln_bwd)
  int blocks = (R + 15) / 16;
  if (blocks > 256) blocks = 256;
  hipLaunchKernelGGL(drop_copy_kernel, dim3(blocks, 1, b.count), dim3(256), 0, s, b, R, C);
  return hipGetLastError();
}

hipError_t mmt_launch_f32_to_bf16(const float* src, bf16_t* dst, int64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(f2bf_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, dst, n);
  return hipGetLastError();
}

// ============================================================================================
// AdamW (torch.optim.AdamW defaults, decoupled decay; main.py:464, 650):
//   p *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// ============================================================================================
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n4, int64_t n,
                                                    float lr, float b1, float b2, float eps, float wd, float bc1,
                                                    float bc2_sqrt) {
  const float step_size = lr / bc1;
  const float decay = 1.f - lr * wd;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    const f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pp[e] *= decay;
      mm[e] += (gg[e] - mm[e]) * (1.f - b1);
      vv[e] = vv[e] * b2 + (1.f - b2) * gg[e] * gg[e];
      const float denom = sqrtf(vv[e]) / bc2_sqrt + eps;
      pp[e] -= step_size * mm[e] / denom;
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
  }
  // scalar tail
  const int64_t t = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) {
    float pp = p[t] * decay;
    const float gg = g[t];
    float mm = m[t] + (gg - m[t]) * (1.f - b1);
    float vv = v[t] * b2 + (1.f - b2) * gg * gg;
    pp -= step_size * mm / (sqrtf(vv) / bc2_sqrt + eps);
    p[t] = pp; m[t] = mm; v[t] = vv;
  }
}

hipError_t mmt_launch_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                            float eps, float wd, float bc1, float bc2_sqrt, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const int64_t n4 = n / 4;
  int64_t blocks = (n4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v, n4, n, lr, b1, b2, eps, wd,
                     bc1, bc2_sqrt);
  return hipGetLastError();
}

// ============================================================================================
// Directional metric (training_utils.py:215-330) for one numeric modality, one wave per sample
//   pred = vocab[argmax(logits[j, T-1])] (first max wins), act = vocab[y[j,T-1]],
//   prev = vocab[x[j,T-1]] (value data) ; win if sign(pred-prev) == sign(act-prev)
//   (percent data: sign(pred) == sign(act)); certainty = softmax mass of same-sign tokens.
// ============================================================================================
__device__ __forceinline__ int dsign(double cur, double prev, int pct) {
  const double c = pct ? cur : cur - prev;
  return c > 0 ? 1 : (c < 0 ? -1 : 0);
}

__global__ __launch_bounds__(64) void eval_dir_kernel(const float* __restrict__ logits, const int64_t* __restrict__ xb,
                                                      const int64_t* __restrict__ yb, const double* __restrict__ vocab,
                                                      int T, int V, int pct, int* wl, double* cert) {
  const int j = blockIdx.x;
  const int lane = threadIdx.x;
  const float* x = logits + ((int64_t)j * T + (T - 1)) * V;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = lane; v < V; v += 64) {
    const float a = x[v];
    if (a > best || (a == best && v < bi)) { best = a; bi = v; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  const double prev = pct ? 0.0 : vocab[xb[(int64_t)j * T + T - 1]];
  const double pv = vocab[bi], av = vocab[yb[(int64_t)j * T + T - 1]];
  const int ps = dsign(pv, prev, pct), as = dsign(av, prev, pct);
  float m = warp_max(best);
  float sum = 0.f, same = 0.f;
  for (int v = lane; v < V; v += 64) {
    const float e = __expf(x[v] - m);
    sum += e;
    if (dsign(vocab[v], prev, pct) == ps) same += e;
  }
  sum = warp_sum(sum);
  same = warp_sum(same);
  if (lane == 0) {
    atomicAdd(wl + (ps == as ? 0 : 1), 1);
    atomicAdd(cert, (double)(same / sum));
  }
}

hipError_t mmt_launch_eval_direction(const float* logits, const int64_t* xb, const int64_t* yb, const double* vocab,
                                     int B, int T, int V, int is_pct, int* wins_losses, double* certainty,
                                     hipStream_t s) {
  if (B == 0) return hipSuccess;
  hipLaunchKernelGGL(eval_dir_kernel, dim3(B), dim3(64), 0, s, logits, xb, yb, vocab, T, V, is_pct, wins_losses,
                     certainty);
  return hipGetLastError();
}

// ============================================================================================
// MX-fp8 quantisation (mmt_common.h): one thread per (row, 32-column block) of each segment
// ============================================================================================
__device__ __forceinline__ void mx_quant_unit(const MxSeg& S, int64_t u, const float* base, uint8_t* dst) {
  const int nb = S.lds8;  // blocks per row including the padding exponents
  if (u >= (int64_t)S.rows * nb) return;
  const int row = (int)(u / nb), kb = (int)(u % nb);
  uint8_t* sp = dst + S.sdst + (int64_t)row * S.lds8 + kb;
  if (kb * 32 >= S.cols) { *sp = 127; return; }
  const float* src = base + S.src + (int64_t)row * S.ld_src + kb * 32;
  f32x4 v[8];
  float am = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    v[q] = reinterpret_cast<const f32x4*>(src)[q];
    am = fmaxf(am, fmaxf(fmaxf(fabsf(v[q][0]), fabsf(v[q][1])), fmaxf(fabsf(v[q][2]), fabsf(v[q][3]))));
  }
  const int ex = mx_exp(am);
  const float inv = mx_inv(ex);
  u32x4 w[2];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    w[q >> 2][q & 3] = pack4fp8(v[q][0] * inv, v[q][1] * inv, v[q][2] * inv, v[q][3] * inv);
  uint8_t* dp = dst + S.dst + (int64_t)row * S.ld8 + kb * 32;
  reinterpret_cast<u32x4*>(dp)[0] = w[0];
  reinterpret_cast<u32x4*>(dp)[1] = w[1];
  *sp = (uint8_t)(ex + 127);
}

__global__ __launch_bounds__(256) void mx_quant_kernel(const MxSeg* segs, const float* base, uint8_t* dst) {
  mx_quant_unit(segs[blockIdx.y], (int64_t)blockIdx.x * 256 + threadIdx.x, base, dst);
}
__global__ __launch_bounds__(256) void mx_quant1_kernel(MxSeg S, const float* base, uint8_t* dst) {
  mx_quant_unit(S, (int64_t)blockIdx.x * 256 + threadIdx.x, base, dst);
}

hipError_t mmt_launch_mx_quant1(const MxSeg& S, const float* base, uint8_t* dst, hipStream_t s) {
  const int64_t units = (int64_t)S.rows * S.lds8;
  if (units == 0) return hipSuccess;
  hipLaunchKernelGGL(mx_quant1_kernel, dim3((unsigned)((units + 255) / 256)), dim3(256), 0, s, S, base, dst);
  return hipGetLastError();
}

hipError_t mmt_launch_mx_quant(const MxSeg* segs_dev, int nseg, int max_units, const float* base, uint8_t* dst,
                               hipStream_t s) {
  if (nseg == 0 || max_units == 0) return hipSuccess;
  hipLaunchKernelGGL(mx_quant_kernel, dim3((max_units + 255) / 256, nseg), dim3(256), 0, s, segs_dev, base, dst);
  return hipGetLastError();
}
