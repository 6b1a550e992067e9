// KV-cache decode attention for generate (reference model.py:404-446): ONE new query position t
// per sequence attends over the cached keys / values of positions 0..t (causal: itself included),
// one independent softmax per KV stream, the per-stream outputs summed (cross-attention,
// model.py:141-158). The cache is the forward's own saved Q/K/V (and cross K/V) layout: row
// b*T + s of a [B*T, ld] bf16 matrix, head h at column h*kv_hstride.
//
// One 256-thread workgroup per (sequence, head, problem). Phase 1: threads over keys, dot products
// of hs bf16 (16-B loads) into an LDS score row, block max / sum; phase 2: four 64-lane groups over
// keys (s = g mod 4), lane d accumulates p_s v[s][d] (one 128-B row segment per wave instruction),
// the groups are summed through LDS. Memory-bound: each K / V row of the window is read once.
#include "mmt_common.h"
#include "mmt_kernels.h"

namespace {

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o, 64);
    v = is_max ? fmaxf(v, u) : v + u;
  }
  __syncthreads();  // red[] free (a previous reduction's readers are done)
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  return r;
}

}  // namespace

template <int HS>
__global__ __launch_bounds__(256) void attn_decode_kernel(DecodeAttnBatch batch, int t, int T, int H, float scale) {
  const DecodeAttnProblem& P = batch.p[blockIdx.z];
  const int bh = blockIdx.x, b = bh / H, head = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
  extern __shared__ float sm[];  // [T] scores, then [4][64] partial outputs, [4] reductions
  float* sc = sm;
  float* part = sm + T;
  float* red = part + 4 * 64;
  const int n = t + 1;
  // the query row in fp32 registers (every thread reads the same 2*HS bytes: one broadcast line)
  float q[HS];
  const bf16_t* qp = P.q + (int64_t)b * P.q_ld + head * HS;
#pragma unroll
  for (int c = 0; c < HS / 8; ++c) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(qp + 8 * c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      q[8 * c + 2 * e] = bf2f(v[e] & 0xffff) * scale;
      q[8 * c + 2 * e + 1] = bf2f(v[e] >> 16) * scale;
    }
  }
  float o = 0.f;  // lane d < HS of group g: output dim d, summed over the streams
  for (int j = 0; j < P.nstreams; ++j) {
    const bf16_t* kb = P.k[j] + (int64_t)b * T * P.kv_ld + head * P.kv_hstride;
    const bf16_t* vb = P.v[j] + (int64_t)b * T * P.kv_ld + head * P.kv_hstride;
    float mx = -INFINITY;
    for (int s = tid; s < n; s += 256) {
      const bf16_t* kr = kb + (int64_t)s * P.kv_ld;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < HS / 8; ++c) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(kr + 8 * c);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc += q[8 * c + 2 * e] * bf2f(v[e] & 0xffff) + q[8 * c + 2 * e + 1] * bf2f(v[e] >> 16);
      }
      sc[s] = acc;
      mx = fmaxf(mx, acc);
    }
    mx = block_reduce(mx, red, true);
    float sum = 0.f;
    for (int s = tid; s < n; s += 256) {
      const float p = __expf(sc[s] - mx);
      sc[s] = p;
      sum += p;
    }
    sum = block_reduce(sum, red, false);  // (its barriers also publish sc[])
    float acc = 0.f;
    if (lane < HS)
      for (int s = g; s < n; s += 4) acc += sc[s] * bf2f(vb[(int64_t)s * P.kv_ld + lane]);
    part[g * 64 + lane] = acc;
    __syncthreads();
    if (g == 0 && lane < HS) o += (part[lane] + part[64 + lane] + part[128 + lane] + part[192 + lane]) / sum;
    __syncthreads();  // sc[] / part[] reused by the next stream
  }
  if (g == 0 && lane < HS) P.o[(int64_t)b * P.o_ld + head * HS + lane] = f2bf(o);
}

hipError_t mmt_launch_attn_decode(const DecodeAttnBatch& b, int B, int t, int T, int H, int hs, float scale,
                                  hipStream_t s) {
  if (b.count == 0) return hipSuccess;
  if (t < 0 || t >= T) return hipErrorInvalidValue;
  const dim3 grid(B * H, 1, b.count);
  const size_t lds = sizeof(float) * ((size_t)T + 4 * 64 + 4);
  switch (hs) {
    case 8: hipLaunchKernelGGL(attn_decode_kernel<8>, grid, dim3(256), lds, s, b, t, T, H, scale); break;
    case 16: hipLaunchKernelGGL(attn_decode_kernel<16>, grid, dim3(256), lds, s, b, t, T, H, scale); break;
    case 24: hipLaunchKernelGGL(attn_decode_kernel<24>, grid, dim3(256), lds, s, b, t, T, H, scale); break;
    case 32: hipLaunchKernelGGL(attn_decode_kernel<32>, grid, dim3(256), lds, s, b, t, T, H, scale); break;
    case 48: hipLaunchKernelGGL(attn_decode_kernel<48>, grid, dim3(256), lds, s, b, t, T, H, scale); break;
    case 64: hipLaunchKernelGGL(attn_decode_kernel<64>, grid, dim3(256), lds, s, b, t, T, H, scale); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
