// bf16 MFMA GEMM for gfx950 with fused epilogues (forward linear, backward data, weight grad).
//
// Tile 128x128x32, 256 threads = 4 waves (2x2), each wave a 64x64 sub-tile as 2x2
// v_mfma_f32_32x32x16_bf16 accumulators. Operand tiles are register-staged (16-B global loads)
// into double-buffered LDS images, one barrier per K-step:
//   K-contiguous operand  -> image [128 rows][32 k], 64-B rows, 16-B chunk XOR swizzle
//                            (chunk ^= (row>>2)&3), fragments by ds_read_b128 (conflict-free)
//   MN-contiguous operand -> image [32 k][128 (+32 pad)], 320-B rows,
//                            fragments by ds_read_b64_tr_b16 (hardware transpose, conflict-free)
// SWAP=true computes C^T tiles (N on accumulator rows, M on lanes) so each lane owns one output
// row and 4 consecutive columns per register group: 8/16-B vector epilogue stores.
// SWAP=false keeps N on lanes: 32 lanes hit 128 contiguous bytes of one row, the shape fp32
// atomics need (weight-grad split-K accumulate).
#include "mmt_common.h"
#include "mmt_kernels.h"

#define GBM 128
#define GBN 128
#define GBK 32
#define KC_ROWB 64
#define MN_ROWB 320
#define IMG_BYTES 10240

template <bool KC>
__device__ __forceinline__ void stage_load(const bf16_t* __restrict__ base, int ld, int rows_total, int K, int r0,
                                           int k0, u32x4 (&reg)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    int row, kk;
    if (KC) { row = c >> 2; kk = (c & 3) * 8; } else { kk = c >> 4; row = (c & 15) * 8; }
    const int grow = r0 + row, gk = k0 + kk;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (KC) {
      if (grow < rows_total) {
        const bf16_t* src = base + (int64_t)grow * ld + gk;
        if (gk + 8 <= K) {
          v = *reinterpret_cast<const u32x4*>(src);
        } else if (gk < K) {
          uint16_t e[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (gk + t < K) ? src[t] : (uint16_t)0;
          v = {e[0] | ((uint32_t)e[1] << 16), e[2] | ((uint32_t)e[3] << 16), e[4] | ((uint32_t)e[5] << 16),
               e[6] | ((uint32_t)e[7] << 16)};
        }
      }
    } else {
      if (gk < K) {
        const bf16_t* src = base + (int64_t)gk * ld + grow;
        if (grow + 8 <= rows_total) {
          v = *reinterpret_cast<const u32x4*>(src);
        } else if (grow < rows_total) {
          uint16_t e[8];
#pragma unroll
          for (int t = 0; t < 8; ++t) e[t] = (grow + t < rows_total) ? src[t] : (uint16_t)0;
          v = {e[0] | ((uint32_t)e[1] << 16), e[2] | ((uint32_t)e[3] << 16), e[4] | ((uint32_t)e[5] << 16),
               e[6] | ((uint32_t)e[7] << 16)};
        }
      }
    }
    reg[i] = v;
  }
}

template <bool KC>
__device__ __forceinline__ void stage_store(char* img, const u32x4 (&reg)[2], int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i;
    int off;
    if (KC) {
      const int row = c >> 2, ch = c & 3;
      off = row * KC_ROWB + ((ch ^ ((row >> 2) & 3)) << 4);
    } else {
      const int kk = c >> 4, mc = c & 15;
      off = kk * MN_ROWB + mc * 16;
    }
    *reinterpret_cast<u32x4*>(img + off) = reg[i];
  }
}

// fragment for "lane row = sb + (lane&31), k = 16*s + 8*(lane>>5) + j"
template <bool KC>
__device__ __forceinline__ bf16x8 frag(const char* img, int sb, int s, int lane) {
  if (KC) {
    const int row = sb + (lane & 31);
    const int ch = 2 * s + (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(img + row * KC_ROWB + ((ch ^ ((row >> 2) & 3)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15;
    const int q = i >> 2, p = i & 3;
    const int col = sb + 16 * (g & 1) + 4 * p;
    const int kr = 16 * s + 8 * (g >> 1) + q;
    s16x4 lo = lds_tr16(img + kr * MN_ROWB + col * 2);
    s16x4 hi = lds_tr16(img + (kr + 4) * MN_ROWB + col * 2);
    return join4(lo, hi);
  }
}

template <int EPI>
__device__ __forceinline__ void epi_vec4(const GemmProblem& P, float alpha, int m, int n, const float (&v)[4]) {
  // n..n+3 all < N (checked by caller), m < M
  const int64_t o = (int64_t)m * P.ldc + n;
  float r[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = alpha * v[e];
  if (EPI == EPI_BIAS_TANH_BF16 || EPI == EPI_BIAS_RELU_BF16 || EPI == EPI_BIAS_RESID_F32 ||
      EPI == EPI_STORE_F32 || EPI == EPI_STORE_BF16) {
    if (P.bias) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(P.bias + n);
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] += b[e];
    }
  }
  if (EPI == EPI_BIAS_TANH_BF16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = tanhf(r[e]);
  }
  if (EPI == EPI_BIAS_RELU_BF16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = fmaxf(r[e], 0.0f);
  }
  if (EPI == EPI_DTANH_BF16 || EPI == EPI_DRELU_BF16) {
    const u32x2 a = *reinterpret_cast<const u32x2*>(P.aux + (int64_t)m * P.ldaux + n);
    const float t[4] = {bf2f(a[0] & 0xffff), bf2f(a[0] >> 16), bf2f(a[1] & 0xffff), bf2f(a[1] >> 16)};
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = (EPI == EPI_DTANH_BF16) ? r[e] * (1.0f - t[e] * t[e]) : (t[e] > 0.0f ? r[e] : 0.0f);
  }
  if (EPI == EPI_BIAS_RESID_F32) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(P.resid + (int64_t)m * P.ldres + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] += x[e];
  }
  if (EPI == EPI_ACC_F32) {
    f32x4* dst = reinterpret_cast<f32x4*>(P.o32 + o);
    f32x4 x = *dst;
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] += r[e];
    *dst = x;
    return;
  }
  if (EPI == EPI_BIAS_RESID_F32 || EPI == EPI_STORE_F32) {
    *reinterpret_cast<f32x4*>(P.o32 + o) = f32x4{r[0], r[1], r[2], r[3]};
    if (EPI == EPI_BIAS_RESID_F32 && P.o16)
      *reinterpret_cast<u32x2*>(P.o16 + (int64_t)m * P.ldo16 + n) = u32x2{pack2bf(r[0], r[1]), pack2bf(r[2], r[3])};
    return;
  }
  // bf16 outputs
  *reinterpret_cast<u32x2*>(P.o16 + (int64_t)m * P.ldo16 + n) = u32x2{pack2bf(r[0], r[1]), pack2bf(r[2], r[3])};
}

template <int EPI>
__device__ __forceinline__ void epi_scalar(const GemmProblem& P, float alpha, int m, int n, float v) {
  float r = alpha * v;
  if (EPI == EPI_BIAS_TANH_BF16 || EPI == EPI_BIAS_RELU_BF16 || EPI == EPI_BIAS_RESID_F32 ||
      EPI == EPI_STORE_F32 || EPI == EPI_STORE_BF16) {
    if (P.bias) r += P.bias[n];
  }
  if (EPI == EPI_BIAS_TANH_BF16) r = tanhf(r);
  if (EPI == EPI_BIAS_RELU_BF16) r = fmaxf(r, 0.0f);
  if (EPI == EPI_DTANH_BF16) { const float t = bf2f(P.aux[(int64_t)m * P.ldaux + n]); r *= (1.0f - t * t); }
  if (EPI == EPI_DRELU_BF16) { const float t = bf2f(P.aux[(int64_t)m * P.ldaux + n]); r = t > 0.0f ? r : 0.0f; }
  if (EPI == EPI_BIAS_RESID_F32) r += P.resid[(int64_t)m * P.ldres + n];
  const int64_t o = (int64_t)m * P.ldc + n;
  if (EPI == EPI_ACC_F32) { P.o32[o] += r; return; }
  if (EPI == EPI_ATOMIC_F32) { atomicAdd(P.o32 + o, r); return; }
  if (EPI == EPI_BIAS_RESID_F32 || EPI == EPI_STORE_F32) {
    P.o32[o] = r;
    if (EPI == EPI_BIAS_RESID_F32 && P.o16) P.o16[(int64_t)m * P.ldo16 + n] = f2bf(r);
    return;
  }
  P.o16[(int64_t)m * P.ldo16 + n] = f2bf(r);
}

template <bool A_KC, bool B_KC, bool SWAP, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(GemmBatch batch) {
  const GemmProblem& P = batch.p[blockIdx.z];
  const int M = P.M, N = P.N, K = P.K;
  const int tiles_n = (N + GBN - 1) / GBN;
  const int tiles_m = (M + GBM - 1) / GBM;
  const int tile = blockIdx.x;
  if (tile >= tiles_m * tiles_n) return;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int nsplit = gridDim.y;
  const int ksteps = (K + GBK - 1) / GBK;
  const int kper = (ksteps + nsplit - 1) / nsplit;
  const int ks0 = blockIdx.y * kper;
  const int ks1 = min(ksteps, ks0 + kper);
  if (EPI == EPI_ATOMIC_F32 && ks0 >= ks1) return;  // nothing to add

  __shared__ __attribute__((aligned(16))) char lds[4 * IMG_BYTES];
#define IMG_A(b) (lds + (b) * IMG_BYTES)
#define IMG_B(b) (lds + (2 + (b)) * IMG_BYTES)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;

  if (ks0 < ks1) {
    u32x4 ra[2], rb[2];
    stage_load<A_KC>(P.A, P.lda, M, K, m0, ks0 * GBK, ra, tid);
    stage_load<B_KC>(P.B, P.ldb, N, K, n0, ks0 * GBK, rb, tid);
    stage_store<A_KC>(IMG_A(0), ra, tid);
    stage_store<B_KC>(IMG_B(0), rb, tid);
    __syncthreads();
    for (int ks = ks0; ks < ks1; ++ks) {
      const int cur = (ks - ks0) & 1;
      const bool more = ks + 1 < ks1;
      if (more) {
        stage_load<A_KC>(P.A, P.lda, M, K, m0, (ks + 1) * GBK, ra, tid);
        stage_load<B_KC>(P.B, P.ldb, N, K, n0, (ks + 1) * GBK, rb, tid);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 fa[2], fb[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) fa[j] = frag<A_KC>(IMG_A(cur), wm * 64 + 32 * j, s, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i) fb[i] = frag<B_KC>(IMG_B(cur), wn * 64 + 32 * i, s, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (SWAP) acc[i][j] = mfma32(fb[i], fa[j], acc[i][j]);
            else acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
          }
      }
      if (more) {
        stage_store<A_KC>(IMG_A(cur ^ 1), ra, tid);
        stage_store<B_KC>(IMG_B(cur ^ 1), rb, tid);
      }
      __syncthreads();
    }
  }

  float alpha = P.alpha;
  if (P.alpha_ptr) alpha *= *P.alpha_ptr;
  const int h = lane >> 5, r = lane & 31;
  // 16-B (f32) / 8-B (bf16) vector epilogue needs every leading dimension to keep 4-column
  // groups aligned; bias pointers are 64-B aligned by the parameter layout.
  const bool vec_ok = ((P.ldc | P.ldres | P.ldo16 | P.ldaux) & 3) == 0;
  if (SWAP) {
    // acc[i][j]: rows = n (sub-tile i), cols = m (sub-tile j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = m0 + wm * 64 + 32 * j + r;
        if (m >= M) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = n0 + wn * 64 + 32 * i + 8 * g + 4 * h;
          const float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
          if (n + 4 <= N && vec_ok && EPI != EPI_ATOMIC_F32) {
            epi_vec4<EPI>(P, alpha, m, n, v);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < N) epi_scalar<EPI>(P, alpha, m, n + e, v[e]);
          }
        }
      }
  } else {
    // acc[i][j]: rows = m (sub-tile i), cols = n (sub-tile j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + 32 * j + r;
        if (n >= N) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wm * 64 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (m < M) epi_scalar<EPI>(P, alpha, m, n, acc[i][j][e]);
        }
      }
  }
}

template <bool A_KC, bool B_KC, bool SWAP, int EPI>
static hipError_t launch_t(const GemmBatch& b, int splits, hipStream_t s) {
  int maxtiles = 0;
  for (int g = 0; g < b.count; ++g) {
    const GemmProblem& P = b.p[g];
    const int t = ((P.M + GBM - 1) / GBM) * ((P.N + GBN - 1) / GBN);
    if (t > maxtiles) maxtiles = t;
  }
  if (maxtiles == 0 || b.count == 0) return hipSuccess;
  dim3 grid(maxtiles, splits, b.count);
  hipLaunchKernelGGL((gemm_kernel<A_KC, B_KC, SWAP, EPI>), grid, dim3(256), 0, s, b);
  return hipGetLastError();
}

hipError_t mmt_launch_gemm(const GemmBatch& b, bool a_kc, bool b_kc, int epi, int splits, hipStream_t s) {
  if (splits < 1) splits = 1;
  if (a_kc && b_kc) {
    switch (epi) {
      case EPI_STORE_BF16: return launch_t<true, true, true, EPI_STORE_BF16>(b, 1, s);
      case EPI_BIAS_TANH_BF16: return launch_t<true, true, true, EPI_BIAS_TANH_BF16>(b, 1, s);
      case EPI_BIAS_RELU_BF16: return launch_t<true, true, true, EPI_BIAS_RELU_BF16>(b, 1, s);
      case EPI_BIAS_RESID_F32: return launch_t<true, true, true, EPI_BIAS_RESID_F32>(b, 1, s);
      case EPI_STORE_F32: return launch_t<true, true, true, EPI_STORE_F32>(b, 1, s);
      case EPI_ACC_F32: return launch_t<true, true, true, EPI_ACC_F32>(b, 1, s);
      default: break;
    }
  } else if (a_kc && !b_kc) {
    switch (epi) {
      case EPI_STORE_BF16: return launch_t<true, false, true, EPI_STORE_BF16>(b, 1, s);
      case EPI_DTANH_BF16: return launch_t<true, false, true, EPI_DTANH_BF16>(b, 1, s);
      case EPI_DRELU_BF16: return launch_t<true, false, true, EPI_DRELU_BF16>(b, 1, s);
      case EPI_STORE_F32: return launch_t<true, false, true, EPI_STORE_F32>(b, 1, s);
      case EPI_ACC_F32: return launch_t<true, false, true, EPI_ACC_F32>(b, 1, s);
      default: break;
    }
  } else if (!a_kc && !b_kc) {
    switch (epi) {
      case EPI_ATOMIC_F32: return launch_t<false, false, false, EPI_ATOMIC_F32>(b, splits, s);
      case EPI_STORE_F32: return launch_t<false, false, true, EPI_STORE_F32>(b, 1, s);
      default: break;
    }
  } else {
    switch (epi) {
      case EPI_ATOMIC_F32: return launch_t<false, true, false, EPI_ATOMIC_F32>(b, splits, s);
      case EPI_STORE_F32: return launch_t<false, true, true, EPI_STORE_F32>(b, 1, s);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}
