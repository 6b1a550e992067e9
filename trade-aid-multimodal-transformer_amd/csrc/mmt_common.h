// Shared device-side definitions for the MI355X (gfx950 / CDNA4) multimodal-transformer kernels.
//
// Storage convention: activations and packed weights are bf16 (raw 16-bit storage `bf16_t`),
// accumulation is fp32 (MFMA f32 accumulators), master params / grads / residual stream fp32.
// Every bf16 matrix that feeds an MFMA GEMM has a leading dimension that is a multiple of 8
// elements and a 16-byte aligned base, so operand tiles stage with 16-byte loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // raw bf16 storage
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define MMT_WAVE 64
#define MMT_MAX_GROUP 8

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  return __builtin_bit_cast(bf16_t, b);
}
// two floats -> packed bf16 pair in ONE v_cvt_pk_bf16_f32 (two scalar conversions joined by an OR
// cost three instructions)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// tanh for fp32 epilogues whose result is stored as bf16: exp-based away from 0, odd Taylor
// polynomial near 0 (avoids the 1 - e cancellation); |error| < 2e-7, far below bf16 rounding.
// Branch-free: both forms are computed and selected (a divide here lowered to the IEEE
// v_div_scale / v_div_fmas sequence and turned the select into a divergent branch per element).
// v_rcp_f32 (1 ulp) keeps the error far below the bf16 rounding of the stored result.
__device__ __forceinline__ float fast_tanh(float x) {
  const float ax = fabsf(x);
  const float e = __expf(-2.0f * ax);
  const float t = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
  const float x2 = x * x;
  const float p = x * (1.0f + x2 * (-0.333333343f + x2 * (0.133333340f + x2 * -0.0539682540f)));
  return ax < 0.125f ? p : __builtin_copysignf(t, x);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// LDS transposed read (ds_read_b64_tr_b16): per 16-lane group, 4 rows x 16 columns of 16-bit
// elements; lane 4q+p supplies the address of row q, columns 4p..4p+3; lane i of the group
// receives column i of the 4 rows (row q in element q).
// `lds_addr` must point into a __shared__ array; the explicit cast is an addrspacecast
// (generic -> LDS), never an integer truncation of the flat address.
__device__ __forceinline__ s16x4 lds_tr16(const void* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds_addr));
}

typedef short s16x8 __attribute__((ext_vector_type(8)));
// whole-vector shuffle + bitcast: element-wise scalar bit_casts of the tr16 result were
// mis-lowered by hipcc (ROCm 7.2) into duplicated register halves
__device__ __forceinline__ bf16x8 join4(s16x4 lo, s16x4 hi) {
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// XCD-aware block order (bijective): hardware block ids b and b+8 share an XCD (and its L2);
// give each XCD a contiguous run of logical tiles so neighbouring tiles that read the two halves of
// the same cache lines (adjacent heads / Q-K-V blocks of one row) run on one XCD at nearly the
// same time. Returns the logical tile of hardware block `bid` out of `nwg`.
// Kernel-argument values pinned as wave-uniform VALUES (readfirstlane): read through the kernel-argument
// struct inside a loop, hipcc re-loads them (s_load + an lgkmcnt wait) every iteration instead of keeping
// them in SGPRs
template <class T>
__device__ __forceinline__ T* sgpr_ptr(T* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
// the same, as a global-address-space pointer: sgpr_ptr's integer round trip loses the address space, and
// the compiler then addresses through FLAT instructions (counted against lgkmcnt too, no SGPR base)
#define MMT_AS1 __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ MMT_AS1 T* sgpr_gptr(T* p) {
  return (MMT_AS1 T*)(uintptr_t)sgpr_ptr(p);
}
__device__ __forceinline__ uint32_t sgpr_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ float sgpr_f32(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

__device__ __forceinline__ int xcd_tile(int bid, int nwg) {
  const int x = bid % 8, q = nwg / 8, rr = nwg % 8;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + bid / 8;
}

// dropout keep test: ONE 32-bit hash per column pair (2c, 2c+1) of a row, its 16-bit halves
// compared against a 16-bit threshold thr = floor(p * 65536) (keep probability 1 - thr/65536):
// half the hashing of one hash per element. `h` = mmt_hash(key, row, col >> 1).
__host__ __device__ __forceinline__ bool mmt_keep(uint32_t h, uint32_t col, uint32_t thr) {
  return ((h >> ((col & 1u) << 4)) & 0xFFFFu) >= thr;
}

// counter-based hash RNG (dropout masks); identical in forward and backward, and restated
// bit-for-bit by the host (mmt_engine.hip: drop keys) and by oracle/mmt_oracle.py (mask_hash)
#define MMT_STREAM_SALT 0x5BD1E995u
__host__ __device__ __forceinline__ uint32_t mmt_hash(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
  return h;
}

// attention-probability keep hash (attn_mask_kernel; restated by oracle/mmt_oracle.py probs):
// the (stream key, score row) part is hashed once per row (mmt_hash), each key pair c then costs
// one add of c * golden-ratio (a compile-time offset plus a per-tile base) and a two-multiply
// finaliser — 2 instead of 5 quarter-rate 32-bit multiplies per pair
#define MMT_PROB_ROW_SALT 0x2545F491u
__host__ __device__ __forceinline__ uint32_t mmt_prob_row(uint32_t stream_key, uint32_t row) {
  return mmt_hash(stream_key, row, MMT_PROB_ROW_SALT);
}
// the finaliser alone: mmt_prob_hash(rh, c) == mmt_prob_fin(rh + c * 0x9E3779B9u) (wrapping arithmetic, so a
// kernel may add a per-tile base and compile-time pair offsets separately)
__host__ __device__ __forceinline__ uint32_t mmt_prob_fin(uint32_t h) {
  h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
  return h;
}
__host__ __device__ __forceinline__ uint32_t mmt_prob_hash(uint32_t row_hash, uint32_t c) {
  return mmt_prob_fin(row_hash + c * 0x9E3779B9u);
}

// ---------------------------------------------------------------------------------------------
// MX-fp8 (OCP e4m3fn values, E8M0 block exponents over 32 consecutive K elements): the operand
// format of v_mfma_scale_f32_32x32x64_f8f6f4 (C4's fp8 path). A 32-element block with absolute
// max `amax` gets the smallest exponent e with amax / 2^e <= 448 (no clipping: every value stays
// finite in e4m3fn, whose conversion does not saturate), stored as the byte e + 127; its values
// are fp8(x * 2^-e) (round to nearest even, v_cvt_pk_fp8_f32). The oracle restates this exactly
// (oracle/mmt_oracle.py mx_fp8).
// ---------------------------------------------------------------------------------------------
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ int mx_exp(float amax) {
  if (!(amax > 0.f)) return -127;
  const uint32_t u = __float_as_uint(amax * (1.0f / 448.0f));
  int e = (int)((u >> 23) & 0xff) - 127;
  if (u & 0x7fffffu) ++e;  // ceil(log2) unless a power of two (denormal quotients: e = -127 or -126)
  return e < -127 ? -127 : (e > 126 ? 126 : e);
}
// 2^-e for e in [-127, 126]
__device__ __forceinline__ float mx_inv(int e) { return __uint_as_float((uint32_t)(127 - e) << 23); }
// four floats (already multiplied by 2^-e) -> four e4m3fn bytes, element 0 in the low byte
__device__ __forceinline__ uint32_t pack4fp8(float a, float b, float c, float d) {
  uint32_t w = 0;
  w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, w, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return w;
}
