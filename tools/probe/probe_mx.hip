// Dev probe (not product): semantics of v_mfma_scale_f32_32x32x64_f8f6f4 (operand k layout, E8M0
// scale byte / block mapping) and of v_cvt_pk_fp8_f32 (OCP e4m3 encoding) on gfx950.
#include <hip/hip_runtime.h>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
__global__ void mx_k(const v8i* a, const v8i* b, const int* sa, const int* sb, v16f* d) {
  const int l = threadIdx.x;
  v16f c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], c, 0, 0, 0, sa[l], 0, sb[l]);
  d[l] = c;
}
__global__ void cvt_k(const float* x, unsigned* y, int n) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n) return;
  unsigned w = 0;
  w = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * l], x[4 * l + 1], w, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * l + 2], x[4 * l + 3], w, true);
  y[l] = w;
}
extern "C" int probe_mx(const void* a, const void* b, const int* sa, const int* sb, float* d) {
  hipLaunchKernelGGL(mx_k, dim3(1), dim3(64), 0, 0, (const v8i*)a, (const v8i*)b, sa, sb, (v16f*)d);
  return hipDeviceSynchronize();
}
extern "C" int probe_cvt(const float* x, unsigned* y, int n) {
  hipLaunchKernelGGL(cvt_k, dim3((n + 255) / 256), dim3(256), 0, 0, x, y, n);
  return hipDeviceSynchronize();
}
