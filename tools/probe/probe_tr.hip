#include <hip/hip_runtime.h>
#include <stdint.h>
typedef short s16x4 __attribute__((ext_vector_type(4)));
// LDS holds a [16 rows][64 cols] u16 image with value row*64+col.
// Each lane supplies the address given by (row_of_lane[lane], col_of_lane[lane]); writes its 4 results.
__global__ void k(const int* rows, const int* cols, int16_t* out) {
  __shared__ __attribute__((aligned(16))) int16_t img[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) img[i] = (int16_t)i;
  __syncthreads();
  const int l = threadIdx.x;
  s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(img + rows[l] * 64 + cols[l]));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = r[e];
}
extern "C" int probe_tr(const int* rows, const int* cols, int16_t* out, void* s) {
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, (hipStream_t)s, rows, cols, out);
  return (int)hipGetLastError();
}
