// Device-resident batcher: the reference get_batch (training_utils.py:333-384) for token streams
// kept in HBM, so a training step needs no host work and no PCIe transfer.
//   jitter   data_utils.py:342-351 (reached through training_utils.py:350-360): in-place
//            x += uniform{0, +-1 .. +-r} where r < x < V - r, on the whole training stream
//   indices  generate_batch_starting_indices (training_utils.py:33-181): uniform over the valid
//            start positions of the split, mapped to (file, position) by binary search
//   gather   x = data[i : i+T], y = data[i+1 : i+T+1] for every modality with the same indices
// Randomness comes from a counter-based hash (seed, counter, element), not Python's `random`
// or torch's CPU generator: the batches are identically distributed, not bit-identical.
#include "mmt_common.h"
#include "mmt.h"

__global__ __launch_bounds__(256) void jitter_kernel(int32_t* __restrict__ data, int64_t n, int r, int V,
                                                     uint32_t s0, uint32_t s1, uint32_t ctr) {
  const int lo = r, hi = V - r;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int x = data[i];
    if (x > lo && x < hi) {
      const uint32_t h = mmt_hash(s0 ^ (uint32_t)(i >> 32), s1 + ctr, (uint32_t)i);
      const int c = (int)(((uint64_t)h * (uint64_t)(2 * r + 1)) >> 32);  // 0 .. 2r
      const int d = (c == 0) ? 0 : ((c & 1) ? (c + 1) / 2 : -(c / 2));
      data[i] = x + d;
    }
  }
}

__global__ void indices_kernel(int batch, const int64_t* __restrict__ cum_valid, const int64_t* __restrict__ fstart,
                               int nfiles, int off, uint32_t s0, uint32_t s1, uint32_t ctr, int64_t* __restrict__ ix) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const int64_t total = cum_valid[nfiles - 1];
  const uint64_t h = ((uint64_t)mmt_hash(s0, s1 + ctr, 2 * b) << 32) | mmt_hash(s0 + 1, s1 + ctr, 2 * b + 1);
  const int64_t u = (int64_t)(h % (uint64_t)total);
  int lo = 0, hi = nfiles - 1;  // first file with cum_valid > u
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cum_valid[mid] > u) hi = mid; else lo = mid + 1;
  }
  const int64_t before = lo ? cum_valid[lo - 1] : 0;
  ix[b] = fstart[lo] + (u - before) + off;
}

struct GatherArgs {
  const int32_t* data[MMT_MAX_MODALITIES];
  int64_t* x[MMT_MAX_MODALITIES];
  int64_t* y[MMT_MAX_MODALITIES];
};

__global__ __launch_bounds__(256) void gather_kernel(GatherArgs a, const int64_t* __restrict__ ix, int batch, int T) {
  const int m = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)batch * T) return;
  const int b = (int)(i / T), t = (int)(i % T);
  const int64_t s = ix[b] + t;
  a.x[m][i] = a.data[m][s];
  a.y[m][i] = a.data[m][s + 1];
}

extern "C" {

int mmt_batch_jitter(void* stream, int32_t* data, int64_t n, int32_t rand_size, int32_t vocab_size, uint64_t seed,
                     uint64_t counter) {
  if (!data || n < 0 || rand_size < 1 || rand_size > 3 || vocab_size < 1) return MMT_ERR_INVALID;
  if (n == 0) return MMT_OK;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(jitter_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, data, n, rand_size,
                     vocab_size, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)counter);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_ERR_HIP;
}

int mmt_batch_indices(void* stream, int32_t batch, const int64_t* cum_valid, const int64_t* file_start, int32_t nfiles,
                      int32_t first_offset, uint64_t seed, uint64_t counter, int64_t* ix) {
  if (batch < 1 || nfiles < 1 || !cum_valid || !file_start || !ix) return MMT_ERR_INVALID;
  hipLaunchKernelGGL(indices_kernel, dim3((batch + 63) / 64), dim3(64), 0, (hipStream_t)stream, batch, cum_valid,
                     file_start, nfiles, first_offset, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)counter, ix);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_ERR_HIP;
}

int mmt_batch_gather(void* stream, int32_t nmod, const int32_t* const* data, const int64_t* ix, int32_t batch,
                     int32_t T, int64_t* const* x, int64_t* const* y) {
  if (nmod < 1 || nmod > MMT_MAX_MODALITIES || batch < 1 || T < 1) return MMT_ERR_INVALID;
  GatherArgs a{};
  for (int m = 0; m < nmod; ++m) { a.data[m] = data[m]; a.x[m] = x[m]; a.y[m] = y[m]; }
  const int64_t n = (int64_t)batch * T;
  hipLaunchKernelGGL(gather_kernel, dim3((unsigned)((n + 255) / 256), nmod), dim3(256), 0, (hipStream_t)stream, a, ix,
                     batch, T);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_ERR_HIP;
}

}  // extern "C"
