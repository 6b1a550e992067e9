// Device-resident batcher: the reference get_batch (training_utils.py:333-384) for token streams
// kept in HBM, so a training step needs no host work and no PCIe transfer.
//   jitter   data_utils.py:342-351 (reached through training_utils.py:350-360): in-place
//            x += uniform{0, +-1 .. +-r} where r < x < V - r, on the whole training stream
//   indices  generate_batch_starting_indices (training_utils.py:33-181): uniform over the valid
//            start positions of the split, mapped to (file, position) by binary search
//   gather   x = data[i : i+T], y = data[i+1 : i+T+1] for every modality with the same indices
// Randomness comes from a counter-based hash (seed, counter, element), not Python's `random`
// or torch's CPU generator: the batches are identically distributed, not bit-identical.
//
// Exact walk (mmt_exact_gen / mmt_exact_walk): the same random walk, bit-identical to the
// reference's Python loop AND to its consumption of Python's global `random` stream, on the device.
// CPython's random is MT19937; random.choice(rand_list) is rand_list[_randbelow(2r + 1)], and
// _randbelow(n) draws getrandbits(k) = genrand_uint32() >> (32 - k) (k = n.bit_length()) until the
// value is < n. So the eligible elements (r < x < V - r before the pass), stream by stream and in
// index order, take the accepted words of ONE MT19937 sequence in order. mmt_exact_gen runs the
// generator (one workgroup, the 624-word twist in three data-parallel phases) from the state
// CPython's random.getstate() holds; mmt_exact_walk turns accept flags and eligibility flags into
// ordinals (prefix sums), gives the o-th eligible element the o-th accepted word, and moves the
// device copy of the generator state to just past the last word the reference loop would draw.
#include <hipcub/hipcub.hpp>

#include <algorithm>

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

// ---------------------------------------------------------------------------------------------
// exact walk: MT19937 as CPython's random (Modules/_randommodule.c genrand_uint32)
// ---------------------------------------------------------------------------------------------
namespace {
constexpr int MT_N = 624, MT_M = 397;
constexpr uint32_t MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu, MT_A = 0x9908b0dfu;
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & MT_UPPER) | (b & MT_LOWER);
  return c ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
}
// words buffer blocks for a stream of `nwords` words from a state at any position (<= 624)
inline int64_t mt_blocks(int64_t nwords) { return (MT_N + nwords + MT_N - 1) / MT_N + 1; }
}  // namespace

// buf block 0 = the state's key (untempered), blocks 1.. = successive twists; stream word s of the
// state (position p0 = state[624]) is temper(buf[p0 + s])
__global__ __launch_bounds__(256) void mt_gen_kernel(const uint32_t* __restrict__ state, uint32_t* __restrict__ buf,
                                                     int nblk) {
  __shared__ uint32_t mt[MT_N];
  const int i = threadIdx.x;
  for (int t = i; t < MT_N; t += 256) {
    mt[t] = state[t];
    buf[t] = state[t];
  }
  __syncthreads();
  for (int b = 1; b < nblk; ++b) {
    // CPython's twist, kk = 0..622 then 623, in three data-parallel phases: [0, 227) reads only old
    // words, [227, 454) reads new words kk - 227 of phase 1, [454, 624) new words of phase 2 (and
    // the new mt[0] for kk = 623)
    uint32_t v = 0;
    if (i < MT_N - MT_M) v = mt_mix(mt[i], mt[i + 1], mt[i + MT_M]);
    __syncthreads();
    if (i < MT_N - MT_M) mt[i] = v;
    __syncthreads();
    const int k2 = MT_N - MT_M + i;  // 227 + i
    if (i < MT_N - MT_M) v = mt_mix(mt[k2], mt[k2 + 1], mt[k2 - (MT_N - MT_M)]);
    __syncthreads();
    if (i < MT_N - MT_M) mt[k2] = v;
    __syncthreads();
    const int k3 = 2 * (MT_N - MT_M) + i;  // 454 + i
    if (k3 < MT_N) v = mt_mix(mt[k3], mt[(k3 + 1) % MT_N], mt[k3 - (MT_N - MT_M)]);
    __syncthreads();
    if (k3 < MT_N) mt[k3] = v;
    __syncthreads();
    for (int t = i; t < MT_N; t += 256) buf[(int64_t)b * MT_N + t] = mt[t];
  }
}

// accept flags over stream words [0, W): word t accepted for this pass iff t >= cursor and
// getrandbits(k) < n
__global__ __launch_bounds__(256) void mt_accept_kernel(const uint32_t* __restrict__ buf, const uint32_t* __restrict__ state,
                                                        int64_t W, const int64_t* __restrict__ cursor, int k, int n,
                                                        int32_t* __restrict__ flags) {
  const int64_t c = *cursor;
  const uint32_t p0 = state[MT_N];
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < W; t += (int64_t)gridDim.x * 256)
    flags[t] = (t >= c && (int)(mt_temper(buf[p0 + t]) >> (32 - k)) < n) ? 1 : 0;
}
__global__ __launch_bounds__(256) void mt_compact_kernel(const uint32_t* __restrict__ buf, const uint32_t* __restrict__ state,
                                                         int64_t W, int k, const int32_t* __restrict__ flags,
                                                         const int32_t* __restrict__ ord, uint8_t* __restrict__ acc_val,
                                                         int32_t* __restrict__ acc_pos) {
  const uint32_t p0 = state[MT_N];
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < W; t += (int64_t)gridDim.x * 256)
    if (flags[t]) {
      acc_val[ord[t]] = (uint8_t)(mt_temper(buf[p0 + t]) >> (32 - k));
      acc_pos[ord[t]] = (int32_t)t;
    }
}
__global__ __launch_bounds__(256) void walk_elig_kernel(const int32_t* __restrict__ data, int64_t n, int r, int V,
                                                        int32_t* __restrict__ flags) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int x = data[i];
    flags[i] = (x > r && x < V - r) ? 1 : 0;
  }
}
// rand_list of data_utils.py:342-345: [0, 1, -1, 2, -2, 3, -3][:2r+1]
__global__ __launch_bounds__(256) void walk_update_kernel(int32_t* __restrict__ data, int64_t n,
                                                          const int32_t* __restrict__ eflags, const int32_t* __restrict__ eord,
                                                          const uint8_t* __restrict__ acc_val, const int32_t* __restrict__ aord,
                                                          const int32_t* __restrict__ aflags, int64_t W) {
  const int64_t navail = (int64_t)aord[W - 1] + aflags[W - 1];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    if (eflags[i] && eord[i] < navail) {
      const int c = acc_val[eord[i]];
      data[i] += (c == 0) ? 0 : ((c & 1) ? (c + 1) / 2 : -(c / 2));
    }
}
// the pass's last draw: cursor = position of the m-th accepted word + 1 (status 1: the generated
// words ran out, the walk is incomplete)
__global__ void walk_cursor_kernel(int64_t n, const int32_t* __restrict__ eflags, const int32_t* __restrict__ eord,
                                   const int32_t* __restrict__ aflags, const int32_t* __restrict__ aord,
                                   const int32_t* __restrict__ acc_pos, int64_t W, int64_t* __restrict__ cursor,
                                   int32_t* __restrict__ status) {
  const int64_t m = (int64_t)eord[n - 1] + eflags[n - 1];
  const int64_t navail = (int64_t)aord[W - 1] + aflags[W - 1];
  if (m > navail) { *status = 1; return; }
  if (m > 0) *cursor = (int64_t)acc_pos[m - 1] + 1;
}
// the device state after the passes: CPython's (key, index) just past the last drawn word
__global__ __launch_bounds__(256) void mt_state_kernel(uint32_t* __restrict__ state, const uint32_t* __restrict__ buf,
                                                       const int64_t* __restrict__ cursor) {
  const int64_t c = *cursor;
  if (c == 0) return;
  const int64_t a = (int64_t)state[MT_N] + c;  // absolute word index in buf of the next draw
  const int64_t b = (a - 1) / MT_N;            // block of the last drawn word: index a - 624 b in 1..624
  __syncthreads();                             // every thread has read the old position
  for (int t = threadIdx.x; t < MT_N; t += 256) state[t] = buf[b * MT_N + t];
  if (threadIdx.x == 0) state[MT_N] = (uint32_t)(a - b * MT_N);
}

extern "C" {

int64_t mmt_exact_words_bytes(int64_t nwords) { return nwords < 0 ? -1 : mt_blocks(nwords) * MT_N * 4; }

int mmt_exact_gen(void* stream, const uint32_t* mt_state, uint32_t* words, int64_t nwords) {
  if (!mt_state || !words || nwords < 1) return MMT_ERR_INVALID;
  hipLaunchKernelGGL(mt_gen_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, mt_state, words,
                     (int)mt_blocks(nwords));
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_ERR_HIP;
}

// scratch layout: cursor (int64) | accept flags, ordinals, positions (int32 x W each) | accepted
// values (u8 x W) | eligibility flags, ordinals (int32 x max_n each) | hipcub temp
static size_t scan_temp_bytes(int64_t items) {
  size_t t = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, (const int32_t*)nullptr, (int32_t*)nullptr, (int)items);
  return t;
}
static int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

int64_t mmt_exact_walk_scratch_bytes(int64_t max_n, int64_t nwords) {
  if (max_n < 1 || nwords < 1) return -1;
  const int64_t mx = std::max(max_n, nwords);
  return 256 + 3 * align256(nwords * 4) + align256(nwords) + 2 * align256(max_n * 4) + align256((int64_t)scan_temp_bytes(mx));
}

int mmt_exact_walk(void* stream, int32_t nmod, int32_t* const* data, const int64_t* n, const int32_t* rand_size,
                   const int32_t* vocab, uint32_t* mt_state, const uint32_t* words, int64_t nwords, void* scratch,
                   int64_t scratch_bytes, int32_t* status) {
  if (nmod < 1 || nmod > MMT_MAX_MODALITIES || !data || !n || !rand_size || !vocab || !mt_state || !words ||
      nwords < 1 || !scratch || !status || nwords > 0x7fffffffLL)
    return MMT_ERR_INVALID;
  int64_t max_n = 1;
  for (int r = 0; r < nmod; ++r) {
    if (rand_size[r] == 0) continue;
    if (rand_size[r] < 1 || rand_size[r] > 3 || vocab[r] < 1 || n[r] < 0 || !data[r]) return MMT_ERR_INVALID;
    max_n = std::max(max_n, n[r]);
  }
  if (mmt_exact_walk_scratch_bytes(max_n, nwords) > scratch_bytes) return MMT_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  char* p = (char*)scratch;
  int64_t* cursor = (int64_t*)p; p += 256;
  int32_t* aflags = (int32_t*)p; p += align256(nwords * 4);
  int32_t* aord = (int32_t*)p; p += align256(nwords * 4);
  int32_t* apos = (int32_t*)p; p += align256(nwords * 4);
  uint8_t* aval = (uint8_t*)p; p += align256(nwords);
  int32_t* eflags = (int32_t*)p; p += align256(max_n * 4);
  int32_t* eord = (int32_t*)p; p += align256(max_n * 4);
  void* tmp = p;
  size_t tmp_bytes = scan_temp_bytes(std::max(max_n, nwords));
  if (hipMemsetAsync(cursor, 0, 8, s) != hipSuccess) return MMT_ERR_HIP;
  const unsigned gw = (unsigned)std::min<int64_t>(8192, (nwords + 255) / 256);
  for (int r = 0; r < nmod; ++r) {
    const int rs = rand_size[r];
    if (rs == 0 || n[r] == 0) continue;
    const int nch = 2 * rs + 1, k = 32 - __builtin_clz((unsigned)nch);  // n.bit_length()
    hipLaunchKernelGGL(mt_accept_kernel, dim3(gw), dim3(256), 0, s, words, mt_state, nwords, cursor, k, nch, aflags);
    if (hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, aflags, aord, (int)nwords, s) != hipSuccess) return MMT_ERR_HIP;
    hipLaunchKernelGGL(mt_compact_kernel, dim3(gw), dim3(256), 0, s, words, mt_state, nwords, k, aflags, aord, aval,
                       apos);
    const unsigned ge = (unsigned)std::min<int64_t>(8192, (n[r] + 255) / 256);
    hipLaunchKernelGGL(walk_elig_kernel, dim3(ge), dim3(256), 0, s, data[r], n[r], rs, vocab[r], eflags);
    if (hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, eflags, eord, (int)n[r], s) != hipSuccess) return MMT_ERR_HIP;
    hipLaunchKernelGGL(walk_update_kernel, dim3(ge), dim3(256), 0, s, data[r], n[r], eflags, eord, aval, aord, aflags,
                       nwords);
    hipLaunchKernelGGL(walk_cursor_kernel, dim3(1), dim3(1), 0, s, n[r], eflags, eord, aflags, aord, apos, nwords,
                       cursor, status);
  }
  hipLaunchKernelGGL(mt_state_kernel, dim3(1), dim3(256), 0, s, mt_state, words, cursor);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_ERR_HIP;
}

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
