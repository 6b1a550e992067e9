// LDS-DMA fill-rate probe (round 5): bytes per second per CU that `buffer_load_dwordx4 ... lds`
// streams into LDS, by source residency (L2 / Infinity Cache / HBM), waves per workgroup, workgroups
// per CU and pieces (1 KiB each) in flight per wave. It bounds what a GEMM main loop that stages its
// operands this way can feed its MFMAs: a 128 x 128 tile needs 16 KiB per BK-32 step (256 MFMA
// cycles per SIMD), a 256 x 256 tile 32 KiB per 1024 cycles.
//
//   hipcc --offload-arch=gfx950 -O3 -o probe_dma tools/probe/probe_dma.hip && ./probe_dma
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int32_t)((a >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int32_t)bytes);
  r[3] = 0x00020000;
  return r;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// every wave streams `iters` 1-KiB pieces into a private ring of SLOTS pieces, keeping INFL in flight
template <int NW, int INFL>
__global__ __launch_bounds__(NW * 64) void dma_rate(const char* buf, uint32_t mask, int iters) {
  constexpr int SLOTS = 16;
  __shared__ __attribute__((aligned(1024))) char lds[NW * SLOTS * 1024];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const i32x4 rs = make_rsrc(buf, mask + 1);
  const uint32_t gw = blockIdx.x * NW + wave, nwt = gridDim.x * NW;
  const uint32_t lbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds + wave * SLOTS * 1024;
  for (int p = 0; p < iters; ++p) {
    const uint32_t off = (((uint32_t)p * nwt + gw) * 1024u + 16u * lane) & mask;
    const uint32_t la = __builtin_amdgcn_readfirstlane(lbase + (p % SLOTS) * 1024);
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(la), "v"(off), "s"(rs)
                 : "memory", "m0");
    wait_vm<INFL>();
  }
  wait_vm<0>();
}

template <int NW, int INFL>
static int run(const char* buf, uint32_t bytes, int blocks_per_cu, const char* tag) {
  const int grid = 256 * blocks_per_cu;
  const int iters = 4096;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((dma_rate<NW, INFL>), dim3(grid), dim3(NW * 64), 0, 0, buf, bytes - 1, iters);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0, 0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((dma_rate<NW, INFL>), dim3(grid), dim3(NW * 64), 0, 0, buf, bytes - 1, iters);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double tot = (double)grid * NW * iters * 1024.0 * reps;
  const double tbs = tot / (ms * 1e-3) / 1e12;
  printf("%-6s src %8.1f MiB  waves/WG %d  WG/CU %d  inflight/wave %2d (%3d KiB/CU): %6.2f TB/s chip, %6.1f GB/s per CU\n",
         tag, bytes / 1048576.0, NW, blocks_per_cu, INFL, NW * blocks_per_cu * INFL, tbs, tbs * 1e3 / 256.0);
  fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main() {
  char* buf = nullptr;
  const uint32_t big = 1u << 31;  // 2 GiB (HBM)
  CHECK(hipMalloc(&buf, big));
  CHECK(hipMemset(buf, 1, big));
  const uint32_t sizes[3] = {2u << 20, 128u << 20, big};
  const char* tags[3] = {"L2", "MALL", "HBM"};
  for (int s = 0; s < 3; ++s) {
    const uint32_t b = sizes[s];
    run<4, 4>(buf, b, 1, tags[s]);
    run<4, 8>(buf, b, 1, tags[s]);
    run<4, 15>(buf, b, 1, tags[s]);
    run<8, 4>(buf, b, 1, tags[s]);
    run<8, 8>(buf, b, 1, tags[s]);
    run<8, 15>(buf, b, 1, tags[s]);
    run<4, 8>(buf, b, 2, tags[s]);
    run<4, 8>(buf, b, 3, tags[s]);
    run<4, 15>(buf, b, 3, tags[s]);
  }
  CHECK(hipFree(buf));
  return 0;
}
