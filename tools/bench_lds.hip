// Microbenchmark (not product): LDS atomic add throughput, random addresses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int RET, int WORDS, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k(int iters, uint32_t *out) {
  extern __shared__ uint32_t w[];
  for (int i = threadIdx.x; i < WORDS; i += BLOCK) w[i] = 0;
  __syncthreads();
  uint32_t x = threadIdx.x * 0x9E3779B1u + blockIdx.x * 0x85EBCA6Bu, acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t a[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { x = x * 1664525u + 1013904223u; a[e] = (x >> 8) & (WORDS - 1); }
    if (RET) {
      uint32_t o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = atomicAdd(&w[a[e]], 1u);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += o[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&w[a[e]], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = w[acc & (WORDS - 1)] + acc;
}
int main() {
  uint32_t *out; hipMalloc(&out, 1 << 20);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 256;
  auto run = [&](auto kern, int block, int lds, const char *name) {
    hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    const int grid = 256 * 8;
    kern<<<grid, block, lds>>>(iters, out); hipDeviceSynchronize();
    hipEventRecord(a); kern<<<grid, block, lds>>>(iters, out); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double ops = (double)grid * block * iters * 8;
    printf("%-28s %.3f ms  %.1f G atomics/s  -> 2^29 keys in %.3f ms\n", name, ms, ops / ms / 1e6, (double)(1u << 29) / (ops / ms));
  };
  run(k<0, 32768, 1024>, 1024, 131072, "noret 32K words blk1024");
  run(k<1, 32768, 1024>, 1024, 131072, "ret   32K words blk1024");
  run(k<0, 16384, 1024>, 1024, 65536, "noret 16K words 2 blk/CU");
  run(k<1, 16384, 1024>, 1024, 65536, "ret   16K words 2 blk/CU");
  run(k<0, 32768, 512>, 512, 131072, "noret 32K words blk512");
  return 0;
}
