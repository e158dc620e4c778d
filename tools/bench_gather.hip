// Microbenchmark (not product): read bandwidth of 1 GiB in random segments
// of S bytes, as (a) one lane per segment, 16-B pieces, and (b) S/16 lanes
// per segment (coalesced), vs (c) a plain stream.  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <random>

__global__ void k_lane(const uint4 *buf, const uint32_t *segs, int64_t nseg, int pieces, uint32_t *out) {
  uint32_t acc = 0;
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < nseg; s += (int64_t)gridDim.x * blockDim.x) {
    const uint4 *p = buf + (int64_t)segs[s] * pieces;
    for (int q = 0; q < pieces; ++q) { uint4 v = p[q]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  }
  if (acc == 0x12345678) out[0] = acc;
}
__global__ void k_group(const uint4 *buf, const uint32_t *segs, int64_t nseg, int pieces, uint32_t *out) {
  uint32_t acc = 0;
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  // lane group of `pieces` lanes per segment
  for (int64_t i = tid; i < nseg * pieces; i += nthr) {
    const int64_t s = i / pieces; const int q = i % pieces;
    uint4 v = buf[(int64_t)segs[s] * pieces + q]; acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}
__global__ void k_stream(const uint4 *buf, int64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint4 v = buf[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}
int main() {
  const int64_t bytes = 1ll << 30;
  uint4 *buf; uint32_t *out, *segs;
  hipMalloc(&buf, bytes); hipMalloc(&out, 4);
  hipMemset(buf, 1, bytes);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto timeit = [&](auto f) { f(); hipDeviceSynchronize(); hipEventRecord(a); for (int i = 0; i < 5; ++i) f(); hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); return ms / 5; };
  float ms = timeit([&] { k_stream<<<8192, 256>>>(buf, bytes / 16, out); });
  printf("stream: %.3f ms %.2f TB/s\n", ms, bytes / ms / 1e9);
  for (int S : {64, 128, 256, 512, 1024}) {
    const int pieces = S / 16;
    const int64_t nseg = bytes / S;
    std::vector<uint32_t> h(nseg);
    for (int64_t i = 0; i < nseg; ++i) h[i] = (uint32_t)i;
    std::shuffle(h.begin(), h.end(), std::mt19937(1));
    hipMalloc(&segs, nseg * 4); hipMemcpy(segs, h.data(), nseg * 4, hipMemcpyHostToDevice);
    float m1 = timeit([&] { k_lane<<<4096, 256>>>(buf, segs, nseg, pieces, out); });
    float m2 = timeit([&] { k_group<<<8192, 256>>>(buf, segs, nseg, pieces, out); });
    printf("S=%4d  lane-per-seg %.3f ms %.2f TB/s   group %.3f ms %.2f TB/s\n", S, m1, bytes / m1 / 1e9, m2, bytes / m2 / 1e9);
    hipFree(segs);
  }
  return 0;
}
