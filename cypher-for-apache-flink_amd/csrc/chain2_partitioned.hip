// chain2_partitioned.hip — radix-partitioned LDS histograms for the fused
// 2-hop count (the k_chain2_hist replacement for large rel tables).
//
// The two per-node histograms of the 2-hop message passing
//   in[b]  = |{r1 : end(r1) = b, start(r1) ∈ S_a}|
//   out[b] = |{r2 : start(r2) = b, end(r2) ∈ S_c}|
// are GROUP BY counts on a 2^24-key domain at R-MAT s24: far larger than LDS,
// and random global atomics run at a small fraction of HBM bandwidth.  This
// is the radix-partitioned hash join of the north star with partitions sized
// to the 160 KiB LDS:
//   P1 k_c2_count   per tile: LDS counts of (side, bucket), bucket = 32 Ki node ids
//   scan            offsets of every (side, bucket, tile) run
//   P2 k_c2_scatter per tile: LDS cursors; each key's low 15 bits → uint16
//                   into its bucket run (self-loop term counted here)
//   P3 k_c2_bucket  per (side, bucket, chunk): 128 KiB LDS histogram, flushed
//                   to the global histogram (plain store when a bucket is one chunk)
//   P4 k_chain2_dot Σ in·out (fused_count.hip)
// Bytes per rel at int64 reference width: P1 16 + P2 16 + 4 + P3 4.
#include <algorithm>
#include <vector>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

constexpr int C2_BITS = 15;
constexpr int C2_BW = 1 << C2_BITS;  // node ids per bucket = uint32 bins in LDS (128 KiB)
constexpr int C2_BLOCK = 256;
constexpr int64_t C2_TILE = 32768;   // rels per P1/P2 tile
constexpr int C2_MAX_BUCKETS = 2048; // 2^26 nodes per side in one LDS count array

struct C2Cols {
  const int64_t *u1, *v1, *u2, *v2;
  int64_t n;
  int64_t lo, hi;  // dense node range of S_a = S_b = S_c (MAP_ONES)
  int nb;          // buckets per side
  int64_t ntiles;
};

// in-key of rel e (-1 = no contribution): end(r1) when start(r1) ∈ S_a and end(r1) ∈ S_b
__device__ inline int64_t c2_in_key(const C2Cols &c, int64_t x1, int64_t y1) {
  return (x1 >= c.lo && x1 <= c.hi && y1 >= c.lo && y1 <= c.hi) ? y1 - c.lo : -1;
}

__global__ __launch_bounds__(C2_BLOCK) void k_c2_count(C2Cols c, uint32_t *counts,
                                                        unsigned long long *loops) {
  __shared__ uint32_t cnt[2 * C2_MAX_BUCKETS];
  for (int i = threadIdx.x; i < 2 * c.nb; i += C2_BLOCK) cnt[i] = 0;
  __syncthreads();
  const int64_t t = blockIdx.x;
  const int64_t e0 = t * C2_TILE, e1 = min(e0 + C2_TILE, c.n);
  unsigned long long lp = 0;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += C2_BLOCK) {
    const int64_t x1 = c.u1[e], y1 = c.v1[e];
    const int64_t x2 = c.u2 == c.u1 ? x1 : c.u2[e];
    const int64_t y2 = c.v2 == c.v1 ? y1 : c.v2[e];
    const int64_t ki = c2_in_key(c, x1, y1);
    const int64_t ko = c2_in_key(c, y2, x2);  // out-key: start(r2) when end(r2) ∈ S_c
    if (ki >= 0) atomicAdd(&cnt[ki >> C2_BITS], 1u);
    if (ko >= 0) atomicAdd(&cnt[c.nb + (ko >> C2_BITS)], 1u);
    lp += (ki >= 0 && ko >= 0 && y1 == x2) ? 1ull : 0ull;
  }
  __syncthreads();
  // layout [side][bucket][tile]: one exclusive scan gives every run's offset
  for (int i = threadIdx.x; i < 2 * c.nb; i += C2_BLOCK) counts[(int64_t)i * c.ntiles + t] = cnt[i];
  lp = wave_reduce_sum(lp);
  if (lane_id() == 0 && lp) atomicAdd(loops, lp);
}

__global__ __launch_bounds__(C2_BLOCK) void k_c2_scatter(C2Cols c, const int64_t *offsets,
                                                          uint16_t *part) {
  __shared__ uint32_t cur[2 * C2_MAX_BUCKETS];
  const int64_t t = blockIdx.x;
  // cursors are relative to the (side, bucket, tile) run start
  for (int i = threadIdx.x; i < 2 * c.nb; i += C2_BLOCK) cur[i] = 0;
  __syncthreads();
  const int64_t e0 = t * C2_TILE, e1 = min(e0 + C2_TILE, c.n);
  for (int64_t e = e0 + threadIdx.x; e < e1; e += C2_BLOCK) {
    const int64_t x1 = c.u1[e], y1 = c.v1[e];
    const int64_t x2 = c.u2 == c.u1 ? x1 : c.u2[e];
    const int64_t y2 = c.v2 == c.v1 ? y1 : c.v2[e];
    const int64_t ki = c2_in_key(c, x1, y1);
    const int64_t ko = c2_in_key(c, y2, x2);
    if (ki >= 0) {
      const int s = (int)(ki >> C2_BITS);
      const uint32_t p = atomicAdd(&cur[s], 1u);
      part[offsets[(int64_t)s * c.ntiles + t] + p] = (uint16_t)(ki & (C2_BW - 1));
    }
    if (ko >= 0) {
      const int s = c.nb + (int)(ko >> C2_BITS);
      const uint32_t p = atomicAdd(&cur[s], 1u);
      part[offsets[(int64_t)s * c.ntiles + t] + p] = (uint16_t)(ko & (C2_BW - 1));
    }
  }
}

__global__ void k_widen_u32(const uint32_t *a, int64_t *b, int64_t m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

struct C2Chunk {
  int64_t begin, end;  // element range in `part`
  int64_t hist_base;   // first global histogram index of the bucket
  int32_t exclusive;   // 1: the bucket is this one chunk → plain store
  int32_t pad;
};

constexpr int C2_HBLOCK = 1024;

__global__ __launch_bounds__(C2_HBLOCK) void k_c2_bucket(const C2Chunk *chunks,
                                                          const uint16_t *part, uint32_t *hist,
                                                          int64_t hist_len) {
  extern __shared__ __attribute__((aligned(16))) uint32_t bins[];  // C2_BW entries
  const C2Chunk ch = chunks[blockIdx.x];
  for (int i = threadIdx.x; i < C2_BW; i += C2_HBLOCK) bins[i] = 0;
  __syncthreads();
  for (int64_t i = ch.begin + threadIdx.x; i < ch.end; i += C2_HBLOCK) atomicAdd(&bins[part[i]], 1u);
  __syncthreads();
  const int64_t lim = min((int64_t)C2_BW, hist_len - ch.hist_base);
  for (int i = threadIdx.x; i < lim; i += C2_HBLOCK) {
    const uint32_t v = bins[i];
    if (ch.exclusive)
      hist[ch.hist_base + i] = v;
    else if (v)
      atomicAdd(&hist[ch.hist_base + i], v);
  }
}

// Returns false if the shape is outside this kernel's limits (caller falls back).
bool chain2_partitioned(Session *s, const int64_t *u1, const int64_t *v1, const int64_t *u2,
                        const int64_t *v2, int64_t n, int64_t lo, int64_t hi, uint32_t *h_in,
                        uint32_t *h_out, uint64_t *loops_out) {
  const int64_t len = hi - lo + 1;
  const int nb = (int)((len + C2_BW - 1) / C2_BW);
  if (len <= 0 || nb > C2_MAX_BUCKETS || n <= 0) return false;
  if (n >= (int64_t(1) << 32)) return false;
  C2Cols c;
  c.u1 = u1;
  c.v1 = v1;
  c.u2 = u2;
  c.v2 = v2;
  c.n = n;
  c.lo = lo;
  c.hi = hi;
  c.nb = nb;
  c.ntiles = (n + C2_TILE - 1) / C2_TILE;
  const int64_t nruns = 2 * (int64_t)nb * c.ntiles;
  BufPtr counts32 = s->alloc(4 * nruns);
  BufPtr counts = s->alloc(8 * nruns), offs = s->alloc(8 * (nruns + 1));
  BufPtr acc = s->alloc(8);
  HIP_CHECK(hipMemsetAsync(acc->p, 0, 8, s->stream));
  {
    KernelTimer kt(s, "c2_count", 16.0 * n);
    hipLaunchKernelGGL(k_c2_count, dim3((unsigned)c.ntiles), dim3(C2_BLOCK), 0, s->stream, c,
                       (uint32_t *)counts32->p, (unsigned long long *)acc->p);
    KERNEL_CHECK();
  }
  // widen to int64 for the generic scan
  hipLaunchKernelGGL(k_widen_u32, dim3(grid_for(nruns, 256)), dim3(256), 0, s->stream,
                     (const uint32_t *)counts32->p, (int64_t *)counts->p, nruns);
  KERNEL_CHECK();
  const int64_t total = exclusive_scan_i64(s, (const int64_t *)counts->p, (int64_t *)offs->p, nruns);
  BufPtr part = s->alloc(2 * std::max<int64_t>(total, 1));
  {
    KernelTimer kt(s, "c2_scatter", 20.0 * n);
    hipLaunchKernelGGL(k_c2_scatter, dim3((unsigned)c.ntiles), dim3(C2_BLOCK), 0, s->stream, c,
                       (const int64_t *)offs->p, (uint16_t *)part->p);
    KERNEL_CHECK();
  }
  // bucket boundaries (first run of every (side, bucket)) → chunk list on the host
  std::vector<int64_t> starts(2 * nb + 1);
  {
    std::vector<int64_t> h(nruns);
    HIP_CHECK(hipMemcpyAsync(h.data(), offs->p, 8 * nruns, hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipMemcpyAsync(s->h_scalars, acc->p, 8, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    for (int k = 0; k < 2 * nb; ++k) starts[k] = h[(int64_t)k * c.ntiles];
    starts[2 * nb] = total;
    *loops_out = (uint64_t)s->h_scalars[0];
  }
  const int64_t per_side = total;
  const int64_t target = std::max<int64_t>(per_side / (4 * 256), 1 << 16);  // ~4 chunks per CU
  std::vector<C2Chunk> chunks;
  for (int k = 0; k < 2 * nb; ++k) {
    const int64_t b0 = starts[k], b1 = starts[k + 1];
    if (b1 <= b0) continue;
    const int64_t nch = (b1 - b0 + target - 1) / target;
    const int64_t side = k / nb, bucket = k % nb;
    for (int64_t q = 0; q < nch; ++q) {
      C2Chunk ch;
      ch.begin = b0 + (b1 - b0) * q / nch;
      ch.end = b0 + (b1 - b0) * (q + 1) / nch;
      ch.hist_base = bucket * C2_BW;
      ch.exclusive = nch == 1;
      ch.pad = (int32_t)side;
      chunks.push_back(ch);
    }
  }
  static bool attr_set = false;
  if (!attr_set) {
    HIP_CHECK(hipFuncSetAttribute((const void *)k_c2_bucket,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 4 * C2_BW));
    attr_set = true;
  }
  HIP_CHECK(hipMemsetAsync(h_in, 0, 4 * len, s->stream));
  HIP_CHECK(hipMemsetAsync(h_out, 0, 4 * len, s->stream));
  // two launches (one per side) so every chunk knows its histogram
  std::vector<C2Chunk> side_chunks[2];
  for (auto &ch : chunks) side_chunks[ch.pad].push_back(ch);
  for (int side = 0; side < 2; ++side) {
    auto &v = side_chunks[side];
    if (v.empty()) continue;
    BufPtr dch = s->alloc(sizeof(C2Chunk) * v.size());
    HIP_CHECK(hipMemcpyAsync(dch->p, v.data(), sizeof(C2Chunk) * v.size(), hipMemcpyHostToDevice,
                             s->stream));
    KernelTimer kt(s, "c2_bucket_hist", 2.0 * (side ? total - starts[nb] : starts[nb]));
    hipLaunchKernelGGL(k_c2_bucket, dim3((unsigned)v.size()), dim3(C2_HBLOCK), 4 * C2_BW,
                       s->stream, (const C2Chunk *)dch->p, (const uint16_t *)part->p,
                       side ? h_out : h_in, len);
    KERNEL_CHECK();
    s->sync();  // host vector `v` must outlive the pageable copy
  }
  return true;
}

}  // namespace capf
