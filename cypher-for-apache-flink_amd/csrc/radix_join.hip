// radix_join.hip — the radix-partitioned equi-join of the north star, for
// Table.join on one key column (FlinkTable.join, FlinkTable.scala:171-187;
// the Expand joins of RelationalPlanner.scala:130-165 are exactly this shape:
// node id = start(r) / end(r) = node id).
//
//   key word w   (the same equality as the hash join: int values / string
//                 codes by value, floats by bits with -0 = 0, NULL never matches)
//   h = fmix64(w)  a bijection on 64 bits: h equal ⇔ w equal, so only h is kept
//   P1 / P2      two radix passes of 8 bits each (h >> 56, then h >> 48 & 255):
//                per 8 Ki-row tile an LDS histogram, one exclusive scan over
//                (bucket, tile) counts, the tile's (h, row) pairs grouped by
//                bucket in LDS and written out run by run (coalesced) into
//                contiguous buckets; the second pass runs per first-level
//                bucket, so (b1, b2) = 65 536 contiguous partitions per side
//   sort         the build partitions sorted by h (segmented radix sort):
//                equal keys are runs
//   J            one workgroup per work item (a partition, or a probe chunk
//                of a big one): a chunk of ≤ 2 Ki sorted build rows becomes an
//                LDS table of runs (h → start, length); COUNT pass → one scan
//                of the per-item counts → EMIT over output ranges (sub-items
//                of ≤ 32 Ki pairs, a hub key's product spread over many
//                workgroups), each step's matches flattened over the
//                workgroup: no global atomics, deterministic placement
//   outer sides  matched flags set in the emit pass, the unmatched rows (NULL
//                keys included) appended by a flag compaction
// The build side is the smaller input (inner and outer joins alike: both
// sides carry matched flags).  Bytes per row and side: P1 read key + write
// 12 B, P2 read 12 B + write 12 B, J read 12 B; output 16 B per pair.
#include <algorithm>
#include <cstring>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

constexpr int RJ_P = 256;          // buckets per radix pass
constexpr int RJ_TILE = 8192;      // rows per partitioning tile
constexpr int RJ_PBLOCK = 512;     // partitioning workgroup
constexpr int RJ_CAP = 2048;       // LDS build rows per chunk × 2 (2 Ki: 3 join workgroups per CU)
constexpr int RJ_CHUNK = RJ_CAP / 2;  // build rows per LDS fill (load ≤ 1/2)
constexpr int RJ_PCHUNK = 8192;    // probe rows per work item (at most)
constexpr int RJ_PCHUNK_MIN = 256; // ... and at least, when the probe side is small
constexpr int RJ_JBLOCK = 256;     // join workgroup

__device__ inline uint64_t rj_word(const ColView &c, int64_t r, bool &nul) {
  if (c.type == CAPF_TYPE_NULL || !c.data || (c.valid && !c.valid[r])) {
    nul = true;
    return 0;
  }
  nul = false;
  if (c.type == CAPF_TYPE_BOOL) return ((const uint8_t *)c.data)[r] ? 1 : 0;
  if (c.type != CAPF_TYPE_FLOAT64) return (uint64_t)ld_int(c, r);
  uint64_t w = ((const uint64_t *)c.data)[r];
  return w == 0x8000000000000000ull ? 0 : w;
}

// ---------------------------------------------------------------- pass 1
__global__ __launch_bounds__(RJ_PBLOCK) void k_rj_hist1(ColView key, int64_t n, int64_t ntiles,
                                                         int64_t *counts) {
  __shared__ uint32_t hist[RJ_P];
  for (int i = threadIdx.x; i < RJ_P; i += RJ_PBLOCK) hist[i] = 0;
  __syncthreads();
  const int64_t t = blockIdx.x, e0 = t * RJ_TILE, e1 = min(e0 + RJ_TILE, n);
  for (int64_t r = e0 + threadIdx.x; r < e1; r += RJ_PBLOCK) {
    bool nul;
    const uint64_t w = rj_word(key, r, nul);
    if (!nul) atomicAdd(&hist[fmix64(w) >> 56], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < RJ_P; b += RJ_PBLOCK) counts[(int64_t)b * ntiles + t] = hist[b];
}

// Scatter of one tile through LDS: every row's rank inside its bucket comes
// from the LDS count atomic, the tile's (h, row) pairs are grouped by bucket
// in LDS, then written out in that order — consecutive lanes write
// consecutive addresses of one bucket's run (a per-row scatter to 256
// cursors makes every 8-B store its own memory transaction: 0.86 TB/s).
// PASS 1 reads the key column (rows [e0, e1)), PASS 2 the pass-1 output
// (h, row) of one first-level bucket's tile; `goff` = this tile's global
// start per bucket.
constexpr int RJ_SBLOCK = 1024;
constexpr int RJ_RPT = RJ_TILE / RJ_SBLOCK;

template <int PASS>
__device__ inline uint32_t rj_bucket(uint64_t h) {
  return PASS == 1 ? (uint32_t)(h >> 56) : (uint32_t)(h >> 48) & (RJ_P - 1);
}

template <int PASS>
__device__ inline void rj_scatter_tile(const ColView &key, const uint64_t *h1, const uint32_t *r1,
                                       int64_t e0, int64_t e1, const int64_t *goff_src,
                                       int64_t goff_stride, uint64_t *oh, uint32_t *orow) {
  __shared__ uint64_t sh[RJ_TILE];
  __shared__ uint32_t sr[RJ_TILE];
  __shared__ uint32_t cnt[RJ_P];
  __shared__ uint32_t loff[RJ_P];
  __shared__ int64_t goff[RJ_P];
  __shared__ uint32_t lds_scan[17];
  for (int i = threadIdx.x; i < RJ_P; i += RJ_SBLOCK) {
    cnt[i] = 0;
    goff[i] = goff_src[(int64_t)i * goff_stride];
  }
  __syncthreads();
  uint64_t h[RJ_RPT];
  uint32_t rk[RJ_RPT];
#pragma unroll
  for (int k = 0; k < RJ_RPT; ++k) {
    const int64_t r = e0 + (int64_t)k * RJ_SBLOCK + threadIdx.x;
    rk[k] = 0xFFFFFFFFu;
    h[k] = 0;
    if (r < e1) {
      bool nul = false;
      h[k] = PASS == 1 ? fmix64(rj_word(key, r, nul)) : h1[r];
      if (!nul) rk[k] = atomicAdd(&cnt[rj_bucket<PASS>(h[k])], 1u);
    }
  }
  __syncthreads();
  uint32_t total;
  const uint32_t c = threadIdx.x < RJ_P ? cnt[threadIdx.x] : 0u;
  const uint32_t ex = block_exclusive_scan(c, lds_scan, total);
  if (threadIdx.x < RJ_P) loff[threadIdx.x] = ex;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RJ_RPT; ++k) {
    if (rk[k] == 0xFFFFFFFFu) continue;
    const uint32_t slot = loff[rj_bucket<PASS>(h[k])] + rk[k];
    sh[slot] = h[k];
    sr[slot] = PASS == 1 ? (uint32_t)(e0 + (int64_t)k * RJ_SBLOCK + threadIdx.x)
                         : r1[e0 + (int64_t)k * RJ_SBLOCK + threadIdx.x];
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < total; i += RJ_SBLOCK) {
    const uint64_t v = sh[i];
    const uint32_t b = rj_bucket<PASS>(v);
    const int64_t pos = goff[b] + (int64_t)(i - loff[b]);
    oh[pos] = v;
    orow[pos] = sr[i];
  }
}

__global__ __launch_bounds__(RJ_SBLOCK) void k_rj_scatter1(ColView key, int64_t n, int64_t ntiles,
                                                            const int64_t *offs, uint64_t *oh,
                                                            uint32_t *orow) {
  const int64_t t = blockIdx.x, e0 = t * RJ_TILE, e1 = min(e0 + RJ_TILE, n);
  rj_scatter_tile<1>(key, nullptr, nullptr, e0, e1, offs + t, ntiles, oh, orow);
}

// ---------------------------------------------------------------- pass 2
// Tiles of the second pass never straddle a first-level bucket.
struct RJTile2 {
  int64_t start, end;   // rows of the pass-1 output
  int64_t region;       // counts2 region base of the bucket: 256·(first tile of the bucket)
  int32_t ntb;          // tiles of the bucket
  int32_t local;        // this tile's index inside its bucket
};

// The grids of pass 2 are an upper bound of the tile count (nt1 + 256: no host
// read of the tile list); a block past *nt2 zeroes the count row its index
// would own (the tiles' rows fill [0, 256·nt2), these [256·nt2, 256·grid)) and exits.
__global__ __launch_bounds__(RJ_PBLOCK) void k_rj_hist2(const uint64_t *h1, const RJTile2 *tiles,
                                                         const int64_t *nt2, int64_t *counts) {
  __shared__ uint32_t hist[RJ_P];
  if ((int64_t)blockIdx.x >= *nt2) {
    for (int b = threadIdx.x; b < RJ_P; b += RJ_PBLOCK) counts[(int64_t)blockIdx.x * RJ_P + b] = 0;
    return;
  }
  for (int i = threadIdx.x; i < RJ_P; i += RJ_PBLOCK) hist[i] = 0;
  __syncthreads();
  const RJTile2 tl = tiles[blockIdx.x];
  for (int64_t r = tl.start + threadIdx.x; r < tl.end; r += RJ_PBLOCK)
    atomicAdd(&hist[(h1[r] >> 48) & (RJ_P - 1)], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < RJ_P; b += RJ_PBLOCK)
    counts[tl.region + (int64_t)b * tl.ntb + tl.local] = hist[b];
}

__global__ __launch_bounds__(RJ_SBLOCK) void k_rj_scatter2(const uint64_t *h1, const uint32_t *r1,
                                                            const RJTile2 *tiles, const int64_t *nt2,
                                                            const int64_t *offs, uint64_t *oh, uint32_t *orow) {
  if ((int64_t)blockIdx.x >= *nt2) return;
  const RJTile2 tl = tiles[blockIdx.x];
  rj_scatter_tile<2>(ColView{}, h1, r1, tl.start, tl.end, offs + tl.region + tl.local, tl.ntb, oh, orow);
}

// Partition starts: pstart[p] for p = b1·256 + b2 (65 536 partitions), + total.
__global__ void k_rj_pstart(const int64_t *offs2, const int64_t *bucket_start, const int32_t *bucket_ntiles,
                            const int64_t *bucket_region, const int64_t *total, int64_t *pstart) {
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p <= RJ_P * RJ_P; p += gridDim.x * blockDim.x) {
    if (p == RJ_P * RJ_P) {
      pstart[p] = *total;
      continue;
    }
    const int b1 = p >> 8, b2 = p & 255;
    const int32_t nt = bucket_ntiles[b1];
    pstart[p] = nt > 0 ? offs2[bucket_region[b1] + (int64_t)b2 * nt] : bucket_start[b1];
  }
}

// The pass-2 tile list on the device (one workgroup of RJ_P lanes, lane b =
// first-level bucket b): tiles of ≤ RJ_TILE rows never straddling a bucket,
// bucket-major; bucket starts / tile counts / count regions for k_rj_pstart.
__global__ __launch_bounds__(RJ_P) void k_rj_tiles2(const int64_t *o1, int64_t nt1, const int64_t *total,
                                                    RJTile2 *tiles, int64_t *bstart, int32_t *bnt, int64_t *breg,
                                                    int64_t *nt2) {
  __shared__ int64_t lds[17];
  const int b = threadIdx.x;
  const int64_t lo = o1[(int64_t)b * nt1];
  const int64_t hi = b + 1 < RJ_P ? o1[(int64_t)(b + 1) * nt1] : *total;
  const int64_t nt = (hi - lo + RJ_TILE - 1) / RJ_TILE;
  int64_t all;
  const int64_t tb = block_exclusive_scan(nt, lds, all);
  bstart[b] = lo;
  bnt[b] = (int32_t)nt;
  breg[b] = (int64_t)RJ_P * tb;
  for (int64_t k = 0; k < nt; ++k)
    tiles[tb + k] = RJTile2{lo + k * RJ_TILE, min(hi, lo + (k + 1) * RJ_TILE), (int64_t)RJ_P * tb, (int32_t)nt,
                            (int32_t)k};
  if (b == 0) *nt2 = all;
}

// Partitioned side: (h, row) in partition order + partition starts.
struct RJSide {
  BufPtr h, row, pstart;
  int64_t n = 0;  // partitioned (non-null) rows
};

// Host-synchronous only when the key column may hold NULLs (the partitioned
// row count is then read back); otherwise every step stays on the stream: the
// partitioned rows are n, the pass-2 tile list is built on the device and the
// pass-2 grids are its upper bound.
static RJSide rj_partition(Session *s, const ColPtr &col, int64_t n) {
  RJSide out;
  out.pstart = s->alloc(8 * (RJ_P * RJ_P + 1));
  const ColView key = view_of(col);
  if (n >= (int64_t(1) << 32)) not_impl("radix join side with 2^32 or more rows");
  const int64_t nt1 = std::max<int64_t>(1, (n + RJ_TILE - 1) / RJ_TILE);
  const int64_t nt2max = nt1 + RJ_P;  // Σ_b ⌈rows_b / TILE⌉ ≤ Σ_b rows_b / TILE + 256
  BufPtr c1 = s->alloc(8 * RJ_P * nt1), o1 = s->alloc(8 * (RJ_P * nt1 + 1));
  // device scalars: [0] partitioned rows, [1] pass-2 tiles, [2] pass-2 scan total (unread)
  BufPtr sc = s->alloc(24);
  int64_t *d_total = (int64_t *)sc->p, *d_nt2 = d_total + 1;
  {
    KernelTimer kt(s, "rj_partition1", 12.0 * n);
    if (n > 0) {
      hipLaunchKernelGGL(k_rj_hist1, dim3((unsigned)nt1), dim3(RJ_PBLOCK), 0, s->stream, key, n, nt1,
                         (int64_t *)c1->p);
      KERNEL_CHECK();
    } else {
      HIP_CHECK(hipMemsetAsync(c1->p, 0, 8 * RJ_P * nt1, s->stream));
    }
    exclusive_scan_i64_async(s, (const int64_t *)c1->p, (int64_t *)o1->p, RJ_P * nt1, d_total);
  }
  const bool all_null = key.type == CAPF_TYPE_NULL || !key.data || n == 0;
  int64_t total = all_null ? 0 : n;
  if (!all_null && key.valid) {  // NULL keys are not partitioned: the count decides the sizes
    HIP_CHECK(hipMemcpyAsync(s->h_scalars, d_total, 8, hipMemcpyDeviceToHost, s->stream));
    s->sync();
    total = s->h_scalars[0];
  }
  out.n = total;
  BufPtr h1 = s->alloc(8 * std::max<int64_t>(total, 1)), r1 = s->alloc(4 * std::max<int64_t>(total, 1));
  if (n > 0) {
    KernelTimer kt(s, "rj_partition1", 12.0 * total);
    hipLaunchKernelGGL(k_rj_scatter1, dim3((unsigned)nt1), dim3(RJ_SBLOCK), 0, s->stream, key, n, nt1,
                       (const int64_t *)o1->p, (uint64_t *)h1->p, (uint32_t *)r1->p);
    KERNEL_CHECK();
  }
  BufPtr dt = s->alloc(sizeof(RJTile2) * nt2max);
  BufPtr meta = s->alloc(8 * RJ_P + 4 * RJ_P + 8 * RJ_P);
  int64_t *d_bstart = (int64_t *)meta->p;
  int32_t *d_bnt = (int32_t *)(d_bstart + RJ_P);
  int64_t *d_breg = (int64_t *)(d_bnt + RJ_P);
  hipLaunchKernelGGL(k_rj_tiles2, dim3(1), dim3(RJ_P), 0, s->stream, (const int64_t *)o1->p, nt1,
                     (const int64_t *)d_total, (RJTile2 *)dt->p, d_bstart, d_bnt, d_breg, d_nt2);
  KERNEL_CHECK();
  out.h = s->alloc(8 * std::max<int64_t>(total, 1));
  out.row = s->alloc(4 * std::max<int64_t>(total, 1));
  BufPtr o2 = s->alloc(8 * (RJ_P * nt2max + 1));
  if (total > 0) {
    KernelTimer kt(s, "rj_partition2", 24.0 * total);
    BufPtr c2 = s->alloc(8 * RJ_P * nt2max);  // (the unused tiles' rows zeroed by k_rj_hist2)
    hipLaunchKernelGGL(k_rj_hist2, dim3((unsigned)nt2max), dim3(RJ_PBLOCK), 0, s->stream,
                       (const uint64_t *)h1->p, (const RJTile2 *)dt->p, (const int64_t *)d_nt2, (int64_t *)c2->p);
    KERNEL_CHECK();
    exclusive_scan_i64_async(s, (const int64_t *)c2->p, (int64_t *)o2->p, RJ_P * nt2max, d_nt2 + 1);
    hipLaunchKernelGGL(k_rj_scatter2, dim3((unsigned)nt2max), dim3(RJ_SBLOCK), 0, s->stream,
                       (const uint64_t *)h1->p, (const uint32_t *)r1->p, (const RJTile2 *)dt->p,
                       (const int64_t *)d_nt2, (const int64_t *)o2->p, (uint64_t *)out.h->p, (uint32_t *)out.row->p);
    KERNEL_CHECK();
  }
  hipLaunchKernelGGL(k_rj_pstart, dim3((RJ_P * RJ_P + 256) / 256), dim3(256), 0, s->stream,
                     (const int64_t *)o2->p, (const int64_t *)d_bstart, (const int32_t *)d_bnt,
                     (const int64_t *)d_breg, (const int64_t *)d_total, (int64_t *)out.pstart->p);
  KERNEL_CHECK();
  return out;  // (the temporaries return to the stream-ordered pool)
}

// ---------------------------------------------------------------- join
struct RJWork {
  int32_t part;    // first partition of the item's group
  int32_t np;      // partitions in the group (consecutive: their sorted build rows are one sorted run of h)
  int64_t p0, p1;  // probe rows of the item (positions in the probe arrays)
};

// COUNT pass of the run-based join: the build partitions are sorted by h
// once (segmented radix sort), so equal keys are runs; an LDS chunk of ≤
// RJ_CHUNK sorted build rows becomes a table of RUNS (h → start, length),
// found from run heads with a ballot bitmask.  A probe row costs one lookup
// whatever its key's multiplicity; out_cnt[item] = the item's pairs (the EMIT
// pass is k_rj_emit_ranges over output ranges).  (Measured and removed: a
// chain-walking multimap join, and an EMIT inside this kernel — one wave wrote
// a hub key's whole product.)
constexpr int RJ_RUNCAP = 2048;  // run-table slots (≤ RJ_CHUNK runs per chunk, load ≤ 1/2)

// (grid: an upper bound of the item count; blocks past *nw count 0 pairs)
__global__ __launch_bounds__(RJ_JBLOCK) void k_rj_join_runs(const RJWork *work, const int64_t *nw,
                                                             const uint64_t *bh, const int64_t *bstart,
                                                             const uint64_t *ph, int64_t *out_cnt) {
  __shared__ uint64_t kk[RJ_CHUNK];
  __shared__ unsigned long long hm[RJ_CHUNK / WAVE];  // run-head bitmask
  __shared__ uint64_t th[RJ_RUNCAP];
  __shared__ uint32_t tv[RJ_RUNCAP];                   // start << 16 | length (chunk-relative), 0 = empty
  constexpr int NW = RJ_JBLOCK / WAVE;
  __shared__ int64_t wsum[NW];
  if ((int64_t)blockIdx.x >= *nw) {
    if (threadIdx.x == 0) out_cnt[blockIdx.x] = 0;
    return;
  }
  const RJWork wk = work[blockIdx.x];
  const int64_t b0 = bstart[wk.part], b1 = bstart[wk.part + wk.np];
  const int wv = threadIdx.x / WAVE, lane = lane_id();
  int64_t item_total = 0;
  for (int64_t c0 = b0; c0 < b1; c0 += RJ_CHUNK) {
    const int nc = (int)min<int64_t>((int64_t)RJ_CHUNK, b1 - c0);
    __syncthreads();  // the previous chunk's table is no longer read
    for (int i = threadIdx.x; i < RJ_RUNCAP; i += RJ_JBLOCK) tv[i] = 0;
    for (int i = threadIdx.x; i < RJ_CHUNK; i += RJ_JBLOCK) kk[i] = i < nc ? bh[c0 + i] : ~0ull;
    __syncthreads();
    for (int i0 = wv * WAVE; i0 < RJ_CHUNK; i0 += RJ_JBLOCK) {  // one ballot per 64 rows
      const int i = i0 + lane;
      const bool head = i < nc && (i == 0 || kk[i] != kk[i - 1]);
      const unsigned long long m = __ballot(head);
      if (lane == 0) hm[i0 / WAVE] = m;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nc; i += RJ_JBLOCK) {
      const unsigned long long m = hm[i / WAVE];
      if (!((m >> (i & (WAVE - 1))) & 1ull)) continue;
      // run end = the next head (or nc): the rest of this word, then the next words
      int e = nc;
      const unsigned long long rest = (i & (WAVE - 1)) == WAVE - 1 ? 0ull : m >> ((i & (WAVE - 1)) + 1);
      if (rest) {
        e = i + 1 + __builtin_ctzll(rest);
      } else {
        for (int w = i / WAVE + 1; w < (nc + WAVE - 1) / WAVE; ++w)
          if (hm[w]) {
            e = w * WAVE + __builtin_ctzll(hm[w]);
            break;
          }
      }
      const uint64_t h = kk[i];
      uint32_t slot = (uint32_t)h & (RJ_RUNCAP - 1);
      while (atomicCAS(&tv[slot], 0u, ((uint32_t)i << 16) | (uint32_t)(e - i)) != 0u)
        slot = (slot + 1) & (RJ_RUNCAP - 1);
      th[slot] = h;
    }
    __syncthreads();
    for (int64_t q0 = wk.p0; q0 < wk.p1; q0 += RJ_JBLOCK) {
      const int64_t q = q0 + threadIdx.x;
      const bool live = q < wk.p1;
      const uint64_t h = live ? ph[q] : 0;
      uint32_t cnt = 0;
      if (live) {
        uint32_t slot = (uint32_t)h & (RJ_RUNCAP - 1);
        for (uint32_t v = tv[slot]; v != 0u; slot = (slot + 1) & (RJ_RUNCAP - 1), v = tv[slot])
          if (th[slot] == h) {
            cnt = v & 0xFFFFu;
            break;
          }
      }
      const uint32_t inc = wave_inclusive_scan(cnt);
      const uint32_t wtot = (uint32_t)__shfl(inc, WAVE - 1, WAVE);
      if (lane == 0) wsum[wv] = wtot;
      __syncthreads();
      int64_t block_tot = 0;
      for (int k = 0; k < NW; ++k) block_tot += wsum[k];
      __syncthreads();  // wsum is rewritten by the next step
      item_total += block_tot;
    }
  }
  if (threadIdx.x == 0) out_cnt[blockIdx.x] = item_total;
}

// EMIT over output ranges.  After COUNT,
// item i (cnt[i] pairs) becomes ⌈cnt[i] / RJ_SUB_OUT⌉ sub-items, each writing
// the pairs [lo, hi) of the item's flattened output sequence (probe-row order,
// then the key's build run): a hub key whose (build run) × (probe rows) product
// is millions of pairs is written by many workgroups instead of one wave of
// one.  A sub-item repeats the item's run-table build and lookups up to its
// range (cheap next to the writes) and flattens each 256-row step over the
// whole workgroup (block scan of the match counts, owner row by an 8-step
// search), 4 outputs per lane in flight.  Probe rows are flagged matched
// (outer joins) by the sub-item holding their first pair.
constexpr int64_t RJ_SUB_OUT = 32768;
// EMIT output positions per lane in flight: 8 (140 VGPRs, the same 3 workgroups per CU
// as 4's 92 — LDS bounds occupancy): var2 s14 filtered EMIT 586 → 568 µs
constexpr int RJ_EMIT_U = 8;
struct RJSub {
  int32_t item;
  int32_t pad;
  int64_t lo, hi;
};

__global__ void k_rj_sub_counts(const int64_t *cnt, int64_t nw, int64_t *nsub) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x)
    nsub[i] = (cnt[i] + RJ_SUB_OUT - 1) / RJ_SUB_OUT;
}

__global__ void k_rj_subs(const int64_t *cnt, const int64_t *soff, int64_t nw, RJSub *subs) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t o = soff[i];
    for (int64_t lo = 0; lo < cnt[i]; lo += RJ_SUB_OUT) subs[o++] = RJSub{(int32_t)i, 0, lo, min(cnt[i], lo + RJ_SUB_OUT)};
  }
}

// A filter over the join's pairs (radix_join_filtered).  Every column operand
// is first materialised per row of its input side as int64 values + a "not
// NULL" byte (k_rj_operand: lazy gathers, FOR decoding, validity folded once
// per input row), in the order the EMIT meets the rows: build operands in the
// sorted build partition order (read at the pair's build position, beside its
// row id: coalesced), probe operands in probe partition order (staged in LDS
// per 256-row step, beside the probe row).  A random 8-B load per pair and
// operand ran at L1's one-line-per-clock rate (s14 var2: 1.1 ms to count).
constexpr int RJ_PMAX = 4;  // probe-side column operands (LDS slots)
struct RjOp {
  const int64_t *val;  // build operand: by sorted build position
  const uint8_t *ok;
  int64_t lit;
  int32_t is_lit;
  int32_t slot;  // probe operand: its LDS slot; −1 = build operand
};
struct RjTerm {
  RjOp a, b;
  int32_t op, neg;
};
struct RjPred {
  RjTerm t[FT_MAX];
  const int64_t *pv[RJ_PMAX];  // probe operands by probe position
  const uint8_t *po[RJ_PMAX];
  int32_t nt, np;
};

__global__ void k_rj_operand(FtOperand o, const uint32_t *rows, int64_t n, int64_t *val, uint8_t *ok) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t v = 0;
    ok[i] = ft_load(o, rows[i], v) ? 1 : 0;
    val[i] = v;
  }
}

// the terms over U pairs (build positions bi, probe step slots bl): all loads
// of a term issued before any compare
template <int U>
__device__ inline void rj_pass(const RjPred &fp, const int64_t (&bi)[U], const uint32_t (&bl)[U],
                               const int64_t (*spv)[RJ_JBLOCK], const uint8_t (*spo)[RJ_JBLOCK], bool (&pass)[U]) {
  for (int t = 0; t < fp.nt; ++t) {
    const RjTerm &tm = fp.t[t];
    int64_t x[U], y[U];
    uint8_t oa[U], ob[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      x[k] = tm.a.is_lit ? tm.a.lit : tm.a.slot >= 0 ? spv[tm.a.slot][bl[k]] : tm.a.val[bi[k]];
      oa[k] = tm.a.is_lit ? (uint8_t)1 : tm.a.slot >= 0 ? spo[tm.a.slot][bl[k]] : tm.a.ok[bi[k]];
      y[k] = tm.b.is_lit ? tm.b.lit : tm.b.slot >= 0 ? spv[tm.b.slot][bl[k]] : tm.b.val[bi[k]];
      ob[k] = tm.b.is_lit ? (uint8_t)1 : tm.b.slot >= 0 ? spo[tm.b.slot][bl[k]] : tm.b.ok[bi[k]];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      bool res = tm.op == OP_EQ   ? x[k] == y[k]
                 : tm.op == OP_NEQ ? x[k] != y[k]
                 : tm.op == OP_LT  ? x[k] < y[k]
                 : tm.op == OP_LE  ? x[k] <= y[k]
                 : tm.op == OP_GT  ? x[k] > y[k]
                                   : x[k] >= y[k];
      if (tm.neg) res = !res;
      pass[k] = pass[k] && oa[k] && ob[k] && res;
    }
  }
}

// MODE 0: every pair of the sub-item's range [lo, hi) at out_off[item] + its
// position.  With a filter (radix_join_filtered): MODE 3 writes the passing
// pairs at the same positions and appends the positions of the failing ones
// to holes[] (the caller then moves tail pairs into the holes: the output is
// a bag — one pass, no count of the passes first); MODE 1 counts the passes
// per sub-item into subcnt[sub] and MODE 2 writes them from suboff[sub] on
// (two passes, when the holes overflow their buffer).
// I: the pair list's row index type (int32 when both sides have < 2^31 rows:
// half the EMIT's bytes and of every gather through the pairs later).
template <int MODE, typename I>
__global__ __launch_bounds__(RJ_JBLOCK) void k_rj_emit_ranges(const RJSub *subs, const RJWork *work,
                                                               const uint64_t *bh, const uint32_t *brow,
                                                               const int64_t *bstart, const uint64_t *ph,
                                                               const uint32_t *prow, const int64_t *out_off,
                                                               I *oprobe, I *obuild,
                                                               uint8_t *pmatched, uint8_t *bmatched,
                                                               const RjPred fp, int build_left, int build_pos,
                                                               int64_t *subcnt, const int64_t *suboff,
                                                               unsigned long long *nholes, int64_t hcap) {
  __shared__ uint64_t kk[RJ_CHUNK];
  __shared__ unsigned long long hm[RJ_CHUNK / WAVE];
  __shared__ uint64_t th[RJ_RUNCAP];
  __shared__ uint32_t tv[RJ_RUNCAP];
  __shared__ uint32_t bex[RJ_JBLOCK + 1], bst[RJ_JBLOCK], bpr[RJ_JBLOCK];
  __shared__ uint32_t lds_sc[17];
  __shared__ int64_t spv[MODE ? RJ_PMAX : 1][RJ_JBLOCK];  // probe operands of the step's rows
  __shared__ uint8_t spo[MODE ? RJ_PMAX : 1][RJ_JBLOCK];
  const RJSub sb = subs[blockIdx.x];
  const RJWork wk = work[sb.item];
  const int64_t b0 = bstart[wk.part], b1 = bstart[wk.part + wk.np];
  const int wv = threadIdx.x / WAVE, lane = lane_id();
  const int64_t obase = MODE == 0 || MODE == 3 ? out_off[sb.item] : 0;
  int64_t fbase = MODE == 2 ? suboff[blockIdx.x] : 0;  // next filtered output position
  uint32_t kept = 0;                                   // MODE 1: passing pairs of this thread
  int64_t rel = 0;  // pairs of the item before the current step
  for (int64_t c0 = b0; c0 < b1 && rel < sb.hi; c0 += RJ_CHUNK) {
    const int nc = (int)min<int64_t>((int64_t)RJ_CHUNK, b1 - c0);
    __syncthreads();
    for (int i = threadIdx.x; i < RJ_RUNCAP; i += RJ_JBLOCK) tv[i] = 0;
    for (int i = threadIdx.x; i < RJ_CHUNK; i += RJ_JBLOCK) kk[i] = i < nc ? bh[c0 + i] : ~0ull;
    __syncthreads();
    for (int i0 = wv * WAVE; i0 < RJ_CHUNK; i0 += RJ_JBLOCK) {
      const int i = i0 + lane;
      const bool head = i < nc && (i == 0 || kk[i] != kk[i - 1]);
      const unsigned long long m = __ballot(head);
      if (lane == 0) hm[i0 / WAVE] = m;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nc; i += RJ_JBLOCK) {
      const unsigned long long m = hm[i / WAVE];
      if (!((m >> (i & (WAVE - 1))) & 1ull)) continue;
      int e = nc;
      const unsigned long long rest = (i & (WAVE - 1)) == WAVE - 1 ? 0ull : m >> ((i & (WAVE - 1)) + 1);
      if (rest) {
        e = i + 1 + __builtin_ctzll(rest);
      } else {
        for (int w = i / WAVE + 1; w < (nc + WAVE - 1) / WAVE; ++w)
          if (hm[w]) {
            e = w * WAVE + __builtin_ctzll(hm[w]);
            break;
          }
      }
      const uint64_t h = kk[i];
      uint32_t slot = (uint32_t)h & (RJ_RUNCAP - 1);
      while (atomicCAS(&tv[slot], 0u, ((uint32_t)i << 16) | (uint32_t)(e - i)) != 0u)
        slot = (slot + 1) & (RJ_RUNCAP - 1);
      th[slot] = h;
    }
    __syncthreads();
    for (int64_t q0 = wk.p0; q0 < wk.p1 && rel < sb.hi; q0 += RJ_JBLOCK) {
      const int64_t q = q0 + threadIdx.x;
      const bool live = q < wk.p1;
      const uint64_t h = live ? ph[q] : 0;
      uint32_t cnt = 0, st = 0;
      if (live) {
        uint32_t slot = (uint32_t)h & (RJ_RUNCAP - 1);
        for (uint32_t v = tv[slot]; v != 0u; slot = (slot + 1) & (RJ_RUNCAP - 1), v = tv[slot])
          if (th[slot] == h) {
            cnt = v & 0xFFFFu;
            st = v >> 16;
            break;
          }
      }
      uint32_t tot;
      const uint32_t ex = block_exclusive_scan(cnt, lds_sc, tot);  // (ends in a barrier)
      if (rel + tot > sb.lo) {  // workgroup-uniform: this step holds pairs of the range
        bex[threadIdx.x] = ex;
        bst[threadIdx.x] = st;
        bpr[threadIdx.x] = live ? prow[q] : 0u;
        if constexpr (MODE != 0)
          for (int j = 0; j < fp.np; ++j) {
            spv[j][threadIdx.x] = live ? fp.pv[j][q] : 0;
            spo[j][threadIdx.x] = live ? fp.po[j][q] : (uint8_t)0;
          }
        if (threadIdx.x == 0) bex[RJ_JBLOCK] = tot;
        if (pmatched && cnt && rel + ex >= sb.lo && rel + ex < sb.hi) pmatched[prow[q]] = 1;
        __syncthreads();
        const uint32_t x0 = (uint32_t)max<int64_t>(0, sb.lo - rel);
        const uint32_t x1 = (uint32_t)min<int64_t>((int64_t)tot, sb.hi - rel);
        constexpr int U = RJ_EMIT_U;
        for (uint32_t xb = x0; xb < x1; xb += U * RJ_JBLOCK) {
          uint32_t br[U], pr[U], bl[U], xs[U];
          int64_t bi[U];
          // owner rows (last row with bex[b] ≤ x) of the U positions, searched in
          // lockstep: the U dependent LDS chains interleave
#pragma unroll
          for (int k = 0; k < U; ++k) {
            xs[k] = min(xb + k * RJ_JBLOCK + threadIdx.x, x1 - 1);
            bl[k] = 0;
          }
#pragma unroll
          for (int st2 = RJ_JBLOCK / 2; st2 > 0; st2 >>= 1) {
            uint32_t v[U];
#pragma unroll
            for (int k = 0; k < U; ++k) v[k] = bex[bl[k] + st2];
#pragma unroll
            for (int k = 0; k < U; ++k) bl[k] = v[k] <= xs[k] ? bl[k] + st2 : bl[k];
          }
#pragma unroll
          for (int k = 0; k < U; ++k) {
            const uint32_t b = bl[k];
            bi[k] = c0 + bst[b] + (xs[k] - bex[b]);
            // build_pos: the build side's sorted position (its columns were permuted
            // into sorted order: later gathers through it stream), else its row
            br[k] = build_pos ? (uint32_t)bi[k] : brow[bi[k]];
            pr[k] = bpr[b];
          }
          if constexpr (MODE == 0) {
#pragma unroll
            for (int k = 0; k < U; ++k) {
              const uint32_t x = xb + k * RJ_JBLOCK + threadIdx.x;
              if (x < x1) {
                oprobe[obase + rel + x] = (I)pr[k];
                obuild[obase + rel + x] = (I)br[k];
                if (bmatched) bmatched[br[k]] = 1;
              }
            }
          } else {
            bool keep[U];
#pragma unroll
            for (int k = 0; k < U; ++k) keep[k] = xb + k * RJ_JBLOCK + threadIdx.x < x1;
            rj_pass<U>(fp, bi, bl, spv, spo, keep);
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < U; ++k) c += keep[k] ? 1u : 0u;
            if constexpr (MODE == 3) {
#pragma unroll
              for (int k = 0; k < U; ++k) {
                const uint32_t x = xb + k * RJ_JBLOCK + threadIdx.x;
                if (x >= x1) continue;
                const int64_t pos = obase + rel + x;
                if (keep[k]) {
                  oprobe[pos] = (I)pr[k];
                  obuild[pos] = (I)br[k];
                } else {
                  const unsigned long long h = atomicAdd(nholes, 1ull);
                  if ((int64_t)h < hcap) subcnt[h] = pos;
                }
              }
              (void)c;
            } else if constexpr (MODE == 1) {
              kept += c;
            } else {
              uint32_t tot2;
              const uint32_t ex2 = block_exclusive_scan(c, lds_sc, tot2);
              int64_t pos = fbase + ex2;
#pragma unroll
              for (int k = 0; k < U; ++k)
                if (keep[k]) {
                  oprobe[pos] = (I)pr[k];
                  obuild[pos] = (I)br[k];
                  ++pos;
                }
              fbase += tot2;
            }
          }
        }
        __syncthreads();  // bex / bst / bpr are rewritten by the next step
      }
      rel += tot;
    }
  }
  if constexpr (MODE == 1) {
    uint32_t tk;
    block_exclusive_scan(kept, lds_sc, tk);
    if (threadIdx.x == 0) subcnt[blockIdx.x] = tk;
  }
}

// MODE 3's holes (sorted): the pairs of the tail [total − nh, total) that are
// not holes move into the holes below it — the k-th hole below the tail
// takes the k-th non-hole tail position counted from the end, p = total − 1 −
// k − #{tail holes > p}, found by fixed-point steps (binary searches of the
// sorted holes) and stepped down past holes.  One workgroup; the filters fused
// here (relationship uniqueness) fail on few pairs (a self-loop rel met twice).
__device__ inline int64_t rj_count_above(const uint64_t *h, int64_t lo, int64_t hi, int64_t p) {
  // entries of the sorted h[lo, hi) greater than p
  int64_t a = lo, b = hi;
  while (a < b) {
    const int64_t mid = (a + b) >> 1;
    if ((int64_t)h[mid] > p) b = mid;
    else a = mid + 1;
  }
  return hi - a;
}

template <typename I>
__global__ __launch_bounds__(1024) void k_rj_fill_holes(const uint64_t *holes, int64_t nh, int64_t total,
                                                        I *op, I *ob) {
  const int64_t m = total - nh;
  // holes below the tail: holes[0, nb)
  int64_t a = 0, b = nh;
  while (a < b) {
    const int64_t mid = (a + b) >> 1;
    if ((int64_t)holes[mid] < m) a = mid + 1;
    else b = mid;
  }
  const int64_t nb = a;
  for (int64_t k = threadIdx.x; k < nb; k += blockDim.x) {
    int64_t p = total - 1 - k;
    for (;;) {
      const int64_t q = total - 1 - k - rj_count_above(holes, nb, nh, p);
      if (q == p) break;
      p = q;
    }
    while (rj_count_above(holes, nb, nh, p - 1) != rj_count_above(holes, nb, nh, p)) --p;  // p is a hole
    const int64_t d = (int64_t)holes[k];
    op[d] = op[p];
    ob[d] = ob[p];
  }
}

// Work items per group g of G consecutive partitions: icnt[g] (heavy build
// side) or icnt[NG + g] (light); the scan of the 2·NG counts lists the heavy
// items first.
__global__ void k_rj_item_counts(const int64_t *bst, const int64_t *pst, int64_t pchunk, int G, int NG,
                                 int64_t *icnt) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= NG) return;
  const int64_t p = (int64_t)g * G;
  const int64_t nb = bst[p + G] - bst[p], np = pst[p + G] - pst[p];
  const int64_t items = nb > 0 && np > 0 ? (np + pchunk - 1) / pchunk : 0;
  const bool heavy = nb > RJ_CHUNK;
  icnt[g] = heavy ? items : 0;
  icnt[NG + g] = heavy ? 0 : items;
}

__global__ void k_rj_items(const int64_t *bst, const int64_t *pst, int64_t pchunk, int G, int NG,
                           const int64_t *ioff, RJWork *work) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= NG) return;
  const int64_t p = (int64_t)g * G;
  const int64_t nb = bst[p + G] - bst[p], q0 = pst[p], q1 = pst[p + G];
  if (nb == 0 || q1 == q0) return;
  int64_t o = ioff[nb > RJ_CHUNK ? g : (int64_t)NG + g];
  for (int64_t a = q0; a < q1; a += pchunk) work[o++] = RJWork{(int32_t)p, G, a, min(q1, a + pchunk)};
}

__global__ void k_rj_unmatched(const uint8_t *matched, int64_t n, uint8_t *flags) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x)
    flags[r] = matched[r] ? 0 : 1;
}

template <typename I>
__global__ void k_rj_append(const int64_t *rows, int64_t m, int64_t off, I *own, I *other) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    own[off + i] = (I)rows[i];
    other[off + i] = I(-1);
  }
}

bool radix_join_applies(const Data &l, const Data &r, const std::vector<std::pair<int, int>> &keys,
                        int32_t join_type) {
  if (keys.size() != 1 || join_type == CAPF_JOIN_CROSS) return false;
  const char *mode = getenv("CAPF_JOIN");  // "radix" | "hash" (default: by size)
  if (mode && strcmp(mode, "hash") == 0) return false;
  if (l.nrows >= (int64_t(1) << 32) || r.nrows >= (int64_t(1) << 32)) return false;
  if (mode && strcmp(mode, "radix") == 0) return true;
  return std::max(l.nrows, r.nrows) >= (int64_t(1) << 18);
}

// The item list stays on the device: *d_nw items, `nw_max` (returned) an upper
// bound sizing the list and the COUNT grid (Σ_g ⌈np_g / pchunk⌉ ≤ NG + probe
// rows / pchunk).
static BufPtr rj_work_items(Session *s, const RJSide &bs, const RJSide &ps, int64_t probe_rows, int64_t &nw_max,
                            int64_t *d_nw) {
  // work items on the device: ⌈probe rows / pchunk⌉ per partition with rows on
  // both sides; partitions whose build side needs several LDS fills ("heavy",
  // skewed keys) are listed first so the dispatcher starts them early.  pchunk
  // shrinks with the probe side (≈16 items per CU when the rows spread evenly,
  // at least RJ_PCHUNK_MIN rows) so one hub key's probe rows — whose output is
  // (its build rows) × (its probe rows) — spread over many workgroups instead
  // of one carrying the whole product.
  constexpr int64_t NPART = (int64_t)RJ_P * RJ_P;
  // partitions grouped G at a time (a group's sorted build rows are one sorted
  // run of h, its probe rows contiguous) so an item holds about half an LDS
  // chunk of build rows: small inputs otherwise spread a few rows over each of
  // 65 536 items (s14 var2: 4 build rows per partition)
  int G = 1;
  while (G < 256 && 2 * G * bs.n <= (int64_t)(RJ_CHUNK / 2) * NPART) G *= 2;
  const int NG = (int)(NPART / G);
  int64_t pchunk = RJ_PCHUNK;
  while (pchunk > RJ_PCHUNK_MIN && pchunk * 16 * s->num_cus > probe_rows) pchunk /= 2;
  BufPtr icnt = s->alloc(8 * 2 * NG), ioff = s->alloc(8 * (2 * NG + 1));
  hipLaunchKernelGGL(k_rj_item_counts, dim3(grid_for(NG, 256)), dim3(256), 0, s->stream,
                     (const int64_t *)bs.pstart->p, (const int64_t *)ps.pstart->p, pchunk, G, NG,
                     (int64_t *)icnt->p);
  KERNEL_CHECK();
  exclusive_scan_i64_async(s, (const int64_t *)icnt->p, (int64_t *)ioff->p, 2 * NG, d_nw);
  nw_max = NG + ps.n / pchunk + 1;
  BufPtr dw = s->alloc(sizeof(RJWork) * nw_max);
  hipLaunchKernelGGL(k_rj_items, dim3(grid_for(NG, 256)), dim3(256), 0, s->stream,
                     (const int64_t *)bs.pstart->p, (const int64_t *)ps.pstart->p, pchunk, G, NG,
                     (const int64_t *)ioff->p, (RJWork *)dw->p);
  KERNEL_CHECK();
  return dw;
}

JoinPairs radix_join(Session *s, const Data &l, const Data &r,
                     const std::vector<std::pair<int, int>> &keys, int32_t join_type, const FtProgram *pred) {
  const bool left_outer = join_type == CAPF_JOIN_LEFT_OUTER || join_type == CAPF_JOIN_FULL_OUTER;
  const bool right_outer = join_type == CAPF_JOIN_RIGHT_OUTER || join_type == CAPF_JOIN_FULL_OUTER;
  // build = the smaller side
  const bool build_left = l.nrows < r.nrows;
  const Data &B = build_left ? l : r, &Pr = build_left ? r : l;
  const ColPtr &bk = B.cols[build_left ? keys[0].first : keys[0].second];
  const ColPtr &pk = Pr.cols[build_left ? keys[0].second : keys[0].first];
  const bool b_outer = build_left ? left_outer : right_outer;
  const bool p_outer = build_left ? right_outer : left_outer;
  RJSide bs = rj_partition(s, bk, B.nrows);
  if (bs.n > 0) {
    // equal keys contiguous inside each build partition (h's top 16 bits are the partition)
    KernelTimer kt(s, "rj_build_sort", 24.0 * (double)bs.n);
    BufPtr sh = s->alloc(8 * bs.n), sr = s->alloc(4 * bs.n);
    const int64_t *off = (const int64_t *)bs.pstart->p;
    size_t tmp = 0;
    // few rows per partition: one sort of the whole side by all 64 bits (the
    // top 16 are the partition, so every partition keeps its range); the
    // segmented sort's per-segment cost dominates below ~64 rows a segment
    const bool whole = bs.n < 64 * (int64_t)RJ_P * RJ_P;
    auto sort = [&](void *t) {
      if (whole)
        return rocprim::radix_sort_pairs(t, tmp, (const uint64_t *)bs.h->p, (uint64_t *)sh->p,
                                         (const uint32_t *)bs.row->p, (uint32_t *)sr->p, (size_t)bs.n, 0, 64,
                                         s->stream);
      return rocprim::segmented_radix_sort_pairs(t, tmp, (const uint64_t *)bs.h->p, (uint64_t *)sh->p,
                                                 (const uint32_t *)bs.row->p, (uint32_t *)sr->p, (unsigned)bs.n,
                                                 (unsigned)(RJ_P * RJ_P), off, off + 1, 0, 48, s->stream);
    };
    HIP_CHECK(sort(nullptr));
    BufPtr t = s->alloc(std::max<size_t>(tmp, 16));
    HIP_CHECK(sort(t->p));
    bs.h = sh;
    bs.row = sr;
  }
  // (A unique build side is the dense / hashed index's join, dense_join.hip;
  // probe-order kernels for it here — a probe of the sorted build partitions
  // and one of LDS tables — ran 3× slower and were removed.)
  RJSide ps = rj_partition(s, pk, Pr.nrows);
  // COUNT, the pair offsets and the EMIT's sub-items are enqueued without a
  // host read; ONE sync then fetches the pair total (the output's size) and
  // the sub-item count (the EMIT grid)
  BufPtr dsc = s->alloc(24);  // [0] items, [1] pairs, [2] sub-items
  int64_t *d_nw = (int64_t *)dsc->p;
  int64_t nw = 0;
  BufPtr dw = rj_work_items(s, bs, ps, Pr.nrows, nw, d_nw);
  BufPtr cnt = s->alloc(8 * nw), off = s->alloc(8 * (nw + 1));
  BufPtr nsub = s->alloc(8 * nw), soff = s->alloc(8 * (nw + 1));
  {
    KernelTimer kt(s, "rj_join_count", 12.0 * (double)(ps.n + bs.n));
    hipLaunchKernelGGL(k_rj_join_runs, dim3((unsigned)nw), dim3(RJ_JBLOCK), 0, s->stream, (const RJWork *)dw->p,
                       (const int64_t *)d_nw, (const uint64_t *)bs.h->p, (const int64_t *)bs.pstart->p,
                       (const uint64_t *)ps.h->p, (int64_t *)cnt->p);
    KERNEL_CHECK();
  }
  exclusive_scan_i64_async(s, (const int64_t *)cnt->p, (int64_t *)off->p, nw, d_nw + 1);
  hipLaunchKernelGGL(k_rj_sub_counts, dim3(grid_for(nw, 256)), dim3(256), 0, s->stream, (const int64_t *)cnt->p,
                     nw, (int64_t *)nsub->p);
  KERNEL_CHECK();
  exclusive_scan_i64_async(s, (const int64_t *)nsub->p, (int64_t *)soff->p, nw, d_nw + 2);
  HIP_CHECK(hipMemcpyAsync(s->h_scalars, d_nw + 1, 16, hipMemcpyDeviceToHost, s->stream));
  s->sync();
  const int64_t total = s->h_scalars[0], ns = s->h_scalars[1];
  // the pair list's row indexes: int32 when both sides have < 2^31 rows (half the
  // EMIT's bytes and half the index bytes of every later gather); CAPF_IDX64=1
  // keeps int64 (tests run both)
  const char *i64env = getenv("CAPF_IDX64");
  const bool idx32 = !(i64env && atoi(i64env) != 0) && l.nrows < (int64_t(1) << 31) && r.nrows < (int64_t(1) << 31);
  // Output far larger than the build side (a hub key's build rows repeat in
  // many pairs): the build side's columns are gathered once into sorted order
  // and the pairs carry sorted positions, so every later gather of a build
  // column reads consecutive rows of a run instead of one random row per pair
  // (var2 s14: the build column's gather 650 → ~200 µs).  Not for an outer
  // build side (its unmatched rows are appended by original row).
  const bool build_pos = idx32 && !b_outer && bs.n > 0 && total >= 4 * bs.n;
  DataPtr bsorted;
  if (build_pos) {
    bsorted = std::make_shared<Data>();
    bsorted->nrows = bs.n;
    for (const ColPtr &c : B.cols) {
      ColPtr pc = c->is_const && c->n > 0 ? const_column(s, *c, bs.n) : gather_column_w(s, c, bs.row->p, 4, bs.n, false);
      // no NULL key: the sorted columns are permutations of the build columns, so
      // their statistics (min / max / non-null / dense-unique, uniqueness) carry
      // over — a base column's are computed once and kept; a later dense join
      // proving its keys match then needs no statistics pass per query
      if (bs.n == B.nrows && !pc->is_const && c->type != Type::List && c->type != Type::Null) {
        std::optional<ColStats> st;
        int8_t uq;
        if (!c->lazy) st = column_stats(s, c);
        {
          std::lock_guard<std::mutex> g(c->mu);
          if (!st && c->stats) st = c->stats;
          uq = c->unique_flag;
        }
        std::lock_guard<std::mutex> g(pc->mu);
        if (st) pc->stats = st;
        pc->unique_flag = uq;
      }
      bsorted->cols.push_back(pc);
    }
  }
  BufPtr subs = s->alloc(sizeof(RJSub) * std::max<int64_t>(ns, 1));
  if (ns > 0) {
    hipLaunchKernelGGL(k_rj_subs, dim3(grid_for(nw, 256)), dim3(256), 0, s->stream, (const int64_t *)cnt->p,
                       (const int64_t *)soff->p, nw, (RJSub *)subs->p);
    KERNEL_CHECK();
  }
  auto emit = [&](auto ityp) -> JoinPairs {
    using I = decltype(ityp);
    BufPtr pm, bm;
    if (p_outer) {
      pm = s->alloc(std::max<int64_t>(Pr.nrows, 1));
      HIP_CHECK(hipMemsetAsync(pm->p, 0, std::max<int64_t>(Pr.nrows, 1), s->stream));
    }
    if (b_outer) {
      bm = s->alloc(std::max<int64_t>(B.nrows, 1));
      HIP_CHECK(hipMemsetAsync(bm->p, 0, std::max<int64_t>(B.nrows, 1), s->stream));
    }
    if (pred) {  // filtered (radix_join_filtered): inner join only
      if (p_outer || b_outer) illegal("radix_join: a filtered join must be inner");
      JoinPairs jp;
      jp.n = 0;
      jp.iw = (int)sizeof(I);
      jp.build_sorted = bsorted;
      jp.build_is_left = build_left;
      BufPtr oprobe = s->alloc(8), obuild = s->alloc(8);
      RjPred rp{};
      std::vector<BufPtr> keep;  // the operand arrays, alive until the EMIT passes are enqueued
      rp.nt = pred->nt;
      rp.np = 0;
      for (int k = 0; k < pred->nt; ++k) {
        const FtOperand *src[2] = {&pred->t[k].a, &pred->t[k].b};
        RjOp *dst[2] = {&rp.t[k].a, &rp.t[k].b};
        for (int j = 0; j < 2; ++j) {
          *dst[j] = RjOp{nullptr, nullptr, src[j]->lit, src[j]->is_lit, -1};
          if (src[j]->is_lit) continue;
          const bool on_build = (src[j]->side == 0) == build_left;
          const RJSide &sd = on_build ? bs : ps;
          BufPtr v = s->alloc(8 * std::max<int64_t>(sd.n, 1)), o = s->alloc(std::max<int64_t>(sd.n, 1));
          if (sd.n > 0) {
            hipLaunchKernelGGL(k_rj_operand, dim3(grid_for(sd.n, 256)), dim3(256), 0, s->stream, *src[j],
                               (const uint32_t *)sd.row->p, sd.n, (int64_t *)v->p, (uint8_t *)o->p);
            KERNEL_CHECK();
          }
          keep.push_back(v);
          keep.push_back(o);
          if (on_build) {
            dst[j]->val = (const int64_t *)v->p;
            dst[j]->ok = (const uint8_t *)o->p;
          } else {
            if (rp.np == RJ_PMAX) illegal("radix_join: too many probe-side filter operands");
            rp.pv[rp.np] = (const int64_t *)v->p;
            rp.po[rp.np] = (const uint8_t *)o->p;
            dst[j]->slot = rp.np++;
          }
        }
        rp.t[k].op = pred->t[k].op;
        rp.t[k].neg = pred->t[k].neg;
      }
      if (total > 0) {
        // one pass: passing pairs at their unfiltered positions, failing ones
        // listed as holes, then the tail's pairs moved into them
        const int64_t hcap = std::min<int64_t>(total, int64_t(1) << 20);
        BufPtr holes = s->alloc(8 * hcap), nh = s->alloc(8);
        HIP_CHECK(hipMemsetAsync(nh->p, 0, 8, s->stream));
        oprobe = s->alloc(sizeof(I) * total);
        obuild = s->alloc(sizeof(I) * total);
        {
          KernelTimer kt(s, "rj_join_filter_emit", 12.0 * (double)(ps.n + bs.n) + 16.0 * (double)total);
          hipLaunchKernelGGL((k_rj_emit_ranges<3, I>), dim3((unsigned)ns), dim3(RJ_JBLOCK), 0, s->stream,
                             (const RJSub *)subs->p, (const RJWork *)dw->p, (const uint64_t *)bs.h->p,
                             (const uint32_t *)bs.row->p, (const int64_t *)bs.pstart->p, (const uint64_t *)ps.h->p,
                             (const uint32_t *)ps.row->p, (const int64_t *)off->p, (I *)oprobe->p,
                             (I *)obuild->p, (uint8_t *)nullptr, (uint8_t *)nullptr, rp, build_left ? 1 : 0, build_pos ? 1 : 0,
                             (int64_t *)holes->p, (const int64_t *)nullptr, (unsigned long long *)nh->p, hcap);
          KERNEL_CHECK();
        }
        int64_t nholes = 0;
        HIP_CHECK(hipMemcpyAsync(&nholes, nh->p, 8, hipMemcpyDeviceToHost, s->stream));
        s->sync();
        if (nholes <= hcap) {
          if (nholes > 0) {
            BufPtr sorted = s->alloc(8 * nholes);
            size_t tmp = 0;
            HIP_CHECK(rocprim::radix_sort_keys(nullptr, tmp, (const uint64_t *)holes->p, (uint64_t *)sorted->p,
                                               (size_t)nholes, 0, 64, s->stream));
            BufPtr t = s->alloc(std::max<size_t>(tmp, 16));
            HIP_CHECK(rocprim::radix_sort_keys(t->p, tmp, (const uint64_t *)holes->p, (uint64_t *)sorted->p,
                                               (size_t)nholes, 0, 64, s->stream));
            hipLaunchKernelGGL(k_rj_fill_holes<I>, dim3(1), dim3(1024), 0, s->stream, (const uint64_t *)sorted->p, nholes,
                               total, (I *)oprobe->p, (I *)obuild->p);
            KERNEL_CHECK();
          }
          jp.n = total - nholes;
        } else {
          // many failing pairs: count the passes per sub-item, then write them
          BufPtr subcnt = s->alloc(8 * ns), suboff = s->alloc(8 * (ns + 1));
          {
            KernelTimer kt(s, "rj_join_filter_count", 12.0 * (double)(ps.n + bs.n));
            hipLaunchKernelGGL((k_rj_emit_ranges<1, I>), dim3((unsigned)ns), dim3(RJ_JBLOCK), 0, s->stream,
                               (const RJSub *)subs->p, (const RJWork *)dw->p, (const uint64_t *)bs.h->p,
                               (const uint32_t *)bs.row->p, (const int64_t *)bs.pstart->p, (const uint64_t *)ps.h->p,
                               (const uint32_t *)ps.row->p, (const int64_t *)off->p, (I *)nullptr,
                               (I *)nullptr, (uint8_t *)nullptr, (uint8_t *)nullptr, rp, build_left ? 1 : 0, build_pos ? 1 : 0,
                               (int64_t *)subcnt->p, (const int64_t *)nullptr, (unsigned long long *)nullptr,
                               (int64_t)0);
            KERNEL_CHECK();
          }
          jp.n = exclusive_scan_i64(s, (const int64_t *)subcnt->p, (int64_t *)suboff->p, ns);
          if (jp.n > 0) {
            KernelTimer kt(s, "rj_join_emit", 12.0 * (double)(ps.n + bs.n) + 16.0 * (double)jp.n);
            hipLaunchKernelGGL((k_rj_emit_ranges<2, I>), dim3((unsigned)ns), dim3(RJ_JBLOCK), 0, s->stream,
                               (const RJSub *)subs->p, (const RJWork *)dw->p, (const uint64_t *)bs.h->p,
                               (const uint32_t *)bs.row->p, (const int64_t *)bs.pstart->p, (const uint64_t *)ps.h->p,
                               (const uint32_t *)ps.row->p, (const int64_t *)off->p, (I *)oprobe->p,
                               (I *)obuild->p, (uint8_t *)nullptr, (uint8_t *)nullptr, rp, build_left ? 1 : 0, build_pos ? 1 : 0,
                               (int64_t *)nullptr, (const int64_t *)suboff->p, (unsigned long long *)nullptr,
                               (int64_t)0);
            KERNEL_CHECK();
          }
        }
      }
      jp.left = build_left ? obuild : oprobe;
      jp.right = build_left ? oprobe : obuild;
      return jp;
    }
    const int64_t cap = total + (p_outer ? Pr.nrows : 0) + (b_outer ? B.nrows : 0);
    BufPtr oprobe = s->alloc(sizeof(I) * std::max<int64_t>(cap, 1)),
           obuild = s->alloc(sizeof(I) * std::max<int64_t>(cap, 1));
    if (total > 0) {
      KernelTimer kt(s, "rj_join_emit", 12.0 * (double)(ps.n + bs.n) + 16.0 * (double)total);
      hipLaunchKernelGGL((k_rj_emit_ranges<0, I>), dim3((unsigned)ns), dim3(RJ_JBLOCK), 0, s->stream, (const RJSub *)subs->p,
                         (const RJWork *)dw->p, (const uint64_t *)bs.h->p, (const uint32_t *)bs.row->p,
                         (const int64_t *)bs.pstart->p, (const uint64_t *)ps.h->p, (const uint32_t *)ps.row->p,
                         (const int64_t *)off->p, (I *)oprobe->p, (I *)obuild->p,
                         p_outer ? (uint8_t *)pm->p : nullptr, b_outer ? (uint8_t *)bm->p : nullptr, RjPred{}, 0, build_pos ? 1 : 0,
                         (int64_t *)nullptr, (const int64_t *)nullptr, (unsigned long long *)nullptr, (int64_t)0);
      KERNEL_CHECK();
    }
    // (total = 0: no pair, the outer sides' flags stay clear — every row is unmatched)
    int64_t m = total;
    // unmatched rows of the outer sides (NULL keys included: never flagged)
    auto append_unmatched = [&](const BufPtr &matched, int64_t n, I *own, I *other) {
      if (n == 0) return;
      BufPtr flags = s->alloc(n);
      hipLaunchKernelGGL(k_rj_unmatched, dim3(grid_for(n, 256)), dim3(256), 0, s->stream,
                         (const uint8_t *)matched->p, n, (uint8_t *)flags->p);
      KERNEL_CHECK();
      int64_t k = 0;
      BufPtr rows = compact_flags(s, (const uint8_t *)flags->p, n, &k);
      if (k > 0) {
        hipLaunchKernelGGL(k_rj_append<I>, dim3(grid_for(k, 256)), dim3(256), 0, s->stream,
                           (const int64_t *)rows->p, k, m, own, other);
        KERNEL_CHECK();
      }
      m += k;
    };
    if (p_outer) append_unmatched(pm, Pr.nrows, (I *)oprobe->p, (I *)obuild->p);
    if (b_outer) append_unmatched(bm, B.nrows, (I *)obuild->p, (I *)oprobe->p);
    JoinPairs jp;
    jp.left = build_left ? obuild : oprobe;
    jp.right = build_left ? oprobe : obuild;
    jp.n = m;
    jp.iw = (int)sizeof(I);
    jp.build_sorted = bsorted;
    jp.build_is_left = build_left;
    return jp;

  };
  return idx32 ? emit(int32_t{}) : emit(int64_t{});
}

// The Filter's names are the join's output names: the left input's columns,
// then the right input's (runtime.cpp, Kind::Join).
bool radix_join_filtered(Session *s, const Program &pred, const std::vector<std::string> &names, const Data &l,
                         const Data &r, const std::vector<std::pair<int, int>> &keys, int32_t join_type,
                         JoinPairs &out) {
  const char *fe = getenv("CAPF_RJ_FILTER");  // 0 (tuning/tests): join, then filter
  if (fe && atoi(fe) == 0) return false;
  if (join_type != CAPF_JOIN_INNER || names.size() != l.cols.size() + r.cols.size()) return false;
  if (!radix_join_applies(l, r, keys, join_type) || dense_join_possible(s, l, r, keys, join_type)) return false;
  Data both;
  both.nrows = 0;
  both.cols = l.cols;
  both.cols.insert(both.cols.end(), r.cols.begin(), r.cols.end());
  FtProgram fp{};
  if (!ft_compile(pred, names, both, fp)) return false;
  // the side of every column operand (ft_compile resolved the same names)
  auto side_of = [&](const std::string &nm) {
    for (size_t k = 0; k < names.size(); ++k)
      if (names[k] == nm) return k < l.cols.size() ? 0 : 1;
    return -1;
  };
  size_t pc = 0;
  const auto &c = pred.code;
  for (int k = 0; k < fp.nt; ++k) {
    FtOperand *ops[2] = {&fp.t[k].a, &fp.t[k].b};
    for (int j = 0; j < 2; ++j) {
      const Instr &in = c[pc + (size_t)j];
      if (in.op == OP_COL) {
        const int sd = side_of(pred.names[(size_t)in.i]);
        if (sd < 0) return false;
        ops[j]->side = sd;
      }
    }
    pc += 3;
    if (pc < c.size() && c[pc].op == OP_NOT) pc += 1;
  }
  int per_side[2] = {0, 0};
  for (int k = 0; k < fp.nt; ++k) {
    if (!fp.t[k].a.is_lit) ++per_side[fp.t[k].a.side];
    if (!fp.t[k].b.is_lit) ++per_side[fp.t[k].b.side];
  }
  if (per_side[0] > RJ_PMAX || per_side[1] > RJ_PMAX) return false;  // (probe operands live in LDS)
  out = radix_join(s, l, r, keys, join_type, &fp);
  return true;
}

}  // namespace capf
