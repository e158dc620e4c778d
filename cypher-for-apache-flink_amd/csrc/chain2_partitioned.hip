// chain2_partitioned.hip — radix-partitioned LDS histograms for the fused
// 2-hop count (replaces the global-atomic k_chain2_hist for large rel tables).
//
// The two per-node histograms of the 2-hop message passing
//   in[b]  = |{r1 : end(r1) = b, start(r1) ∈ S_a}|
//   out[b] = |{r2 : start(r2) = b, end(r2) ∈ S_c}|
// are GROUP BY counts on a 2^24-key domain at R-MAT s24: far larger than LDS,
// and random device-scope atomics run at ~11 G/s on MI355X (measured: 47.7 ms
// for the 5.4e8 updates at s24).  This is the radix-partitioned hash join of
// the north star, partitions sized to the 160 KiB LDS:
//   P1 k_c2_count   per tile of 32 Ki rels: LDS counts per run = (side, bucket),
//                   bucket = 32 Ki consecutive node ids; self-loop term
//   scan            uint32 exclusive scan → offset of every (run, tile)
//   P2 k_c2_scatter per tile, in 4 steps of 8 Ki rels held in registers: LDS
//                   counting sort of the step's keys by run, then every run
//                   written out coalesced as uint16 (the key's low 15 bits);
//                   48 KiB LDS → 3 blocks per CU overlap load and write-out
//   P3 k_c2_bucket  per (run, chunk): 128 KiB LDS histogram from 16-B loads,
//                   flushed to the global histogram (plain store when the run
//                   is one chunk)
//   P4 k_chain2_dot Σ in·out (fused_count.hip)
// Bytes per rel at int64 reference width: P1 16, P2 16 + 4, P3 4.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "capf_internal.h"
#include "device_common.h"

namespace capf {

constexpr int C2_BITS = 15;
constexpr int C2_BW = 1 << C2_BITS;   // node ids per bucket = uint32 bins in LDS (128 KiB)
constexpr int C2_BLOCK = 256;         // P1
constexpr int64_t C2_TILE = 32768;    // rels per P1/P2 tile
constexpr int C2_MAX_RUNS = 2048;     // 2 sides × 1024 buckets (2^25 nodes)
constexpr int C2_SBLOCK = 512;        // P2
constexpr int C2_SPT = 16;            // P2 rels per thread per step
constexpr int C2_STEP = C2_SBLOCK * C2_SPT;  // 8 Ki rels per step, 16 Ki keys staged

// F32: the four id columns are FOR32-encoded (uint32 + per-column base);
// otherwise plain int64.  Half the P1/P2 read bytes.
template <bool F32>
struct C2Cols {
  const void *u1, *v1, *u2, *v2;
  int64_t bu1, bv1, bu2, bv2;  // FOR32 bases (0 for plain columns)
  int64_t n;
  int64_t lo, hi;  // dense node range of S_a = S_b = S_c (MAP_ONES)
  int nb;          // buckets per side
  int64_t ntiles;
  NodeMix mix;     // histogram index = node_mix(id − lo) on a 2^k domain
  int64_t hist_len;  // 2^k (a multiple of C2_BW)
};

// key of b = `to` when both endpoints lie in the node range, else -1
template <bool F32>
__device__ inline int64_t c2_ld(const void *p, int64_t base, int64_t e) {
  if (F32) return base + (int64_t)((const uint32_t *)p)[e];
  return ((const int64_t *)p)[e];
}

template <bool F32>
__device__ inline int64_t c2_key(const C2Cols<F32> &c, int64_t from, int64_t to) {
  const uint64_t len = (uint64_t)(c.hi - c.lo) + 1;
  const bool ok = ((uint64_t)(from - c.lo) < len) & ((uint64_t)(to - c.lo) < len);  // branch-free
  return ok ? (int64_t)node_mix((uint32_t)(to - c.lo), c.mix) : -1;
}

// LDS bank spreading.  R-MAT ids are skewed bit by bit (each bit is 0 with
// probability .76), so ids whose low 5 bits are all zero — one LDS bank —
// take ~25 % of the keys.  Folding bits 5-14 into the bank bits (a bijection
// that only rewrites the low 5 bits) cuts that bank's share to ~6 %.
__device__ inline uint32_t lds_slot(uint32_t x) { return x ^ ((x >> 5) & 31) ^ ((x >> 10) & 31); }

struct C2Keys {
  int64_t ki, ko;
  bool loop;
};

template <bool F32>
__device__ inline C2Keys c2_load(const C2Cols<F32> &c, int64_t e) {
  const int64_t x1 = c2_ld<F32>(c.u1, c.bu1, e), y1 = c2_ld<F32>(c.v1, c.bv1, e);
  const int64_t x2 = c.u2 == c.u1 ? x1 : c2_ld<F32>(c.u2, c.bu2, e);
  const int64_t y2 = c.v2 == c.v1 ? y1 : c2_ld<F32>(c.v2, c.bv2, e);
  C2Keys k;
  k.ki = c2_key(c, x1, y1);  // in-key:  end(r1)   when start(r1) ∈ S_a
  k.ko = c2_key(c, y2, x2);  // out-key: start(r2) when end(r2)   ∈ S_c
  k.loop = k.ki >= 0 && k.ko >= 0 && y1 == x2;
  return k;
}

template <bool F32>
__global__ __launch_bounds__(C2_BLOCK) void k_c2_count(C2Cols<F32> c, uint32_t *counts,
                                                        unsigned long long *loops) {
  __shared__ uint32_t cnt[C2_MAX_RUNS];
  for (int i = threadIdx.x; i < 2 * c.nb; i += C2_BLOCK) cnt[i] = 0;
  __syncthreads();
  const int64_t t = blockIdx.x;
  const int64_t e0 = t * C2_TILE, e1 = min(e0 + C2_TILE, c.n);
  unsigned long long lp = 0;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += C2_BLOCK) {
    const C2Keys k = c2_load(c, e);
    if (k.ki >= 0) atomicAdd(&cnt[k.ki >> C2_BITS], 1u);
    if (k.ko >= 0) atomicAdd(&cnt[c.nb + (k.ko >> C2_BITS)], 1u);
    lp += k.loop ? 1ull : 0ull;
  }
  __syncthreads();
  // layout [run][tile]: one exclusive scan gives every (run, tile) offset
  for (int i = threadIdx.x; i < 2 * c.nb; i += C2_BLOCK) counts[(int64_t)i * c.ntiles + t] = cnt[i];
  lp = wave_reduce_sum(lp);
  if (lane_id() == 0 && lp) atomicAdd(loops, lp);
}

template <bool F32>
__global__ __launch_bounds__(C2_SBLOCK) void k_c2_scatter(C2Cols<F32> c, const uint32_t *offsets,
                                                           uint16_t *part) {
  __shared__ uint16_t stage[2 * C2_STEP];          // 32 KiB
  __shared__ uint32_t cur[C2_MAX_RUNS];            // step counts → cursors → run ends
  __shared__ uint16_t start[C2_MAX_RUNS];          // run starts in the stage
  __shared__ uint16_t tilepos[C2_MAX_RUNS];        // elements of the run written by earlier steps
  __shared__ uint32_t lds_scan[17];
  const int64_t t = blockIdx.x;
  const int nr = 2 * c.nb;
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  for (int i = threadIdx.x; i < nr; i += C2_SBLOCK) tilepos[i] = 0;
  const int64_t e0 = t * C2_TILE, e1 = min(e0 + C2_TILE, c.n);
  for (int64_t s0 = e0; s0 < e1; s0 += C2_STEP) {
    for (int i = threadIdx.x; i < nr; i += C2_SBLOCK) cur[i] = 0;
    __syncthreads();
    uint32_t kin[C2_SPT], kout[C2_SPT];  // run << 15 | low bits
#pragma unroll
    for (int j = 0; j < C2_SPT; ++j) {
      const int64_t e = s0 + (int64_t)j * C2_SBLOCK + threadIdx.x;
      kin[j] = kout[j] = NONE;
      if (e < e1) {
        const C2Keys k = c2_load(c, e);
        if (k.ki >= 0) kin[j] = (uint32_t)k.ki;
        if (k.ko >= 0) kout[j] = (uint32_t)(k.ko + ((int64_t)c.nb << C2_BITS));
      }
      if (kin[j] != NONE) atomicAdd(&cur[kin[j] >> C2_BITS], 1u);
      if (kout[j] != NONE) atomicAdd(&cur[kout[j] >> C2_BITS], 1u);
    }
    __syncthreads();
    // exclusive scan of the step's run counts (4 runs per thread)
    uint32_t cs[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 4 * threadIdx.x + q;
      cs[q] = r < nr ? cur[r] : 0u;
      sum += cs[q];
    }
    uint32_t total;
    uint32_t ex = block_exclusive_scan(sum, lds_scan, total);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 4 * threadIdx.x + q;
      if (r < nr) {
        start[r] = (uint16_t)ex;
        cur[r] = ex;
      }
      ex += cs[q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < C2_SPT; ++j) {
      if (kin[j] != NONE) stage[atomicAdd(&cur[kin[j] >> C2_BITS], 1u)] = (uint16_t)(kin[j] & (C2_BW - 1));
      if (kout[j] != NONE) stage[atomicAdd(&cur[kout[j] >> C2_BITS], 1u)] = (uint16_t)(kout[j] & (C2_BW - 1));
    }
    __syncthreads();
    // write-out: consecutive stage slots of a run go to consecutive addresses
    for (uint32_t i = threadIdx.x; i < total; i += C2_SBLOCK) {
      int lo = 0, hi = nr;  // last run r with start[r] <= i (the one holding slot i)
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (start[mid] <= i) lo = mid; else hi = mid;
      }
      part[(int64_t)offsets[(int64_t)lo * c.ntiles + t] + tilepos[lo] + (i - start[lo])] = stage[i];
    }
    __syncthreads();
    for (int r = threadIdx.x; r < nr; r += C2_SBLOCK) tilepos[r] += (uint16_t)(cur[r] - start[r]);
    __syncthreads();
  }
}

__global__ void k_run_starts(const uint32_t *offs, int64_t ntiles, int nr, const uint32_t *total,
                             int64_t *starts) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nr) starts[k] = offs[(int64_t)k * ntiles];
  if (k == nr) starts[k] = *total;
}

struct C2Chunk {
  int64_t begin, end;  // element range in `part`
  int64_t hist_base;   // first global histogram index of the bucket
  int32_t exclusive;   // 1: the bucket is this one chunk → plain store
  int32_t side;
};

constexpr int C2_HBLOCK = 1024;

__global__ __launch_bounds__(C2_HBLOCK) void k_c2_bucket(const C2Chunk *chunks,
                                                          const uint16_t *part, uint32_t *h_in,
                                                          uint32_t *h_out, int64_t hist_len) {
  extern __shared__ __attribute__((aligned(16))) uint32_t bins[];  // C2_BW entries
  const C2Chunk ch = chunks[blockIdx.x];
  uint32_t *hist = ch.side ? h_out : h_in;
  for (int i = threadIdx.x; i < C2_BW; i += C2_HBLOCK) bins[i] = 0;
  __syncthreads();
  // scalar head/tail, 16-B (8 keys) loads in the aligned body
  const int64_t a0 = min(ch.end, (ch.begin + 7) & ~int64_t(7));
  const int64_t a1 = max(a0, ch.end & ~int64_t(7));
  for (int64_t i = ch.begin + threadIdx.x; i < a0; i += C2_HBLOCK) atomicAdd(&bins[lds_slot(part[i])], 1u);
  for (int64_t i = a1 + threadIdx.x; i < ch.end; i += C2_HBLOCK) atomicAdd(&bins[lds_slot(part[i])], 1u);
  const uint4 *p4 = (const uint4 *)(part + a0);
  const int64_t n4 = (a1 - a0) / 8;
  for (int64_t i = threadIdx.x; i < n4; i += C2_HBLOCK) {
    const uint4 v = p4[i];
    atomicAdd(&bins[lds_slot(v.x & 0xFFFF)], 1u);
    atomicAdd(&bins[lds_slot(v.x >> 16)], 1u);
    atomicAdd(&bins[lds_slot(v.y & 0xFFFF)], 1u);
    atomicAdd(&bins[lds_slot(v.y >> 16)], 1u);
    atomicAdd(&bins[lds_slot(v.z & 0xFFFF)], 1u);
    atomicAdd(&bins[lds_slot(v.z >> 16)], 1u);
    atomicAdd(&bins[lds_slot(v.w & 0xFFFF)], 1u);
    atomicAdd(&bins[lds_slot(v.w >> 16)], 1u);
  }
  __syncthreads();
  const int64_t lim = min((int64_t)C2_BW, hist_len - ch.hist_base);
  for (int i = threadIdx.x; i < lim; i += C2_HBLOCK) {
    const uint32_t v = bins[lds_slot(i)];
    if (ch.exclusive)
      hist[ch.hist_base + i] = v;
    else if (v)
      atomicAdd(&hist[ch.hist_base + i], v);
  }
}

// ===================================================================== v3
// Single-pass partitioning: every tile of 16 Ki rels sorts its keys by run in
// LDS (keys held in registers, counted, scanned, staged) and writes them
// CONTIGUOUSLY into a tile-private region of `part` (fixed stride 2·TILE),
// together with one packed (start | count << 16) word per run.  No count
// pass, no global scan: the rels are read once (16-B loads, 4 rels per lane).
// P3 then gathers, for a run, its segments across a range of tiles into the
// LDS histogram — one tile per lane, 16-B loads along the segment.  The
// P3 work list is built on the device, so the whole count runs without a
// host round trip.
constexpr int64_t C3_TILE = 16384;
constexpr int C3_BLOCK = 512;
constexpr int C3_GROUPS = (int)(C3_TILE / (4 * C3_BLOCK));  // 8 groups of 4 rels per thread
constexpr int C3_SPT = 4 * C3_GROUPS;                       // 32 rels per thread

// 4 consecutive ids starting at e (16-B aligned when e % 4 == 0)
template <bool F32>
__device__ inline void c3_load4(const void *p, int64_t base, int64_t e, int64_t e1, int64_t v[4]) {
  if (e + 4 <= e1) {
    if (F32) {
      const uint4 q = *(const uint4 *)((const uint32_t *)p + e);
      v[0] = base + (int64_t)q.x;
      v[1] = base + (int64_t)q.y;
      v[2] = base + (int64_t)q.z;
      v[3] = base + (int64_t)q.w;
    } else {
      const longlong2 q0 = *(const longlong2 *)((const int64_t *)p + e);
      const longlong2 q1 = *(const longlong2 *)((const int64_t *)p + e + 2);
      v[0] = q0.x;
      v[1] = q0.y;
      v[2] = q1.x;
      v[3] = q1.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = e + k < e1 ? c2_ld<F32>(p, base, e + k) : 0;
  }
}

template <bool F32>
__global__ __launch_bounds__(C3_BLOCK) void k_c3_partition(C2Cols<F32> c, uint16_t *part,
                                                            uint32_t *meta,
                                                            unsigned long long *loops,
                                                            int64_t t_base) {
  __shared__ __attribute__((aligned(16))) uint16_t stage[2 * C3_TILE];  // 64 KiB
  __shared__ uint32_t cur[C2_MAX_RUNS];
  __shared__ uint32_t lds_scan[17];
  const int64_t t = t_base + blockIdx.x;
  const int nr = 2 * c.nb;
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  for (int i = threadIdx.x; i < nr; i += C3_BLOCK) cur[i] = 0;
  __syncthreads();
  const int64_t e0 = t * C3_TILE, e1 = min(e0 + C3_TILE, c.n);
  uint32_t kin[C3_SPT], kout[C3_SPT];  // run << 15 | low bits
  unsigned long long lp = 0;
  const bool alias_u = c.u2 == c.u1, alias_v = c.v2 == c.v1;
#pragma unroll
  for (int g = 0; g < C3_GROUPS; ++g) {
    const int64_t e = e0 + 4 * ((int64_t)g * C3_BLOCK + threadIdx.x);
    int64_t x1[4], y1[4], x2[4], y2[4];
    c3_load4<F32>(c.u1, c.bu1, e, e1, x1);
    c3_load4<F32>(c.v1, c.bv1, e, e1, y1);
    if (alias_u) {
#pragma unroll
      for (int k = 0; k < 4; ++k) x2[k] = x1[k];
    } else {
      c3_load4<F32>(c.u2, c.bu2, e, e1, x2);
    }
    if (alias_v) {
#pragma unroll
      for (int k = 0; k < 4; ++k) y2[k] = y1[k];
    } else {
      c3_load4<F32>(c.v2, c.bv2, e, e1, y2);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = 4 * g + k;
      kin[j] = kout[j] = NONE;
      if (e + k < e1) {
        const int64_t ki = c2_key(c, x1[k], y1[k]);  // end(r1)   when start(r1) ∈ S_a
        const int64_t ko = c2_key(c, y2[k], x2[k]);  // start(r2) when end(r2)   ∈ S_c
        if (ki >= 0) kin[j] = (uint32_t)ki;
        if (ko >= 0) kout[j] = (uint32_t)(ko + ((int64_t)c.nb << C2_BITS));
        lp += (ki >= 0 && ko >= 0 && y1[k] == x2[k]) ? 1ull : 0ull;
      }
      if (kin[j] != NONE) atomicAdd(&cur[kin[j] >> C2_BITS], 1u);
      if (kout[j] != NONE) atomicAdd(&cur[kout[j] >> C2_BITS], 1u);
    }
  }
  __syncthreads();
  uint32_t cs[4], sum = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 4 * threadIdx.x + q;
    cs[q] = r < nr ? cur[r] : 0u;
    sum += cs[q];
  }
  uint32_t total;
  uint32_t ex = block_exclusive_scan(sum, lds_scan, total);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 4 * threadIdx.x + q;
    if (r < nr) {
      cur[r] = ex;
      meta[t * nr + r] = ex | (cs[q] << 16);  // [tile][run], transposed later
    }
    ex += cs[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < C3_SPT; ++j) {
    if (kin[j] != NONE) stage[atomicAdd(&cur[kin[j] >> C2_BITS], 1u)] = (uint16_t)(kin[j] & (C2_BW - 1));
    if (kout[j] != NONE) stage[atomicAdd(&cur[kout[j] >> C2_BITS], 1u)] = (uint16_t)(kout[j] & (C2_BW - 1));
  }
  __syncthreads();
  // the stage IS the region's layout: contiguous 16-B copy-out
  uint4 *dst = (uint4 *)(part + t * 2 * C3_TILE);
  const uint4 *src = (const uint4 *)stage;
  const uint32_t n16 = (total + 7) / 8;
  for (uint32_t i = threadIdx.x; i < n16; i += C3_BLOCK) dst[i] = src[i];
  lp = wave_reduce_sum(lp);
  if (lane_id() == 0 && lp) atomicAdd(loops, lp);
}

// P1, second form: full tiles only (the ragged last tile goes through
// k_c3_partition), branch-free keys, and each key's rank inside its run taken
// from the counting atomic itself — one LDS atomic per key instead of two.
// Keys outside the node range go to a dummy run nr (counted and staged like
// the others, never read back), so no lane is ever masked off.
template <bool F32>
__device__ inline void c4_load4(const void *p, int64_t base, int64_t e, int64_t v[4]) {
  if (F32) {
    const uint4 q = *(const uint4 *)((const uint32_t *)p + e);
    v[0] = base + (int64_t)q.x;
    v[1] = base + (int64_t)q.y;
    v[2] = base + (int64_t)q.z;
    v[3] = base + (int64_t)q.w;
  } else {
    const longlong2 q0 = *(const longlong2 *)((const int64_t *)p + e);
    const longlong2 q1 = *(const longlong2 *)((const int64_t *)p + e + 2);
    v[0] = q0.x;
    v[1] = q0.y;
    v[2] = q1.x;
    v[3] = q1.y;
  }
}

template <bool F32, int BLOCK, bool ALIAS>
__global__ __launch_bounds__(BLOCK) void k_c4_partition(C2Cols<F32> c, uint16_t *part,
                                                         uint32_t *meta,
                                                         unsigned long long *loops) {
  constexpr int RPT = (int)(C3_TILE / BLOCK);
  constexpr int GROUPS = RPT / 4;
  constexpr int RUNS_PT = (C2_MAX_RUNS + BLOCK - 1) / BLOCK;
  __shared__ __attribute__((aligned(16))) uint16_t stage[2 * C3_TILE];  // 64 KiB
  __shared__ uint32_t cur[C2_MAX_RUNS];
  __shared__ uint32_t lds_scan[17];
  const int64_t t = blockIdx.x;
  const int nr = 2 * c.nb;
  for (int i = threadIdx.x; i < C2_MAX_RUNS; i += BLOCK) cur[i] = 0;
  __syncthreads();
  const int64_t e0 = t * C3_TILE;
  const uint64_t len = (uint64_t)(c.hi - c.lo) + 1;
  const uint32_t out_run0 = (uint32_t)c.nb << C2_BITS;
  const uint32_t dummy = (uint32_t)nr << C2_BITS;
  uint32_t kin[RPT], kout[RPT], rank[RPT];
  uint32_t lp = 0;
#pragma unroll
  for (int g = 0; g < GROUPS; ++g) {
    const int64_t e = e0 + 4 * ((int64_t)g * BLOCK + threadIdx.x);
    int64_t x1[4], y1[4], x2[4], y2[4];
    c4_load4<F32>(c.u1, c.bu1, e, x1);
    c4_load4<F32>(c.v1, c.bv1, e, y1);
    if (!ALIAS) {
      c4_load4<F32>(c.u2, c.bu2, e, x2);
      c4_load4<F32>(c.v2, c.bv2, e, y2);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = 4 * g + k;
      const int64_t a = x1[k] - c.lo, bq = y1[k] - c.lo;
      const int64_t cq = (ALIAS ? x1[k] : x2[k]) - c.lo;
      const int64_t d = (ALIAS ? y1[k] : y2[k]) - c.lo;
      const bool in_ok = ((uint64_t)a < len) & ((uint64_t)bq < len);   // start(r1) ∈ S_a
      const bool out_ok = ((uint64_t)d < len) & ((uint64_t)cq < len);  // end(r2) ∈ S_c
      // in range ⇒ the offsets fit 32 bits: only those stay live
      const uint32_t b32 = (uint32_t)bq, c32 = (uint32_t)cq;
      kin[j] = in_ok ? node_mix(b32, c.mix) : dummy;
      kout[j] = out_ok ? node_mix(c32, c.mix) + out_run0 : dummy;
      lp += (in_ok & out_ok & (b32 == c32)) ? 1u : 0u;
      const uint32_t ri = atomicAdd(&cur[lds_slot(kin[j] >> C2_BITS)], 1u);
      const uint32_t ro = atomicAdd(&cur[lds_slot(kout[j] >> C2_BITS)], 1u);
      rank[j] = ri | (ro << 16);
    }
    __builtin_amdgcn_sched_barrier(0);  // bound what the scheduler keeps in flight
  }
  // launder the keys: stops the compiler from keeping the count phase's LDS
  // addresses alive across the scan (32 extra VGPRs → spills)
#pragma unroll
  for (int j = 0; j < RPT; ++j) asm volatile("" : "+v"(kin[j]), "+v"(kout[j]));
  __syncthreads();
  uint32_t cs[RUNS_PT], sum = 0;
#pragma unroll
  for (int q = 0; q < RUNS_PT; ++q) {
    const int r = RUNS_PT * threadIdx.x + q;
    cs[q] = r <= nr ? cur[lds_slot(r)] : 0u;
    sum += cs[q];
  }
  uint32_t total;
  uint32_t ex = block_exclusive_scan(sum, lds_scan, total);
#pragma unroll
  for (int q = 0; q < RUNS_PT; ++q) {
    const int r = RUNS_PT * threadIdx.x + q;
    if (r <= nr) cur[lds_slot(r)] = ex;
    if (r < nr) meta[t * nr + r] = ex | (cs[q] << 16);  // [tile][run], transposed later
    ex += cs[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    stage[cur[lds_slot(kin[j] >> C2_BITS)] + (rank[j] & 0xFFFF)] = (uint16_t)(kin[j] & (C2_BW - 1));
    stage[cur[lds_slot(kout[j] >> C2_BITS)] + (rank[j] >> 16)] = (uint16_t)(kout[j] & (C2_BW - 1));
    if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  // the stage IS the region's layout: contiguous 16-B copy-out
  uint4 *dst = (uint4 *)(part + t * 2 * C3_TILE);
  const uint4 *src = (const uint4 *)stage;
  const uint32_t n16 = (total + 7) / 8;
  for (uint32_t i = threadIdx.x; i < n16; i += BLOCK) dst[i] = src[i];
  unsigned long long lp64 = wave_reduce_sum((unsigned long long)lp);
  if (lane_id() == 0 && lp64) atomicAdd(loops, lp64);
}

template <bool F32, int BLOCK>
static void launch_c4(Session *s, const C2Cols<F32> &c, uint16_t *part, uint32_t *meta,
                      unsigned long long *d_loops) {
  const int64_t nfull = c.n / C3_TILE;
  if (nfull > 0) {
    if (c.u2 == c.u1 && c.v2 == c.v1)
      hipLaunchKernelGGL((k_c4_partition<F32, BLOCK, true>), dim3((unsigned)nfull), dim3(BLOCK), 0,
                         s->stream, c, part, meta, d_loops);
    else
      hipLaunchKernelGGL((k_c4_partition<F32, BLOCK, false>), dim3((unsigned)nfull), dim3(BLOCK),
                         0, s->stream, c, part, meta, d_loops);
    KERNEL_CHECK();
  }
  if (nfull < c.ntiles) {  // the ragged last tile
    hipLaunchKernelGGL(k_c3_partition<F32>, dim3(1), dim3(C3_BLOCK), 0, s->stream, c, part, meta,
                       d_loops, nfull);
    KERNEL_CHECK();
  }
}

// [tile][run] → [run][tile] and per-run totals.  A block moves 32 runs ×
// 256 tiles through a 32×33 LDS tile (8 steps) and adds each run's count
// once per block (one atomic per run per 256 tiles, not per 32).
constexpr int C3_TT = 256;
__global__ __launch_bounds__(256) void k_c3_transpose(const uint32_t *meta, uint32_t *meta_t,
                                                       int64_t ntiles, int nr,
                                                       unsigned long long *run_total) {
  __shared__ uint32_t tilebuf[32][33];
  const int r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads = 32 × 8
  unsigned int cnt[4] = {0, 0, 0, 0};                       // runs r0 + ty + 8q
  for (int64_t t0 = (int64_t)blockIdx.x * C3_TT; t0 < min(ntiles, ((int64_t)blockIdx.x + 1) * C3_TT);
       t0 += 32) {
    for (int k = ty; k < 32; k += 8) {
      const int64_t t = t0 + k;
      const int r = r0 + tx;
      tilebuf[k][tx] = (t < ntiles && r < nr) ? meta[t * nr + r] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = ty + 8 * q;
      const int r = r0 + k;
      const int64_t t = t0 + tx;
      const uint32_t v = tilebuf[tx][k];
      if (t < ntiles && r < nr) meta_t[(int64_t)r * ntiles + t] = v;
      cnt[q] += v >> 16;
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned int c = cnt[q];
    for (int d = 16; d > 0; d >>= 1) c += __shfl_xor(c, d, 32);
    const int r = r0 + ty + 8 * q;
    if (tx == 0 && c && r < nr) atomicAdd(&run_total[r], (unsigned long long)c);
  }
}

struct C3Unit {
  int32_t run;
  int32_t exclusive;   // the run is this one unit → plain store
  int64_t t0, t1;      // tile range
};

constexpr int C3_UBLOCK = 1024;

// Work list of P3 on the device.  With hash-partitioned runs the run sizes
// are near-uniform (max/mean ≈ 1.6 at s24), so every run is ONE unit — an
// exclusive one, whose plain stores cover all 2^15 bins of its bucket: the
// histograms need no memset, empty runs included (they store zeros).  A run
// holding more than twice the mean (a hub-heavy bucket) is split into tile
// ranges that flush with atomic adds into bins cleared by k_c3_zero.  Units
// stay in run order: k_c3_bucket maps them onto XCDs in groups of
// consecutive runs (c3_unit_of).
__global__ __launch_bounds__(C3_UBLOCK) void k_c3_units(const unsigned long long *run_total,
                                                         int nr, int64_t ntiles, C3Unit *units,
                                                         int32_t *nunits, int32_t *split) {
  __shared__ unsigned long long lds64[17];
  __shared__ uint32_t lds32[17];
  unsigned long long cnt[2], tot = 0;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 2 * threadIdx.x + q;
    cnt[q] = r < nr ? run_total[r] : 0ull;
    tot += cnt[q];
  }
  unsigned long long total;
  block_exclusive_scan(tot, lds64, total);
  const unsigned long long target = max(2 * total / (unsigned long long)max(nr, 1), 65536ull);
  const int64_t maxsplit = max<int64_t>(1, ntiles / 256);
  uint32_t nu[2], nsum = 0;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 2 * threadIdx.x + q;
    nu[q] = r >= nr ? 0u
            : cnt[q] ? (uint32_t)min<int64_t>((int64_t)((cnt[q] + target - 1) / target), maxsplit)
                     : 1u;
    nsum += nu[q];
  }
  uint32_t ntot;
  uint32_t off = block_exclusive_scan(nsum, lds32, ntot);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 2 * threadIdx.x + q;
    if (!nu[q]) continue;
    for (uint32_t k = 0; k < nu[q]; ++k) {
      C3Unit u;
      u.run = r;
      u.exclusive = nu[q] == 1;
      u.t0 = cnt[q] ? ntiles * k / nu[q] : 0;
      u.t1 = cnt[q] ? ntiles * (k + 1) / nu[q] : 0;
      units[off + k] = u;
    }
    off += nu[q];
    split[r] = nu[q] > 1;
  }
  if (threadIdx.x == 0) *nunits = (int32_t)ntot;
}

// XCD-aware unit placement.  Workgroup i runs on XCD i mod 8, and P3 holds
// one workgroup per CU (128 KiB LDS), 32 per XCD.  Runs r and r+1 are
// adjacent in every tile's region, so their ~64-B segments share 128-B
// lines: giving each XCD 32 CONSECUTIVE units per 256-workgroup wave lets
// those blocks (sweeping the tiles in the same order at the same pace) hit
// the shared lines in their own L2 instead of fetching each line per run.
__device__ inline int c3_unit_of(int i) {
  return (i / 256) * 256 + (i % 8) * 32 + (i % 256) / 8;
}

// Clears the buckets of split runs (their units flush with atomic adds).
__global__ __launch_bounds__(256) void k_c3_zero(const int32_t *split, int nb, uint32_t *h_in,
                                                  uint32_t *h_out) {
  const int r = blockIdx.y;
  if (!split[r]) return;
  uint4 *p = (uint4 *)((r >= nb ? h_out : h_in) + (int64_t)(r % nb) * C2_BW);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < C2_BW / 4; i += gridDim.x * 256)
    p[i] = make_uint4(0, 0, 0, 0);
}

template <int K, int Q>
__global__ __launch_bounds__(C2_HBLOCK) void k_c3_bucket(const C3Unit *units,
                                                          const int32_t *nunits,
                                                          const uint16_t *part,
                                                          const uint32_t *meta_t, int64_t ntiles,
                                                          int nb, uint32_t *h_in, uint32_t *h_out,
                                                          int64_t hist_len) {
  const int ui = c3_unit_of((int)blockIdx.x);
  if (ui >= *nunits) return;
  extern __shared__ __attribute__((aligned(16))) uint32_t bins[];  // C2_BW entries
  const C3Unit u = units[ui];
  uint32_t *hist = u.run >= nb ? h_out : h_in;
  const int64_t hist_base = (int64_t)(u.run % nb) * C2_BW;
  for (int i = threadIdx.x; i < C2_BW; i += C2_HBLOCK) bins[i] = 0;
  __syncthreads();
  const int wave = threadIdx.x / WAVE, lane = lane_id();
  constexpr int NW = C2_HBLOCK / WAVE;
  const uint32_t *m = meta_t + (int64_t)u.run * ntiles;
  // One tile per lane, C3_K tiles per lane at once, C3_Q 16-B pieces of each
  // segment per step: the segments are short (≈32 keys) and scattered, so the
  // kernel is bound by memory latency unless many loads are in flight.
  // the unit's tiles are split contiguously over the waves
  const int64_t ut = u.t1 - u.t0;
  const int64_t w0 = u.t0 + ut * wave / NW, w1 = u.t0 + ut * (wave + 1) / NW;
  for (int64_t tb = w0; tb < w1; tb += (int64_t)WAVE * K) {
    uint32_t st[K], len[K], a0[K], nq[K];
    const uint4 *seg[K];
    uint32_t maxq = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int64_t t = tb + k * WAVE + lane;
      const uint32_t w = t < w1 ? m[t] : 0u;
      st[k] = w & 0xFFFF;
      len[k] = w >> 16;
      a0[k] = st[k] & ~7u;
      nq[k] = len[k] ? ((st[k] + len[k] + 7) / 8 - a0[k] / 8) : 0u;
      seg[k] = (const uint4 *)(part + t * 2 * C3_TILE) + a0[k] / 8;
      maxq = max(maxq, nq[k]);
    }
#pragma unroll
    for (int d = WAVE / 2; d > 0; d >>= 1) maxq = max(maxq, (uint32_t)__shfl_xor((int)maxq, d, WAVE));
    for (uint32_t q0 = 0; q0 < maxq; q0 += Q) {
      uint4 v[K][Q];
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int qq = 0; qq < Q; ++qq)
          if (q0 + qq < nq[k]) v[k][qq] = seg[k][q0 + qq];
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int qq = 0; qq < Q; ++qq) {
          if (q0 + qq >= nq[k]) continue;
          const uint32_t b = a0[k] + 8 * (q0 + qq);  // element index of v.x's low half
          const uint32_t words[4] = {v[k][qq].x, v[k][qq].y, v[k][qq].z, v[k][qq].w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t idx = b + e;
            if (idx >= st[k] && idx < st[k] + len[k])
              atomicAdd(&bins[lds_slot((words[e >> 1] >> (16 * (e & 1))) & 0xFFFF)], 1u);
          }
        }
    }
  }
  __syncthreads();
  const int64_t lim = min((int64_t)C2_BW, hist_len - hist_base);
  for (int i = threadIdx.x; i < lim; i += C2_HBLOCK) {
    const uint32_t v = bins[lds_slot(i)];
    if (u.exclusive)
      hist[hist_base + i] = v;
    else if (v)
      atomicAdd(&hist[hist_base + i], v);
  }
}

template <bool F32>
static bool chain2_single_pass(Session *s, const C2Cols<F32> &c0, uint32_t *h_in,
                               uint32_t *h_out, unsigned long long *d_loops, int p1) {
  C2Cols<F32> c = c0;
  c.ntiles = (c.n + C3_TILE - 1) / C3_TILE;
  const int nr = 2 * c.nb;
  static bool attr_set = false;
  if (!attr_set) {
    for (const void *f : {(const void *)k_c3_bucket<1, 1>, (const void *)k_c3_bucket<2, 1>,
                          (const void *)k_c3_bucket<4, 1>, (const void *)k_c3_bucket<1, 2>,
                          (const void *)k_c3_bucket<2, 2>, (const void *)k_c3_bucket<4, 2>})
      HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * C2_BW));
    attr_set = true;
  }
  const int max_units = (2 * nr + 1 + 255) / 256 * 256;  // runs + splits, whole XCD waves
  BufPtr part = s->alloc(2 * 2 * C3_TILE * c.ntiles);
  BufPtr meta = s->alloc(4 * nr * c.ntiles), meta_t = s->alloc(4 * nr * c.ntiles);
  BufPtr acc = s->alloc(8 * nr + 16 + 4 * nr + sizeof(C3Unit) * max_units);
  unsigned long long *run_total = (unsigned long long *)acc->p;
  int32_t *nunits = (int32_t *)(run_total + nr);
  int32_t *split = nunits + 4;
  C3Unit *units = (C3Unit *)(split + nr);
  HIP_CHECK(hipMemsetAsync(acc->p, 0, 8 * nr + 16, s->stream));
  if (p1 == 1 || p1 == 2) {
    KernelTimer kt(s, "c4_partition", (F32 ? 12.0 : 20.0) * c.n);
    if (p1 == 1)
      launch_c4<F32, 512>(s, c, (uint16_t *)part->p, (uint32_t *)meta->p, d_loops);
    else
      launch_c4<F32, 1024>(s, c, (uint16_t *)part->p, (uint32_t *)meta->p, d_loops);
  } else {
    KernelTimer kt(s, "c3_partition", (F32 ? 12.0 : 20.0) * c.n);
    hipLaunchKernelGGL(k_c3_partition<F32>, dim3((unsigned)c.ntiles), dim3(C3_BLOCK), 0,
                       s->stream, c, (uint16_t *)part->p, (uint32_t *)meta->p, d_loops,
                       (int64_t)0);
    KERNEL_CHECK();
  }
  {
    KernelTimer kt(s, "c3_transpose", 8.0 * nr * c.ntiles);
    hipLaunchKernelGGL(k_c3_transpose, dim3((unsigned)((c.ntiles + C3_TT - 1) / C3_TT), (nr + 31) / 32),
                       dim3(256), 0, s->stream, (const uint32_t *)meta->p, (uint32_t *)meta_t->p,
                       c.ntiles, nr, run_total);
    KERNEL_CHECK();
  }
  hipLaunchKernelGGL(k_c3_units, dim3(1), dim3(C3_UBLOCK), 0, s->stream,
                     (const unsigned long long *)run_total, nr, c.ntiles, units, nunits, split);
  KERNEL_CHECK();
  hipLaunchKernelGGL(k_c3_zero, dim3(4, nr), dim3(256), 0, s->stream, (const int32_t *)split, c.nb,
                     h_in, h_out);
  KERNEL_CHECK();
  {
    KernelTimer kt(s, "c3_bucket_hist", 4.0 * c.n);
    // P3 shape (tiles per lane, pieces per step); CAPF_P3="k,q" overrides
    int pk = 1, pq = 2;
    if (const char *e = getenv("CAPF_P3")) sscanf(e, "%d,%d", &pk, &pq);
    auto kern = k_c3_bucket<1, 2>;
    if (pk == 1 && pq == 1) kern = k_c3_bucket<1, 1>;
    if (pk == 2 && pq == 1) kern = k_c3_bucket<2, 1>;
    if (pk == 4 && pq == 1) kern = k_c3_bucket<4, 1>;
    if (pk == 2 && pq == 2) kern = k_c3_bucket<2, 2>;
    if (pk == 4 && pq == 2) kern = k_c3_bucket<4, 2>;
    hipLaunchKernelGGL(kern, dim3((unsigned)max_units), dim3(C2_HBLOCK), 4 * C2_BW,
                       s->stream, (const C3Unit *)units, (const int32_t *)nunits,
                       (const uint16_t *)part->p, (const uint32_t *)meta_t->p, c.ntiles, c.nb,
                       h_in, h_out, c.hist_len);
    KERNEL_CHECK();
  }
  return true;
}

template <bool F32>
static bool chain2_run(Session *s, const ColView *cols, int64_t n, int64_t lo, int64_t hi,
                       uint32_t *h_in, uint32_t *h_out, unsigned long long *d_loops) {
  const int kbits = chain2_hist_bits(hi - lo + 1);
  const int64_t hlen = int64_t(1) << kbits;
  const int nb = (int)(hlen / C2_BW);
  static bool attr_set = false;
  if (!attr_set) {
    HIP_CHECK(hipFuncSetAttribute((const void *)k_c2_bucket,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 4 * C2_BW));
    attr_set = true;
  }
  C2Cols<F32> c;
  c.u1 = cols[0].data;
  c.v1 = cols[1].data;
  c.u2 = cols[2].data;
  c.v2 = cols[3].data;
  c.bu1 = F32 ? cols[0].base : 0;
  c.bv1 = F32 ? cols[1].base : 0;
  c.bu2 = F32 ? cols[2].base : 0;
  c.bv2 = F32 ? cols[3].base : 0;
  c.n = n;
  c.lo = lo;
  c.hi = hi;
  c.nb = nb;
  c.ntiles = (n + C2_TILE - 1) / C2_TILE;
  c.mix = node_mix_for(kbits);
  c.hist_len = hlen;
  // single-pass P1 forms: "c4" (default, 512 threads) | "c4w" (1024) | "single" (c3);
  // "twopass": P1 count + scan + P2 scatter
  const char *variant = getenv("CAPF_C2");
  if (!variant || strcmp(variant, "twopass") != 0) {
    const int p1 = !variant || strcmp(variant, "c4w") == 0 ? 2 : strcmp(variant, "c4") == 0 ? 1 : 0;
    return chain2_single_pass(s, c, h_in, h_out, d_loops, p1);
  }
  const int nr = 2 * nb;
  const int64_t nruns = (int64_t)nr * c.ntiles;
  HIP_CHECK(hipMemsetAsync(h_in, 0, 4 * hlen, s->stream));  // chunks of a split run add atomically
  HIP_CHECK(hipMemsetAsync(h_out, 0, 4 * hlen, s->stream));
  BufPtr counts = s->alloc(4 * nruns), offs = s->alloc(4 * nruns);
  BufPtr acc = s->alloc(8 * (nr + 3));  // [1..nr+1] run starts, [nr+2] total
  uint32_t *d_total = (uint32_t *)((int64_t *)acc->p + nr + 2);
  {
    KernelTimer kt(s, "c2_count", (F32 ? 8.0 : 16.0) * n);
    hipLaunchKernelGGL(k_c2_count<F32>, dim3((unsigned)c.ntiles), dim3(C2_BLOCK), 0, s->stream, c,
                       (uint32_t *)counts->p, d_loops);
    KERNEL_CHECK();
  }
  exclusive_scan_u32_async(s, (const uint32_t *)counts->p, (uint32_t *)offs->p, nruns, d_total);
  hipLaunchKernelGGL(k_run_starts, dim3((nr + 1 + 255) / 256), dim3(256), 0, s->stream,
                     (const uint32_t *)offs->p, c.ntiles, nr, d_total, (int64_t *)acc->p + 1);
  KERNEL_CHECK();
  std::vector<int64_t> hbuf(nr + 2);
  HIP_CHECK(hipMemcpyAsync(hbuf.data(), acc->p, 8 * (nr + 2), hipMemcpyDeviceToHost, s->stream));
  s->sync();
  const int64_t *starts = hbuf.data() + 1;
  const int64_t total = starts[nr];
  BufPtr part = s->alloc(2 * std::max<int64_t>(total, 8) + 16);
  {
    KernelTimer kt(s, "c2_scatter", (F32 ? 8.0 : 16.0) * n + 2.0 * total);
    hipLaunchKernelGGL(k_c2_scatter<F32>, dim3((unsigned)c.ntiles), dim3(C2_SBLOCK), 0, s->stream, c,
                       (const uint32_t *)offs->p, (uint16_t *)part->p);
    KERNEL_CHECK();
  }
  const int64_t target = std::max<int64_t>(total / (4 * 256), 1 << 16);  // ~4 chunks per CU
  std::vector<C2Chunk> chunks;
  for (int k = 0; k < nr; ++k) {
    const int64_t b0 = starts[k], b1 = starts[k + 1];
    if (b1 <= b0) continue;
    const int64_t nch = (b1 - b0 + target - 1) / target;
    for (int64_t q = 0; q < nch; ++q) {
      C2Chunk ch;
      ch.begin = b0 + (b1 - b0) * q / nch;
      ch.end = b0 + (b1 - b0) * (q + 1) / nch;
      ch.hist_base = (int64_t)(k % nb) * C2_BW;
      ch.exclusive = nch == 1;
      ch.side = k / nb;
      chunks.push_back(ch);
    }
  }
  if (!chunks.empty()) {
    BufPtr dch = s->alloc(sizeof(C2Chunk) * chunks.size());
    HIP_CHECK(hipMemcpyAsync(dch->p, chunks.data(), sizeof(C2Chunk) * chunks.size(),
                             hipMemcpyHostToDevice, s->stream));
    KernelTimer kt(s, "c2_bucket_hist", 2.0 * total);
    hipLaunchKernelGGL(k_c2_bucket, dim3((unsigned)chunks.size()), dim3(C2_HBLOCK), 4 * C2_BW,
                       s->stream, (const C2Chunk *)dch->p, (const uint16_t *)part->p, h_in,
                       h_out, hlen);
    KERNEL_CHECK();
    s->sync();  // the host chunk vector must outlive the pageable copy
  }
  return true;
}

int chain2_hist_bits(int64_t len) {
  int k = C2_BITS;
  while (k < 62 && (int64_t(1) << k) < len) ++k;
  return k;
}

int64_t chain2_hist_len(int64_t len) { return int64_t(1) << chain2_hist_bits(len); }

// cols = {start(r1), end(r1), start(r2), end(r2)}: non-null INTEGER columns,
// all plain or all FOR32.  h_in / h_out hold chain2_hist_len(hi − lo + 1)
// counters each, indexed by node_mix(id − lo); every counter is written (no
// memset needed).  The self-loop count is added to *d_loops (device).
// Returns false — before launching anything — if the shape is outside this
// kernel's limits (the caller falls back to k_chain2_hist).
bool chain2_partitioned(Session *s, const ColView *cols, int64_t n, int64_t lo, int64_t hi,
                        uint32_t *h_in, uint32_t *h_out, unsigned long long *d_loops) {
  const int64_t len = hi - lo + 1;
  if (len <= 0 || n <= 0) return false;
  const int64_t nb = chain2_hist_len(len) / C2_BW;
  if (2 * nb + 1 > C2_MAX_RUNS) return false;  // + the dummy run
  if (n >= (int64_t(1) << 31)) return false;  // 2·n keys must fit the uint32 scan
  int nf = 0;
  for (int i = 0; i < 4; ++i) {
    if (cols[i].valid || !cols[i].data) return false;
    if ((uintptr_t)cols[i].data & 15) return false;  // 16-B vector loads
    nf += cols[i].enc == ENC_FOR32;
  }
  if (nf == 4) return chain2_run<true>(s, cols, n, lo, hi, h_in, h_out, d_loops);
  if (nf == 0) return chain2_run<false>(s, cols, n, lo, hi, h_in, h_out, d_loops);
  return false;
}

}  // namespace capf
